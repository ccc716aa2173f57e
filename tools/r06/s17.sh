#!/bin/bash
# Round 6, session 17: the precompiled kernel against the field-specialised one (a cold
# first solve without the hiprtc compile?), with the round's compile routing.
O=gpurun_out/r06s17
source "$(dirname "$0")/common.sh"
step precompiled 300 python -u tools/r06/precompiled_probe.py
cat $O/precompiled.log
cat $O/status.txt
