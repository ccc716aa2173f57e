#!/bin/bash
# Round 6, session 41: the whole GPU suite and smoke at the final code (feb6ae8).
O=gpurun_out/r06s41
source "$(dirname "$0")/common.sh"
step gputests 1000 python -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread
step smoke 200 python -c "import __graft_entry__ as g; g.smoke()"
tail -3 $O/gputests.log
cat $O/status.txt
