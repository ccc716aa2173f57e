#!/bin/bash
# Round 6, session 13: the whole GPU suite and smoke after the round's main changes.
O=gpurun_out/r06s13
source "$(dirname "$0")/common.sh"
step gputests 1100 python -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
tail -3 $O/gputests.log
cat $O/status.txt
