#!/bin/bash
# Round 6, session 43: the whole GPU suite and smoke at the final code (08ff289).
O=gpurun_out/r06s43
source "$(dirname "$0")/common.sh"
step gputests 1000 python -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread
step smoke 200 python -c "import __graft_entry__ as g; g.smoke()"
tail -3 $O/gputests.log
cat $O/status.txt
