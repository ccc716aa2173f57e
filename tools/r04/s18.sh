#!/bin/bash
# Round 4, session 18: the whole GPU suite and smoke at HEAD (after the oracle's thread
# default and the new pool tests).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r04s18
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/gputests.log 2>&1
rc=$?; echo "gputests rc=$rc" | tee -a $O/status.txt; [ $rc -ge 124 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
echo "smoke rc=$?" | tee -a $O/status.txt
tail -2 $O/gputests.log; tail -3 $O/smoke.log
