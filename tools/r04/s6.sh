#!/bin/bash
# Round 4, session 6: the whole GPU test suite and smoke at HEAD.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r04s6
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/gputests.log 2>&1
echo "gputests rc=$?" | tee -a $O/status.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
echo "smoke rc=$?" | tee -a $O/status.txt
tail -3 $O/gputests.log
