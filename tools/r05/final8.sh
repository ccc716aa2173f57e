#!/bin/bash
# Round 5 end, eighth pass (the chunk rate floor): the whole GPU suite (with the queue-shape tests) and smoke on the
# final code.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r05final8
mkdir -p $O
step() {   # name limit command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > $O/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc" | tee -a $O/status.txt
  [ $rc -ge 124 ] && exit $rc
  return 0
}
step gputests_queue 300 python -u -m pytest -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_queue.py
step gputests 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
tail -3 $O/gputests.log
cat $O/status.txt
