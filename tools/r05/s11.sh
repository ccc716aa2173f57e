#!/bin/bash
# Round 5, session 11: the work queue's chunk at C2's BASELINE size (64 points x 10k walks,
# ~2.4 walks per lane): A/B of the minimum walks per dequeue (WOST_CHUNK_MIN; today
# count / (4 waves) = 19 walks, i.e. ~34k dequeues of one global counter per launch).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r05s11
mkdir -p $O
step() {   # name limit command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" >> $O/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc" | tee -a $O/status.txt
  [ $rc -ge 124 ] && exit $rc
  return 0
}
for C in 1 64 256 1024 1 64 256 1024; do
  echo "== WOST_CHUNK_MIN=$C" >> $O/c2_chunk.log
  export WOST_CHUNK_MIN=$C
  step c2_chunk 300 python bench.py --workload poisson_square --steps 50 --warmup 5 --no-cpu
done
unset WOST_CHUNK_MIN
cat $O/status.txt
