#!/bin/bash
# Round 5, session 16: the C5 survey (17 launches per field, 3 handle pairs) under the
# round-5 work queue: default, without the static first chunk (WOST_CHUNK0=0), and round
# 4's queue (WOST_CHUNK0=0 WOST_CHUNK_MIN=1), alternating; then C2 under the short-walk grid
# rule, its bench-command profile, and the GPU suite.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r05s16
mkdir -p $O
step() {   # name limit command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" >> $O/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc" | tee -a $O/status.txt
  [ $rc -ge 124 ] && exit $rc
  return 0
}
for V in "def" "0 -" "0 1" "def" "0 -" "0 1"; do
  unset WOST_CHUNK0 WOST_CHUNK_MIN
  set -- $V
  [ "$1" != def ] && export WOST_CHUNK0=$1
  [ -n "$2" ] && [ "$2" != - ] && export WOST_CHUNK_MIN=$2
  echo "== $V" >> $O/c5_queue.log
  step c5_queue 400 python bench.py --workload wenner_topography --steps 3 --warmup 1 --no-cpu --no-rho
done
unset WOST_CHUNK0 WOST_CHUNK_MIN
# the short-walk grid rule (fewer resident workgroups after a solve of < 32 steps per walk)
for r in 1 2; do step c2_grid 300 python bench.py --workload poisson_square --no-cpu --no-rho --steps 30 --warmup 3; done
step prof_c2 600 bash tools/r05/profile_bench.sh poisson_square 50 5
step gputests 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
cat $O/status.txt
