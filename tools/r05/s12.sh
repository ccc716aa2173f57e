#!/bin/bash
# Round 5, session 12: the work queue's static first fill (chunk0 = 64 walks per wave) and
# 64-walk minimum dequeues, against round 4's queue (WOST_CHUNK0=0 WOST_CHUNK_MIN=1):
# the GPU suite first (every kernel's walks go through the queue), then alternating
# bench lines for C2, C4, C3 and the scenario bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r05s12
mkdir -p $O
step() {   # name limit command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" >> $O/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc" | tee -a $O/status.txt
  [ $rc -ge 124 ] && exit $rc
  return 0
}
step gputests 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
for V in "0 1" "64 64" "64 256" "0 1" "64 64" "64 256"; do
  set -- $V
  export WOST_CHUNK0=$1 WOST_CHUNK_MIN=$2
  for W in poisson_square dcr_dipole variable_coefficients; do
    echo "== WOST_CHUNK0=$1 WOST_CHUNK_MIN=$2 $W" >> $O/queue_ab.log
    step queue_ab 300 python bench.py --workload $W --no-cpu --no-rho --steps 20 --warmup 3
  done
  echo "== WOST_CHUNK0=$1 WOST_CHUNK_MIN=$2 scenarios" >> $O/scen_ab.log
  step scen_ab 400 python -u tools/scenario_bench.py --reps 2
done
unset WOST_CHUNK0 WOST_CHUNK_MIN
cat $O/status.txt
