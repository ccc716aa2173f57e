#!/bin/bash
# Round 5, session 13: the work queue's dynamic chunk after the static first fill:
# count / (4 waves) (default), the same on the rest (WOST_CHUNK_REST), a 64-walk floor,
# and round 4's queue (WOST_CHUNK0=0), on C2 (bench) and the scenario bench (C5, notebook).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r05s13
mkdir -p $O
step() {   # name limit command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" >> $O/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc" | tee -a $O/status.txt
  [ $rc -ge 124 ] && exit $rc
  return 0
}
for V in "64 1 -" "0 1 -" "64 64 -" "64 1 rest" "64 1 -" "0 1 -" "64 64 -" "64 1 rest"; do
  set -- $V
  export WOST_CHUNK0=$1 WOST_CHUNK_MIN=$2
  if [ "$3" = rest ]; then export WOST_CHUNK_REST=1; else unset WOST_CHUNK_REST; fi
  echo "== WOST_CHUNK0=$1 WOST_CHUNK_MIN=$2 $3 poisson_square" >> $O/queue_ab.log
  step queue_ab 300 python bench.py --workload poisson_square --no-cpu --no-rho --steps 30 --warmup 3
  echo "== WOST_CHUNK0=$1 WOST_CHUNK_MIN=$2 $3 scenarios" >> $O/scen_ab.log
  step scen_ab 400 python -u tools/scenario_bench.py --reps 2 --only notebook_dcr,wenner_topography,wenner_topography_physical,variable_coefficients,manufactured_polynomial
done
unset WOST_CHUNK0 WOST_CHUNK_MIN WOST_CHUNK_REST
export TMPDIR=/tmp
# where a C2 solve's host time goes: HIP API calls and copies around the kernels
step c2_hiptrace 300 rocprofv3 --hip-trace --kernel-trace --memory-copy-trace --stats --output-format csv \
  -d $O/c2_hiptrace -o run -- python3 bench.py --workload poisson_square --no-cpu --no-rho --steps 30 --warmup 3
cat $O/status.txt
