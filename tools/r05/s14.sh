#!/bin/bash
# Round 5, session 14: the solve's host path (pinned staging of the small copies, the queue
# head reset by the block reduce, one wait for the last batch) and the queue's adaptive
# chunk floor: the GPU suite, C2 / C4 / C3 bench lines, the scenario bench, the C2 HIP trace.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r05s14
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
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
for r in 1 2; do
  for W in poisson_square dcr_dipole variable_coefficients; do
    step bench_$W 300 python bench.py --workload $W --no-cpu --no-rho --steps 30 --warmup 3
  done
done
WOST_BENCH_FORCE_COMM=1 step bench_forcecomm 300 python3 bench.py --gpus 1 --steps 5 --warmup 2 --no-cpu --no-rho
step scen 400 python -u tools/scenario_bench.py --reps 2
export TMPDIR=/tmp
step c2_hiptrace 300 rocprofv3 --hip-trace --kernel-trace --memory-copy-trace --stats --output-format csv \
  -d $O/c2_hiptrace -o run -- python3 bench.py --workload poisson_square --no-cpu --no-rho --steps 30 --warmup 3
cat $O/status.txt
