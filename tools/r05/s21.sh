#!/bin/bash
# Round 5, session 21: the dynamic chunk's rate floor (at most ~40M dequeues per second at
# the previous solve's rate): every scenario, the four bench lines, the queue tests, smoke.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r05s21
mkdir -p $O
step() {   # name limit command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > $O/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc" | tee -a $O/status.txt
  [ $rc -ge 124 ] && exit $rc
  return 0
}
step scenarios 400 python -u tools/scenario_bench.py --reps 2
step bench_c4 300 python bench.py --no-cpu --no-rho --steps 20 --warmup 3
step bench_c3 300 python bench.py --workload variable_coefficients --no-cpu --no-rho --steps 20 --warmup 3
step bench_c2 300 python bench.py --workload poisson_square --no-cpu --no-rho --steps 30 --warmup 3
step bench_c5 400 python bench.py --workload wenner_topography --steps 3 --warmup 1 --no-cpu --no-rho
step gputests_queue 300 python -u -m pytest -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_queue.py tests/test_gpu_parity.py
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
cat $O/status.txt
