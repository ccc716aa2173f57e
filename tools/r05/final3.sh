#!/bin/bash
# Round 5 end, third pass (the queue's static chunks only for short walks, the short-walk
# grid rule): GPU parity subsets and smoke, the four default bench lines, the C2 and C5
# bench-command profiles.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r05final3
mkdir -p $O
step() {   # name limit command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > $O/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc" | tee -a $O/status.txt
  [ $rc -ge 124 ] && exit $rc
  return 0
}
step gputests_sub 600 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_c5.py
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench_c4_full 400 python3 bench.py
step bench_c5_full 600 python3 bench.py --workload wenner_topography --steps 3 --warmup 1
step bench_c3_full 300 python3 bench.py --workload variable_coefficients
step bench_c2_full 300 python3 bench.py --workload poisson_square --steps 50 --warmup 5
step prof_c2 600 bash tools/r05/profile_bench.sh poisson_square 50 5
step prof_c5 900 bash tools/r05/profile_bench.sh wenner_topography 2 1 --no-bruteforce
cat $O/status.txt
