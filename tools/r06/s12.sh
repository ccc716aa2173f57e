#!/bin/bash
# Round 6, session 12: the longest walk from the wave records (no per-workgroup atomics in
# the block reduce of the scan kernels): queue tests, C2/C4 bench lines, scenarios vs round 5.
O=gpurun_out/r06s12
source "$(dirname "$0")/common.sh"
step gputests_queue 400 python -u -m pytest -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_queue.py
step bench_c4 300 python bench.py --no-cpu --no-rho --steps 20 --warmup 3
step bench_c2 300 python bench.py --workload poisson_square --no-cpu --no-rho --steps 30 --warmup 3
step r05_a 400 python -u abtest/r05/tools/scenario_bench.py --reps 3
step r06_a 400 python -u tools/scenario_bench.py --reps 3
step r05_b 400 python -u abtest/r05/tools/scenario_bench.py --reps 3
step r06_b 400 python -u tools/scenario_bench.py --reps 3
cat $O/status.txt
