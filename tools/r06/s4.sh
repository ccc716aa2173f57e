#!/bin/bash
# Round 6, session 4: the completion-rate dequeue floor capped by the share; no wave state in the tree kernels and the launch
# statistics behind the queue head: queue tests, then A/B against round 5 on every scenario.
O=gpurun_out/r06s4
source "$(dirname "$0")/common.sh"
export TMPDIR=/tmp
step gputests_queue 400 python -u -m pytest -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_queue.py
step r05_a 400 python -u abtest/r05/tools/scenario_bench.py --reps 3
step r06_a 400 python -u tools/scenario_bench.py --reps 3
step r05_b 400 python -u abtest/r05/tools/scenario_bench.py --reps 3
step r06_b 400 python -u tools/scenario_bench.py --reps 3
step r06_chunk0_0 400 python -u tools/scenario_bench.py --reps 3 --opt chunk0=0
step bench_c2 300 python bench.py --workload poisson_square --no-cpu --no-rho --steps 30 --warmup 3
step bench_c4 300 python bench.py --no-cpu --no-rho --steps 20 --warmup 3
cat $O/status.txt
