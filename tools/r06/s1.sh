#!/bin/bash
# Round 6, session 1: the launch shape as a function of the call (adaptive dequeues),
# launch statistics, the options API; queue tests first, then every scenario and the bench lines.
O=gpurun_out/r06s1
source "$(dirname "$0")/common.sh"
step gputests_queue 400 python -u -m pytest -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_queue.py
step scenarios 400 python -u tools/scenario_bench.py --reps 2
step bench_c4 300 python bench.py --no-cpu --no-rho --steps 20 --warmup 3
step bench_c2 300 python bench.py --workload poisson_square --no-cpu --no-rho --steps 30 --warmup 3
step bench_c3 300 python bench.py --workload variable_coefficients --no-cpu --no-rho --steps 20 --warmup 3
step bench_c5 400 python bench.py --workload wenner_topography --steps 3 --warmup 1 --no-cpu --no-rho
step gputests_opts 600 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_c5.py tests/test_segment_tree.py
cat $O/status.txt
