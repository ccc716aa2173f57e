#!/bin/bash
# Round 6, session 10: literal multi-source kernels (param_sources an option) compiled
# concurrently: multi-source and C5 tests, the C5 bench line (cold first survey, warm rate).
O=gpurun_out/r06s10
source "$(dirname "$0")/common.sh"
step gputests_ms 900 python -u -m pytest -v -s --timeout 400 --timeout-method thread -m gpu tests/test_gpu_multisource.py tests/test_gpu_c5.py tests/test_gpu_c5_reference.py
step bench_c5 700 python bench.py --workload wenner_topography --steps 3 --warmup 1 --no-cpu
cat $O/status.txt
