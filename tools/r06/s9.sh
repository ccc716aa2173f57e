#!/bin/bash
# Round 6, session 9: multi-source kernels reading their sources' parameters from the
# program buffer (one compile per survey instead of one per electrode group): the
# multi-source bit tests, the C5 reference tests, the C5 bench line (cold first survey).
O=gpurun_out/r06s9
source "$(dirname "$0")/common.sh"
step gputests_ms 900 python -u -m pytest -v -s --timeout 400 --timeout-method thread -m gpu tests/test_gpu_multisource.py tests/test_gpu_c5.py tests/test_gpu_c5_reference.py
step bench_c5 700 python bench.py --workload wenner_topography --steps 3 --warmup 1 --no-cpu
cat $O/status.txt
