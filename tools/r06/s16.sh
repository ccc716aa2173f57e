#!/bin/bash
# Round 6, session 16: survey kernels prepared from a thread pool (wost_prepare_sources). The multi-source and
# C5 GPU tests, the C5 survey's cold start with the helpers and in-process, the C5 and C4
# bench lines (cold numbers).
O=gpurun_out/r06s16
source "$(dirname "$0")/common.sh"
step tests 400 python -u -m pytest tests/test_gpu_multisource.py tests/test_gpu_c5.py tests/test_gpu_queue.py -x -v --timeout 200 --timeout-method thread
step cold_helper 300 python -u tools/r06/cold_survey.py 1
step cold_inproc 300 python -u tools/r06/cold_survey.py 0
step bench_c5 400 python -u bench.py --workload wenner_topography --steps 3 --warmup 1 --no-cpu --no-rho
step bench_c4 300 python -u bench.py --steps 10 --warmup 3 --no-cpu --no-rho
tail -3 $O/tests.log
cat $O/cold_helper.log $O/cold_inproc.log
cat $O/status.txt
