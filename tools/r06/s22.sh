#!/bin/bash
# Round 6, session 22: the queue tests (jit_race excluded from their option checks), the C5
# survey's cold start twice per route, the C5 bench line.
O=gpurun_out/r06s22
source "$(dirname "$0")/common.sh"
step queue 300 python -u -m pytest tests/test_gpu_queue.py -x -q --timeout 200 --timeout-method thread
step cold_helper_a 300 python -u tools/r06/cold_survey.py 1
step cold_helper_b 300 python -u tools/r06/cold_survey.py 1
step cold_inproc 300 python -u tools/r06/cold_survey.py 0
step bench_c5 400 python -u bench.py --workload wenner_topography --steps 3 --warmup 2 --no-cpu --no-rho
tail -3 $O/queue.log
cat $O/cold_*.log
grep -o '"cold": {[^}]*' $O/bench_c5.log
cat $O/status.txt
