#!/bin/bash
# Round 6, session 33: the static first chunk for short walks (all of a launch's walks when at
# most 6 per lane, else 256): queue and parity tests, the C2 bench line, the scenario table.
O=gpurun_out/r06s33
source "$(dirname "$0")/common.sh"
step tests 500 python -u -m pytest tests/test_gpu_queue.py tests/test_gpu_parity.py tests/test_gpu_race.py tests/test_gpu_multisource.py -x -q --timeout 300 --timeout-method thread
step bench_c2 300 python -u bench.py --workload poisson_square --steps 20 --warmup 5 --no-cpu --no-rho
step bench_c4 300 python -u bench.py --steps 20 --warmup 5 --no-cpu --no-rho
step scenarios 400 python3 tools/scenario_bench.py
tail -3 $O/tests.log
grep -o '"value": [0-9.e+]*' $O/bench_c2.log $O/bench_c4.log
head -9 $O/scenarios.log
cat $O/status.txt
