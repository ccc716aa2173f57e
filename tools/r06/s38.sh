#!/bin/bash
# Round 6, session 38: ~2 short walks per lane for the grid: queue tests, the C2 bench line,
# the scenario table, C2-size probes.
O=gpurun_out/r06s38
source "$(dirname "$0")/common.sh"
step tests 400 python -u -m pytest tests/test_gpu_queue.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread
step bench_c2 300 python -u bench.py --workload poisson_square --steps 20 --warmup 5 --no-cpu --no-rho
step p005 120 python3 tools/scenario_bench.py --only poisson_square --reps 9 --scale 0.05
step l005 120 python3 tools/scenario_bench.py --only laplace_square --reps 9 --scale 0.05
step p02 120 python3 tools/scenario_bench.py --only poisson_square --reps 9 --scale 0.2
step scenarios 400 python3 tools/scenario_bench.py
tail -2 $O/tests.log
grep -o '"value": [0-9.e+]*' $O/bench_c2.log
grep -h "steps/s" $O/p005.log $O/l005.log $O/p02.log
head -8 $O/scenarios.log
cat $O/status.txt
