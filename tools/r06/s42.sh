#!/bin/bash
# Round 6, session 42: the facade's solve passes plain addresses (host time per solve).
O=gpurun_out/r06s42
source "$(dirname "$0")/common.sh"
step tests 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_queue.py tests/test_gpu_race.py tests/test_gpu_callables.py -x -q --timeout 300 --timeout-method thread
step bench_c2 300 python -u bench.py --workload poisson_square --steps 20 --warmup 5 --no-cpu --no-rho
step bench_c2b 300 python -u bench.py --workload poisson_square --steps 20 --warmup 5 --no-cpu --no-rho
tail -2 $O/tests.log
grep -o '"value": [0-9.e+]*' $O/bench_c2.log $O/bench_c2b.log
grep -o '"solve_wall_ms": [0-9.]*, "libwost_span_ms": [0-9.]*' $O/bench_c2.log $O/bench_c2b.log
cat $O/status.txt
