#!/bin/bash
# Round 6, session 40: one copy for the points and the first batch's block ranges; the waves'
# records reduced by an extra workgroup. Tests touching every solve path, C2/C4 bench lines.
O=gpurun_out/r06s40
source "$(dirname "$0")/common.sh"
step tests 600 python -u -m pytest tests/test_gpu_queue.py tests/test_gpu_parity.py tests/test_gpu_race.py tests/test_gpu_multisource.py tests/test_gpu_c5.py tests/test_gpu_distributed.py tests/test_gpu_fixed.py -x -q --timeout 300 --timeout-method thread
step bench_c2 300 python -u bench.py --workload poisson_square --steps 20 --warmup 5 --no-cpu --no-rho
step bench_c2b 300 python -u bench.py --workload poisson_square --steps 20 --warmup 5 --no-cpu --no-rho
step bench_c4 300 python -u bench.py --steps 20 --warmup 5 --no-cpu --no-rho
tail -2 $O/tests.log
grep -o '"value": [0-9.e+]*' $O/bench_c2.log $O/bench_c2b.log $O/bench_c4.log
grep -o '"host_breakdown": {[^}]*' $O/bench_c2.log | cut -c1-400
cat $O/status.txt
