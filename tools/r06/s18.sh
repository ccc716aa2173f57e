#!/bin/bash
# Round 6, session 18: cold solves race the compile (jit_race): the race tests, the
# multi-source / C5 / queue / parity tests, the bench lines' cold blocks.
O=gpurun_out/r06s18
source "$(dirname "$0")/common.sh"
step race 300 python -u -m pytest tests/test_gpu_race.py -x -v -s --timeout 200 --timeout-method thread
step tests 500 python -u -m pytest tests/test_gpu_multisource.py tests/test_gpu_c5.py tests/test_gpu_queue.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread
step bench_c4 300 python -u bench.py --steps 10 --warmup 5 --no-cpu --no-rho
step bench_c2 300 python -u bench.py --workload poisson_square --steps 10 --warmup 5 --no-cpu --no-rho
step bench_c5 400 python -u bench.py --workload wenner_topography --steps 3 --warmup 2 --no-cpu --no-rho
tail -5 $O/race.log
tail -3 $O/tests.log
cat $O/status.txt
