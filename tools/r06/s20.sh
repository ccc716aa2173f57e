#!/bin/bash
# Round 6, session 20: threaded sampler tables, their prefetch and the helper probe at wost_create; the race
# tests, the multi-source / parity tests, cold first solves phase by phase, bench lines.
O=gpurun_out/r06s20
source "$(dirname "$0")/common.sh"
step race 300 python -u -m pytest tests/test_gpu_race.py -x -v -s --timeout 200 --timeout-method thread
step tests 500 python -u -m pytest tests/test_gpu_multisource.py tests/test_gpu_parity.py tests/test_gpu_queue.py -x -q --timeout 300 --timeout-method thread
for sc in "poisson_square 64 10000" "variable_coefficients 256 100000" "dcr_dipole 48 1000000" "wenner_topography 256 2000"; do
  set -- $sc
  step cold_${1}_race 120 python -u tools/r06/cold_first_solve.py $1 $2 $3 1
  step cold_${1}_wait 120 python -u tools/r06/cold_first_solve.py $1 $2 $3 0
done
step bench_c4 300 python -u bench.py --steps 10 --warmup 5 --no-cpu --no-rho
step bench_c2 300 python -u bench.py --workload poisson_square --steps 10 --warmup 5 --no-cpu --no-rho
tail -12 $O/race.log
tail -3 $O/tests.log
cat $O/cold_*.log
cat $O/status.txt
