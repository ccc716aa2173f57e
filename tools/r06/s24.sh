#!/bin/bash
# Round 6, session 24: every handle compile in a helper again (no lone in-process route);
# race tests, the C5 cold survey twice, cold first solves, bench lines (C4 full, C2, C5).
O=gpurun_out/r06s24
source "$(dirname "$0")/common.sh"
step race 300 python -u -m pytest tests/test_gpu_race.py tests/test_gpu_multisource.py -x -q --timeout 200 --timeout-method thread
step cold_survey_a 300 python -u tools/r06/cold_survey.py 1
step cold_survey_b 300 python -u tools/r06/cold_survey.py 1
for sc in "poisson_square 64 10000" "variable_coefficients 256 100000" "dcr_dipole 48 1000000" "wenner_topography 256 2000"; do
  set -- $sc
  step cold_${1}_race 120 python -u tools/r06/cold_first_solve.py $1 $2 $3 1
  step cold_${1}_wait 120 python -u tools/r06/cold_first_solve.py $1 $2 $3 0
done
step bench_c4 300 python -u bench.py --steps 20 --warmup 5
step bench_c2 300 python -u bench.py --workload poisson_square --steps 20 --warmup 5 --no-cpu --no-rho
step bench_c5 400 python -u bench.py --workload wenner_topography --steps 3 --warmup 2 --no-cpu --no-rho
tail -3 $O/race.log
for f in $O/cold_survey_*; do echo "$f $(grep -o '"survey0_ms": [0-9.]*' $f)"; done
cat $O/status.txt
