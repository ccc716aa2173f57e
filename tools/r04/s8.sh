#!/bin/bash
# Round 4, session 8: 6 vs 7 waves per SIMD for the scan kernels (WOST_JIT_WAVES), alternated
# four times on one box, then the bench line both ways.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r04s8
mkdir -p $O
for i in 1 2 3 4; do
  for w in 6 7; do
    WOST_JIT_WAVES=$w timeout -k 10 300 python tools/scenario_bench.py \
        --only dcr_dipole,variable_coefficients,laplace_square,notebook_dcr,poisson_square,manufactured_polynomial \
        --reps 2 > $O/w${w}_$i.log 2>&1
    echo "w$w run $i rc=$?" >> $O/status.txt
  done
done
for w in 6 7 6 7; do
  WOST_JIT_WAVES=$w timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu --no-rho >> $O/bench_w$w.log 2>&1
  echo "bench w$w rc=$?" >> $O/status.txt
done
cat $O/status.txt
