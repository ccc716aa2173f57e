#!/bin/bash
# A/B of libwost builds: tools/ab_bench.sh lib1.so lib2.so ... (runs on the GPU box)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for lib in "$@"; do
  for rep in 1 2; do
    echo "== $lib rep $rep"
    WOST_LIB="$PWD/$lib" timeout -k 10 300 python tools/scenario_bench.py --reps 2 --only dcr_dipole,variable_coefficients,laplace_square,poisson_square 2>&1 | grep -v JSON || exit $?
  done
done
