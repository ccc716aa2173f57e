#!/bin/bash
# A/B of libwost builds on chosen scenarios: AB_ONLY=a,b [AB_COMPAT=fixed] tools/ab_libs.sh lib1.so lib2.so ...
# (runs on the GPU box; each library twice, alternating)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for rep in 1 2; do
  for lib in "$@"; do
    echo "== $lib rep $rep"
    WOST_LIB="$PWD/$lib" timeout -k 10 300 python tools/scenario_bench.py --reps 2 --compat "${AB_COMPAT:-reference}" \
      --only "${AB_ONLY:-dcr_dipole,variable_coefficients}" 2>&1 | grep -v JSON || exit $?
  done
done
