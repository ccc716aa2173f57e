#!/bin/bash
# A/B of libwost builds on chosen scenarios: AB_ONLY=a,b [AB_COMPAT=fixed] tools/ab_libs.sh lib1.so lib2.so ...
# (runs on the GPU box; each library twice, alternating). lib.so:VAR=VAL[,VAR=VAL] sets
# environment variables for that library's runs.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for rep in 1 2; do
  for arg in "$@"; do
    lib="${arg%%:*}"; extra=""; [ "$arg" != "$lib" ] && extra="${arg#*:}"
    echo "== $arg rep $rep"
    env ${extra//,/ } WOST_LIB="$PWD/$lib" timeout -k 10 300 python tools/scenario_bench.py --reps 2 --compat "${AB_COMPAT:-reference}" \
      --only "${AB_ONLY:-dcr_dipole,variable_coefficients}" 2>&1 | grep -v JSON || exit $?
  done
done
