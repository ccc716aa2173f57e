#!/bin/bash
# A/B of the compiled-in polyline size limit (WOST_JIT_CONST_VERTICES): tools/ab_constverts.sh 16 40 64
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for v in "$@"; do
  echo "== WOST_JIT_CONST_VERTICES=$v"
  WOST_JIT_CONST_VERTICES=$v timeout -k 10 300 python tools/scenario_bench.py --reps 2 --only variable_coefficients,dcr_dipole,notebook_dcr 2>&1 | grep -v JSON || exit $?
done
