#!/bin/bash
# A/B of the walk kernel's exact fast paths (WOST_EXP_FLAGS bit mask, see
# wost_jit.cpp exp_flags): tools/ab_flags.sh 0 1 2 3  (runs on the GPU box);
# AB_COMPAT=fixed and AB_ONLY=a,b select the estimator and the scenarios
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for f in "$@"; do
  echo "== WOST_EXP_FLAGS=$f"
  WOST_EXP_FLAGS=$f timeout -k 10 300 python tools/scenario_bench.py --reps 2 --compat "${AB_COMPAT:-reference}" \
    --only "${AB_ONLY:-dcr_dipole,variable_coefficients,laplace_square,poisson_square}" 2>&1 | grep -v JSON || exit $?
done
