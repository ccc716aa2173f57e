#!/bin/bash
# A/B of the AMDGPU scheduler strategy for the field-specialised kernels
# (WOST_JIT_SCHED, wost_jit.cpp): AB_ONLY=a,b tools/ab_sched.sh default max-ilp ... (GPU box)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for st in "$@"; do
  echo "== WOST_JIT_SCHED=$st"
  if [ "$st" = default ]; then unset WOST_JIT_SCHED; else export WOST_JIT_SCHED=$st; fi
  timeout -k 10 300 python tools/scenario_bench.py --reps 2 \
    --only "${AB_ONLY:-dcr_dipole,variable_coefficients,laplace_square,wenner_topography}" 2>&1 | grep -v JSON || exit $?
done
