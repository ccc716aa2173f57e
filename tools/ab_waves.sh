#!/bin/bash
# A/B of the field-specialised kernels' register budget (WOST_JIT_WAVES: waves per SIMD
# the launch bounds size registers for): AB_ONLY=a,b tools/ab_waves.sh 6 8 ... (GPU box)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for w in "$@"; do
  echo "== WOST_JIT_WAVES=$w"
  WOST_JIT_WAVES=$w timeout -k 10 200 python tools/scenario_bench.py --reps 2 --only "${AB_ONLY:-wenner_topography}" 2>&1 | grep -v JSON || exit $?
done
