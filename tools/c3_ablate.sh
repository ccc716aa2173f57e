#!/bin/bash
# C3 (variable_coefficients) step cost split by ablation switches (timing only: they
# change the walks): 4 no Philox, 8 no alpha(z), 16 no sigma', 32 no Neumann ray query,
# 65536 no silhouette query, 65568 neither Neumann query.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for f in ${C3_FLAGS:-0 4 8 16 32 65536 65568}; do
  WOST_EXP_FLAGS=$f timeout -k 10 120 python tools/scenario_bench.py --only variable_coefficients --reps 2 2>&1 | grep -v JSON | sed "s/^/flags $f: /"
done
