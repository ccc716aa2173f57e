#!/bin/bash
# C5 time split by ablation / A/B switches (flags 32 / 65536 change the walks: timing only).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for f in ${C5_FLAGS:-0 32 65536 65568}; do
  WOST_EXP_FLAGS=$f timeout -k 10 120 python tools/scenario_bench.py --only wenner_topography --reps 2 2>&1 | grep -v JSON | sed "s/^/flags $f: /"
done
