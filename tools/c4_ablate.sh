#!/bin/bash
# C4 step cost split by ablation switches (timing only: they change the walks).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for f in ${C4_FLAGS:-0 4 8 16 32 4096}; do
  WOST_EXP_FLAGS=$f timeout -k 10 120 python tools/scenario_bench.py --only dcr_dipole --reps 2 2>&1 | grep -v JSON | sed "s/^/flags $f: /"
done
