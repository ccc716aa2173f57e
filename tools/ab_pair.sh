#!/bin/bash
# Alternating walk-rate A/B of two libwost builds on $AB_ONLY, $AB_REPS rounds (GPU box).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for rep in $(seq 1 ${AB_REPS:-3}); do
  for lib in "$@"; do
    WOST_LIB="$PWD/$lib" timeout -k 10 300 python tools/scenario_bench.py --reps 2 --only "${AB_ONLY:-wenner_topography}" 2>&1 \
      | grep -v JSON | sed "s|^|$lib: |" || exit $?
  done
done
