#!/bin/bash
# Round 4, session 22: the tree queries' loop counters (study build) with the silhouette
# query's wave-level visit issues (counter 15).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r04s22
mkdir -p $O
for sc in wenner_topography wenner_topography_physical; do
  WOST_TREE_ITER_STATS=1 timeout -k 10 200 python tools/scenario_bench.py --only $sc --reps 1 > $O/stats_$sc.log 2>&1
  echo "stats $sc rc=$?" >> $O/status.txt
  grep -E "tree_iter_stats|steps/s" $O/stats_$sc.log | cut -c1-250
done
cat $O/status.txt
