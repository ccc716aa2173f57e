#!/bin/bash
# Round 4, session 16: refill batch x walk pools, and the pools' near-wave count and
# margin for both C5 variants (scenario_bench, alternated).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r04s16
mkdir -p $O
run() {  # label, env...
  local lab=$1; shift
  env "$@" timeout -k 10 200 python tools/scenario_bench.py --only wenner_topography,wenner_topography_physical --reps 2 > $O/$lab.log 2>&1
  local rc=$?; echo "$lab rc=$rc" >> $O/status.txt; grep -v JSON $O/$lab.log | awk -v l=$lab '{print l, $1, $7}'
  return $rc
}
for i in 1 2; do
  run base_$i || exit 1
  run nopool_$i WOST_TREE_POOL=0 || exit 1
  run r1_$i WOST_JIT_REFILL_MIN=1 || exit 1
  run r2_$i WOST_JIT_REFILL_MIN=2 || exit 1
  run r3_$i WOST_JIT_REFILL_MIN=3 || exit 1
  run r2nopool_$i WOST_JIT_REFILL_MIN=2 WOST_TREE_POOL=0 || exit 1
  run r2nw3_$i WOST_JIT_REFILL_MIN=2 WOST_POOL_NEAR_WAVES=3 || exit 1
  run r2nw4_$i WOST_JIT_REFILL_MIN=2 WOST_POOL_NEAR_WAVES=4 || exit 1
  run r2near03_$i WOST_JIT_REFILL_MIN=2 WOST_POOL_NEAR=0.03 || exit 1
  run r2near30_$i WOST_JIT_REFILL_MIN=2 WOST_POOL_NEAR=0.3 || exit 1
done
cat $O/status.txt
