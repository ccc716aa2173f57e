#!/bin/bash
# Round 4, session 15: the C5 tree kernel's knobs re-swept with the walk pools on
# (leaf size, refill batch, hand-out threshold, tree batch), alternated with the defaults.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r04s15
mkdir -p $O
run() {  # label, env...
  local lab=$1; shift
  env "$@" timeout -k 10 200 python tools/scenario_bench.py --only wenner_topography,wenner_topography_physical --reps 2 > $O/$lab.log 2>&1
  local rc=$?; echo "$lab rc=$rc" >> $O/status.txt; grep -v JSON $O/$lab.log | awk -v l=$lab '{print l, $1, $7}'
  return $rc
}
run base1 || exit 1
run leaf4 WOST_TREE_LEAF=4 || exit 1
run leaf6 WOST_TREE_LEAF=6 || exit 1
run leaf12 WOST_TREE_LEAF=12 || exit 1
run leaf16 WOST_TREE_LEAF=16 || exit 1
run base2 || exit 1
run refill2 WOST_JIT_REFILL_MIN=2 || exit 1
run refill8 WOST_JIT_REFILL_MIN=8 || exit 1
run refill16 WOST_JIT_REFILL_MIN=16 || exit 1
run share16 WOST_JIT_TREE_SHARE=16 || exit 1
run share48 WOST_JIT_TREE_SHARE=48 || exit 1
run base3 || exit 1
run batch2 WOST_JIT_TREE_BATCH=2 || exit 1
run nopool WOST_TREE_POOL=0 || exit 1
run sharemin2 WOST_JIT_TREE_SHARE_MIN=2 || exit 1
run base4 || exit 1
cat $O/status.txt
