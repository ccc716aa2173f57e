#!/bin/bash
# Round 4, session 25: the silhouette visit's per-child update as selects
# (WOST_JIT_TREE_SELECT_UPDATE=1) against the branches -- bits, C5 rates.
# (Not adopted: the select variant and its knob were not kept; profiles/r04_ab/c5_select_update_ab.log.)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r04s25
mkdir -p $O
L=dcrmontecarlo_amd/libwost.so
timeout -k 10 300 python tools/ab_bitwise.py $L $L:WOST_JIT_TREE_SELECT_UPDATE=1 > $O/bitwise.log 2>&1
rc=$?; echo "bitwise rc=$rc" | tee -a $O/status.txt; tail -1 $O/bitwise.log; [ $rc -ne 0 ] && exit $rc
run() {
  local lab=$1; shift
  env "$@" timeout -k 10 200 python tools/scenario_bench.py --only wenner_topography,wenner_topography_physical --reps 2 > $O/$lab.log 2>&1
  local rc=$?; echo "$lab rc=$rc" >> $O/status.txt; grep -v JSON $O/$lab.log | awk -v l=$lab '{print l, $1, $7}'
  return $rc
}
for i in 1 2 3; do
  run base_$i || exit 1
  run sel_$i WOST_JIT_TREE_SELECT_UPDATE=1 || exit 1
done
