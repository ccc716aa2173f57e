#!/bin/bash
# Round 4, session 13: walk pools with the near walks taken by the workgroup's first
# wave(s) (WOST_POOL_NEAR_WAVES) -- bits against WOST_TREE_POOL=0, then C5 rates.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r04s13
mkdir -p $O
L=dcrmontecarlo_amd/libwost.so
timeout -k 10 240 python tools/ab_bitwise.py $L:WOST_TREE_POOL=0 $L > $O/bitwise.log 2>&1
rc=$?; echo "bitwise rc=$rc" | tee -a $O/status.txt; tail -1 $O/bitwise.log
[ $rc -ge 124 ] && exit $rc
run() {  # label, env...
  local lab=$1; shift
  env "$@" timeout -k 10 200 python tools/scenario_bench.py --only wenner_topography,wenner_topography_physical --reps 2 > $O/$lab.log 2>&1
  local rc=$?; echo "$lab rc=$rc" >> $O/status.txt; grep -v JSON $O/$lab.log | sed "s|^|$lab |"
  return $rc
}
for i in 1 2; do
  run off_$i WOST_TREE_POOL=0 || exit 1
  run nw1_$i WOST_POOL_NEAR_WAVES=1 || exit 1
  run nw2_$i WOST_POOL_NEAR_WAVES=2 || exit 1
  run nw0_$i WOST_POOL_NEAR_WAVES=0 || exit 1
done
run nw1_near10 WOST_POOL_NEAR_WAVES=1 WOST_POOL_NEAR=0.1 || exit 1
run nw2_near10 WOST_POOL_NEAR_WAVES=2 WOST_POOL_NEAR=0.1 || exit 1
run nw3_near10 WOST_POOL_NEAR_WAVES=3 WOST_POOL_NEAR=0.1 || exit 1
run nw1_near01 WOST_POOL_NEAR_WAVES=1 WOST_POOL_NEAR=0.01 || exit 1
run nw1_s256 WOST_POOL_NEAR_WAVES=1 WOST_POOL_SLOTS=256 || exit 1
cat $O/status.txt
