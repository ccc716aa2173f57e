#!/bin/bash
# Round 4, session 23: quad-cooperative ray visits (WOST_JIT_TREE_QUAD=1: one child test
# per lane, 16 visits per batch) against the per-lane visits -- bits, C5 tests, rates.
# (The quad variant exists only in commit c799ffa; profiles/r04_ab/c5_quad_ray_visits_ab.log.)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r04s23
mkdir -p $O
L=dcrmontecarlo_amd/libwost.so
timeout -k 10 300 python tools/ab_bitwise.py $L $L:WOST_JIT_TREE_QUAD=1 > $O/bitwise.log 2>&1
rc=$?; echo "bitwise rc=$rc" | tee -a $O/status.txt; tail -3 $O/bitwise.log | cut -c1-150; [ $rc -ne 0 ] && exit $rc
WOST_JIT_TREE_QUAD=1 timeout -k 10 500 python -u -m pytest tests/test_gpu_c5.py tests/test_gpu_long_polylines.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc" | tee -a $O/status.txt; tail -2 $O/tests.log; [ $rc -ge 124 ] && exit $rc
run() {  # label, env...
  local lab=$1; shift
  env "$@" timeout -k 10 200 python tools/scenario_bench.py --only wenner_topography,wenner_topography_physical --reps 2 > $O/$lab.log 2>&1
  local rc=$?; echo "$lab rc=$rc" >> $O/status.txt; grep -v JSON $O/$lab.log | awk -v l=$lab '{print l, $1, $7}'
  return $rc
}
for i in 1 2 3; do
  run base_$i || exit 1
  run quad_$i WOST_JIT_TREE_QUAD=1 || exit 1
done
WOST_JIT_TREE_QUAD=1 WOST_TREE_ITER_STATS=1 timeout -k 10 200 python tools/scenario_bench.py --only wenner_topography --reps 1 > $O/stats_quad.log 2>&1
grep tree_iter_stats $O/stats_quad.log
cat $O/status.txt
