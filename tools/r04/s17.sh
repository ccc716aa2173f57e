#!/bin/bash
# Round 4, session 17: the new multi-source pool test, then the tree staging level and
# waves per SIMD re-checked with the walk pools on (C5 scenario_bench, alternated).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r04s17
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_c5.py -m gpu -x -q -k pools --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc" | tee -a $O/status.txt; tail -1 $O/tests.log; [ $rc -ge 124 ] && exit $rc
run() {  # label, env...
  local lab=$1; shift
  env "$@" timeout -k 10 200 python tools/scenario_bench.py --only wenner_topography,wenner_topography_physical --reps 2 > $O/$lab.log 2>&1
  local rc=$?; echo "$lab rc=$rc" >> $O/status.txt; grep -v JSON $O/$lab.log | awk -v l=$lab '{print l, $1, $7}'
  return $rc
}
for i in 1 2; do
  run base_$i || exit 1
  run lds1_$i WOST_TREE_LDS=1 || exit 1
  run lds1b1024_$i WOST_TREE_LDS=1 WOST_TREE_LDS_BLOCK=1024 || exit 1
  run lds0_$i WOST_TREE_LDS=0 || exit 1
  run w5lds1_$i WOST_TREE_LDS=1 WOST_JIT_WAVES=5 WOST_TREE_LDS_BLOCK=640 || exit 1
done
cat $O/status.txt
