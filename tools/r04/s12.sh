#!/bin/bash
# Round 4, session 12: walk pools in the tree kernels (wost_walk.h): bits against
# WOST_TREE_POOL=0, the C5 GPU tests, then C5 rates with and without the pools and
# with other near margins / pool sizes, alternated on one box.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r04s12
mkdir -p $O
L=dcrmontecarlo_amd/libwost.so
timeout -k 10 240 python tools/ab_bitwise.py $L:WOST_TREE_POOL=0 $L > $O/bitwise.log 2>&1
rc=$?; echo "bitwise rc=$rc" | tee -a $O/status.txt; tail -3 $O/bitwise.log
[ $rc -ge 124 ] && exit $rc
timeout -k 10 400 python -u -m pytest tests/test_gpu_c5.py tests/test_gpu_c5_reference.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc" | tee -a $O/status.txt; tail -2 $O/tests.log
[ $rc -ge 124 ] && exit $rc
run() {  # label, env...
  local lab=$1; shift
  env "$@" timeout -k 10 200 python tools/scenario_bench.py --only wenner_topography,wenner_topography_physical --reps 2 > $O/$lab.log 2>&1
  local rc=$?; echo "$lab rc=$rc" >> $O/status.txt; grep -v JSON $O/$lab.log | sed "s|^|$lab |"
  return $rc
}
for i in 1 2 3; do
  run off_$i WOST_TREE_POOL=0 || exit 1
  run on_$i WOST_TREE_POOL=1 || exit 1
done
run near01 WOST_POOL_NEAR=0.01 || exit 1
run near003 WOST_POOL_NEAR=0.003 || exit 1
run near10 WOST_POOL_NEAR=0.1 || exit 1
run slots64 WOST_POOL_SLOTS=64 || exit 1
run slots256 WOST_POOL_SLOTS=256 || exit 1
run push4 WOST_JIT_POOL_MIN_PUSH=4 || exit 1
for p in 0 1; do
  WOST_TREE_POOL=$p timeout -k 10 300 python3 bench.py --workload wenner_topography --steps 2 --warmup 1 --no-cpu --no-rho > $O/bench_c5_pool$p.log 2>&1
  echo "bench pool$p rc=$?" | tee -a $O/status.txt
done
cat $O/status.txt
