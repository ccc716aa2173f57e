#!/bin/bash
# Round 4, session 21: the tree queries' loop counters (study build, WOST_TREE_ITER_STATS=1)
# on C5, and the shipped kernels with the (compiled-away) counter hooks against the
# previous library: bits and rates.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r04s21
mkdir -p $O
L=dcrmontecarlo_amd/libwost.so
timeout -k 10 300 python tools/ab_bitwise.py ablib/libwost_base.so $L > $O/bitwise.log 2>&1
rc=$?; echo "bitwise rc=$rc" | tee -a $O/status.txt; tail -1 $O/bitwise.log; [ $rc -ge 124 ] && exit $rc
for i in 1 2 3; do
  for lib in ablib/libwost_base.so $L; do
    WOST_LIB=$PWD/$lib timeout -k 10 200 python tools/scenario_bench.py --only wenner_topography,wenner_topography_physical --reps 2 > $O/rate_$(basename $lib .so)_$i.log 2>&1
    echo "rate $lib $i rc=$?" >> $O/status.txt
    grep -v JSON $O/rate_$(basename $lib .so)_$i.log | awk -v l=$(basename $lib .so)_$i '{print l, $1, $7}'
  done
done
for sc in wenner_topography wenner_topography_physical; do
  WOST_TREE_ITER_STATS=1 timeout -k 10 200 python tools/scenario_bench.py --only $sc --reps 1 > $O/stats_$sc.log 2>&1
  echo "stats $sc rc=$?" >> $O/status.txt
  grep -E "tree_iter_stats|steps/s" $O/stats_$sc.log | cut -c1-250
done
cat $O/status.txt
