#!/bin/bash
# Round 4, session 19: two walks per lane (WOST_JIT_X2=1, walk_body_x2)
# against one -- bits, then the scan scenarios' rates at 5 and 6 waves per SIMD,
# alternated, then the bench line both ways.
set -o pipefail
# (Not adopted: the two-walk kernel exists only in commit e65523c; profiles/r04_ab/two_walks_per_lane_ab.log.)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r04s19
mkdir -p $O
L=dcrmontecarlo_amd/libwost.so
timeout -k 10 300 python tools/ab_bitwise.py $L $L:WOST_JIT_X2=1 > $O/bitwise.log 2>&1
rc=$?; echo "bitwise rc=$rc" | tee -a $O/status.txt; cat $O/bitwise.log | cut -c1-160; [ $rc -ne 0 ] && exit $rc
run() {  # label, env...
  local lab=$1; shift
  env "$@" timeout -k 10 300 python tools/scenario_bench.py --only dcr_dipole,notebook_dcr,variable_coefficients,laplace_square,poisson_square --reps 2 > $O/$lab.log 2>&1
  local rc=$?; echo "$lab rc=$rc" >> $O/status.txt; grep -v JSON $O/$lab.log | awk -v l=$lab '{print l, $1, $7, "grid", $(NF-3)}'
  return $rc
}
for i in 1 2; do
  run x1_$i || exit 1
  run x2w5_$i WOST_JIT_X2=1 WOST_JIT_WAVES=5 || exit 1
  run x2w6_$i WOST_JIT_X2=1 WOST_JIT_WAVES=6 || exit 1
  run x2w7_$i WOST_JIT_X2=1 WOST_JIT_WAVES=7 || exit 1
done
for x in 0 1 0 1; do
  WOST_JIT_X2=$x WOST_JIT_WAVES=$([ $x = 1 ] && echo 6 || echo 7) timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu --no-rho >> $O/bench_x$x.log 2>&1
  echo "bench x$x rc=$?" >> $O/status.txt
done
grep -h '"value"' $O/bench_x0.log | cut -c1-70
grep -h '"value"' $O/bench_x1.log | cut -c1-70
cat $O/status.txt
