#!/bin/bash
# Round 4, session 14: poly_distance_axis (the Dirichlet distance of axis-parallel
# compiled-in polylines from the one segment a point is certainly nearest to) against
# WOST_JIT_AXIS_DISTANCE=0: bits, parity tests, then rates alternated, then the bench line.
# (Not adopted: the axis path and its knob were removed again; profiles/r04_ab/axis_distance_ab.log.)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r04s14
mkdir -p $O
L=dcrmontecarlo_amd/libwost.so
timeout -k 10 300 python tools/ab_bitwise.py $L:WOST_JIT_AXIS_DISTANCE=0 $L > $O/bitwise.log 2>&1
rc=$?; echo "bitwise rc=$rc" | tee -a $O/status.txt; tail -1 $O/bitwise.log
[ $rc -ge 124 ] && exit $rc
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc" | tee -a $O/status.txt; tail -1 $O/tests.log
[ $rc -ge 124 ] && exit $rc
for i in 1 2 3; do
  for a in 0 1; do
    WOST_JIT_AXIS_DISTANCE=$a timeout -k 10 300 python tools/scenario_bench.py \
        --only dcr_dipole,notebook_dcr,variable_coefficients,laplace_square,poisson_square,wenner_topography --reps 2 > $O/a${a}_$i.log 2>&1
    echo "axis$a run $i rc=$?" >> $O/status.txt
    grep -v JSON $O/a${a}_$i.log | awk -v l=a${a}_$i '{print l, $1, $7}'
  done
done
for a in 0 1 0 1; do
  WOST_JIT_AXIS_DISTANCE=$a timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu --no-rho >> $O/bench_a$a.log 2>&1
  echo "bench a$a rc=$?" >> $O/status.txt
done
grep -h '"value"' $O/bench_a0.log | cut -c1-80
grep -h '"value"' $O/bench_a1.log | cut -c1-80
cat $O/status.txt
