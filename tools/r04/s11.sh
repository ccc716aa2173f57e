#!/bin/bash
# Round 4, session 11: the field-specialised kernels without the staged copy of a short
# compiled-in Neumann polyline (C4: 20,512 -> 20,480 B per 256-thread workgroup, 7 -> 8
# workgroups per CU) against WOST_STAGE_NEUMANN=1 (staged as before): bits, then the rates
# alternated four times on one box, then the bench line both ways.
# (Not adopted: the knob and the unstaged variant were removed again; profiles/r04_ab/neumann_staging_ab.log.)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r04s11
mkdir -p $O
L=dcrmontecarlo_amd/libwost.so
timeout -k 10 400 python tools/ab_bitwise.py $L:WOST_STAGE_NEUMANN=1 $L > $O/bitwise.log 2>&1
echo "bitwise rc=$?" | tee -a $O/status.txt
tail -1 $O/bitwise.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fixed.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
echo "tests rc=$?" | tee -a $O/status.txt
tail -2 $O/tests.log
for i in 1 2 3 4; do
  for s in 1 0; do
    WOST_STAGE_NEUMANN=$s timeout -k 10 300 python tools/scenario_bench.py \
        --only dcr_dipole,notebook_dcr,variable_coefficients --reps 2 > $O/s${s}_$i.log 2>&1
    echo "stage$s run $i rc=$?" >> $O/status.txt
  done
done
for s in 1 0 1 0; do
  WOST_STAGE_NEUMANN=$s timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu --no-rho >> $O/bench_s$s.log 2>&1
  echo "bench s$s rc=$?" >> $O/status.txt
done
cat $O/status.txt
