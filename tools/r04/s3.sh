#!/bin/bash
# Round 4, session 3: Philox one step ahead (WOST_JIT_PHILOX_AHEAD 0-3), timing A/B on
# every scenario, then the bits of variant 1..3 against 0 (tools/ab_bitwise.py).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r04s3
mkdir -p $O
L=dcrmontecarlo_amd/libwost.so
for v in 0 1 2 3 0 1 2 3; do
    WOST_JIT_PHILOX_AHEAD=$v timeout -k 10 240 python tools/scenario_bench.py \
        --only dcr_dipole,variable_coefficients,laplace_square,notebook_dcr,wenner_topography --reps 2 \
        >> $O/ahead_$v.log 2>&1
    echo "ahead $v rc=$?" >> $O/status.txt
done
timeout -k 10 400 python tools/ab_bitwise.py $L $L:WOST_JIT_PHILOX_AHEAD=1 > $O/bitwise_1.log 2>&1
echo "bitwise 1 rc=$?" >> $O/status.txt
timeout -k 10 400 python tools/ab_bitwise.py $L $L:WOST_JIT_PHILOX_AHEAD=2 > $O/bitwise_2.log 2>&1
echo "bitwise 2 rc=$?" >> $O/status.txt
cat $O/status.txt
for v in 0 1 2 3; do echo "== $v"; grep -h "steps/s" $O/ahead_$v.log; done
