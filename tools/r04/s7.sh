#!/bin/bash
# Round 4, session 7: occupancy of the scan kernels with larger workgroups (WOST_WALK_BLOCK:
# one LDS copy of the sampler / G_norm tables per workgroup, so 7-8 waves per SIMD fit;
# 256-thread workgroups are LDS-bound at 7). Timing only (the bits do not depend on it).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r04s7
mkdir -p $O
run() {
    local tag=$1; shift
    env "$@" timeout -k 10 300 python tools/scenario_bench.py \
        --only dcr_dipole,variable_coefficients,laplace_square,notebook_dcr,poisson_square --reps 2 > $O/$tag.log 2>&1
    echo "$tag rc=$? $*" >> $O/status.txt
}
run base
run b512w6 WOST_WALK_BLOCK=512 WOST_JIT_WAVES=6
run b512w7 WOST_WALK_BLOCK=512 WOST_JIT_WAVES=7
run b512w8 WOST_WALK_BLOCK=512 WOST_JIT_WAVES=8
run b1024w8 WOST_WALK_BLOCK=1024 WOST_JIT_WAVES=8
run b256w7 WOST_JIT_WAVES=7
run base2
cat $O/status.txt
for t in base b512w6 b512w7 b512w8 b1024w8 b256w7 base2; do echo "== $t"; grep -h "steps/s" $O/$t.log | awk '{print "  ", $1, $7, $NF}'; done
