#!/bin/bash
# Round 4, session 2: C5 tree-kernel occupancy A/B (timing only; every staging level
# gives the same bits). A = default (records + vertices in LDS, one 1024-thread
# workgroup per CU, 4 waves/SIMD, 101 VGPRs); B-E = records only in LDS, larger
# workgroups, two per CU, 5-6 waves/SIMD with fewer VGPRs (batch 2: 87 VGPRs).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r04s2
mkdir -p $O
run() {   # tag, env...
    local tag=$1; shift
    env "$@" timeout -k 10 240 python tools/scenario_bench.py --only wenner_topography,wenner_topography_physical --reps 3 \
        > $O/$tag.log 2>&1
    echo "$tag rc=$? $*" >> $O/status.txt
}
run A0
run B WOST_TREE_LDS=1 WOST_TREE_LDS_BLOCK=640 WOST_JIT_WAVES=5 WOST_JIT_TREE_BATCH=2
run C WOST_TREE_LDS=1 WOST_TREE_LDS_BLOCK=640 WOST_JIT_WAVES=5 WOST_JIT_TREE_BATCH=4
run D WOST_TREE_LDS=1 WOST_TREE_LDS_BLOCK=768 WOST_JIT_WAVES=6 WOST_JIT_TREE_BATCH=2
run E WOST_JIT_TREE_BATCH=2
run F WOST_TREE_LDS=1 WOST_TREE_LDS_BLOCK=512 WOST_JIT_WAVES=4 WOST_JIT_TREE_BATCH=4
run A1
cat $O/status.txt
grep -h "wenner" $O/*.log | head -40
