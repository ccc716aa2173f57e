#!/bin/bash
# C5 walk-kernel LDS counters with the tree's records staged in LDS (default) and without
# (WOST_TREE_LDS=0): bank conflicts, LDS instructions, waits.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/tree_lds_pmc
for v in 1 0; do
  WOST_TREE_LDS=$v timeout -k 10 200 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_LDS \
    --output-format csv -d gpurun_out/tree_lds_pmc/lds$v -o run -- python3 tools/scenario_bench.py --only wenner_topography --reps 1 \
    > gpurun_out/tree_lds_pmc/lds$v.log 2>&1 || exit $?
  grep wenner gpurun_out/tree_lds_pmc/lds$v.log | head -1
done
