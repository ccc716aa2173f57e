#!/bin/bash
# Round 5, session 10: counters of the fused brute-force scan kernel (C5, set_segment_tree(-1))
# on one chip-filling launch: instruction mix, waits, lane utilisation, one group per run.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd "$R"
O="$R/gpurun_out/r05s10"
mkdir -p "$O"
export TMPDIR=/tmp
CMD="$R/tools/scenario_bench.py --scan --only wenner_topography --reps 1"
P="--output-format csv"
bash tools/gpu_session.sh \
  "scan_bench|300|python3 $CMD" \
  "scan_stats|300|rocprofv3 --kernel-trace --stats $P -d $O/stats -o run -- python3 $CMD" \
  "scan_sq1|300|rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES $P -d $O/pmc_sq1 -o run -- python3 $CMD" \
  "scan_sq2|300|rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_SALU SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH GRBM_GUI_ACTIVE $P -d $O/pmc_sq2 -o run -- python3 $CMD" \
  "scan_util|300|rocprofv3 --pmc SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU $P -d $O/pmc_util -o run -- python3 $CMD"
