#!/bin/bash
# C5 (wenner_topography) walk-kernel counters: stats, instruction mix, waits, lane
# utilisation; one counter group per rocprofv3 run.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
SC="${1:-wenner_topography}"
O="$R/gpurun_out/prof_$SC"
mkdir -p "$O"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
CMD="$R/tools/scenario_bench.py --only $SC --reps 1"
bash tools/gpu_session.sh \
  "${SC}_stats|240|rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o run -- python3 $CMD" \
  "${SC}_sq1|240|rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d $O/pmc_sq1 -o run -- python3 $CMD" \
  "${SC}_sq2|240|rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_SALU SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE --output-format csv -d $O/pmc_sq2 -o run -- python3 $CMD" \
  "${SC}_util|240|rocprofv3 --pmc SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU --output-format csv -d $O/pmc_util -o run -- python3 $CMD"
