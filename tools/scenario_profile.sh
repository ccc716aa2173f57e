#!/bin/bash
# rocprofv3 stats + PMC passes of one scenario's walk kernel (tools/scenario_bench.py),
# one counter group per run, no tracing domains beside the counters. Counter groups
# that rocprofv3 --list-avail (gpurun_out/counters.txt, tools/box_info.sh) does not
# name are skipped.
# Usage (on the GPU box): tools/scenario_profile.sh <scenario> [extra scenario_bench args]
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
SC="$1"; shift
O="$R/gpurun_out/prof_$SC"
mkdir -p "$O"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
CMD="$R/tools/scenario_bench.py --only $SC --reps 1 $*"
AVAIL="$R/profiles/gfx950_counters.txt"
have() { [ -s "$AVAIL" ] && grep -q "\b$1\b" "$AVAIL"; }
specs=(
  "${SC}_stats|240|rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o run -- python3 $CMD"
  "${SC}_sq1|240|rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d $O/pmc_sq1 -o run -- python3 $CMD"
  "${SC}_sq2|240|rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_SALU SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE --output-format csv -d $O/pmc_sq2 -o run -- python3 $CMD"
)
if have SQ_INSTS_VALU_TRANS_F32; then
  specs+=("${SC}_trans|240|rocprofv3 --pmc SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU --output-format csv -d $O/pmc_trans -o run -- python3 $CMD")
fi
if have TCC_HIT_sum && have TCP_TCC_READ_REQ_sum; then
  specs+=("${SC}_cache|240|rocprofv3 --pmc TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum --output-format csv -d $O/pmc_cache -o run -- python3 $CMD")
fi
"$R/tools/gpu_session.sh" "${specs[@]}"
