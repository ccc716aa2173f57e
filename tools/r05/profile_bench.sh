#!/bin/bash
# Round 5: rocprofv3 of the exact bench.py command (as tools/r04/profile_bench.sh): the command alone (its JSON
# line: ms_per_step), its kernel-trace --stats summary, and PMC passes of the same
# command (one counter group per run, nothing traced beside them), for one workload.
# Usage (GPU box): tools/r05/profile_bench.sh <workload> <steps> <warmup> [extra bench args]
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd "$R"
W=$1; K=$2; WU=$3; shift 3
O="gpurun_out/r05prof/$W"
mkdir -p "$O"
export TMPDIR=/tmp
CMD="python3 bench.py --gpus 1 --steps $K --warmup $WU --no-cpu --no-rho --workload $W $*"
P="--output-format csv"
bash tools/gpu_session.sh \
  "${W}_bench|400|$CMD" \
  "${W}_stats|400|rocprofv3 --kernel-trace --stats $P -d $O/stats -o run -- $CMD" \
  "${W}_sq1|400|rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES $P -d $O/pmc_sq1 -o run -- $CMD" \
  "${W}_sq2|400|rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_SALU SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE $P -d $O/pmc_sq2 -o run -- $CMD" \
  "${W}_trans|400|rocprofv3 --pmc SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU $P -d $O/pmc_trans -o run -- $CMD" \
  "${W}_util|400|rocprofv3 --pmc SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU $P -d $O/pmc_util -o run -- $CMD" \
  "${W}_fetch|400|rocprofv3 --pmc FETCH_SIZE $P -d $O/pmc_fetch -o run -- $CMD" \
  "${W}_write|400|rocprofv3 --pmc WRITE_SIZE $P -d $O/pmc_write -o run -- $CMD"
