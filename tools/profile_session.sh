#!/bin/bash
# Measurement session on the GPU box: the bench line, a rocprofv3 kernel-trace
# summary of the same bench command, and PMC passes (one counter group per
# run, no tracing domains beside them). Output under gpurun_out/prof/.
# Usage (via gpurun): tools/profile_session.sh [tag]
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/prof"
mkdir -p "$O"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
B="$R/bench.py"
S="$R/tools/gpu_session.sh"
PMC_ARGS="--steps 2 --warmup 1 --no-cpu --no-rho"
"$S" \
  "bench|300|python3 $B" \
  "stats|300|rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o run -- python3 $B --steps 4 --warmup 1 --no-cpu --no-rho" \
  "pmc_fetch|300|rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o run -- python3 $B $PMC_ARGS" \
  "pmc_write|300|rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o run -- python3 $B $PMC_ARGS" \
  "pmc_sq1|300|rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d $O/pmc_sq1 -o run -- python3 $B $PMC_ARGS" \
  "pmc_sq2|300|rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_SALU SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE --output-format csv -d $O/pmc_sq2 -o run -- python3 $B $PMC_ARGS" \
  "pmc_trans|300|rocprofv3 --pmc SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU --output-format csv -d $O/pmc_trans -o run -- python3 $B $PMC_ARGS"
