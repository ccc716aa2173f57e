#!/bin/bash
# Round 6 end (second pass, part A: the profiles): rocprofv3 of exactly the code that ships (the commit in $O/commit.txt):
# the bench commands of C4 (the headline), C2 and C3 -- their kernel-trace --stats
# summaries and PMC passes, one counter group per run -- and the C5 tree kernel's single
# launch (tools/scenario_bench.py, the bench's speedup_vs_bruteforce sample); then the
# default bench line, the C2/C3/C5 bench lines and the scenario table. Each step has its own time limit; a crash or timeout ends the session.
O=gpurun_out/r06prof6a
source "$(dirname "$0")/common.sh"
export TMPDIR=/tmp
git_rev="$(cat tools/r06/COMMIT 2>/dev/null || echo unknown)"
echo "$git_rev" > $O/commit.txt
P="--output-format csv"
prof() {   # workload command...
  local W=$1; shift
  local D=$O/$W
  mkdir -p $D
  step ${W}_stats 400 rocprofv3 --kernel-trace --stats $P -d $D/stats -o run -- "$@"
  step ${W}_sq1 400 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES $P -d $D/pmc_sq1 -o run -- "$@"
  step ${W}_sq2 400 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_SALU SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE $P -d $D/pmc_sq2 -o run -- "$@"
  step ${W}_trans 400 rocprofv3 --pmc SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU $P -d $D/pmc_trans -o run -- "$@"
  step ${W}_util 400 rocprofv3 --pmc SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU $P -d $D/pmc_util -o run -- "$@"
  step ${W}_fetch 400 rocprofv3 --pmc FETCH_SIZE $P -d $D/pmc_fetch -o run -- "$@"
  step ${W}_write 400 rocprofv3 --pmc WRITE_SIZE $P -d $D/pmc_write -o run -- "$@"
}
prof dcr_dipole python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu --no-rho --workload dcr_dipole
prof poisson_square python3 bench.py --gpus 1 --steps 30 --warmup 3 --no-cpu --no-rho --workload poisson_square
prof variable_coefficients python3 bench.py --gpus 1 --steps 20 --warmup 3 --no-cpu --no-rho --workload variable_coefficients
prof wenner_topography_single python3 tools/scenario_bench.py --only wenner_topography --reps 1
cat $O/status.txt
