#!/bin/bash
# Round 6, session 2: A/B of the round-5 library (abtest/r05, a worktree of e9f4c23) against
# this round's (adaptive dequeues, launch statistics, options): every scenario, interleaved
# twice; this round's with the round-5 queue shape forced; PMC instruction counts of C4.
O=gpurun_out/r06s2
source "$(dirname "$0")/common.sh"
export TMPDIR=/tmp
step r05_a 400 python -u abtest/r05/tools/scenario_bench.py --reps 3
step r06_a 400 python -u tools/scenario_bench.py --reps 3
step r05_b 400 python -u abtest/r05/tools/scenario_bench.py --reps 3
step r06_b 400 python -u tools/scenario_bench.py --reps 3
step r06_noadapt 400 python -u tools/scenario_bench.py --reps 3 --opt adaptive_chunk=0
step r06_chunk0_0 400 python -u tools/scenario_bench.py --reps 3 --opt chunk0=0
P="--output-format csv"
step pmc_r05 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD $P -d $O/pmc_r05 -o run -- python3 abtest/r05/tools/scenario_bench.py --only dcr_dipole,poisson_square --reps 1
step pmc_r06 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD $P -d $O/pmc_r06 -o run -- python3 tools/scenario_bench.py --only dcr_dipole,poisson_square --reps 1
cat $O/status.txt
