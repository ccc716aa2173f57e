#!/bin/bash
# Round 6 end (second pass, part B: the bench lines of the same commit): rocprofv3 of exactly the code that ships (the commit in $O/commit.txt):
# the bench commands of C4 (the headline), C2 and C3 -- their kernel-trace --stats
# summaries and PMC passes, one counter group per run -- and the C5 tree kernel's single
# launch (tools/scenario_bench.py, the bench's speedup_vs_bruteforce sample); then the
# default bench line, the C2/C3/C5 bench lines and the scenario table. Each step has its own time limit; a crash or timeout ends the session.
O=gpurun_out/r06prof6b
source "$(dirname "$0")/common.sh"
export TMPDIR=/tmp
git_rev="$(cat tools/r06/COMMIT 2>/dev/null || echo unknown)"
echo "$git_rev" > $O/commit.txt
step bench_c4_plain 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu --no-rho --workload dcr_dipole
step bench_default 600 python3 bench.py
step bench_c2 400 python3 bench.py --workload poisson_square
step bench_c3 400 python3 bench.py --workload variable_coefficients
step bench_c5 600 python3 bench.py --workload wenner_topography --steps 3 --warmup 1
step scenarios 400 python3 tools/scenario_bench.py
cat $O/status.txt
