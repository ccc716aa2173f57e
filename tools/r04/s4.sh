#!/bin/bash
# Round 4, session 4: bench-reproducible profiles at HEAD for C4 (the bench workload),
# C3 and C5, then the full bench line.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
bash tools/r04/profile_bench.sh dcr_dipole 20 5 && \
bash tools/r04/profile_bench.sh variable_coefficients 20 5 && \
bash tools/r04/profile_bench.sh wenner_topography 2 1 --no-bruteforce && \
timeout -k 10 400 python3 bench.py > gpurun_out/r04prof/bench_full.log 2>&1
echo "session rc=$?"
