#!/bin/bash
# Round 5, session 20: every scenario with the round's last code (kernel walk-steps/s), and
# C5's brute-force scan kernel.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r05s20
mkdir -p $O
timeout -k 10 400 python -u tools/scenario_bench.py --reps 2 > $O/scenarios.log 2>&1 && \
timeout -k 10 300 python -u tools/scenario_bench.py --scan --reps 2 --only wenner_topography,wenner_topography_physical > $O/scan.log 2>&1
echo "rc=$?" | tee $O/status.txt
