#!/bin/bash
# Measurement session B (GPU box): every scenario with the CPU oracle beside it, the
# compat="fixed" scenarios, the C4 bench under rocprofv3 (stats + PMC passes), and the
# C5 / C3 walk kernels' counters.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
bash tools/gpu_session.sh \
  "scen|600|python tools/scenario_bench.py --reps 2 --cpu --cpu-seconds 4" \
  "scen_fixed|300|python tools/scenario_bench.py --reps 2 --compat fixed" \
  && bash tools/profile_session.sh \
  && bash tools/c5_profile.sh wenner_topography \
  && bash tools/c5_profile.sh variable_coefficients
