#!/bin/bash
# End-of-round measurement on the GPU box: every scenario (reference and fixed
# estimators), then the profile session (bench line, rocprofv3 stats, PMC passes).
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
bash tools/gpu_session.sh \
  "scen|400|python tools/scenario_bench.py --reps 2" \
  "scen_fixed|300|python tools/scenario_bench.py --reps 2 --compat fixed" && bash tools/profile_session.sh
