#!/bin/bash
# Round 4, session 5: the single-launch C5 counters at HEAD (tools/c5_profile.sh).
# (PC sampling is not run on this pool.)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
bash tools/c5_profile.sh wenner_topography > gpurun_out/c5_profile_session.log 2>&1
echo "c5 profile rc=$?"
