#!/bin/bash
# Round 4, session 5: PC sampling (rocprofv3 beta, stochastic) of the C4 and C5 walk
# kernels with their code objects kept for offline disassembly; then the single-launch
# C5 counters at HEAD (tools/c5_profile.sh).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
bash tools/r04/pcsample.sh dcr_dipole c4
rc=$?
echo "c4 pcsample rc=$rc"
if [ $rc -lt 124 ]; then
    bash tools/r04/pcsample.sh wenner_topography c5
    rc=$?
    echo "c5 pcsample rc=$rc"
fi
if [ $rc -lt 124 ]; then
    bash tools/c5_profile.sh wenner_topography > gpurun_out/c5_profile_session.log 2>&1
    echo "c5 profile rc=$?"
fi
