#!/bin/bash
# Round 5, session 4: the walk step's dynamic VALU per phase (phase_dup.sh) for C4 and C3.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
timeout -k 10 900 bash tools/r05/phase_dup.sh dcr_dipole > gpurun_out/r05dup_c4.log 2>&1
echo "c4 rc=$?"
timeout -k 10 600 bash tools/r05/phase_dup.sh variable_coefficients > gpurun_out/r05dup_c3.log 2>&1
echo "c3 rc=$?"
