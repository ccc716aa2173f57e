#!/bin/bash
# round-2 session: sqrt_rn on top of -fno-slp-vectorize (WOST_EXP_FLAGS=2048 = sqrtf)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
AB_ONLY=dcr_dipole,variable_coefficients,wenner_topography,notebook_dcr timeout -k 10 800 bash tools/ab_libs.sh ab/libwost_cur.so ab/libwost_cur.so:WOST_EXP_FLAGS=2048 > gpurun_out/ab_sqrt2_time.log 2>&1 || exit $?
