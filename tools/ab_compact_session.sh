#!/bin/bash
# A/B: compiled-in Neumann ray scan in two passes (WOST_EXP_FLAGS=16384) vs the unrolled per-segment exact tests
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
L=ab/libwost_cmp.so
timeout -k 10 300 python tools/ab_bitwise.py "$L" "$L:WOST_EXP_FLAGS=16384" > gpurun_out/ab_compact_bits.log 2>&1 || exit $?
AB_ONLY=variable_coefficients,dcr_dipole,notebook_dcr timeout -k 10 600 bash tools/ab_libs.sh "$L" "$L:WOST_EXP_FLAGS=16384" > gpurun_out/ab_compact_time.log 2>&1 || exit $?
