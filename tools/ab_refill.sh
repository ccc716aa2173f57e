#!/bin/bash
# A/B of the refill batch size (WOST_JIT_REFILL_MIN idle lanes per refill, wost_walk.h
# WOST_REFILL_MIN) on the field-specialised kernels, plus the bitwise check of the batched
# refill against refills every iteration. Runs on the GPU box.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
L=${AB_LIB:-dcrmontecarlo_amd/libwost.so}
timeout -k 10 300 python tools/ab_bitwise.py "$L:WOST_JIT_REFILL_MIN=1" "$L" > gpurun_out/ab_refill_bits.log 2>&1 || exit $?
AB_ONLY=${AB_ONLY:-dcr_dipole,variable_coefficients,wenner_topography,laplace_square,notebook_dcr} timeout -k 10 900 \
  bash tools/ab_libs.sh "$L:WOST_JIT_REFILL_MIN=1" "$L:WOST_JIT_REFILL_MIN=2" "$L" "$L:WOST_JIT_REFILL_MIN=8" > gpurun_out/ab_refill_time.log 2>&1 || exit $?
