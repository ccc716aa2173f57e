#!/bin/bash
# A/B: walk terminations batched with the refills (ab/libwost_term.so) vs refills alone batched (ab/libwost_refill.so)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python tools/ab_bitwise.py ab/libwost_refill.so ab/libwost_term.so > gpurun_out/ab_term_bits.log 2>&1 || exit $?
AB_ONLY=dcr_dipole,variable_coefficients,wenner_topography,laplace_square,notebook_dcr timeout -k 10 900 \
  bash tools/ab_libs.sh ab/libwost_refill.so ab/libwost_term.so ab/libwost_term.so:WOST_JIT_REFILL_MIN=8 > gpurun_out/ab_term_time.log 2>&1 || exit $?
