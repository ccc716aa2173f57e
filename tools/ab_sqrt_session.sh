#!/bin/bash
# round-2 session: sqrt_rn and -fno-slp-vectorize A/B (bits + time), VALU-utilisation counters
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python tools/ab_bitwise.py ab/libwost_old.so ab/libwost_cur.so > gpurun_out/ab_sqrt_slp_bits.log 2>&1 || exit $?
AB_ONLY=dcr_dipole,variable_coefficients,wenner_topography,laplace_square timeout -k 10 700 bash tools/ab_libs.sh ab/libwost_old.so ab/libwost_new.so ab/libwost_cur.so > gpurun_out/ab_sqrt_slp_time.log 2>&1 || exit $?
timeout -k 10 700 bash tools/pmc_util.sh || exit $?
