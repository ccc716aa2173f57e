#!/bin/bash
# Round 5, session 6: A/B of unit_direction's (n, y) table (WOST_EXP_FLAGS 2^29) -- bitwise on
# every scenario, then the rates, alternating.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r05s6
mkdir -p $O
L=dcrmontecarlo_amd/libwost.so
timeout -k 10 300 python -u tools/ab_bitwise.py $L "$L:WOST_EXP_FLAGS=536870912" > $O/bitwise_unit_tab.log 2>&1
echo "bitwise rc=$?" >> $O/status.txt
AB_ONLY=dcr_dipole,variable_coefficients,notebook_dcr,laplace_square,poisson_square \
  timeout -k 10 900 bash tools/ab_flags.sh 0 536870912 0 536870912 0 536870912 > $O/ab_unit_tab.log 2>&1
echo "ab rc=$?" >> $O/status.txt
cat $O/status.txt
