#!/bin/bash
# Round 5, session 2: correctly rounded walk directions (sincos_rn) and host atan2f segment
# angles. C5 replay agreement with the new default and with the hardware trig (A/B flag
# 131072), the trig's rate cost on every scenario, then the whole GPU suite and smoke.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r05s2
mkdir -p $O
timeout -k 10 300 python -u tools/r05/c5_hist_dump.py $O/hist_exact.npz > $O/hist_exact.log 2>&1
echo "hist exact rc=$?" >> $O/status.txt
WOST_EXP_FLAGS=131072 timeout -k 10 300 python -u tools/r05/c5_hist_dump.py $O/hist_fast.npz > $O/hist_fast.log 2>&1
echo "hist fast rc=$?" >> $O/status.txt
AB_ONLY=dcr_dipole,variable_coefficients,wenner_topography,laplace_square,poisson_square,notebook_dcr,manufactured_polynomial \
  timeout -k 10 900 bash tools/ab_flags.sh 0 131072 0 131072 > $O/ab_trig.log 2>&1
echo "ab trig rc=$?" >> $O/status.txt
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > $O/gputests.log 2>&1
echo "gputests rc=$?" >> $O/status.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
echo "smoke rc=$?" >> $O/status.txt
cat $O/status.txt $O/hist_exact.log $O/hist_fast.log
tail -3 $O/gputests.log
