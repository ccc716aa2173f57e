#!/bin/bash
# Round 5, session 1: where the device's C5 walks leave the reference's.
# The device's trigonometry vs the host C library, and the C5 replay with return_history
# under the default kernels and with the device library's sinf/cosf (WOST_EXP_FLAGS=128).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r05s1
mkdir -p $O
python tools/r05/trig_inputs.py $O/trig_in.bin && \
timeout -k 10 60 tools/r05/trig_probe $O/trig_in.bin $O/trig_out.bin > $O/trig.log 2>&1
echo "trig rc=$?" >> $O/status.txt
timeout -k 10 300 python -u tools/r05/c5_hist_dump.py $O/hist_f0.npz > $O/hist_f0.log 2>&1
echo "hist f0 rc=$?" >> $O/status.txt
WOST_EXP_FLAGS=128 timeout -k 10 300 python -u tools/r05/c5_hist_dump.py $O/hist_f128.npz > $O/hist_f128.log 2>&1
echo "hist f128 rc=$?" >> $O/status.txt
timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu --no-rho > $O/bench_c4.log 2>&1
echo "bench c4 rc=$?" >> $O/status.txt
cat $O/status.txt $O/hist_f0.log $O/hist_f128.log
