#!/bin/bash
# Round 4 end-of-round session: the bits of HEAD against the 6-wave register budget
# (tools/ab_bitwise.py), the GPU suite and smoke, the bench-command profiles (C4, C3, C5)
# and the default bench line with its CPU and rho_a legs.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r04final
mkdir -p $O
L=dcrmontecarlo_amd/libwost.so
timeout -k 10 400 python tools/ab_bitwise.py $L:WOST_JIT_WAVES=6 $L > $O/bitwise_w6_vs_head.log 2>&1
echo "bitwise rc=$?" | tee -a $O/status.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/gputests.log 2>&1
echo "gputests rc=$?" | tee -a $O/status.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
echo "smoke rc=$?" | tee -a $O/status.txt
bash tools/r04/profile_bench.sh dcr_dipole 20 5 > $O/prof_c4.log 2>&1
echo "prof c4 rc=$?" | tee -a $O/status.txt
bash tools/r04/profile_bench.sh variable_coefficients 20 5 > $O/prof_c3.log 2>&1
echo "prof c3 rc=$?" | tee -a $O/status.txt
timeout -k 10 400 python3 bench.py > $O/bench_c4_full.log 2>&1
echo "bench c4 rc=$?" | tee -a $O/status.txt
timeout -k 10 400 python3 bench.py --workload wenner_topography --steps 3 --warmup 1 > $O/bench_c5_full.log 2>&1
echo "bench c5 rc=$?" | tee -a $O/status.txt
timeout -k 10 300 python3 bench.py --workload variable_coefficients > $O/bench_c3_full.log 2>&1
echo "bench c3 rc=$?" | tee -a $O/status.txt
tail -3 $O/gputests.log
