#!/bin/bash
# Round 4 end-of-round session (after the walk pools): bits of HEAD against the pools
# off, the GPU suite and smoke, the bench-command profiles (C4, C3, C5 survey) and the
# single-launch C5 counters, the default bench lines, and the launcher paths at N = 1.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r04final2
mkdir -p $O
L=dcrmontecarlo_amd/libwost.so
timeout -k 10 400 python tools/ab_bitwise.py $L:WOST_TREE_POOL=0 $L > $O/bitwise_pools_off_vs_head.log 2>&1
rc=$?; echo "bitwise rc=$rc" | tee -a $O/status.txt; [ $rc -ge 124 ] && exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/gputests.log 2>&1
rc=$?; echo "gputests rc=$rc" | tee -a $O/status.txt; [ $rc -ge 124 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc" | tee -a $O/status.txt; [ $rc -ge 124 ] && exit $rc
bash tools/r04/profile_bench.sh dcr_dipole 20 5 > $O/prof_c4.log 2>&1
rc=$?; echo "prof c4 rc=$rc" | tee -a $O/status.txt; [ $rc -ge 124 ] && exit $rc
bash tools/r04/profile_bench.sh variable_coefficients 20 5 > $O/prof_c3.log 2>&1
rc=$?; echo "prof c3 rc=$rc" | tee -a $O/status.txt; [ $rc -ge 124 ] && exit $rc
bash tools/r04/profile_bench.sh wenner_topography 2 1 --no-bruteforce > $O/prof_c5.log 2>&1
rc=$?; echo "prof c5 rc=$rc" | tee -a $O/status.txt; [ $rc -ge 124 ] && exit $rc
bash tools/c5_profile.sh wenner_topography > $O/prof_c5_single.log 2>&1
rc=$?; echo "prof c5 single rc=$rc" | tee -a $O/status.txt; [ $rc -ge 124 ] && exit $rc
timeout -k 10 400 python3 bench.py > $O/bench_c4_full.log 2>&1
rc=$?; echo "bench c4 rc=$rc" | tee -a $O/status.txt; [ $rc -ge 124 ] && exit $rc
timeout -k 10 400 python3 bench.py --workload wenner_topography --steps 3 --warmup 1 > $O/bench_c5_full.log 2>&1
rc=$?; echo "bench c5 rc=$rc" | tee -a $O/status.txt; [ $rc -ge 124 ] && exit $rc
timeout -k 10 300 python3 bench.py --workload variable_coefficients > $O/bench_c3_full.log 2>&1
rc=$?; echo "bench c3 rc=$rc" | tee -a $O/status.txt; [ $rc -ge 124 ] && exit $rc
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 \
    bench.py --gpus 1 --steps 5 --warmup 2 --no-cpu --no-rho > $O/bench_torchrun_n1.log 2>&1
rc=$?; echo "torchrun n1 rc=$rc" | tee -a $O/status.txt; [ $rc -ge 124 ] && exit $rc
WOST_BENCH_FORCE_COMM=1 timeout -k 10 300 python3 bench.py --gpus 1 --steps 5 --warmup 2 --no-cpu --no-rho > $O/bench_forcecomm_n1.log 2>&1
rc=$?; echo "forcecomm n1 rc=$rc" | tee -a $O/status.txt
# --gpus 2 on a one-GPU box must fail clearly (rank 1 has no device) and stop rank 0
timeout -k 10 180 python3 bench.py --gpus 2 --steps 2 --warmup 1 --no-cpu --no-rho > $O/bench_gpus2_on_one_gpu.log 2>&1
echo "gpus2 on one gpu rc=$? (expected nonzero, not 124/137)" | tee -a $O/status.txt
tail -3 $O/gputests.log
cat $O/status.txt
