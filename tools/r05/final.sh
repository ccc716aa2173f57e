#!/bin/bash
# Round 5 end-of-round session: the GPU suite and smoke, the bench-command profiles (C4, C3,
# C5 survey, C2) and the single-launch C5 counters, the default bench lines, and the
# launcher paths at N = 1. Each GPU step under its own limit; stops at a crash or timeout.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r05final
mkdir -p $O
step() {   # name limit command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > $O/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc" | tee -a $O/status.txt
  [ $rc -ge 124 ] && exit $rc
  return 0
}
step gputests 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step prof_c4 900 bash tools/r05/profile_bench.sh dcr_dipole 20 5
step prof_c3 900 bash tools/r05/profile_bench.sh variable_coefficients 20 5
step prof_c5 900 bash tools/r05/profile_bench.sh wenner_topography 2 1 --no-bruteforce
step prof_c2 600 bash tools/r05/profile_bench.sh poisson_square 50 5
step prof_c5_single 600 bash tools/c5_profile.sh wenner_topography
step bench_c4_full 400 python3 bench.py
step bench_c5_full 600 python3 bench.py --workload wenner_topography --steps 3 --warmup 1
step bench_c3_full 300 python3 bench.py --workload variable_coefficients
step bench_c2_full 300 python3 bench.py --workload poisson_square --steps 50 --warmup 5
step bench_torchrun_n1 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
    --master-port 29533 bench.py --gpus 1 --steps 5 --warmup 2 --no-cpu --no-rho
WOST_BENCH_FORCE_COMM=1 step bench_forcecomm_n1 300 python3 bench.py --gpus 1 --steps 5 --warmup 2 --no-cpu --no-rho
# --gpus 2 on a one-GPU box must fail clearly (rank 1 has no device) and stop rank 0
timeout -k 10 180 python3 bench.py --gpus 2 --steps 2 --warmup 1 --no-cpu --no-rho > $O/bench_gpus2_on_one_gpu.log 2>&1
echo "gpus2 on one gpu rc=$? (expected nonzero, not 124/137)" | tee -a $O/status.txt
tail -3 $O/gputests.log
cat $O/status.txt
