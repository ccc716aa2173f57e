#!/bin/bash
# Round 5 end (sixth pass, the cap of 16 after long walks), part A: the GPU
# suite and smoke, the default bench lines of the four workloads, the launcher paths at N = 1.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r05final6
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
step bench_c4_full 400 python3 bench.py
step bench_c5_full 600 python3 bench.py --workload wenner_topography --steps 3 --warmup 1
step bench_c3_full 300 python3 bench.py --workload variable_coefficients
step bench_c2_full 300 python3 bench.py --workload poisson_square --steps 50 --warmup 5
step bench_torchrun_n1 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
    --master-port 29533 bench.py --gpus 1 --steps 5 --warmup 2 --no-cpu --no-rho
WOST_BENCH_FORCE_COMM=1 step bench_forcecomm_n1 300 python3 bench.py --gpus 1 --steps 5 --warmup 2 --no-cpu --no-rho
timeout -k 10 180 python3 bench.py --gpus 2 --steps 2 --warmup 1 --no-cpu --no-rho > $O/bench_gpus2_on_one_gpu.log 2>&1
echo "gpus2 on one gpu rc=$? (expected nonzero, not 124/137)" | tee -a $O/status.txt
tail -3 $O/gputests.log
cat $O/status.txt
