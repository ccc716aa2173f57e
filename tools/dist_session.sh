#!/bin/bash
# The driver's multi-GPU launch path at N=1 (torchrun, one rank over RCCL through libwost's
# communicator), weak and strong, plus the C5 Wenner survey end to end. Runs on the GPU box.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for sc in weak strong; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29517 \
    bench.py --gpus 1 --steps 5 --warmup 1 --no-cpu --no-rho --scaling $sc > gpurun_out/bench_torchrun_1rank_$sc.log 2>&1 || exit $?
done
timeout -k 10 300 python tools/c5_survey.py --walks 10000 > gpurun_out/c5_survey_10k.log 2>&1 || exit $?
timeout -k 10 400 python tools/c5_survey.py --walks 100000 > gpurun_out/c5_survey_100k.log 2>&1 || exit $?
