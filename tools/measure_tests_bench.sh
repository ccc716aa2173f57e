#!/bin/bash
# Measurement session A (GPU box): the GPU test suite, smoke, the C4 bench line (with its
# CPU baseline and rho_a legs), the C5 bench line, and both through a one-rank
# torchrun + RCCL communicator (WOST_BENCH_FORCE_COMM). Stops at a crash or time-out.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
export HSA_ENABLE_IPC_MODE_LEGACY=0
TR="python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533"
bash tools/gpu_session.sh \
  "gputests|700|python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
  "smoke|300|python -c 'import __graft_entry__ as g; g.smoke()'" \
  "bench|400|python bench.py" \
  "bench_c5|400|python bench.py --workload wenner_topography --steps 5 --warmup 1" \
  "bench_comm|300|WOST_BENCH_FORCE_COMM=1 $TR bench.py --steps 5 --warmup 1 --no-cpu" \
  "bench_c5_comm|300|WOST_BENCH_FORCE_COMM=1 $TR bench.py --workload wenner_topography --steps 3 --warmup 1 --no-cpu --no-bruteforce"
