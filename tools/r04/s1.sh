#!/bin/bash
# Round 4, first GPU session: the new and changed GPU tests, smoke, bench.py --gpus 2 on a
# one-GPU box (must exit non-zero, clearly), one-rank communicator benches of C4/C5 (the
# socket-store bootstrap and the ordered survey path), and a first C3 bench line.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r04s1
mkdir -p $O
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu \
    tests/test_gpu_c5_reference.py tests/test_gpu_c5.py tests/test_gpu_fixed.py tests/test_gpu_long_polylines.py \
    tests/test_gpu_distributed.py > $O/gputests.log 2>&1
echo "gputests rc=$?" >> $O/status.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
echo "smoke rc=$?" >> $O/status.txt
timeout -k 10 120 python bench.py --gpus 2 --steps 2 --warmup 1 --no-cpu --no-rho > $O/bench_gpus2.log 2>&1
echo "bench --gpus 2 rc=$? (expected non-zero on a one-GPU box)" >> $O/status.txt
WOST_BENCH_FORCE_COMM=1 timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu --no-rho \
    > $O/bench_c4_comm.log 2>&1
echo "bench c4 comm rc=$?" >> $O/status.txt
WOST_BENCH_FORCE_COMM=1 MASTER_PORT=29533 timeout -k 10 300 python bench.py --workload wenner_topography --steps 2 \
    --warmup 1 --no-cpu --no-bruteforce > $O/bench_c5_comm.log 2>&1
echo "bench c5 comm rc=$?" >> $O/status.txt
timeout -k 10 300 python bench.py --workload variable_coefficients --steps 10 --warmup 2 --cpu-seconds 8 \
    > $O/bench_c3.log 2>&1
echo "bench c3 rc=$?" >> $O/status.txt
cat $O/status.txt
