#!/bin/bash
# Round 6, session 27: the bench's communicator path end to end on one GPU (a one-rank RCCL
# communicator: the protocol, all-gather and merge the N-GPU run takes), C4 and C5, and
# the --gpus 2 refusal on a one-GPU box.
O=gpurun_out/r06s27
source "$(dirname "$0")/common.sh"
export WOST_BENCH_FORCE_COMM=1
step comm_c4 300 python -u bench.py --steps 5 --warmup 2 --no-cpu --no-rho
step comm_c5 400 python -u bench.py --workload wenner_topography --steps 2 --warmup 1 --no-cpu --no-rho
unset WOST_BENCH_FORCE_COMM
step gpus2 120 python -u bench.py --gpus 2 --steps 2 --warmup 1 --no-cpu --no-rho
grep -o '"value": [0-9.e+]*' $O/comm_c4.log $O/comm_c5.log
grep -o '"parallelism": "[^"]*"' $O/comm_c4.log $O/comm_c5.log
tail -3 $O/gpus2.log
cat $O/status.txt
