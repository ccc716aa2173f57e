#!/bin/bash
# Round 6, session 8: the C5 reference tests (histories against the oracle's floor, both
# surveys' rho_a replays), the queue tests, and the C5 bench line with both replay legs.
O=gpurun_out/r06s8
source "$(dirname "$0")/common.sh"
step gputests_c5ref 900 python -u -m pytest -v -s --timeout 400 --timeout-method thread -m gpu tests/test_gpu_c5_reference.py
step bench_c5 700 python bench.py --workload wenner_topography --steps 3 --warmup 1 --no-cpu
cat $O/status.txt
