#!/bin/bash
# Round 6, session 28: kernel trace of the C5 survey bench (how busy the GPU is between the
# survey's 34 launches on its 6 streams).
O=gpurun_out/r06s28
source "$(dirname "$0")/common.sh"
export TMPDIR=/tmp
step trace 400 rocprofv3 --kernel-trace --output-format csv -d $O/trace -o run -- python3 bench.py --workload wenner_topography --steps 2 --warmup 1 --no-cpu --no-rho --no-bruteforce
ls -R $O/trace | head
cat $O/status.txt
