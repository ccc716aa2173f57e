#!/bin/bash
# Round 6, session 21: the whole GPU suite with jit_race (tests compile before their first
# solve; tests/test_gpu_race.py races), smoke (both solves per scenario), bench lines.
O=gpurun_out/r06s21
source "$(dirname "$0")/common.sh"
step gputests 1000 python -u -m pytest tests -m gpu -q --timeout 400 --timeout-method thread
step smoke 200 python -c "import __graft_entry__ as g; g.smoke()"
step bench_c4 300 python -u bench.py --steps 20 --warmup 5
step bench_c5 400 python -u bench.py --workload wenner_topography --steps 3 --warmup 2 --no-cpu --no-rho
tail -5 $O/gputests.log
cat $O/smoke.log
cat $O/status.txt
