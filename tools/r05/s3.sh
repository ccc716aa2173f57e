#!/bin/bash
# Round 5, session 3: the trig policy (AUTO) timings, C5 reference tests (walk replay, rho_a
# replay, stats), small-solve host overhead, the C2 bench line, the per-rank breakdown on
# one GPU through the communicator (C4, C5), the C5 bench with its rho_a replay leg.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r05s3
mkdir -p $O
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_c5_reference.py \
  "tests/test_gpu_parity.py::test_statistics_vs_reference_rng" > $O/gputests_c5.log 2>&1
echo "gputests c5 rc=$?" >> $O/status.txt
timeout -k 10 300 python -u tools/scenario_bench.py --reps 2 \
  --only dcr_dipole,variable_coefficients,wenner_topography,laplace_square,poisson_square,notebook_dcr,manufactured_polynomial \
  > $O/scenarios_auto.log 2>&1
echo "scenarios rc=$?" >> $O/status.txt
timeout -k 10 300 python -u tools/r05/host_overhead.py --reps 20 > $O/host_overhead.log 2>&1
echo "host overhead rc=$?" >> $O/status.txt
timeout -k 10 300 python bench.py --workload poisson_square --steps 50 --warmup 5 --cpu-seconds 8 > $O/bench_c2.log 2>&1
echo "bench c2 rc=$?" >> $O/status.txt
WOST_BENCH_FORCE_COMM=1 timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu --no-rho > $O/bench_c4_comm.log 2>&1
echo "bench c4 comm rc=$?" >> $O/status.txt
WOST_BENCH_FORCE_COMM=1 timeout -k 10 600 python bench.py --workload wenner_topography --steps 2 --warmup 1 --no-cpu \
  --no-bruteforce > $O/bench_c5_comm.log 2>&1
echo "bench c5 comm rc=$?" >> $O/status.txt
cat $O/status.txt
