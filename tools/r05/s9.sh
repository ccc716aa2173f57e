#!/bin/bash
# Round 5, session 9 (the staged scan in batches of eight vertices): the fused brute-force scan (neumann_scan_both): bitwise tests, its rate
# against the separate scans (WOST_EXP_FLAGS 2^28), the C5 bench's speedup leg.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r05s9
mkdir -p $O
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_c5.py > $O/gputests_c5.log 2>&1
echo "gputests c5 rc=$?" >> $O/status.txt
for F in 0 268435456 0 268435456; do
  echo "== WOST_EXP_FLAGS=$F" >> $O/scan_ab.log
  WOST_EXP_FLAGS=$F timeout -k 10 300 python -u tools/scenario_bench.py --scan --reps 2 \
    --only wenner_topography,wenner_topography_physical >> $O/scan_ab.log 2>&1 || break
done
echo "scan ab rc=$?" >> $O/status.txt
timeout -k 10 600 python bench.py --workload wenner_topography --steps 3 --warmup 1 --no-cpu > $O/bench_c5.log 2>&1
echo "bench c5 rc=$?" >> $O/status.txt
cat $O/status.txt
timeout -k 10 600 python -u tools/r05/trig_parity.py > gpurun_out/r05s9/trig_parity.log 2>&1
echo "trig parity rc=$?" >> gpurun_out/r05s9/status.txt
