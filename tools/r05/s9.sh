#!/bin/bash
# Round 5, session 9 (the staged scan in batches of eight vertices): the fused brute-force
# scan (neumann_scan_both): bitwise tests, its rate against the separate scans
# (WOST_EXP_FLAGS 2^28) and the round-5 per-vertex bits (2^17), the C5 bench's speedup leg,
# the trig parity probe. Each GPU step under its own limit; stops at a crash or timeout.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r05s9
mkdir -p $O
step() {   # name limit command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" >> $O/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc" | tee -a $O/status.txt
  [ $rc -ge 124 ] && exit $rc
  return 0
}
step gputests_c5 600 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_c5.py
for F in 0 268435456 131072 0 268435456 131072; do
  echo "== WOST_EXP_FLAGS=$F" >> $O/scan_ab.log
  export WOST_EXP_FLAGS=$F
  step scan_ab 300 python -u tools/scenario_bench.py --scan --reps 2 \
    --only wenner_topography,wenner_topography_physical
done
unset WOST_EXP_FLAGS
export WOST_EXP_FLAGS=131072
step gputests_bits 300 python -u -m pytest -v --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_c5.py -k "fused or global"
unset WOST_EXP_FLAGS
step bench_c5 600 python bench.py --workload wenner_topography --steps 3 --warmup 1 --no-cpu
step trig_parity 600 python -u tools/r05/trig_parity.py
cat $O/status.txt
