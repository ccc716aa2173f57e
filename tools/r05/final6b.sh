#!/bin/bash
# Round 5 end (sixth pass), part B: rocprofv3 of the exact bench commands (stats and PMC
# passes) for the four workloads and the single-launch C5 counters.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r05final6
mkdir -p $O
step() {   # name limit command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > $O/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc" | tee -a $O/status_b.txt
  [ $rc -ge 124 ] && exit $rc
  return 0
}
step prof_c4 900 bash tools/r05/profile_bench.sh dcr_dipole 20 5
step prof_c3 900 bash tools/r05/profile_bench.sh variable_coefficients 20 5
step prof_c2 600 bash tools/r05/profile_bench.sh poisson_square 50 5
step prof_c5 900 bash tools/r05/profile_bench.sh wenner_topography 2 1 --no-bruteforce
step prof_c5_single 600 bash tools/c5_profile.sh wenner_topography
cat $O/status_b.txt
