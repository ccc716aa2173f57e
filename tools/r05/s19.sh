#!/bin/bash
# Round 5, session 19: the C5 survey under smaller dynamic-chunk caps (its launches' own
# count / (4 waves) is ~90 walks, so the 64 cap binds): 64 (default), 32, 16, alternating.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r05s19
mkdir -p $O
step() {   # name limit command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" >> $O/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc" | tee -a $O/status.txt
  [ $rc -ge 124 ] && exit $rc
  return 0
}
for C in 64 32 16 64 32 16; do
  export WOST_CHUNK_MAX=$C
  echo "== WOST_CHUNK_MAX=$C wenner_topography" >> $O/cap_c5.log
  step cap_c5 400 python bench.py --workload wenner_topography --steps 3 --warmup 1 --no-cpu --no-rho
done
cat $O/status.txt
