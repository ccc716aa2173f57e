#!/bin/bash
# Round 5, session 15: C2 (64 points x 10k walks, ~1.2 walks per lane at full occupancy):
# fewer resident workgroups per CU (WOST_GRID_BLOCKS_PER_CU) -- faster steps per wave at
# the launch's tail against fewer lanes.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r05s15
mkdir -p $O
step() {   # name limit command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" >> $O/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc" | tee -a $O/status.txt
  [ $rc -ge 124 ] && exit $rc
  return 0
}
for B in 8 4 2 1 8 4 2 1; do
  echo "== WOST_GRID_BLOCKS_PER_CU=$B" >> $O/grid_ab.log
  export WOST_GRID_BLOCKS_PER_CU=$B
  step grid_ab 300 python bench.py --workload poisson_square --no-cpu --no-rho --steps 30 --warmup 3
done
cat $O/status.txt
