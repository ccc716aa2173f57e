#!/bin/bash
# Round 5, session 18: the dynamic chunk's cap around the new default (64): 32, 64, 128 on
# C4 and C3, and the C5 survey at the default against round 4's cap (1024).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r05s18
mkdir -p $O
step() {   # name limit command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" >> $O/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc" | tee -a $O/status.txt
  [ $rc -ge 124 ] && exit $rc
  return 0
}
for C in 64 32 128 64 32 128; do
  export WOST_CHUNK_MAX=$C
  for W in dcr_dipole variable_coefficients; do
    echo "== WOST_CHUNK_MAX=$C $W" >> $O/cap_ab.log
    step cap_ab 300 python bench.py --workload $W --no-cpu --no-rho --steps 20 --warmup 3
  done
done
for C in 64 1024 64 1024; do
  export WOST_CHUNK_MAX=$C
  echo "== WOST_CHUNK_MAX=$C wenner_topography" >> $O/cap_c5.log
  step cap_c5 400 python bench.py --workload wenner_topography --steps 3 --warmup 1 --no-cpu --no-rho
done
cat $O/status.txt
