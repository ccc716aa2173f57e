#!/bin/bash
# Round 5, session 17: the dynamic chunk's cap (WOST_CHUNK_MAX; 1024 walks = 16 per lane,
# ~4 ms of a C4 wave's work at the launch's end) on C4 and C3, alternating.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r05s17
mkdir -p $O
step() {   # name limit command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" >> $O/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc" | tee -a $O/status.txt
  [ $rc -ge 124 ] && exit $rc
  return 0
}
for C in 1024 256 64 1024 256 64; do
  export WOST_CHUNK_MAX=$C
  for W in dcr_dipole variable_coefficients; do
    echo "== WOST_CHUNK_MAX=$C $W" >> $O/cap_ab.log
    step cap_ab 300 python bench.py --workload $W --no-cpu --no-rho --steps 20 --warmup 3
  done
  echo "== WOST_CHUNK_MAX=$C scenarios" >> $O/cap_scen.log
  step cap_scen 300 python -u tools/scenario_bench.py --reps 2 --only dcr_dipole,notebook_dcr,wenner_topography
done
cat $O/status.txt
