#!/bin/bash
# Round 6, session 34: the static first chunk for the Neumann (long-walk) kernels: C3 at the
# scenario size and at its BASELINE size (scale 5: 256 x 100k), notebook DCR; 64 (default)
# vs 128 / 256, baselines interleaved.
O=gpurun_out/r06s34
source "$(dirname "$0")/common.sh"
run() {   # tag scenario scale opts...
  local tag=$1 sc=$2 scale=$3; shift 3
  local args=""
  for o in "$@"; do args="$args --opt $o"; done
  step ${sc}_${scale}_$tag 120 python3 tools/scenario_bench.py --only $sc --reps 7 --scale $scale $args
}
for r in 0 1; do
  for x in "variable_coefficients 1" "variable_coefficients 5" "notebook_dcr 1"; do
    set -- $x
    run base$r $1 $2
    run c128_$r $1 $2 chunk0=128
    run c256_$r $1 $2 chunk0=256
  done
done
cat $O/status.txt
