#!/bin/bash
# Round 6, session 31: the static first chunk (chunk0) for short walks: 64 (default) vs 128 /
# 256 on Poisson, Laplace and manufactured at the scenario sizes and at C2's BASELINE size
# (scale 0.05: 64 x 10k), and on C4; baselines interleaved.
O=gpurun_out/r06s31
source "$(dirname "$0")/common.sh"
run() {   # tag scenario scale opts...
  local tag=$1 sc=$2 scale=$3; shift 3
  local args=""
  for o in "$@"; do args="$args --opt $o"; done
  step ${sc}_${scale}_$tag 120 python3 tools/scenario_bench.py --only $sc --reps 7 --scale $scale $args
}
for r in 0 1; do
  for sc in poisson_square laplace_square manufactured_polynomial; do
    run base$r $sc 1
    run c128_$r $sc 1 chunk0=128
    run c256_$r $sc 1 chunk0=256
  done
  run base$r poisson_square 0.05
  run c128_$r poisson_square 0.05 chunk0=128
  run c256_$r poisson_square 0.05 chunk0=256
  run base$r dcr_dipole 1
  run c128_$r dcr_dipole 1 chunk0=128
done
cat $O/status.txt
