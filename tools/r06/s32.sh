#!/bin/bash
# Round 6, session 32: the static first chunk for short walks, wider: chunk0 256 / 320 / 512 /
# 1024 at C2's BASELINE size and the scenario sizes; the dynamic chunk cap at 256.
O=gpurun_out/r06s32
source "$(dirname "$0")/common.sh"
run() {   # tag scenario scale opts...
  local tag=$1 sc=$2 scale=$3; shift 3
  local args=""
  for o in "$@"; do args="$args --opt $o"; done
  step ${sc}_${scale}_$tag 120 python3 tools/scenario_bench.py --only $sc --reps 7 --scale $scale $args
}
for r in 0 1; do
  run base$r poisson_square 0.05
  run c256_$r poisson_square 0.05 chunk0=256
  run c320_$r poisson_square 0.05 chunk0=320
  run c512_$r poisson_square 0.05 chunk0=512
  run c256m256_$r poisson_square 0.05 chunk0=256 chunk_max=256
  for sc in poisson_square laplace_square manufactured_polynomial; do
    run base$r $sc 1
    run c256_$r $sc 1 chunk0=256
    run c512_$r $sc 1 chunk0=512
    run c1024_$r $sc 1 chunk0=1024
    run c256m256_$r $sc 1 chunk0=256 chunk_max=256
  done
done
cat $O/status.txt
