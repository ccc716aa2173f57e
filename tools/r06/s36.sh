#!/bin/bash
# Round 6, session 36: more launch-shape options at the final code -- C2's grid with the
# all-static chunk, the short walks' dynamic chunk cap, the tree kernel's chunk cap, C3's
# dynamic chunk cap at its BASELINE size; baselines interleaved.
O=gpurun_out/r06s36
source "$(dirname "$0")/common.sh"
run() {   # tag scenario scale opts...
  local tag=$1 sc=$2 scale=$3; shift 3
  local args=""
  for o in "$@"; do args="$args --opt $o"; done
  step ${sc}_${scale}_$tag 120 python3 tools/scenario_bench.py --only $sc --reps 7 --scale $scale $args
}
for r in 0 1; do
  run base$r poisson_square 0.05
  run g1_$r poisson_square 0.05 grid_blocks_per_cu=1
  run g3_$r poisson_square 0.05 grid_blocks_per_cu=3
  run g4_$r poisson_square 0.05 grid_blocks_per_cu=4
  run base$r laplace_square 1
  run cm128_$r laplace_square 1 chunk_max=128
  run cm256_$r laplace_square 1 chunk_max=256
  run base$r wenner_topography 1
  run cm8_$r wenner_topography 1 chunk_max=8
  run cm32_$r wenner_topography 1 chunk_max=32
  run base$r variable_coefficients 5
  run cm32_$r variable_coefficients 5 chunk_max=32
  run cm128_$r variable_coefficients 5 chunk_max=128
done
cat $O/status.txt
