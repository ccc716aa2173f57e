#!/bin/bash
# Round 6, session 37: resident workgroups for few short walks with the all-static first
# chunk: C2's size (Poisson and Laplace, 64 x 10k) and a 4x larger one, 2 (default) to 8 per CU.
O=gpurun_out/r06s37
source "$(dirname "$0")/common.sh"
run() {   # tag scenario scale opts...
  local tag=$1 sc=$2 scale=$3; shift 3
  local args=""
  for o in "$@"; do args="$args --opt $o"; done
  step ${sc}_${scale}_$tag 120 python3 tools/scenario_bench.py --only $sc --reps 9 --scale $scale $args
}
for r in 0 1; do
  for x in "poisson_square 0.05" "laplace_square 0.05" "poisson_square 0.2"; do
    set -- $x
    run base$r $1 $2
    run g4_$r $1 $2 grid_blocks_per_cu=4
    run g5_$r $1 $2 grid_blocks_per_cu=5
    run g6_$r $1 $2 grid_blocks_per_cu=6
    run g8_$r $1 $2 grid_blocks_per_cu=8
  done
done
cat $O/status.txt
