#!/bin/bash
# Round 6, session 29: a bit-preserving option sweep at the final code on C4 and C3
# (tools/scenario_bench.py, 5 reps, best kernel rate), baselines interleaved.
O=gpurun_out/r06s29
source "$(dirname "$0")/common.sh"
run() {   # tag scenario opts...
  local tag=$1 sc=$2; shift 2
  local args=""
  for o in "$@"; do args="$args --opt $o"; done
  step ${sc}_$tag 120 python3 tools/scenario_bench.py --only $sc --reps 5 $args
  echo "$sc $tag $(grep -o 'steps/s (kernel)' -B0 $O/${sc}_$tag.log >/dev/null; grep "^$sc " $O/${sc}_$tag.log | awk '{print $6}')" >> $O/summary.txt
}
for sc in dcr_dipole variable_coefficients; do
  run base0 $sc
  run wb512 $sc walk_block=512
  run wb1024 $sc walk_block=1024
  run w6 $sc jit_waves=6
  run w8 $sc jit_waves=8
  run base1 $sc
  run pa1 $sc philox_ahead=1
  run pa2 $sc philox_ahead=2
  run rm16 $sc refill_min=16
  run rm48 $sc refill_min=48
  run base2 $sc
  run g6 $sc grid_blocks_per_cu=6
  run g8 $sc grid_blocks_per_cu=8
  run base3 $sc
done
cat $O/summary.txt
cat $O/status.txt
