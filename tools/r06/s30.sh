#!/bin/bash
# Round 6, session 30: the same bit-preserving option sweep on C5's tree kernel (one launch of
# 256 electrodes x 2000 walks) and C2, baselines interleaved.
O=gpurun_out/r06s30
source "$(dirname "$0")/common.sh"
run() {   # tag scenario opts...
  local tag=$1 sc=$2; shift 2
  local args=""
  for o in "$@"; do args="$args --opt $o"; done
  step ${sc}_$tag 120 python3 tools/scenario_bench.py --only $sc --reps 5 $args
}
sc=wenner_topography
run base0 $sc
run lds1 $sc tree_lds=1
run lds0 $sc tree_lds=0
run pool0 $sc tree_pool=0
run slots64 $sc pool_slots=64
run slots256 $sc pool_slots=256
run base1 $sc
run near05 $sc pool_near=0.05
run near2 $sc pool_near=0.2
run share0 $sc tree_share=0
run share16 $sc tree_share=16
run batch2 $sc tree_batch=2
run w5 $sc jit_waves=5
run base2 $sc
sc=poisson_square
run base0 $sc
run c0_16 $sc chunk0=16
run c0_128 $sc chunk0=128
run adapt0 $sc adaptive_chunk=0
run base1 $sc
cat $O/status.txt
