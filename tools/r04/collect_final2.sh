#!/bin/bash
# Copies the end-of-round profiles of tools/r04/final2.sh from gpurun_out/ into
# profiles/ and regenerates the issue / traffic JSON the bench line reads (CPU side).
set -e
cd "$(dirname "$0")/../.."
G=gpurun_out
for W in dcr_dipole variable_coefficients wenner_topography; do
  D=profiles/r04_prof/$W
  rm -rf $D; mkdir -p $D
  cp $G/r04prof/$W/stats/run_kernel_stats.csv $D/kernel_stats.csv
  cp $G/${W}_bench.log $D/bench.log
  [ $W != wenner_topography ] && cp $G/${W}_stats.log $D/stats.log   # (C5's was overwritten by the single-launch run)
  for p in $G/r04prof/$W/pmc_*; do mkdir -p $D/$(basename $p); cp $p/run_counter_collection.csv $D/$(basename $p)/; done
done
D=profiles/r04_prof/wenner_topography_single
rm -rf $D; mkdir -p $D/stats
cp $G/prof_wenner_topography/stats/run_kernel_stats.csv $D/stats/
cp $G/wenner_topography_stats.log $D/stats.log
for p in sq1 sq2 util; do mkdir -p $D/pmc_$p; cp $G/prof_wenner_topography/pmc_$p/run_counter_collection.csv $D/pmc_$p/; cp $G/wenner_topography_$p.log $D/$p.log; done
mkdir -p profiles/r04_final2
cp $G/r04final2/*.log $G/r04final2/status.txt profiles/r04_final2/
