cd $GRAFT_REPO_ROOT
for cfg in "WOST_TREE_LEAF=8" "WOST_TREE_LEAF=10" "WOST_TREE_LEAF=16" "WOST_TREE_LEAF=10 WOST_JIT_WAVES=7" "WOST_TREE_LEAF=10 WOST_JIT_WAVES=8" "WOST_TREE_LEAF=8 WOST_JIT_WAVES=8"; do
  env $cfg timeout -k 10 120 python tools/scenario_bench.py --only wenner_topography --reps 3 2>&1 | grep -v JSON | sed "s/^/$cfg: /"
done
