cd "${GRAFT_REPO_ROOT:-.}"
for v in none 511 255 none 511 1023; do
  echo "== WOST_TREE_LDS=$v"
  if [ "$v" = none ]; then timeout -k 10 200 python tools/scenario_bench.py --reps 2 --only wenner_topography 2>&1 | grep -v JSON || exit $?
  else WOST_TREE_LDS=$v timeout -k 10 200 python tools/scenario_bench.py --reps 2 --only wenner_topography 2>&1 | grep -v JSON || exit $?; fi
done
