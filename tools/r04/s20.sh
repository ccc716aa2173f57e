#!/bin/bash
# Round 4, session 20: C5 survey handle pairs 3 (default) vs 4 and 5, with the walk pools.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r04s20
mkdir -p $O
for i in 1 2; do
  for p in 3 4 5; do
    timeout -k 10 300 python3 bench.py --workload wenner_topography --steps 3 --warmup 1 --no-cpu --no-bruteforce --handle-pairs $p > $O/pairs${p}_$i.log 2>&1
    rc=$?; echo "pairs$p run $i rc=$rc" >> $O/status.txt; [ $rc -ge 124 ] && exit $rc
    python3 -c "
import json
for l in open('$O/pairs${p}_$i.log'):
    if l.startswith('{'): d=json.loads(l); print('pairs $p run $i', d['value'], d['ms_per_step'])"
  done
done
cat $O/status.txt
