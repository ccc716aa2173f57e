#!/bin/bash
# The C5 survey bench line (bench.py --workload wenner_topography) at each tree staging
# level (WOST_TREE_LDS 2 / 1 / 0). GPU box.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for lv in ${C5_LEVELS:-2 1 0}; do
  WOST_TREE_LDS=$lv timeout -k 10 400 python bench.py --workload wenner_topography --steps 3 --warmup 1 --no-cpu --no-bruteforce \
    > gpurun_out/c5_bench_lds$lv.log 2>&1 || exit $?
  python3 -c "
import json; l=[x for x in open('gpurun_out/c5_bench_lds$lv.log') if x.startswith('{')][-1]; d=json.loads(l)
print('WOST_TREE_LDS=$lv', 'survey walk-steps/s %.4g' % d['value'], 'ms_per_step %.1f' % d['ms_per_step'])"
done
