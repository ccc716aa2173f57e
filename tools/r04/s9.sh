#!/bin/bash
# Round 4, session 9: the C5 survey with 1, 2 and 3 (model, background) handle pairs
# (2, 4, 6 concurrent launches), alternated; the new C3 full-size tests and the survey
# GPU tests.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r04s9
mkdir -p $O
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_c3_full.py \
    tests/test_gpu_distributed.py tests/test_gpu_c5.py -k "c3 or wenner or survey" > $O/gputests.log 2>&1
echo "gputests rc=$?" >> $O/status.txt
for i in 1 2; do
  for k in 1 2 3; do
    timeout -k 10 300 python bench.py --workload wenner_topography --steps 3 --warmup 1 --no-cpu --no-bruteforce \
        --handle-pairs $k > $O/c5_pairs${k}_$i.log 2>&1
    echo "c5 pairs $k run $i rc=$?" >> $O/status.txt
  done
done
cat $O/status.txt
for f in $O/c5_pairs*.log; do python - "$f" <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith("{"):
        d = json.loads(l); print(sys.argv[1].split("/")[-1], d["value"], d["ms_per_step"], d["config"]["handle_pairs"])
PY
done
