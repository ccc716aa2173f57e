#!/bin/bash
# Round 6, session 11: C5 survey, literal vs parameter-buffer multi-source kernels (the latter
# now sharing identical factors' words), alternating, fresh caches per process.
O=gpurun_out/r06s11
source "$(dirname "$0")/common.sh"
step lit_a 300 python tools/r06/survey_ab.py 0 6
step par_a 300 python tools/r06/survey_ab.py 1 6
step lit_b 300 python tools/r06/survey_ab.py 0 6
step par_b 300 python tools/r06/survey_ab.py 1 6
step gputests_ms 400 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_multisource.py
tail -n 1 $O/lit_a.log $O/par_a.log $O/lit_b.log $O/par_b.log
cat $O/status.txt
