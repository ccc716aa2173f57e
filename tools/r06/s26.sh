#!/bin/bash
# Round 6, session 26: the race tests after the switch test's widening (16M walks).
O=gpurun_out/r06s26
source "$(dirname "$0")/common.sh"
step race 300 python -u -m pytest tests/test_gpu_race.py -v -s --timeout 200 --timeout-method thread
grep -E "PASSED|FAILED|raced:" $O/race.log
cat $O/status.txt
