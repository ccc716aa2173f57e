#!/bin/bash
# Round 6, session 23: A/B of the C5 survey's cold start on one box -- HEAD against the
# s16 code (2cd7e66: every compile in a helper) and the s18 code (8fa764c: a lone compile
# in-process), interleaved.
O=gpurun_out/r06s23
source "$(dirname "$0")/common.sh"
for r in 1 2; do
  step new_$r 300 python -u tools/r06/cold_survey.py 1
  step old_$r 300 python -u abtest/r06/old/tools/r06/cold_survey.py 1
  step mid_$r 300 python -u abtest/r06/mid/tools/r06/cold_survey.py 1
done
for f in $O/new_* $O/old_* $O/mid_*; do echo "$f $(grep -o '"survey0_ms": [0-9.]*' $f)"; done
cat $O/status.txt
