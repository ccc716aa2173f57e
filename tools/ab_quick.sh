#!/bin/bash
# Bitwise check of ab/libwost_base.so vs the working tree's libwost, the GPU tests in
# $AB_TESTS, then an alternating rate A/B of $AB_LIBS on $AB_ONLY (GPU box).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python tools/ab_bitwise.py ab/libwost_base.so dcrmontecarlo_amd/libwost.so > gpurun_out/ab_bitwise.log 2>&1
echo "ab_bitwise rc $?"; tail -1 gpurun_out/ab_bitwise.log
if [ -n "$AB_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest $AB_TESTS -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/ab_tests.log 2>&1
  rc=$?; echo "tests rc $rc"; tail -2 gpurun_out/ab_tests.log
  [ $rc -ge 124 ] && exit $rc
fi
AB_REPS=${AB_REPS:-3} bash tools/ab_pair.sh $AB_LIBS
