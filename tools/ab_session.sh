#!/bin/bash
# A/B session on the GPU box: bitwise equality of a baseline library (ab/libwost_base.so)
# and the working tree's, the GPU tests named in $AB_TESTS, then both libraries' walk
# rates on $AB_ONLY (tools/ab_libs.sh).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python tools/ab_bitwise.py ab/libwost_base.so dcrmontecarlo_amd/libwost.so > gpurun_out/ab_bitwise.log 2>&1
echo "ab_bitwise rc $?"; tail -9 gpurun_out/ab_bitwise.log
if [ -n "$AB_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest $AB_TESTS -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/ab_tests.log 2>&1
  rc=$?; echo "tests rc $rc"; tail -3 gpurun_out/ab_tests.log
  [ $rc -ge 124 ] && exit $rc
fi
bash tools/ab_libs.sh ab/libwost_base.so dcrmontecarlo_amd/libwost.so 2>&1 | tee gpurun_out/ab_libs.log
