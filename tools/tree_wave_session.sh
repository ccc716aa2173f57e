#!/bin/bash
# GPU box: the cooperative tree queries against ab/libwost_base.so -- bits on every
# scenario (TW_BITWISE: lib[:ENV] to compare with the base), the C5 GPU tests, then
# C5 walk rates of the variants given as arguments (lib[:VAR=VAL,...], tools/ab_libs.sh).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in ${TW_BITWISE:-dcrmontecarlo_amd/libwost.so}; do
  timeout -k 10 300 python tools/ab_bitwise.py ab/libwost_base.so "$v" > gpurun_out/tw_bitwise.log 2>&1
  rc=$?; echo "ab_bitwise $v rc $rc"; tail -1 gpurun_out/tw_bitwise.log
  [ $rc -ne 0 ] && exit $rc
done
if [ -n "$TW_TESTS" ]; then
  timeout -k 10 400 python -u -m pytest $TW_TESTS -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/tw_tests.log 2>&1
  rc=$?; echo "tests rc $rc"; tail -3 gpurun_out/tw_tests.log
  [ $rc -ne 0 ] && exit $rc
fi
AB_ONLY=${AB_ONLY:-wenner_topography,wenner_topography_physical} bash tools/ab_libs.sh "$@" 2>&1 | tee gpurun_out/tw_rates.log
