#!/bin/bash
# End-of-session check on the GPU box: bitwise A/B of the final library against the previous
# one, the GPU test suite, smoke, then tools/final_session.sh (scenarios, bench, rocprofv3).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python tools/ab_bitwise.py ab/libwost_refill.so ab/libwost_final.so > gpurun_out/ab_final_bits.log 2>&1 || exit $?
AB_ONLY=wenner_topography timeout -k 10 300 bash tools/ab_libs.sh ab/libwost_refill.so ab/libwost_final.so > gpurun_out/ab_final_time.log 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gputests.log 2>&1 || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
bash tools/final_session.sh > gpurun_out/final_session.log 2>&1
