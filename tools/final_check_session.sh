#!/bin/bash
# End-of-session check on the GPU box: the GPU test suite, smoke, then tools/final_session.sh
# (scenarios, bench, rocprofv3 stats + PMC).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gputests.log 2>&1 || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
bash tools/final_session.sh > gpurun_out/final_session.log 2>&1
