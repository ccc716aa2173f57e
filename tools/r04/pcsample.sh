#!/bin/bash
# PC sampling (rocprofv3, beta) of one scenario's walk kernel: where its waves spend
# their cycles, per instruction. The field-specialised code objects are kept
# (WOST_JIT_CACHE) for offline disassembly. Usage: tools/r04/pcsample.sh <scenario> <tag>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
SC=$1; TAG=$2
O=gpurun_out/r04pcs/$TAG
mkdir -p $O/jit
export TMPDIR=/tmp
WOST_JIT_CACHE=$O/jit timeout -k 10 300 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method stochastic \
    --pc-sampling-unit cycles --pc-sampling-interval 1048576 --output-format csv -d $O/pcs -o run -- \
    python3 tools/scenario_bench.py --only $SC --reps 1 > $O/run.log 2>&1
echo "pcsample $SC stochastic rc=$?" | tee -a $O/status.txt
