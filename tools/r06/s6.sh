#!/bin/bash
# Round 6, session 6: the C5 parity tests (history replay of both variants, the tightened
# device-vs-oracle bounds), the fused-scan clamp, the parity suite and smoke.
O=gpurun_out/r06s6
source "$(dirname "$0")/common.sh"
step gputests_c5 900 python -u -m pytest -v -s --timeout 300 --timeout-method thread -m gpu tests/test_gpu_c5.py tests/test_gpu_c5_reference.py
step gputests_parity 600 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
cat $O/status.txt
