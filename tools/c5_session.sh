set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_segment_tree.py tests/test_gpu_c5.py tests/test_gpu_fixed.py tests/test_gpu_long_polylines.py tests/test_gpu_distributed.py tests/test_gpu_rho_reference.py tests/test_survey.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gputests_tree.log 2>&1; echo "tests rc $?"
tail -3 gpurun_out/gputests_tree.log
for L in 8 10 16; do WOST_TREE_LEAF=$L timeout -k 10 120 python tools/scenario_bench.py --only wenner_topography,variable_coefficients --reps 2 2>&1 | grep -v JSON | sed "s/^/leaf $L: /"; done
