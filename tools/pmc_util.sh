set -e
export TMPDIR=/tmp
O=gpurun_out/util; mkdir -p $O
for sc in dcr_dipole variable_coefficients wenner_topography; do
  timeout -k 10 240 rocprofv3 --pmc SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAVES --output-format csv -d $O/$sc -o run -- python3 tools/scenario_bench.py --only $sc --reps 1 > $O/$sc.log 2>&1
  echo done $sc
done
