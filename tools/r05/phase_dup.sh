#!/bin/bash
# Round 5: the walk step's dynamic VALU per phase. For each phase bit
# (wost_walk.h WOST_ABL_DUP: the phase computed twice, the walks unchanged), one rocprofv3
# PMC pass of one solve (tools/r05/dup_driver.py); the VALU/SALU per wave-step minus the
# baseline's is that phase's cost (+ ~3 merge instructions). Usage: phase_dup.sh SCENARIO
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
SC=${1:-dcr_dipole}
O=gpurun_out/r05dup/$SC
mkdir -p $O
export TMPDIR=/tmp
for b in 0 1 2 3 4 5 6 7 8 9 base; do
  if [ "$b" = base ]; then F=0; else F=$(( (1 << b) << 18 )); fi
  WOST_EXP_FLAGS=$F timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VALU_TRANS_F32 \
    SQ_INSTS_LDS --output-format csv -d $O/f$F -o run -- python3 tools/r05/dup_driver.py $SC > $O/f$F.log 2>&1 || exit $?
  echo "flags $F done" >> $O/status.txt
done
