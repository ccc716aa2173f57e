#!/bin/bash
# Round 5, session 16: the C5 survey (17 launches per field, 3 handle pairs) under the
# round-5 work queue: default, without the static first chunk (WOST_CHUNK0=0), and round
# 4's queue (WOST_CHUNK0=0 WOST_CHUNK_MIN=1), alternating.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r05s16
mkdir -p $O
step() {   # name limit command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" >> $O/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc" | tee -a $O/status.txt
  [ $rc -ge 124 ] && exit $rc
  return 0
}
for V in "def" "0 -" "0 1" "def" "0 -" "0 1"; do
  unset WOST_CHUNK0 WOST_CHUNK_MIN
  set -- $V
  [ "$1" != def ] && export WOST_CHUNK0=$1
  [ -n "$2" ] && [ "$2" != - ] && export WOST_CHUNK_MIN=$2
  echo "== $V" >> $O/c5_queue.log
  step c5_queue 400 python bench.py --workload wenner_topography --steps 3 --warmup 1 --no-cpu --no-rho
done
cat $O/status.txt
