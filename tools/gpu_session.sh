#!/bin/bash
# Runs a sequence of GPU steps on the gpurun box, each under its own time
# limit. Stops at the first step that crashes, aborts or times out (exit
# status >= 124); a plain test failure (exit 1) does not stop the session.
# Usage: tools/gpu_session.sh "<name>|<seconds>|<command>" ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
status=0
for spec in "$@"; do
  name="${spec%%|*}"; rest="${spec#*|}"; secs="${rest%%|*}"; cmd="${rest#*|}"
  echo "=== [$name] (limit ${secs}s): $cmd" | tee -a gpurun_out/session.log
  start=$(date +%s)
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "=== [$name] exit $rc after $(( $(date +%s) - start ))s" | tee -a gpurun_out/session.log
  tail -n 15 "gpurun_out/$name.log"
  if [ $rc -ge 124 ]; then echo "fatal exit $rc in $name: stopping"; exit $rc; fi
  [ $rc -ne 0 ] && status=$rc
done
exit $status
