# sourced by the round-6 session scripts: O (output dir) must be set
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p $O
step() {   # name limit command...: a GPU step under its own time limit; a crash or timeout ends the session
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > $O/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc" | tee -a $O/status.txt
  [ $rc -ge 124 ] && exit $rc
  return 0
}
