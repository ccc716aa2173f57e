#!/bin/bash
# Round 4, session 10: sessions 8 (6 vs 7 waves) and 9 (C5 handle pairs, C3 full-size tests) in one box.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
bash tools/r04/s9.sh
bash tools/r04/s8.sh
