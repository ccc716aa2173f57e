#!/bin/bash
# Round 6, session 7: C5 device histories on both replay fixtures (host-side diagnosis of the
# history test's record mismatches).
O=gpurun_out/r06s7
source "$(dirname "$0")/common.sh"
step dump_lit 300 python tools/r05/c5_hist_dump.py $O/hist_literal.npz replay_wenner_topography.npz
step dump_phys 300 python -c "import sys; sys.path.insert(0, 'tools/r05'); import c5_hist_dump as d; d.main('$O/hist_physical.npz', 'replay_wenner_topography_physical.npz', physical=True)"
cat $O/status.txt
