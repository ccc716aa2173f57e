#!/usr/bin/env python3
"""Round 6 A/B: the C5 Wenner survey (bench.py's workload: 256 electrodes x 100k walks,
3 handle pairs) with the multi-source kernels' sources as literals (one hiprtc compile per
electrode group and field) or read from the program buffer (option param_sources: one per
source structure). Fresh caches per process (WOST_JIT_CACHE, AMD_COMGR_CACHE_DIR): the first
survey's wall time is the cold start; then K warm surveys. Usage: survey_ab.py PARAM [K]"""
import json
import os
import sys
import tempfile
import time

d = tempfile.mkdtemp(prefix="wost_ab_")
os.environ["WOST_JIT_CACHE"] = d
os.environ["AMD_COMGR_CACHE_DIR"] = os.path.join(d, "comgr")
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from dcrmontecarlo_amd import scenarios as S  # noqa: E402
from dcrmontecarlo_amd import survey  # noqa: E402

param = int(sys.argv[1])
K = int(sys.argv[2]) if len(sys.argv) > 2 else 5
sc = S.wenner_topography(n_electrodes=256, n_walks=100_000)
pairs = []
for _ in range(3):
    m = sc.solver(device=0)
    pairs += [m, survey.homogeneous_solver(sc, 1e-2, m, device=0)]
for s in pairs:
    s.set_option("param_sources", param)
t0 = time.perf_counter()
survey.run_wenner_survey(sc, 1e-2, 100_000, seed=1000, solvers=tuple(pairs))
first = time.perf_counter() - t0
times, steps = [], 0
for k in range(K):
    t0 = time.perf_counter()
    res = survey.run_wenner_survey(sc, 1e-2, 100_000, seed=k, solvers=tuple(pairs))
    times.append(time.perf_counter() - t0)
    steps = int(res.walk_steps)
print(json.dumps({"param_sources": param, "first_survey_s": first, "warm_s": times,
                  "warm_walk_steps_per_s": steps / min(times), "median_walk_steps_per_s": steps / sorted(times)[K // 2]}))
