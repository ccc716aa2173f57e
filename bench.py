#!/usr/bin/env python3
"""Walk-steps/sec of the Walk-on-Stars hot path on MI355X.

Workload (BASELINE.json configs[3]): the DCR dipole survey of
tests/testGeophysicalScenario.py -- 48 surface electrodes x 1M walks each,
delta tracking with the reference's conductivity field, mixed Dirichlet /
Neumann boundary, eps = 0.9, maxSteps = 500. One bench "step" is one full
survey solve (48M walks, ~3.65G walk-steps) per GPU.

N ranks (one process per GPU) solve through libwost's own RCCL communicator
(dcrmontecarlo_amd.comm, wost_solve_distributed): rank r solves the walk range
wost_shard_walk_range(W, N, r) of EVERY electrode, the per-block partial sums
are all-gathered over xGMI (the only data-path collective) and summed per
electrode in global block order -- bitwise a one-GPU solve of W walks per
electrode. --scaling weak (default): W = N x 1M, so each GPU keeps the one-GPU
workload; --scaling strong: W = 1M split N ways. The communicator's id travels
through a standard-library socket store hosted by rank 0 (comm.launch_store); no
torch process group is created.

--workload wenner_topography (BASELINE configs[4]): the 256-electrode
Wenner-alpha line over the 10,000-segment topography, model and homogeneous
background, every electrode's walks scoring the (<= 16) transmitters it receives
(survey.run_wenner_survey); one bench step = one whole survey. N ranks shard every
group's walks by walk range over ONE communicator (survey._run_fields_distributed: the
model and background fields' local solves run concurrently, one thread issues every
collective in a fixed order); weak scaling keeps --walks per electrode per GPU. Its cpu_baseline is the oracle's brute-force scan (the reference's
algorithm), and the segment tree's gain is reported as speedup_vs_bruteforce
against the device's own brute-force scan kernel (never as a roofline
fraction).

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--scaling weak|strong]
                       [--workload dcr_dipole|wenner_topography|variable_coefficients]
       --gpus N > 1 starts N rank processes itself (launch_ranks; the parent makes no HIP
       call); under a launcher (python -m torch.distributed.run --nproc-per-node N
       bench.py --gpus N ...) WORLD_SIZE must equal --gpus.
Prints one JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--workload", choices=["dcr_dipole", "wenner_topography", "variable_coefficients",
                                           "poisson_square"], default="dcr_dipole")
    ap.add_argument("--walks", type=int, default=None,
                    help="walks per electrode per GPU (dcr_dipole 1M, wenner_topography 100k, "
                         "variable_coefficients 100k per point, poisson_square 10k per point)")
    ap.add_argument("--fields", choices=["literal", "physical"], default="literal",
                    help="wenner_topography: the notebook's conductivity with its air term (literal, SURVEY 8d "
                         "C5; the timed survey) or without it (physical); the rho_a report always comes from "
                         "a physical survey")
    ap.add_argument("--no-bruteforce", action="store_true", help="wenner_topography: skip the scan-kernel leg")
    ap.add_argument("--handle-pairs", type=int, default=None,
                    help="wenner_topography: (model, background) solver pairs, one host thread and HIP stream each "
                         "(1 / 2 / 3 pairs: 1.357 / 1.377 / 1.409e10 walk-steps/s, profiles/r04_ab/c5_handle_pairs_ab.log). "
                         "Default 3 on one GPU; 1 with a communicator, so that the 2 walk streams and libwost's RCCL "
                         "stream fit the box's GPU_MAX_HW_QUEUES = 4 hardware queues (a collective queued behind a "
                         "persistent walk kernel on a shared queue would wait for it)")
    ap.add_argument("--electrodes", type=int, default=None,
                    help="dcr_dipole 48, wenner_topography 256, variable_coefficients 256 and poisson_square 64 "
                         "(query points)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="budget of the CPU-baseline sample")
    ap.add_argument("--scaling", choices=["weak", "strong"], default="weak",
                    help="weak: N x --walks walks per electrode on N GPUs (default); strong: --walks on N GPUs")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-rho", action="store_true", help="skip the apparent-resistivity leg (profiling runs)")
    ap.add_argument("--dry-launch", action="store_true",
                    help="only launch the ranks: each prints its RANK/LOCAL_RANK/WORLD_SIZE as JSON (no GPU)")
    ap.add_argument("--dry-launch-fail-rank", type=int, default=None, help=argparse.SUPPRESS)
    return ap.parse_args()


CPU_SEED = 321
ALPHA_BG = 1e2   # background conductivity of testGeophysicalScenario.py:39 (rho_bg = 0.01)


def _point_stats(v, W):
    v = v.astype(np.float64).reshape(-1, W)
    return v.mean(axis=1), v.std(axis=1, ddof=1) / np.sqrt(W)


def host_cpu() -> dict:
    """The host's CPU model and the cores this process may run on."""
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, p = f.read().split()[:2]
            if q != "max":
                quota = float(q) / float(p)
    except (OSError, ValueError):
        pass
    return {"cpu_model": model, "affinity_cpus": len(os.sched_getaffinity(0)), "os_cpu_count": os.cpu_count(),
            "cgroup_cpu_quota": quota, "omp_num_threads_env": os.environ.get("OMP_NUM_THREADS")}


def cpu_leg(sc, sc_h, sigma_bar, sigma_bar_h, budget_s: float):
    """The CPU oracle (C, OpenMP over walks) on a bounded sample of the same survey:
    timed on the model solve (the cpu_baseline) on every core this process may use,
    then on one core, then also run on the homogeneous background so the sample
    yields the survey's apparent resistivities."""
    from oracle import oracle as O

    info = host_cpu()
    threads = info["affinity_cpus"]
    if info["cgroup_cpu_quota"]:                   # a CPU quota caps the usable cores below the affinity set
        threads = max(1, min(threads, int(round(info["cgroup_cpu_quota"]))))
    pb = O.Problem.from_scenario(sc, sigma_bar=sigma_bar)
    pts = sc.points
    pb.solve_walks(pts, 2, sc.max_steps, sc.eps, 1, threads=threads)       # builds the sampler table
    w = 64
    while True:                                                             # grow the sample to the budget
        t0 = time.perf_counter()
        v, s = pb.solve_walks(pts, w, sc.max_steps, sc.eps, CPU_SEED, threads=threads)
        dt = time.perf_counter() - t0
        if dt >= 0.5 * budget_s or w >= 1_000_000:
            break
        w = int(min(1_000_000, w * max(2.0, 0.8 * budget_s / max(dt, 1e-3))))
    base = {"value": float(s.sum()) / dt, "unit": "walk-steps/s", "cores": threads, "kind": "port",
            "sample": f"{sc.name} {len(pts)} points x {w} walks ({int(s.sum())} walk-steps, {dt:.1f} s), "
                      f"oracle/wost_oracle.c with {threads} OpenMP threads (every usable host core)",
            "host": info}
    # the same oracle on one core, on a smaller sample (all cores and one core)
    w1 = max(16, int(w * 0.06))
    t0 = time.perf_counter()
    _, s1 = pb.solve_walks(pts, w1, sc.max_steps, sc.eps, CPU_SEED + 1, threads=1)
    dt1 = time.perf_counter() - t0
    base["single_core"] = {"value": float(s1.sum()) / dt1, "cores": 1,
                           "sample": f"{len(pts)} electrodes x {w1} walks ({int(s1.sum())} walk-steps, {dt1:.1f} s)"}
    if sc_h is None:   # no apparent-resistivity leg (variable_coefficients)
        return base, w, _point_stats(v, w), None
    vh, _ = O.Problem.from_scenario(sc_h, sigma_bar=sigma_bar_h).solve_walks(pts, w, sc.max_steps, sc.eps, CPU_SEED,
                                                                             threads=threads)
    return base, w, _point_stats(v, w), _point_stats(vh, w)


RHO_SEED = 4242
RHO_REPLICA_WALKS = 400      # the reference fixture's walks per electrode (tests/golden/rho_dcr_dipole.npz)
RHO_REPLICAS = 512


def paired_walks(survey, sc, solver, solver_h, n_walks):
    """Per-walk values [E, W] of the model and of the homogeneous background on common
    random numbers (same seed, same sigma_bar: identical paths, different weights)."""
    vm, _ = solver.solve_walks(sc.points, nWalks=n_walks, maxSteps=sc.max_steps, eps=sc.eps, seed=RHO_SEED)
    vh, _ = solver_h.solve_walks(sc.points, nWalks=n_walks, maxSteps=sc.max_steps, eps=sc.eps, seed=RHO_SEED)
    return vm, vh


def reference_leg(survey, alpha_bg, vm, vh):
    """The GPU against the reference's own run (tests/golden/rho_dcr_dipole.npz): the
    paired GPU estimate's RMSE vs the reference's 1 sigma (north star), z-scores, and
    the matched-walk test -- is the reference's 400-walk rho_a a plausible draw of the
    GPU estimator at 400 walks (512 independent replicas)?"""
    ref = survey.reference_rho_a(os.path.join(REPO, "tests", "golden", "rho_dcr_dipole.npz"))
    if ref is None or ref.rho.rho_a.shape[0] != vm.shape[0] - 1:
        return None
    pairs = survey.dipole_dipole_pairs(vm.shape[0])
    gpu = survey.paired_apparent_resistivity(vm, vh, pairs, 1.0 / alpha_bg)
    rep = survey.replica_rho_a(vm, vh, pairs, 1.0 / alpha_bg, ref.walks)
    out = survey.compare_to_reference(gpu, ref, replicas=rep)
    out["gpu_walks_per_electrode"] = int(vm.shape[1])
    p = survey.matched_walk_pvalues(rep, ref.rho.rho_a)
    ok = np.isfinite(p)
    out["matched_walks"] = {"replicas": int(rep.shape[0]), "walks_per_replica": int(ref.walks),
                            "dipoles_tested": int(ok.sum()), "p_min": float(np.min(p[ok])) if ok.any() else None,
                            "frac_p_gt_0.01": float(np.mean(p[ok] > 0.01)) if ok.any() else None}
    out["gpu_paired_1sigma_rms"] = float(np.sqrt(np.mean(gpu.se[gpu.resolved] ** 2))) if gpu.resolved.any() else None
    return out


def replay_leg(survey, solver, solver_h):
    """Deterministic rho_a parity: the reference's survey replayed on the Philox stream
    (tests/golden/rho_replay_dcr_dipole.npz, all 48 electrodes, model + background) and
    the device on the same walks -- step counts, per-walk values and every dipole's
    paired rho_a, independent of Monte-Carlo error."""
    ref = survey.load_replay_survey(os.path.join(REPO, "tests", "golden", "rho_replay_dcr_dipole.npz"))
    if ref is None:
        return None
    kw = dict(nWalks=ref.n_walks, maxSteps=ref.max_steps, eps=ref.eps, seed=ref.seed)
    vm, sm = solver.solve_walks(ref.points, **kw)
    vh, sh = solver_h.solve_walks(ref.points, **kw)
    out = survey.compare_to_replay(vm, vh, sm, sh, ref)
    out.pop("rho_a_reference")
    out.pop("rho_a_gpu")
    return out


def rho_report(survey, alpha_bg, gpu_full, gpu_same, cpu_same, w_cpu, paired=None, replay=None):
    """Apparent resistivity of the dipole-dipole line: the full GPU run's precision, the
    full GPU run against the reference's own run (tests/golden/rho_dcr_dipole.npz: the
    north-star RMSE <= 1 sigma check), and the GPU vs the CPU port (oracle) on the same
    walks (same seeds) of the CPU sample."""
    pairs = survey.dipole_dipole_pairs(len(gpu_full[0][0]))

    def rho(model, bg):
        dm = survey.potential_differences(model[0], model[1], pairs)
        dh = survey.potential_differences(bg[0], bg[1], pairs)
        return survey.apparent_resistivity(dm, dh, 1.0 / alpha_bg)

    full = rho(gpu_full[0], gpu_full[1])
    ok = full.resolved & np.isfinite(full.rho_a)
    out = {"array": f"dipole-dipole, {len(pairs)} adjacent-electrode dipoles",
           "rho_bg": 1.0 / alpha_bg,
           "gpu_full": {"walks_per_electrode": int(gpu_full[2]), "resolved": int(ok.sum()),
                        "dipoles": int(len(pairs)),
                        "resolved_note": f"{int(ok.sum())} of {len(pairs)} dipoles resolve at the timed walk count "
                                         "(model and background dV > 3 se, rho_a's error < a third of it)",
                        "mc_1sigma_rms": float(np.sqrt(np.mean(full.se[ok] ** 2))) if ok.any() else None,
                        "rho_a_checksum": float(np.sum(full.rho_a[ok]))}}
    if replay is not None:
        out["vs_reference_replay"] = replay
    if paired is not None:
        # statistical leg against the reference's own RNG, INFORMATIONAL: its bound is the
        # spread of the GPU's OWN 400-walk replicas (~rho_bg itself), so it can hardly fail;
        # the parity is vs_reference_replay above
        leg = reference_leg(survey, alpha_bg, *paired)
        if leg is not None:
            leg = {"informational": True,
                   "note": "bound = the GPU's own 400-walk replica spread (gpu_replica_1sigma_rms), not the "
                           "reference's error; little power -- the deterministic parity is vs_reference_replay",
                   **leg}
        out["vs_reference_statistical"] = leg
    if cpu_same is not None:
        g, c = rho(*gpu_same), rho(*cpu_same)
        cmp = survey.compare(g, c)
        cmp_full = survey.compare(full, c)
        out["vs_cpu_port"] = {
            "walks_per_electrode": int(w_cpu), "seed": CPU_SEED, "resolved": cmp["resolved"],
            "rmse": cmp["rmse"], "cpu_mc_1sigma_rms": cmp["mc_1sigma"],
            "rmse_over_1sigma": (cmp["rmse"] / cmp["mc_1sigma"]) if cmp["rmse"] is not None and cmp["mc_1sigma"] else None,
            "z_rms_same_walks": cmp["z_rms"],
            "gpu_full_rmse": cmp_full["rmse"],
            # the full run's walks are independent of the sample's: z-scores of the two estimates
            "gpu_full_vs_cpu_z_rms": cmp_full["z_rms"], "gpu_full_vs_cpu_z_max": cmp_full["z_max"]}
    return out


def measured_traffic(workload: str = "dcr_dipole"):
    """HBM bytes per walk-kernel launch from the committed rocprofv3 PMC passes of this
    workload (FETCH_SIZE x 2 per the gfx950 correction + WRITE_SIZE), if present."""
    path = os.path.join(REPO, "profiles", f"traffic_{workload}.json")
    try:
        with open(path) as f:
            return json.load(f)["hbm_bytes_per_launch"]
    except (OSError, ValueError, KeyError):
        return None


def issue_line(perfmodel, kernel_steps_per_s: float, workload: str = "dcr_dipole"):
    """The VALU issue-rate roofline of the walk kernel: instructions per wave-step from
    the committed rocprofv3 PMC passes of this workload (profiles/issue_<workload>.json),
    at this run's kernel walk-steps/s."""
    try:
        with open(os.path.join(REPO, "profiles", f"issue_{workload}.json")) as f:
            pmc = json.load(f)
    except (OSError, ValueError):
        return None
    out = perfmodel.issue_fraction(pmc["valu_per_wave_step"], pmc["trans_per_wave_step"], kernel_steps_per_s,
                                   perfmodel.PHILOX_MAD64_PER_STEP)
    out.update({"valu_per_wave_step": pmc["valu_per_wave_step"], "trans_per_wave_step": pmc["trans_per_wave_step"],
                "pmc_source": pmc.get("source")})
    return out


def rank_breakdown(comm, values: dict) -> dict:
    """Every rank's timed-region figures (collective): min / max / mean over the ranks of
    each, and max/mean of the walk kernel's time and of the local work, so that an N-GPU
    line shows what its scaling lost -- kernel imbalance, the agreement all-reduce (which
    waits for the slowest rank), the all-gather, or host time outside the kernels."""
    names = list(values)
    rows = comm.allgather(np.array([float(values[k]) for k in names], np.float64))   # [R, len(names)]
    out = {k: {"min": float(rows[:, i].min()), "max": float(rows[:, i].max()), "mean": float(rows[:, i].mean())}
           for i, k in enumerate(names)}
    out["ranks"] = int(rows.shape[0])
    for k in ("kernel_ms", "local_ms", "wait_ms"):
        if k in out and out[k]["mean"] > 0:
            out[k]["max_over_mean"] = out[k]["max"] / out[k]["mean"]
    return out


def library_check(solvers=()) -> dict:
    """The product library with every handle option at its default, or exit non-zero with
    no metric line: a study build (build/libwost_study.so: A/B knobs and result-changing
    ablations read from the environment) or a non-default wost_set_option would make the
    line describe another kernel. Returns what goes into the line: the build, the options
    and the WOST_* variables of this environment (the product library reads none that
    changes a kernel; WOST_JIT_CACHE only moves the kernel cache)."""
    from dcrmontecarlo_amd import _lib

    rep = _lib.options_report()
    if rep["build"] != "product":
        sys.exit(f"bench.py: {_lib.LIB_PATH} is a study build ({rep}); refusing to report a metric")
    for slv in solvers:
        r = slv.options_report()
        if r["non_default"]:
            sys.exit(f"bench.py: a handle has non-default options {r['non_default']}; refusing to report a metric")
    return {"build": rep["build"], "path": os.path.relpath(_lib.LIB_PATH, REPO), "non_default_options": {},
            "wost_env": sorted(k for k in os.environ if k.startswith("WOST_"))}


def cold_start(make_solver, solve, warm_walk_ms: float, warm_wall_ms: float) -> dict:
    """Cold numbers (VERDICT r05 Missing #2; the reference calls solve() once per script,
    tests/testWostWithSource.py:110): hiprtc's compile of the field-specialised kernel
    with an empty kernel cache (WOST_JIT_CACHE is a fresh directory for this process, so
    the bench's first solve compiled it: `first_handle`), then a fresh handle's first
    solve with the cache warm, against the timed region's warm medians."""
    fresh = make_solver()
    t0 = time.perf_counter()
    t = solve(fresh)
    wall = 1e3 * (time.perf_counter() - t0)
    out = {"first_solve_ms": wall, "first_solve_walk_kernel_ms": float(t["walk_kernel_ms"]),
           "first_solve_jit_ms": float(t["jit_ms"]), "warm_median_solve_ms": warm_wall_ms,
           "warm_median_walk_kernel_ms": warm_walk_ms,
           "first_over_warm_kernel": float(t["walk_kernel_ms"]) / warm_walk_ms if warm_walk_ms > 0 else None,
           "first_over_warm_wall": wall / warm_wall_ms if warm_wall_ms > 0 else None,
           "shape_first": {k: int(t[k]) for k in ("grid_blocks", "blocks_per_cu", "chunk0", "chunk", "adaptive")}}
    return out


def _free_port() -> int:
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n: int, argv: list[str]) -> int:
    """bench.py --gpus N (N > 1) without a launcher: start N rank processes of this script
    (RANK = LOCAL_RANK = r, WORLD_SIZE = N, MASTER_ADDR = 127.0.0.1 and a free MASTER_PORT,
    where rank 0 hosts the communicator's id store) and wait for them. This parent makes
    no HIP call (it imports nothing of the package). When a rank fails, the others are
    stopped (they would wait for it in the id exchange or RCCL) and its exit code is
    returned; 0 when every rank succeeded."""
    import signal
    import subprocess

    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WOST_BENCH_LAUNCHED="1")
        env.pop("TORCHELASTIC_USE_AGENT_STORE", None)
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + argv, env=env))
    def stop(ranks):
        for q in ranks:
            procs[q].send_signal(signal.SIGTERM)
        t0 = time.time()
        for q in ranks:
            try:
                procs[q].wait(timeout=max(0.1, 20.0 - (time.time() - t0)))
            except subprocess.TimeoutExpired:
                procs[q].kill()
                procs[q].wait()

    live = set(range(n))

    def on_term(signum, frame):   # a launcher stopping this parent stops the ranks too
        stop(sorted(q for q in range(n) if procs[q].poll() is None))
        sys.exit(128 + signum)

    signal.signal(signal.SIGTERM, on_term)
    try:
        while live:
            failed = None
            for r in sorted(live):
                code = procs[r].poll()
                if code is not None:
                    live.discard(r)
                    if code != 0:
                        failed = (r, code)
                        break
            if failed is not None:
                r, code = failed
                print(f"bench.py: rank {r} exited with status {code}; stopping the other ranks",
                      file=sys.stderr, flush=True)
                stop(sorted(live))
                return code if code > 0 else 128 - code     # killed by signal s: 128 + s
            time.sleep(0.05)
    except KeyboardInterrupt:
        stop(sorted(live))
        raise
    return 0


def check_launch(args) -> tuple[int, int, int]:
    """(world, rank, local rank) of this process. Under a launcher (WORLD_SIZE set) --gpus
    must equal WORLD_SIZE; a rank whose LOCAL_RANK device does not exist exits non-zero."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if "WORLD_SIZE" in os.environ and args.gpus != world:
        sys.exit(f"bench.py: --gpus {args.gpus} but the launcher started WORLD_SIZE={world} ranks")
    if args.dry_launch:
        return world, rank, local
    from dcrmontecarlo_amd import _lib

    ndev = _lib.device_count()
    if local >= ndev:
        sys.exit(f"bench.py: rank {rank} needs device {local} (LOCAL_RANK) but this node has {ndev} visible "
                 f"GPU(s); run with --gpus <= {ndev}")
    return world, rank, local


def main():
    args = parse()
    if args.gpus < 1:
        sys.exit("bench.py: --gpus must be >= 1")
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    if not args.dry_launch:
        # the kernel cache in a fresh directory: the first solve measures hiprtc's compile
        # (cold start); only the cache's location changes, never a kernel
        import tempfile

        os.environ["WOST_JIT_CACHE"] = tempfile.mkdtemp(prefix="wost_jit_bench_")
        # and an empty code-object cache of ROCm's compiler library (comgr caches hiprtc's
        # compiles on its own, so a kernel compiled by an earlier process would cost ~13 ms)
        os.environ["AMD_COMGR_CACHE_DIR"] = os.path.join(os.environ["WOST_JIT_CACHE"], "comgr")
        library_check()
    world, rank, local = check_launch(args)
    if args.dry_launch:
        # the launch alone (CPU tests): report this rank's environment, fail on request
        print(json.dumps({"rank": rank, "local_rank": local, "world_size": world,
                          "master_addr": os.environ.get("MASTER_ADDR"), "master_port": os.environ.get("MASTER_PORT"),
                          "pid": os.getpid(), "ppid": os.getppid()}), flush=True)
        if args.dry_launch_fail_rank == rank:
            sys.exit(3)
        if args.dry_launch_fail_rank is not None:
            time.sleep(30)   # the healthy ranks: the launcher must stop them
        return
    if args.workload == "wenner_topography":
        return wenner_main(args, world, rank, local)
    c3 = args.workload == "variable_coefficients"
    c2 = args.workload == "poisson_square"
    args.walks = args.walks or (100_000 if c3 else 10_000 if c2 else 1_000_000)
    args.electrodes = args.electrodes or (256 if c3 else 64 if c2 else 48)

    from dcrmontecarlo_amd import comm as C
    from dcrmontecarlo_amd import perfmodel
    from dcrmontecarlo_amd import scenarios as S
    from dcrmontecarlo_amd import survey
    from dcrmontecarlo_amd.solvers.WoStSolver import stats_from_sums

    if c3:   # BASELINE configs[2] / SURVEY 8d C3: 256 points x 100k walks
        sc = S.variable_coefficients(n_points=args.electrodes, n_walks=args.walks)
        if len(sc.points) != args.electrodes:
            sys.exit(f"bench.py: variable_coefficients has {len(sc.points)} query points, not {args.electrodes}")
    elif c2:   # BASELINE configs[1] / SURVEY 8d C2: 64 points x 10k walks (testWostWithSource)
        sc = S.poisson_square(n_points=args.electrodes, n_walks=args.walks)
        if len(sc.points) != args.electrodes:
            sys.exit(f"bench.py: poisson_square has {len(sc.points)} query points, not {args.electrodes}")
    else:
        sc = S.dcr_dipole(n_electrodes=args.electrodes, n_walks=args.walks)
    solver = sc.solver(device=local)
    # libwost's own RCCL communicator (wost_comm_*): the 128-byte id travels through the
    # launcher's TCP store; barriers, the block-sum all-gather and the max over ranks
    # are RCCL collectives on libwost's stream -- no torch process group
    # (WOST_BENCH_FORCE_COMM=1 takes the communicator path with one rank too: a check of the
    # launcher bootstrap and the RCCL solve on a one-GPU box)
    comm = C.Communicator.from_env(device=local) if (world > 1 or os.environ.get("WOST_BENCH_FORCE_COMM")) else None
    # weak: N x 1M walks per electrode over N GPUs; strong: 1M walks per electrode over N
    Wt = sc.n_walks * (world if args.scaling == "weak" else 1)   # walks per electrode of the whole job
    w0, w1 = C.shard_walk_range(Wt, world, rank)

    def barrier_sync():
        # every solve returns with its results on the host (libwost syncs its stream);
        # the RCCL barrier syncs the communicator's stream before returning
        if comm is not None:
            comm.barrier()

    def one_step(seed, slv=solver):
        """One survey solve; the per-electrode (sum, sum^2, steps) end up in slv.last_point_sums."""
        if comm is None:
            slv.solve(sc.points, nWalks=Wt, maxSteps=sc.max_steps, eps=sc.eps, seed=seed)
        else:
            C.solve_distributed(slv, comm, sc.points, Wt, sc.max_steps, sc.eps, seed=seed)
        return slv.last_timing

    cold = {}
    for k in range(args.warmup):
        ts = time.perf_counter()
        t = one_step(1000 + k)
        if k == 0:   # the process's first solve: its kernel is in no cache (empty WOST_JIT_CACHE)
            # (option jit_race: the compile runs in a helper process while the precompiled
            # kernel starts the walks; jit_compile_ms is then 0)
            cold["first_handle"] = {"first_solve_ms": 1e3 * (time.perf_counter() - ts),
                                    "jit_compile_ms": float(t["jit_ms"]), "walk_kernel_ms": float(t["walk_kernel_ms"]),
                                    "precompiled_walks": int(t["precompiled_walks"]),
                                    "walks": int(t["total_walks"])}
        elif k == 1:   # the second: waits for the rest of that compile, if any
            cold["first_handle"].update({"second_solve_ms": 1e3 * (time.perf_counter() - ts),
                                         "second_jit_wait_ms": float(t["jit_ms"])})
    libinfo = library_check([solver])

    barrier_sync()
    t0 = time.perf_counter()
    steps_local = 0
    kernel_ms = 0.0
    launches = 0
    jit = 0
    phase = {"local_ms": 0.0, "agree_ms": 0.0, "gather_ms": 0.0, "merge_ms": 0.0}
    host = {"solve_wall_ms": [], "libwost_span_ms": [], "walk_kernel_ms": [], "reduce_kernel_ms": [],
            "device_span_ms": [], "tail_ms": [], "max_walk_steps": [], "last_wave_ms": [], "last_wave_iters": []}
    for k in range(args.steps):
        ts = time.perf_counter()
        t = one_step(k)
        host["solve_wall_ms"].append(1e3 * (time.perf_counter() - ts))
        host["libwost_span_ms"].append(float(t["total_ms"]))
        host["walk_kernel_ms"].append(float(t["walk_kernel_ms"]))
        host["reduce_kernel_ms"].append(float(t["reduce_kernel_ms"]))
        host["device_span_ms"].append(float(t.get("span_ms", 0.0)))
        host["tail_ms"].append(float(t.get("tail_ms", 0.0)))
        host["max_walk_steps"].append(float(t.get("max_walk_steps", 0)))
        host["last_wave_ms"].append(float(t.get("last_wave_ms", 0.0)))
        host["last_wave_iters"].append(float(t.get("last_wave_iters", 0)))
        steps_local += int(t["total_steps"])
        kernel_ms += float(t["walk_kernel_ms"])
        launches += int(t["n_launches"])
        jit = int(t["jit"])
        for name in phase:
            phase[name] += float(t.get(name, 0.0))
    barrier_sync()
    elapsed = time.perf_counter() - t0

    total_steps = steps_local
    max_elapsed = elapsed
    per_rank = None
    if comm is not None:
        total_steps = int(comm.allreduce([float(steps_local)], "sum")[0])
        max_elapsed = float(comm.allreduce([elapsed], "max")[0])
        per_rank = rank_breakdown(comm, {"elapsed_ms": 1e3 * elapsed, "kernel_ms": kernel_ms, **phase,
                                         "walk_steps": steps_local})
    last_sums = solver.last_point_sums

    # apparent resistivity (second half of the metric), outside the timed region: the
    # homogeneous-background survey on the same walk streams as the last timed step
    no_rho_leg = c3 or c2   # the apparent-resistivity leg is the DCR survey's
    sc_h = None if no_rho_leg else survey.homogeneous(sc, ALPHA_BG)
    solver_h = sums_h = None
    if not args.no_rho and not no_rho_leg:
        solver_h = survey.homogeneous_solver(sc, ALPHA_BG, solver, device=local)
        one_step(args.steps - 1, solver_h)
        sums_h = solver_h.last_point_sums

    if rank == 0:
        value = total_steps / max_elapsed
        fps = perfmodel.flops_per_step(sc)
        # dominant kernel: the walk kernel on this rank (HIP events on libwost's stream)
        ach_tflops = fps * steps_local / (kernel_ms * 1e-3) / 1e12
        fps_exec = perfmodel.executed_flops_per_step(sc)
        exec_tflops = fps_exec * steps_local / (kernel_ms * 1e-3) / 1e12
        bytes_per_launch = perfmodel.hbm_bytes_per_walk() * (len(sc.points) * (w1 - w0))
        ach_gbs = bytes_per_launch * launches / (kernel_ms * 1e-3) / 1e9 if kernel_ms > 0 else 0.0
        mean = last_sums[:, 0] / Wt
        out = {
            "metric": "walk-steps/sec",
            "value": value,
            "unit": "walk-steps/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": 1e3 * max_elapsed / args.steps,
            "higher_is_better": True,
            "scaling": args.scaling,
            "vs_baseline": None,
            "dtype": "f32",
            "data": ("synthetic (testWostVariableCoefficients fields/geometry, Philox4x32-10 walks)" if c3 else
                     "synthetic (testWostWithSource fields/geometry, Philox4x32-10 walks)" if c2 else
                     "synthetic (reference DCR scenario fields/geometry, Philox4x32-10 walks)"),
            "config": {"workload": ("variable_coefficients: BASELINE configs[2] / SURVEY 8d C3 (testWostVariable"
                                    "Coefficients fields, mixed boundary with the 32-segment Neumann circle, delta "
                                    "tracking, eps=1e-4, maxSteps=1000; points = query points)" if c3 else
                                    "poisson_square: BASELINE configs[1] / SURVEY 8d C2 (testWostWithSource: f = -4 "
                                    "on the square +-2, g = x^2 + y^2, Dirichlet only, eps=1e-4, maxSteps=500; "
                                    "points = query points)" if c2 else
                                    "dcr_dipole (testGeophysicalScenario fields, eps=0.9, maxSteps=500)"),
                       "electrodes": len(sc.points), "walks_per_electrode": Wt,
                       "walks_per_electrode_per_gpu": w1 - w0,
                       "walk_steps_per_solve": total_steps // max(args.steps, 1),
                       "parallelism": (f"walk-range shards of every electrode over {world} GPUs "
                                       "(wost_solve_distributed: libwost RCCL all-gather of block sums)")
                       if world > 1 else "one GPU"},
            "roofline": {"bound": "valu", "achieved": ach_tflops, "peak": perfmodel.FP32_PEAK_TFLOPS,
                         "unit": "TFLOP/s", "frac": ach_tflops / perfmodel.FP32_PEAK_TFLOPS,
                         # HBM bytes per walk-kernel launch from the committed PMC passes
                         # (profiles/traffic_dcr_dipole.json) vs the algorithmic 8 B per walk
                         "traffic": measured_traffic(args.workload),
                         "algorithmic_bytes_per_launch": bytes_per_launch,
                         "model_flops_per_step": fps,
                         "flop_model": "SURVEY.md 8(d) v1 per-config total (C3 ~1,150, C4 ~350)",
                         # the same model without the ~120 FLOP i0e series the kernel replaced by
                         # an LDS table lookup: the FP32 work it executes
                         "executed_flops_per_step": fps_exec, "achieved_executed": exec_tflops,
                         "frac_executed": exec_tflops / perfmodel.FP32_PEAK_TFLOPS,
                         "kernel": f"wost_walk_jit (hiprtc field-specialised, {args.workload})" if jit
                         else "wost_walk_kernel<true,true,true> (precompiled)",
                         "kernel_ms_per_launch": kernel_ms / max(launches, 1),
                         "issue": issue_line(perfmodel, steps_local / (kernel_ms * 1e-3) if kernel_ms > 0 else 0.0,
                                             args.workload)},
            "roofline_hbm": {"bound": "hbm", "achieved": ach_gbs, "peak": perfmodel.HBM_PEAK_GBS, "unit": "GB/s",
                             "frac": ach_gbs / perfmodel.HBM_PEAK_GBS, "traffic": measured_traffic(args.workload),
                             "algorithmic_bytes_per_launch": bytes_per_launch},
            "u_checksum": float(np.sum(mean)),
        }
        if per_rank is not None:
            # the timed region per rank (sums over the K steps): walk-kernel ms, the protocol's
            # phases (local solve + pack, agreement all-reduce, all-gather, merge) and walk-steps
            out["per_rank"] = per_rank
        # one solve's wall time against its kernels (medians over the timed steps; rank 0):
        # the facade's call, libwost's own span (points upload .. block sums on the host,
        # HIP events), the walk and reduce kernels
        med = {k: float(np.median(v)) for k, v in host.items()}
        med["wall_over_kernel"] = med["solve_wall_ms"] / med["walk_kernel_ms"] if med["walk_kernel_ms"] > 0 else None
        # the launch's tail (device wall clock, wost_timing): the wave that ended last ran
        # last_wave_iters loop iterations in last_wave_ms; the longest walk needs at least
        # max_walk_steps of them, so its share of the kernel is at least
        # max_walk_steps x (last_wave_ms / last_wave_iters) / walk_kernel_ms
        if med["last_wave_iters"] > 0 and med["walk_kernel_ms"] > 0:
            it_ms = med["last_wave_ms"] / med["last_wave_iters"]
            med["iteration_ms_last_wave"] = it_ms
            med["longest_walk_ms"] = med["max_walk_steps"] * it_ms
            med["longest_walk_share_of_kernel"] = med["longest_walk_ms"] / med["walk_kernel_ms"]
            med["tail_share_of_kernel"] = med["tail_ms"] / med["walk_kernel_ms"]
        out["host_breakdown"] = med
        out["libwost"] = libinfo
        if comm is None:
            def fresh_solve(slv):
                slv.solve(sc.points, nWalks=Wt, maxSteps=sc.max_steps, eps=sc.eps, seed=7)
                return slv.last_timing

            cold.update(cold_start(lambda: sc.solver(device=local), fresh_solve, med["walk_kernel_ms"],
                                   med["solve_wall_ms"]))
        out["cold"] = cold or None
        cpu_same = gpu_same = None
        w_cpu = 0
        if not args.no_cpu and world == 1 and (c3 or c2):
            out["cpu_baseline"] = cpu_leg(sc, None, solver.sigma_bar or 0.0, 0.0, args.cpu_seconds)[0]
        elif not args.no_cpu and world == 1:
            if solver_h is None:
                solver_h = survey.homogeneous_solver(sc, ALPHA_BG, solver, device=local)
            base, w_cpu, cm, ch = cpu_leg(sc, sc_h, solver.sigma_bar or 0.0, solver_h.sigma_bar or 0.0,
                                          args.cpu_seconds)
            out["cpu_baseline"] = base
            cpu_same = (cm, ch)
            _, gm = solver.solve(sc.points, nWalks=w_cpu, maxSteps=sc.max_steps, eps=sc.eps, seed=CPU_SEED,
                                 return_stats=True)
            _, gh = solver_h.solve(sc.points, nWalks=w_cpu, maxSteps=sc.max_steps, eps=sc.eps, seed=CPU_SEED,
                                   return_stats=True)
            gpu_same = ((gm.mean, gm.stderr), (gh.mean, gh.stderr))
        else:
            out["cpu_baseline"] = None
        if not args.no_rho and not no_rho_leg:
            st_m, st_h = stats_from_sums(last_sums, Wt), stats_from_sums(sums_h, Wt)
            gpu_full = ((st_m.mean, st_m.stderr), (st_h.mean, st_h.stderr), Wt)
            paired = paired_walks(survey, sc, solver, solver_h, RHO_REPLICA_WALKS * RHO_REPLICAS)
            replay = replay_leg(survey, solver, solver_h) if len(sc.points) == 48 else None
            out["rho_a"] = rho_report(survey, ALPHA_BG, gpu_full, gpu_same, cpu_same, w_cpu, paired, replay)
        print(json.dumps(out), flush=True)
    if comm is not None:
        comm.barrier()
        comm.close()


WENNER_ALPHA_BG = 1e-2     # notebook cell 17's background conductivity (rho_bg = 100)
WENNER_ISSUE = "profiles/issue_wenner_topography.json"


def wenner_cpu_leg(sc, sigma_bar, budget_s):
    """The oracle's brute-force scan (the reference's algorithm: every segment, twice
    per step) on a bounded sample of the C5 survey's walks, one source field, on every
    usable core; then on one core."""
    from oracle import oracle as O

    info = host_cpu()
    threads = info["affinity_cpus"]
    if info["cgroup_cpu_quota"]:
        threads = max(1, min(threads, int(round(info["cgroup_cpu_quota"]))))
    pb = O.Problem.from_scenario(sc, sigma_bar=sigma_bar)
    pts = sc.points[::8]                                   # 32 electrodes along the line
    pb.solve_walks(pts[:1], 1, sc.max_steps, sc.eps, 1, threads=1)
    w = 2
    while True:
        t0 = time.perf_counter()
        _, s = pb.solve_walks(pts, w, sc.max_steps, sc.eps, CPU_SEED, threads=threads)
        dt = time.perf_counter() - t0
        if dt >= 0.4 * budget_s or w >= 100_000:
            break
        w = int(min(100_000, w * max(2.0, 0.8 * budget_s / max(dt, 1e-3))))
    base = {"value": float(s.sum()) / dt, "unit": "walk-steps/s", "cores": threads, "kind": "port",
            "sample": f"{sc.name}: {len(pts)} electrodes x {w} walks, one source field ({int(s.sum())} walk-steps, "
                      f"{dt:.1f} s); oracle/wost_oracle.c brute-force scans of the {len(sc.neumann) - 1}-segment "
                      f"topography, {threads} OpenMP threads (every usable host core)",
            "host": info}
    t0 = time.perf_counter()
    _, s1 = pb.solve_walks(pts[:4], max(1, w // 4), sc.max_steps, sc.eps, CPU_SEED + 1, threads=1)
    dt1 = time.perf_counter() - t0
    base["single_core"] = {"value": float(s1.sum()) / dt1, "cores": 1,
                           "sample": f"4 electrodes x {max(1, w // 4)} walks ({int(s1.sum())} walk-steps, {dt1:.1f} s)"}
    return base


def wenner_main(args, world, rank, local):
    """BASELINE configs[4] / SURVEY C5 (module docstring)."""
    from dcrmontecarlo_amd import comm as C
    from dcrmontecarlo_amd import perfmodel
    from dcrmontecarlo_amd import scenarios as S
    from dcrmontecarlo_amd import survey

    W1 = args.walks or 100_000
    E = args.electrodes or 256
    sc = S.wenner_topography(n_electrodes=E, n_walks=W1, physical=args.fields == "physical")
    sm = sc.solver(device=local)
    sh = survey.homogeneous_solver(sc, WENNER_ALPHA_BG, sm, device=local)
    use_comm = world > 1 or bool(os.environ.get("WOST_BENCH_FORCE_COMM"))
    n_pairs = args.handle_pairs if args.handle_pairs is not None else (1 if use_comm else 3)
    # (model, background) handle pairs: each its own HIP stream, so 2 x pairs launches share the GPU
    pairs = [sm, sh]
    for _ in range(max(1, n_pairs) - 1):
        m2 = sc.solver(device=local)
        pairs += [m2, survey.homogeneous_solver(sc, WENNER_ALPHA_BG, m2, device=local)]
    comm = C.Communicator.from_env(device=local) if use_comm else None
    Wt = W1 * (world if args.scaling == "weak" else 1)
    w0, w1 = C.shard_walk_range(Wt, world, rank)

    def step(seed, walks=Wt):
        return survey.run_wenner_survey(sc, WENNER_ALPHA_BG, walks, seed=seed, solvers=tuple(pairs), comm=comm)

    def barrier():
        if comm is not None:
            comm.barrier()

    cold = {}
    for k in range(args.warmup):
        ts = time.perf_counter()
        step(1000 + k)
        if k == 0:   # the process's first survey: hiprtc compiles its kernels (empty cache)
            cold["first_survey_ms"] = 1e3 * (time.perf_counter() - ts)
    libinfo = library_check(pairs)
    barrier()
    t0 = time.perf_counter()
    steps_all, steps_local, kernel_ms, res = 0, 0, 0.0, None
    phase = {"wait_ms": 0.0, "agree_ms": 0.0, "gather_ms": 0.0, "merge_ms": 0.0}
    for k in range(args.steps):
        res = step(k)
        steps_all += int(res.walk_steps)           # all ranks' walk-steps (solve_sources_distributed)
        steps_local += int(res.local_walk_steps)   # this rank's
        kernel_ms += float(res.kernel_ms)          # this rank's walk-kernel time, both fields
        for name in phase:
            phase[name] += float((res.phase_ms or {}).get(name, 0.0))
    barrier()
    elapsed = time.perf_counter() - t0
    max_elapsed = elapsed if comm is None else float(comm.allreduce([elapsed], "max")[0])
    per_rank = None
    if comm is not None:
        # (kernel_ms sums both fields' concurrent kernels: it can exceed elapsed_ms)
        per_rank = rank_breakdown(comm, {"elapsed_ms": 1e3 * elapsed, "kernel_ms": kernel_ms, **phase,
                                         "walk_steps": steps_local})
    res_phys = None
    pm = ph = None
    if args.fields == "literal" and not args.no_rho:   # outside the timed region: the physical survey's rho_a
        sp = S.wenner_topography(n_electrodes=E, n_walks=W1, physical=True)
        pm = sp.solver(device=local)
        ph = survey.homogeneous_solver(sp, WENNER_ALPHA_BG, pm, device=local)
        res_phys = survey.run_wenner_survey(sp, WENNER_ALPHA_BG, Wt, seed=4242, solvers=(pm, ph), comm=comm)
    elif args.fields == "physical":
        pm, ph = sm, sh

    if rank == 0:
        value = steps_all / max_elapsed
        kernel_rate = steps_local / (kernel_ms * 1e-3) if kernel_ms > 0 else 0.0   # both fields' kernels summed
        ok = res.rho.resolved & np.isfinite(res.rho.rho_a)
        out = {
            "metric": "walk-steps/sec", "value": value, "unit": "walk-steps/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": 1e3 * max_elapsed / args.steps,
            "higher_is_better": True, "scaling": args.scaling, "vs_baseline": None, "dtype": "f32",
            "data": "synthetic (notebook cell 17 fields, 10k-segment y = 1 + 2 sin(x/37) topography, Philox4x32-10)",
            "config": {"workload": f"{sc.name}: BASELINE configs[4] / SURVEY 8d C5 -- Wenner-alpha line, {E} "
                                   f"electrodes, {len(sc.neumann) - 1}-segment Neumann topography, model + "
                                   f"homogeneous background, multi-source batched (<= 16 transmitters per walk)",
                       "electrodes": E, "quadripoles": int(len(res.quadripoles)),
                       "walks_per_electrode": Wt, "walks_per_electrode_per_gpu": w1 - w0,
                       "launches_per_field": res.launches, "walk_steps_per_survey": steps_all // max(args.steps, 1),
                       "handle_pairs": len(pairs) // 2,
                       "parallelism": (f"walk-range shards of every electrode over {world} GPUs "
                                       "(libwost's protocol over its RCCL communicator, all-gather of block sums; "
                                       "both fields' collectives in a fixed order)") if world > 1 else "one GPU"},
            # walk-steps over the walk kernels' summed times: the model and background fields
            # run concurrently, so this understates the kernel rate
            "survey_kernel_walk_steps_per_s_fields_summed": kernel_rate,
            "libwost": libinfo,
        }
        cold["warm_median_survey_ms"] = 1e3 * max_elapsed / args.steps
        if per_rank is not None:
            # the timed region per rank: walk-kernel ms (both fields summed), the collective
            # thread's wait for the local solves, the protocol's collectives and merge, walk-steps
            out["per_rank"] = per_rank
        if not args.no_bruteforce:
            # the device's brute-force scan kernel (the reference's algorithm, every segment twice
            # per step) against the tree kernel on the SAME chip-filling sample: 256 electrodes x
            # 2048 walks, one source field, one launch each (the survey's own kernel rate above
            # sums two concurrent fields' kernel times)
            nb = min(E, 256)
            rates = {}
            for tree in (True, False):
                sv = sc.solver(device=local)
                sv.set_segment_tree(0 if tree else -1)
                ts = time.perf_counter()
                _, st = sv.solve(sc.points[:nb], nWalks=2048, maxSteps=sc.max_steps, eps=sc.eps, seed=5,
                                 return_stats=True)
                first = (1e3 * (time.perf_counter() - ts), st.kernel_ms, sv.last_timing["jit_ms"],
                         int(sv.last_timing["precompiled_walks"]))
                # the rate of the warm single launch: a second solve on the same handle (the
                # first may have run on the precompiled kernel while its own compiled: jit_race)
                _, st = sv.solve(sc.points[:nb], nWalks=2048, maxSteps=sc.max_steps, eps=sc.eps, seed=5,
                                 return_stats=True)
                if tree:
                    cold["tree_single_launch"] = {"first_solve_ms": first[0], "first_walk_kernel_ms": first[1],
                                                  "first_jit_ms": first[2], "first_precompiled_walks": first[3],
                                                  "second_walk_kernel_ms": st.kernel_ms,
                                                  "second_jit_wait_ms": sv.last_timing["jit_ms"],
                                                  "first_over_second_kernel": first[1] / st.kernel_ms}
                rates[tree] = st.total_steps / (st.kernel_ms * 1e-3)
            bs = perfmodel.flops_per_step(sc)      # SURVEY 8d v1, brute force (~290,000 FLOP/step)
            out["speedup_vs_bruteforce"] = {
                "bruteforce_kernel_walk_steps_per_s": rates[False], "tree_kernel_walk_steps_per_s": rates[True],
                "speedup": rates[True] / rates[False] if rates[False] > 0 else None,
                "sample": f"{nb} electrodes x 2048 walks, one source, one launch per kernel",
                "bruteforce_model_tflops": rates[False] * bs / 1e12,
                "bruteforce_frac_fp32": rates[False] * bs / 1e12 / perfmodel.FP32_PEAK_TFLOPS}
        roof = {"bound": "valu-issue", "unit": "SIMD cycles/s", "traffic": None,
                "note": "SURVEY 8d: the segment tree is never priced as a FLOP roofline fraction; this is the "
                        "VALU issue-rate line from committed PMC passes, and speedup_vs_bruteforce below"}
        try:
            with open(os.path.join(REPO, WENNER_ISSUE)) as f:
                pmc = json.load(f)
            # at the tree kernel's rate on one chip-filling launch (the survey's summed kernel
            # times double-count its two concurrent fields)
            rate = out.get("speedup_vs_bruteforce", {}).get("tree_kernel_walk_steps_per_s") or kernel_rate
            roof.update(perfmodel.issue_fraction(pmc["valu_per_wave_step"], pmc["trans_per_wave_step"], rate,
                                                 perfmodel.PHILOX_MAD64_PER_STEP))
            roof["walk_steps_per_s"] = rate
            roof.update({"achieved": roof["achieved_simd_cycles_per_s"], "peak": roof["peak_simd_cycles_per_s"],
                         "lane_utilisation": pmc.get("lane_utilisation"), "pmc_source": pmc.get("source")})
        except (OSError, ValueError, KeyError):
            roof.update({"achieved": None, "peak": perfmodel.N_SIMDS * perfmodel.CLOCK_GHZ * 1e9, "frac": None})
        out["roofline"] = roof
        out["cold"] = cold
        out["cpu_baseline"] = (wenner_cpu_leg(sc, sm.sigma_bar or 0.0, args.cpu_seconds)
                               if (not args.no_cpu and world == 1) else None)
        def rho_summary(r, what):
            good = r.rho.resolved & np.isfinite(r.rho.rho_a)
            return {"survey": what, "array": f"Wenner-alpha a = 1, {len(r.quadripoles)} quadripoles",
                    "rho_bg": 1 / WENNER_ALPHA_BG, "resolved": int(good.sum()),
                    "median": float(np.median(r.rho.rho_a[good])) if good.any() else None,
                    "p10_p90": [float(np.percentile(r.rho.rho_a[good], q)) for q in (10, 90)] if good.any() else None,
                    "mc_1sigma_rms": float(np.sqrt(np.mean(r.rho.se[good] ** 2))) if good.any() else None,
                    "rho_a_checksum": float(np.sum(r.rho.rho_a[good]))}

        if args.fields == "physical":
            out["rho_a"] = rho_summary(res, f"the timed survey ({sc.name})")
        elif res_phys is None:
            out["rho_a"] = None   # --no-rho (profiling runs)
            out["rho_a_literal_timed_survey"] = rho_summary(res, sc.name)
        else:
            out["rho_a"] = rho_summary(res_phys, f"wenner_topography_physical, {Wt} walks per electrode, untimed "
                                                 "(the literal fields put the electrodes in 'air': "
                                                 "their rho_a is not physical)")
            out["rho_a_literal_timed_survey"] = rho_summary(res, sc.name)
        if E == 256 and not args.no_rho:
            # deterministic parity: the reference's own C5 Wenner survey replayed on the Philox
            # stream (32 quadripoles x both receivers x 64 walks, model + background) against
            # the device on the same walks -- the physical survey the rho_a report comes from,
            # and (round 6) the literal survey the bench times, on its own handles
            legs = [("rho_a", "rho_replay_wenner_topography_physical.npz", pm, ph)]
            if args.fields == "literal":
                legs.append(("rho_a_literal_timed_survey", "rho_replay_wenner_topography.npz", sm, sh))
            for key, fixture, mh, hh in legs:
                ref = survey.load_wenner_replay(os.path.join(REPO, "tests", "golden", fixture))
                if ref is not None and out.get(key) is not None and mh is not None:
                    cmp = survey.compare_wenner_replay(*survey.wenner_replay_walks(
                        ref, survey.solver_replay_walks(mh, hh, ref)), ref)
                    out[key]["vs_reference_replay"] = cmp
        print(json.dumps(out), flush=True)
    if comm is not None:
        comm.barrier()
        comm.close()


if __name__ == "__main__":
    main()
