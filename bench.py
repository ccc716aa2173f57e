#!/usr/bin/env python3
"""Walk-steps/sec of the Walk-on-Stars hot path on MI355X.

Workload (BASELINE.json configs[3]): the DCR dipole survey of
tests/testGeophysicalScenario.py -- 48 surface electrodes x 1M walks each,
delta tracking with the reference's conductivity field, mixed Dirichlet /
Neumann boundary, eps = 0.9, maxSteps = 500. One bench "step" is one full
survey solve (48M walks, ~3.9G walk-steps). With N ranks the survey's walk
blocks are split into N contiguous shards (strong scaling); each rank solves
its shard on its own GPU and the per-block partial sums are combined with one
RCCL all_gather over xGMI (the only data-path collective), then summed in
block order, so the result is bitwise independent of N.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W]
       (N > 1: python -m torch.distributed.run --nproc-per-node N bench.py --gpus N ...)
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
    ap.add_argument("--walks", type=int, default=1_000_000, help="walks per electrode")
    ap.add_argument("--electrodes", type=int, default=48)
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="budget of the CPU-baseline sample")
    ap.add_argument("--no-cpu", action="store_true")
    return ap.parse_args()


def cpu_baseline(sc, budget_s: float):
    """The CPU oracle (C, OpenMP over walks) on a bounded sample of the same survey."""
    from oracle import oracle as O

    threads = min(16, len(os.sched_getaffinity(0)))
    pb = O.Problem.from_scenario(sc, sigma_bar=10.0)
    pts = sc.points
    pb.solve_walks(pts, 1, sc.max_steps, sc.eps, 1, threads=threads)       # builds the sampler table
    w = 64
    while True:                                                             # grow the sample to the budget
        t0 = time.perf_counter()
        _, s = pb.solve_walks(pts, w, sc.max_steps, sc.eps, 321, threads=threads)
        dt = time.perf_counter() - t0
        if dt >= 0.5 * budget_s or w >= 1_000_000:
            break
        w = int(min(1_000_000, w * max(2.0, 0.8 * budget_s / max(dt, 1e-3))))
    return {"value": float(s.sum()) / dt, "unit": "walk-steps/sec", "cores": threads, "kind": "port",
            "sample": f"dcr_dipole {len(pts)} electrodes x {w} walks ({int(s.sum())} walk-steps, {dt:.1f} s), "
                      f"oracle/wost_oracle.c with {threads} OpenMP threads"}


def measured_traffic():
    """HBM bytes per walk-kernel launch from the committed rocprofv3 PMC passes of this
    workload (FETCH_SIZE x 2 per the gfx950 correction + WRITE_SIZE), if present."""
    path = os.path.join(REPO, "profiles", "traffic_dcr_dipole.json")
    try:
        with open(path) as f:
            return json.load(f)["hbm_bytes_per_launch"]
    except (OSError, ValueError, KeyError):
        return None


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch
        import torch.distributed as dist

        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    from dcrmontecarlo_amd import distributed as D
    from dcrmontecarlo_amd import perfmodel
    from dcrmontecarlo_amd import scenarios as S

    sc = S.dcr_dipole(n_electrodes=args.electrodes, n_walks=args.walks)
    solver = sc.solver(device=local)
    W = sc.n_walks
    nb = solver.num_blocks(len(sc.points), W)
    b0, b1 = D.shard_range(nb, rank, world)

    def barrier_sync():
        if dist is not None:
            import torch

            dist.barrier()
            torch.cuda.synchronize()

    def one_step(seed):
        bs = solver.solve_blocks(sc.points, W, b0, b1, sc.max_steps, sc.eps, seed=seed)
        t = solver.last_timing
        full = D.gather_block_stats(bs, nb, device=f"cuda:{local}") if dist is not None else bs   # RCCL all_gather
        return D.point_sums(full, len(sc.points)), t

    for k in range(args.warmup):
        one_step(1000 + k)

    barrier_sync()
    t0 = time.perf_counter()
    steps_local = 0
    kernel_ms = 0.0
    launches = 0
    jit = 0
    sums = None
    for k in range(args.steps):
        sums, t = one_step(k)
        steps_local += int(t["total_steps"])
        kernel_ms += float(t["walk_kernel_ms"])
        launches += int(t["n_launches"])
        jit = int(t["jit"])
    barrier_sync()
    elapsed = time.perf_counter() - t0

    total_steps = steps_local
    max_elapsed = elapsed
    if dist is not None:
        import torch

        v = torch.tensor([float(steps_local), elapsed], dtype=torch.float64, device=f"cuda:{local}")
        s_all = v.clone()
        dist.all_reduce(s_all[0:1], op=dist.ReduceOp.SUM)
        e_max = v[1:2].clone()
        dist.all_reduce(e_max, op=dist.ReduceOp.MAX)
        total_steps = int(s_all[0].item())
        max_elapsed = float(e_max.item())

    if rank == 0:
        value = total_steps / max_elapsed
        fps = perfmodel.flops_per_step(sc)
        # dominant kernel: wost_walk_kernel<NEU,SRC,DELTA> on this rank (HIP events on its stream)
        ach_tflops = fps * steps_local / (kernel_ms * 1e-3) / 1e12
        bytes_per_launch = perfmodel.hbm_bytes_per_walk() * (len(sc.points) * W / world)
        ach_gbs = bytes_per_launch * launches / (kernel_ms * 1e-3) / 1e9 if kernel_ms > 0 else 0.0
        mean = sums[:, 0] / W
        out = {
            "metric": "walk-steps/sec",
            "value": value,
            "unit": "walk-steps/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": 1e3 * max_elapsed / args.steps,
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (reference DCR scenario fields/geometry, Philox4x32-10 walks)",
            "config": {"workload": "dcr_dipole (testGeophysicalScenario fields, eps=0.9, maxSteps=500)",
                       "electrodes": len(sc.points), "walks_per_electrode": W,
                       "walk_steps_per_solve": total_steps // max(args.steps, 1),
                       "parallelism": f"walk-block shards x{world}, RCCL all_gather of block sums"},
            "roofline": {"bound": "valu", "achieved": ach_tflops, "peak": perfmodel.FP32_PEAK_TFLOPS,
                         "unit": "TFLOP/s", "frac": ach_tflops / perfmodel.FP32_PEAK_TFLOPS, "traffic": None,
                         "model_flops_per_step": fps,
                         "kernel": "wost_walk_jit (hiprtc field-specialised, mixed+delta)" if jit
                         else "wost_walk_kernel<true,true,true> (precompiled)",
                         "kernel_ms_per_launch": kernel_ms / max(launches, 1)},
            "roofline_hbm": {"bound": "hbm", "achieved": ach_gbs, "peak": perfmodel.HBM_PEAK_GBS, "unit": "GB/s",
                             "frac": ach_gbs / perfmodel.HBM_PEAK_GBS, "traffic": measured_traffic(),
                             "algorithmic_bytes_per_launch": bytes_per_launch},
            "u_checksum": float(np.sum(mean)),
        }
        if not args.no_cpu and world == 1:
            out["cpu_baseline"] = cpu_baseline(S.dcr_dipole(n_electrodes=args.electrodes, n_walks=8),
                                               args.cpu_seconds)
        else:
            out["cpu_baseline"] = None
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
