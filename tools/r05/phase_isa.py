#!/usr/bin/env python3
"""Round 5: the walk step's instruction budget per phase, offline.

Builds the field-specialised kernel libwost would hand to hiprtc for a scenario with the
step's phase markers on (wost_walk.h WOST_PHASE, an assembly comment per phase: a study
build only -- the comments bound the scheduler's regions), compiles it for gfx950 with
hiprtc's options and counts the instructions of each phase in program order: VALU (and
of those transcendental, 64-bit multiply-add and double-precision), SALU, LDS, memory.
Static counts: straight-line phases execute as counted, the rare branches (the clip's
square roots, sigma' at collisions, termination and refill) are listed separately so
their per-step weight can be applied.
Usage: python tools/r05/phase_isa.py dcr_dipole [--trig auto|exact|fast]"""
import argparse
import collections
import os
import re
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)


def classify(op):
    if re.match(r"v_(exp|log|rcp|rsq|sqrt|sin|cos)_f32", op):
        return "valu_trans"
    if op.startswith("v_mad_u64_u32") or op.startswith("v_mad_i64_i32"):
        return "valu_mad64"
    if re.match(r"v_.*_f64", op):
        return "valu_f64"
    if op.startswith("v_"):
        return "valu"
    if op.startswith("s_"):
        return "salu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("global_", "buffer_", "flat_", "scratch_")):
        return "vmem"
    return "other"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("scenario")
    ap.add_argument("--out", default=os.path.join(REPO, "build", "phase"))
    ap.add_argument("--trig", default=None)
    a = ap.parse_args()
    if a.trig:
        os.environ["WOST_TRIG"] = a.trig
    from dcrmontecarlo_amd import scenarios as S

    sc = S.ALL[a.scenario](n_electrodes=4, n_walks=1) if a.scenario in ("dcr_dipole", "wenner_topography") \
        else S.ALL[a.scenario]()
    src = "#define WOST_PHASE_MARKS 1\n" + sc.kernel_source()
    os.makedirs(a.out, exist_ok=True)
    hip = os.path.join(a.out, f"{a.scenario}.hip")
    with open(hip, "w") as f:
        f.write(src)
    asm = os.path.join(a.out, f"{a.scenario}.s")
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "--offload-device-only", "-S", "-O3", "-std=c++17",
                    "-fhip-fp32-correctly-rounded-divide-sqrt", "-ffp-contract=fast-honor-pragmas", "-fno-slp-vectorize",
                    "-I", os.path.join(REPO, "include"), "-I", os.path.join(REPO, "dcrmontecarlo_amd", "csrc"), hip,
                    "-o", asm], check=True)
    body = open(asm).read().split("wost_walk_jit:", 1)[1].split(".Lfunc_end", 1)[0]
    phase = "prologue"
    order = [phase]
    counts = collections.defaultdict(collections.Counter)
    for line in body.splitlines():
        s = line.strip()
        m = re.search(r"@phase (\w+)", s)
        if m:
            phase = m.group(1)
            if phase not in order:
                order.append(phase)
            continue
        if not s or s.startswith((";", ".", "//")) or s.endswith(":"):
            continue
        op = s.split()[0]
        counts[phase][classify(op)] += 1
        counts[phase]["all"] += 1
    cols = ["valu", "valu_trans", "valu_mad64", "valu_f64", "salu", "lds", "vmem", "all"]
    print(f"{a.scenario} (static instructions per phase, program order; trig {os.environ.get('WOST_TRIG', 'auto')})")
    print(f"{'phase':22s}" + "".join(f"{c:>11s}" for c in cols))
    tot = collections.Counter()
    for p in order:
        c = counts[p]
        tot.update(c)
        print(f"{p:22s}" + "".join(f"{c[k]:11d}" for k in cols))
    print(f"{'total':22s}" + "".join(f"{tot[k]:11d}" for k in cols))


if __name__ == "__main__":
    main()
