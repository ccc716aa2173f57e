#!/usr/bin/env python3
"""Offline ISA of a scenario's field-specialised walk kernel (no GPU needed).

Generates the kernel source libwost would hand to hiprtc (wost_kernel_source),
compiles it with hipcc for gfx950 with hiprtc's options, and prints the
kernel's resource usage and an instruction histogram (static counts).
Usage: python tools/jit_isa.py dcr_dipole [--out build/jit] [--show]"""
import argparse
import collections
import os
import re
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("scenario")
    ap.add_argument("--out", default=os.path.join(REPO, "build", "jit"))
    ap.add_argument("--show", action="store_true", help="print the ISA")
    ap.add_argument("--waves", default=None, help="WOST_JIT_WAVES for the generator")
    a = ap.parse_args()
    if a.waves:
        os.environ["WOST_JIT_WAVES"] = a.waves
    from dcrmontecarlo_amd import scenarios as S

    kw = {"n_walks": 1}
    sc = S.ALL[a.scenario](**({"n_electrodes": 4} if a.scenario in ("dcr_dipole", "wenner_topography") else {}), **kw) \
        if a.scenario in ("dcr_dipole", "wenner_topography") else S.ALL[a.scenario]()
    src = sc.kernel_source()
    os.makedirs(a.out, exist_ok=True)
    hip = os.path.join(a.out, f"{a.scenario}.hip")
    with open(hip, "w") as f:
        f.write(src)
    asm = os.path.join(a.out, f"{a.scenario}.s")
    cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "--offload-device-only", "-S", "-O3", "-std=c++17",
           "-fhip-fp32-correctly-rounded-divide-sqrt", "-ffp-contract=fast-honor-pragmas",
           *([] if os.environ.get("WOST_JIT_SLP") == "1" else ["-fno-slp-vectorize"]),
           "-I", os.path.join(REPO, "include"), "-I", os.path.join(REPO, "dcrmontecarlo_amd", "csrc"), hip, "-o", asm]
    subprocess.run(cmd, check=True)
    text = open(asm).read()
    body = text.split("wost_walk_jit:", 1)[1].split(".Lfunc_end", 1)[0]
    hist = collections.Counter()
    n = 0
    for line in body.splitlines():
        s = line.strip()
        if not s or s.startswith((";", ".", "//")) or s.endswith(":"):
            continue
        op = s.split()[0]
        hist[op] += 1
        n += 1
    meta = {k: re.search(rf"\.{k}:\s+(\d+)", text) for k in ("vgpr_count", "sgpr_count", "lds_size")}
    print(f"{a.scenario}: {n} instructions;", ", ".join(f"{k}={m.group(1)}" for k, m in meta.items() if m))
    for pre in ("v_", "s_", "ds_", "global_", "buffer_", "scratch_"):
        print(f"  {pre}*: {sum(c for o, c in hist.items() if o.startswith(pre))}")
    trans = [o for o in hist if re.match(r"v_(exp|log|rcp|rsq|sqrt|sin|cos)_f32", o)]
    print("  transcendental:", {o: hist[o] for o in trans})
    print("  top:", hist.most_common(25))
    if a.show:
        print(body)


if __name__ == "__main__":
    main()
