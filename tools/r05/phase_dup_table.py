"""Round 5: the phase-duplication PMC passes (tools/r05/phase_dup.sh) as a per-phase table:
dynamic VALU / SALU / transcendentals per wave-step of the measured solve's walk kernel,
and each phase's cost = (duplicated - baseline). Usage: phase_dup_table.py DIR"""
import csv
import glob
import os
import re
import sys

NAMES = {0: "baseline", 1: "Dirichlet distance (box)", 2: "Philox draw", 4: "direction cos/sin",
         8: "Neumann ray query", 16: "radial sampler", 32: "screened G_norm", 64: "alpha jet at the sample",
         128: "alpha at the ray's point (accepted)", 256: "source f", 512: "sigma' (collisions)"}


def load(d):
    log = open(d + ".log").read()
    steps = int(re.search(r"steps=(\d+)", log).group(1))
    rows = {}
    for r in csv.DictReader(open(os.path.join(d, "run_counter_collection.csv"))):
        if "wost_walk" not in r["Kernel_Name"]:
            continue
        rows.setdefault(int(r["Dispatch_Id"]), {})[r["Counter_Name"]] = float(r["Counter_Value"])
    last = rows[max(rows)]   # the measured solve (the warm-up's dispatch comes first)
    ws = steps / 64.0
    return {k: v / ws for k, v in last.items() if k.startswith("SQ_INSTS")}, steps


def main(root):
    res = {}
    for d in sorted(glob.glob(os.path.join(root, "f*"))):
        if not os.path.isdir(d):
            continue
        bit = int(os.path.basename(d)[1:]) >> 18
        res[bit], _ = load(d)
    base = res[0]
    print(f"{os.path.basename(root)}: per wave-step (64 walk-steps); cost = duplicated - baseline (incl. ~3 merge VALU)")
    print(f"{'phase':38s} {'VALU':>8s} {'SALU':>8s} {'TRANS':>7s} {'LDS':>7s}")
    b = base
    print(f"{'baseline (whole step)':38s} {b['SQ_INSTS_VALU']:8.1f} {b['SQ_INSTS_SALU']:8.1f} "
          f"{b['SQ_INSTS_VALU_TRANS_F32']:7.1f} {b['SQ_INSTS_LDS']:7.1f}")
    for bit in sorted(res):
        if bit == 0:
            continue
        r = res[bit]
        print(f"{NAMES.get(bit, bit):38s} {r['SQ_INSTS_VALU'] - b['SQ_INSTS_VALU']:8.1f} "
              f"{r['SQ_INSTS_SALU'] - b['SQ_INSTS_SALU']:8.1f} {r['SQ_INSTS_VALU_TRANS_F32'] - b['SQ_INSTS_VALU_TRANS_F32']:7.1f} "
              f"{r['SQ_INSTS_LDS'] - b['SQ_INSTS_LDS']:7.1f}")


if __name__ == "__main__":
    main(sys.argv[1])
