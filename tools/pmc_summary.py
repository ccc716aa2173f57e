#!/usr/bin/env python3
"""Per walk-kernel dispatch summary of rocprofv3 --pmc CSVs (one or more passes).
Usage: tools/pmc_summary.py [--steps N] dir1 [dir2 ...]
With --steps (walk-steps of one dispatch) also prints instructions per wave-step."""
import argparse
import collections
import csv

ap = argparse.ArgumentParser()
ap.add_argument("dirs", nargs="+")
ap.add_argument("--steps", type=float, default=0.0)
a = ap.parse_args()
rows = collections.defaultdict(dict)
for d in a.dirs:
    for r in csv.DictReader(open(f"{d}/run_counter_collection.csv")):
        if "wost_walk" not in r["Kernel_Name"]:
            continue
        k = r["Dispatch_Id"]
        rows[k]["kernel"] = r["Kernel_Name"][:60]
        rows[k]["grid"] = r["Grid_Size"]
        rows[k][r["Counter_Name"]] = float(r["Counter_Value"])
for k, v in sorted(rows.items(), key=lambda kv: int(kv[0])):
    out = {kk: (f"{vv:.4g}" if isinstance(vv, float) else vv) for kk, vv in v.items()}
    if a.steps and "SQ_INSTS_VALU" in v:
        ws = a.steps / 64.0
        out["VALU/wave-step"] = f"{v['SQ_INSTS_VALU'] / ws:.0f}"
        out["SALU/wave-step"] = f"{v.get('SQ_INSTS_SALU', 0) / ws:.0f}"
    if "FETCH_SIZE" in v:
        out["fetch_bytes(x2 gfx950 wide-read correction)"] = f"{v['FETCH_SIZE'] * 1024 * 2:.4g}"
    if "WRITE_SIZE" in v:
        out["write_bytes"] = f"{v['WRITE_SIZE'] * 1024:.4g}"
    print(k, out)
