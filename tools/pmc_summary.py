#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc CSVs per walk-kernel dispatch: instruction mix per
wave-step and issue utilisation. Usage: tools/pmc_summary.py dir1 [dir2 ...]
(walk-steps per dispatch are taken from the matching scenario_bench log if given
with --steps-json)."""
import collections
import csv
import sys

rows = collections.defaultdict(dict)
for d in sys.argv[1:]:
    for r in csv.DictReader(open(f"{d}/run_counter_collection.csv")):
        if "walk_kernel" not in r["Kernel_Name"]:
            continue
        key = (r["Dispatch_Id"] if False else None, r["Kernel_Name"].split("<")[1].split(">")[0], r["Grid_Size"])
        rows[(d, r["Dispatch_Id"])]["kernel"] = r["Kernel_Name"].split("<")[1].split(">")[0]
        rows[(d, r["Dispatch_Id"])]["vgpr"] = r["VGPR_Count"]
        rows[(d, r["Dispatch_Id"])]["sgpr"] = r["SGPR_Count"]
        rows[(d, r["Dispatch_Id"])][r["Counter_Name"]] = float(r["Counter_Value"])
for k, v in sorted(rows.items()):
    print(k, {kk: (f"{vv:.4g}" if isinstance(vv, float) else vv) for kk, vv in v.items()})
