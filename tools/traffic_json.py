#!/usr/bin/env python3
"""Writes profiles/traffic_dcr_dipole.json (read by bench.py for roofline.traffic)
from the rocprofv3 FETCH_SIZE and WRITE_SIZE passes of tools/profile_session.sh:
per walk-kernel dispatch, FETCH_SIZE x 2 (the gfx950 correction of
MI355X_MICROARCH.md) + WRITE_SIZE, KB -> bytes, averaged over dispatches.
Usage: tools/traffic_json.py <pmc_fetch dir> <pmc_write dir> <source label> [<workload> [<kernel label>]]
(workload default dcr_dipole -> profiles/traffic_<workload>.json)"""
import csv
import json
import os
import sys


def per_dispatch(d, counter):
    vals = {}
    for r in csv.DictReader(open(os.path.join(d, "run_counter_collection.csv"))):
        # (the field-specialised walk kernel only: a raced first solve also runs the
        # precompiled wost_walk_kernel on walk ranges, jit_race)
        if "wost_walk_jit" in r["Kernel_Name"] and r["Counter_Name"] == counter:
            vals[r["Dispatch_Id"]] = vals.get(r["Dispatch_Id"], 0.0) + float(r["Counter_Value"])
    return list(vals.values())


def main():
    fetch = per_dispatch(sys.argv[1], "FETCH_SIZE")
    write = per_dispatch(sys.argv[2], "WRITE_SIZE")
    f = 2.0 * 1024.0 * sum(fetch) / len(fetch)
    w = 1024.0 * sum(write) / len(write)
    wl = sys.argv[4] if len(sys.argv) > 4 else "dcr_dipole"
    label = sys.argv[5] if len(sys.argv) > 5 else "wost_walk_jit (dcr_dipole, 48 x 1M walks)"
    out = {"kernel": label, "dispatches": [len(fetch), len(write)],
           "fetch_bytes_corrected": f, "write_bytes": w, "hbm_bytes_per_launch": f + w,
           "source": sys.argv[3] + " (rocprofv3 --pmc, separate passes; FETCH_SIZE x2 gfx950 correction, KB -> bytes)"}
    path = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles",
                        f"traffic_{wl}.json")
    with open(path, "w") as fh:
        json.dump(out, fh, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
