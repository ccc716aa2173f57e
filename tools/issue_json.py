#!/usr/bin/env python3
"""Writes profiles/issue_dcr_dipole.json (read by bench.py for roofline.issue) from the
rocprofv3 PMC passes of tools/profile_session.sh: VALU and transcendental VALU
instructions per wave-step of the walk kernel (SQ_INSTS_VALU, SQ_INSTS_VALU_TRANS_F32
per dispatch, over walk-steps / 64).
Usage: tools/issue_json.py <pmc_sq1 dir> <pmc_trans dir> <walk-steps per dispatch> <source label>"""
import csv
import json
import os
import sys


def per_dispatch(d, counter):
    vals = {}
    for r in csv.DictReader(open(os.path.join(d, "run_counter_collection.csv"))):
        if "wost_walk" in r["Kernel_Name"] and r["Counter_Name"] == counter:
            vals[r["Dispatch_Id"]] = vals.get(r["Dispatch_Id"], 0.0) + float(r["Counter_Value"])
    return list(vals.values())


def main():
    valu = per_dispatch(sys.argv[1], "SQ_INSTS_VALU")
    trans = per_dispatch(sys.argv[2], "SQ_INSTS_VALU_TRANS_F32")
    steps = float(sys.argv[3])
    ws = steps / 64.0
    out = {"kernel": "wost_walk_jit (dcr_dipole, 48 x 1M walks)", "dispatches": [len(valu), len(trans)],
           "walk_steps_per_dispatch": steps,
           "valu_per_wave_step": sum(valu) / len(valu) / ws, "trans_per_wave_step": sum(trans) / len(trans) / ws,
           "source": sys.argv[4] + " (rocprofv3 --pmc SQ_INSTS_VALU / SQ_INSTS_VALU_TRANS_F32, separate passes)"}
    path = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles",
                        "issue_dcr_dipole.json")
    with open(path, "w") as fh:
        json.dump(out, fh, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
