#!/usr/bin/env python3
"""Writes profiles/issue_dcr_dipole.json (read by bench.py for roofline.issue) from the
rocprofv3 PMC passes of tools/profile_session.sh: VALU and transcendental VALU
instructions per wave-step of the walk kernel (SQ_INSTS_VALU, SQ_INSTS_VALU_TRANS_F32
per dispatch, over walk-steps / 64).
Usage: tools/issue_json.py <pmc_sq1 dir> <pmc_trans dir> <walk-steps per dispatch> <source label>
                           [<scenario> [<pmc dir with SQ_THREAD_CYCLES_VALU, SQ_ACTIVE_INST_VALU>]]
(scenario default dcr_dipole -> profiles/issue_<scenario>.json; with the third dir the
lane utilisation SQ_THREAD_CYCLES_VALU / (64 SQ_ACTIVE_INST_VALU) is recorded too)"""
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
    valu = per_dispatch(sys.argv[1], "SQ_INSTS_VALU")
    trans = per_dispatch(sys.argv[2], "SQ_INSTS_VALU_TRANS_F32")
    if len(sys.argv) > 5:   # a scenario_bench run: a warm-up launch, then the measured one (the largest)
        i = max(range(len(valu)), key=lambda j: valu[j])
        valu, trans = [valu[i]], [trans[max(range(len(trans)), key=lambda j: trans[j])]]
    steps = float(sys.argv[3])
    ws = steps / 64.0
    sc = sys.argv[5] if len(sys.argv) > 5 else "dcr_dipole"
    out = {"kernel": f"wost_walk_jit ({sc})", "dispatches": [len(valu), len(trans)],
           "walk_steps_per_dispatch": steps,
           "valu_per_wave_step": sum(valu) / len(valu) / ws, "trans_per_wave_step": sum(trans) / len(trans) / ws,
           "source": sys.argv[4] + " (rocprofv3 --pmc SQ_INSTS_VALU / SQ_INSTS_VALU_TRANS_F32, separate passes)"}
    if len(sys.argv) > 6:
        tc = per_dispatch(sys.argv[6], "SQ_THREAD_CYCLES_VALU")
        ai = per_dispatch(sys.argv[6], "SQ_ACTIVE_INST_VALU")
        out["lane_utilisation"] = max(tc) / (64.0 * max(ai))
    path = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles",
                        f"issue_{sc}.json")
    with open(path, "w") as fh:
        json.dump(out, fh, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
