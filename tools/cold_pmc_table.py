#!/usr/bin/env python3
"""Warm against cold MatMult counters from tools/pmc_kernels.sh passes over
tools/cold_probe.py (REGEX matching the flush and the SpMV kernels): a SpMV
dispatch whose previous dispatch is the flush (dot_partials_kernel) is cold.
Median per counter and class.
    python tools/cold_pmc_table.py gpurun_out/pmc_TAG"""
import csv, glob, statistics, sys

for f in sorted(glob.glob(sys.argv[1] + "/p*/**/*counter_collection.csv", recursive=True)):
    disp = {}
    for r in csv.DictReader(open(f)):
        d = disp.setdefault(int(r["Dispatch_Id"]), {"name": r["Kernel_Name"], "c": {}})
        d["c"][r["Counter_Name"]] = d["c"].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    ids = sorted(disp)
    cls = {"warm": {}, "cold": {}}
    for i, k in enumerate(ids):
        if "dot_partials" in disp[k]["name"]:
            continue
        prev = disp[ids[i - 1]]["name"] if i else ""
        c = "cold" if "dot_partials" in prev else "warm"
        for cn, v in disp[k]["c"].items():
            cls[c].setdefault(cn, []).append(v)
    print(f)
    for cn in sorted(set(cls["warm"]) | set(cls["cold"])):
        w, c = cls["warm"].get(cn, []), cls["cold"].get(cn, [])
        mw = statistics.median(w) if w else float("nan")
        mc = statistics.median(c) if c else float("nan")
        print(f"    {cn:40s} warm {mw:16.1f} (n={len(w)})  cold {mc:16.1f} (n={len(c)})  cold/warm {mc / mw if mw else float('nan'):.3f}")
