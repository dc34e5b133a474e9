#!/usr/bin/env python3
"""Per-kernel median of every counter collected by tools/pmc_kernels.sh.
    python tools/pmc_table.py gpurun_out/pmc_TAG [kernel-substring ...]"""
import csv
import glob
import re
import statistics
import sys


def short(name):
    n = re.sub(r"^void\s+", "", name).split("(")[0].replace("mx::", "").replace(" ", "")
    return n


vals = {}
for f in glob.glob(sys.argv[1] + "/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = short(r["Kernel_Name"])
        if len(sys.argv) > 2 and not any(s in k for s in sys.argv[2:]):
            continue
        vals.setdefault(k, {}).setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
names = sorted({c for v in vals.values() for c in v})
for k, v in sorted(vals.items()):
    print(k)
    for c in names:
        if c in v:
            print(f"    {c:32s} {statistics.median(v[c]):16.1f}   (n={len(v[c])})")
