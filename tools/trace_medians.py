#!/usr/bin/env python3
"""Median / mean / min kernel duration (us) per kernel from rocprofv3 --kernel-trace csv files.
    python tools/trace_medians.py DIR [min_us]   (launches shorter than min_us, default 10, are dropped:
    no-op launches after a solve has stopped)"""
import csv, glob, re, statistics, sys
d = {}
lo = float(sys.argv[2]) if len(sys.argv) > 2 else 10.0
for f in glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = re.sub(r"^void\s+", "", r["Kernel_Name"]).split("(")[0].replace("mx::", "").replace(" ", "")
        d.setdefault(k, []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for k, v in sorted(d.items(), key=lambda t: -sum(t[1])):
    w = [t for t in v if t >= lo]
    if not w:
        continue
    print(f"{k[:70]:70s} n={len(w):5d} (dropped {len(v)-len(w):4d})  med {statistics.median(w):8.2f}  mean {statistics.mean(w):8.2f}  min {min(w):8.2f}")
