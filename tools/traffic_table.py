#!/usr/bin/env python3
"""Per-kernel HBM-side traffic and duration from tools/pmc_kernels.sh passes
(TCC_EA0_RDREQ_{64B,128B}_sum, WRITE_SIZE) and a rocprofv3 kernel trace:
median bytes read (128-B requests x 128 + 64-B x 64 -- FETCH_SIZE tallies the
128-B ones at 64 B on gfx950), written (WRITE_SIZE KiB x 1024) and duration
per kernel name.
    python tools/traffic_table.py PMC_DIR TRACE_DIR"""
import csv, glob, statistics, sys
from collections import defaultdict


def short(n):
    n = n.replace("void ", "").replace("(anonymous namespace)::", "").replace("mx::", "")
    return n.split("(")[0] if not n.startswith("(") else n


cnt = defaultdict(lambda: defaultdict(list))
for f in glob.glob(sys.argv[1] + "/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        cnt[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
dur = defaultdict(list)
for f in glob.glob(sys.argv[2] + "/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        dur[short(r["Kernel_Name"])].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
print(f"{'kernel':70s} {'n':>5s} {'us':>8s} {'read MB':>9s} {'write MB':>9s} {'TB/s':>6s}")
for k, c in sorted(cnt.items(), key=lambda kv: -statistics.median(dur.get(kv[0], [0]))):
    med = lambda name: statistics.median(c[name]) if name in c else 0.0
    rd = med("TCC_EA0_RDREQ_128B_sum") * 128 + med("TCC_EA0_RDREQ_64B_sum") * 64 + med("TCC_EA0_RDREQ_32B_sum") * 32
    wr = med("WRITE_SIZE") * 1024
    us = statistics.median(dur[k]) if dur.get(k) else float("nan")
    print(f"{k[:70]:70s} {len(dur.get(k, [])):5d} {us:8.1f} {rd / 1e6:9.1f} {wr / 1e6:9.1f} {(rd + wr) / us / 1e6 if us == us and us > 0 else float('nan'):6.2f}")
