#!/usr/bin/env python3
"""HIP runtime calls slower than a threshold in a rocprofv3 --hip-runtime-trace
(any run_hip_api_trace.csv under DIR), with the totals per function.
    python tools/slow_calls.py DIR [MIN_MS]"""
import csv, glob, os, sys
from collections import defaultdict

d = sys.argv[1]
min_ms = float(sys.argv[2]) if len(sys.argv) > 2 else 10.0
files = glob.glob(os.path.join(d, "**", "*hip_api_trace.csv"), recursive=True)
tot = defaultdict(lambda: [0, 0.0, 0.0])
slow = []
for f in files:
    for h in csv.DictReader(open(f)):
        ms = (int(h["End_Timestamp"]) - int(h["Start_Timestamp"])) / 1e6
        t = tot[h["Function"]]
        t[0] += 1; t[1] += ms; t[2] = max(t[2], ms)
        if ms >= min_ms:
            slow.append((int(h["Start_Timestamp"]), ms, h["Function"]))
slow.sort()
t0 = slow[0][0] if slow else 0
print(f"calls >= {min_ms} ms: {len(slow)}")
for s, ms, fn in slow:
    print(f"  t={(s - t0) / 1e6:10.1f} ms  {ms:9.1f} ms  {fn}")
print("per function (calls, total ms, max ms), by total:")
for fn, (n, ms, mx) in sorted(tot.items(), key=lambda t: -t[1][1])[:15]:
    print(f"  {fn:36s} {n:7d} {ms:10.1f} {mx:9.1f}")
