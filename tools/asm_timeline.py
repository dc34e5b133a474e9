#!/usr/bin/env python3
"""One assembly's host/device timeline from a rocprofv3 trace with
--kernel-trace --hip-runtime-trace (tools/asm_phases.py as the program):
kernels and HIP calls of the LAST assembly (from its generator launch on),
each with its start offset and duration; HIP calls under MIN_US are summed.
python tools/asm_timeline.py TRACE_DIR [FIRST_KERNEL_REGEX] [MIN_US]"""
import csv, os, re, sys
from collections import defaultdict

d = sys.argv[1]
first = re.compile(sys.argv[2] if len(sys.argv) > 2 else r"stencil_kernel")
min_us = float(sys.argv[3]) if len(sys.argv) > 3 else 50.0
K = list(csv.DictReader(open(os.path.join(d, "run_kernel_trace.csv"))))
H = list(csv.DictReader(open(os.path.join(d, "run_hip_api_trace.csv"))))
starts = [int(k["Start_Timestamp"]) for k in K if first.search(k["Kernel_Name"])]
t0 = starts[-1]
ev = [(int(k["Start_Timestamp"]), int(k["End_Timestamp"]), "K", k["Kernel_Name"][:60]) for k in K
      if int(k["Start_Timestamp"]) >= t0]
hs = [(int(h["Start_Timestamp"]), int(h["End_Timestamp"]), "H", h["Function"]) for h in H
      if int(h["Start_Timestamp"]) >= t0 - 200_000]
small = defaultdict(lambda: [0, 0.0])
for s, e, kind, name in sorted(ev + hs):
    us = (e - s) / 1e3
    if kind == "H" and us < min_us:
        small[name][0] += 1
        small[name][1] += us
        continue
    print(f"{(s - t0) / 1e3:10.1f} us  {us:9.1f}  {kind}  {name}")
print("HIP calls under", min_us, "us:")
for name, (n, us) in sorted(small.items(), key=lambda t: -t[1][1]):
    print(f"  {name:40s} n={n:5d} total {us:9.1f} us")
