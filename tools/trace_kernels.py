#!/usr/bin/env python3
"""Median duration per (kernel, grid) of a rocprofv3 kernel trace, the kernels
whose total time is largest first.

    python tools/trace_kernels.py run_kernel_trace.csv [regex] [top]
"""
import csv
import re
import statistics
import sys
from collections import defaultdict

path = sys.argv[1]
pat = re.compile(sys.argv[2] if len(sys.argv) > 2 else ".")
top = int(sys.argv[3]) if len(sys.argv) > 3 else 20
d = defaultdict(list)
for r in csv.DictReader(open(path)):
    n = re.sub(r"\(.*", "", r["Kernel_Name"].replace("void ", "").replace("mx::", "")).replace(" ", "")
    if pat.search(n):
        d[(n, int(r["Grid_Size_X"]) // int(r["Workgroup_Size_X"]))].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for (n, g), v in sorted(d.items(), key=lambda kv: -sum(kv[1]))[:top]:
    print(f"{statistics.median(v):9.1f} us median  {len(v):6d} calls  grid {g:6d}  {n}")
