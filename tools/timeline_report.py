#!/usr/bin/env python3
"""Per-kernel start offsets, durations and gaps of the LAST solve in a
rocprofv3 kernel trace of tools/solve_timeline.py.
    python tools/timeline_report.py TRACE_DIR"""
import csv, glob, re, sys
rows = []
for f in glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = re.sub(r"^void\s+", "", r["Kernel_Name"]).split("(")[0].replace("mx::", "").replace(" ", "")
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), k))
rows.sort()
# the last solve starts at its state-init kernel (the last cg_norms kernel
# in builds without one)
first = "ksp_state_init" if any(r[2].startswith("ksp_state_init") for r in rows) else "cg_norms"
start = max(i for i, r in enumerate(rows) if r[2].startswith(first))
t0 = rows[start][0]
prev_end = None
for s, e, k in rows[start:]:
    gap = (s - prev_end) / 1e3 if prev_end else 0.0
    print(f"{(s - t0) / 1e3:9.1f} us  dur {(e - s) / 1e3:8.1f}  gap {gap:6.1f}  {k[:60]}")
    prev_end = e
print(f"total {(rows[-1][1] - t0) / 1e3:.1f} us")
