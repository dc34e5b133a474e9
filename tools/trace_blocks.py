#!/usr/bin/env python3
"""Per-block medians of a kernel's launches in a rocprofv3 kernel trace, in
launch order -- for interleaved knob A/B runs whose variants share a kernel
name (tools/c5_trace.py runs one solve per setting).
    python tools/trace_blocks.py TRACE_DIR REGEX BLOCK [SKIP]   (SKIP: leading launches dropped, e.g. a warm-up)"""
import csv, glob, re, statistics, sys
rx, blk = re.compile(sys.argv[2]), int(sys.argv[3])
rows = []
for f in glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if rx.search(r["Kernel_Name"]):
            rows.append((int(r["Start_Timestamp"]), (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3))
rows.sort()
rows = rows[int(sys.argv[4]) if len(sys.argv) > 4 else 0:]
for i in range(0, len(rows), blk):
    v = [t for _, t in rows[i:i + blk]]
    print(f"block {i // blk}: n={len(v)} median {statistics.median(v):.2f} mean {statistics.mean(v):.2f} us")
