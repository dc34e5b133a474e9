#!/usr/bin/env python3
"""Per-iteration kernel time of the interior rank in a rocprofv3 kernel trace
of tools/rank_proxy.py (variants 9=1, 9=2, 9=5 in that order, one round):
the host thread with the most kernel time is rank 1 (32 planes); its launches
are cut into the three variants' windows by each mode's MatMult kernel, and
per window the kernels' summed durations are divided by the iterations run
(32 warm-up + its timed).

    python tools/proxy_trace.py gpurun_out/proxytrace/run_kernel_trace.csv [its]

(__amd_rocclr_copyBuffer and local_sum_kernel are the in-process transport's
payload copies and all-reduce sums; RCCL replaces them on the 8-GPU node.)
"""
import csv
import re
import statistics
import sys
from collections import defaultdict

path = sys.argv[1]
its = int(sys.argv[2]) if len(sys.argv) > 2 else 100
rows = list(csv.DictReader(open(path)))
short = lambda n: re.sub(r"\(.*", "", n.replace("void ", "").replace("mx::", "")).replace(" ", "")
by_thread = defaultdict(list)
for r in rows:
    by_thread[r["Thread_Id"]].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"])))
tid = max(by_thread, key=lambda t: sum(e - s for s, e, _ in by_thread[t]))
ks = sorted(by_thread[tid])
marks = {1: "spmv_sell_kernel<3,", 2: "spmv_pair_zm_kernel<2,", 5: "spmv_pair_zm_kernel<6,"}
out = {}
for mode, pre in marks.items():
    idx = [i for i, k in enumerate(ks) if k[2].startswith(pre)]
    if not idx:
        continue
    # the window: from the launch after the previous mode's last MatMult to this mode's last one
    lo, hi = idx[0], idx[-1]
    while lo > 0 and not any(ks[lo - 1][2].startswith(p) for p in marks.values()) and ks[lo - 1][2] != "ksp_state_init_kernel":
        lo -= 1
    win = ks[lo:hi + 3]
    per = defaultdict(list)
    for s, e, n in win:
        per[n].append((e - s) / 1e3)
    nit = len(idx)
    tot = sum(sum(v) for v in per.values())
    out[mode] = {"iterations": nit, "kernel_us_per_iteration": round(tot / nit, 1),
                 "kernels": {n: {"calls": len(v), "median_us": round(statistics.median(v), 1),
                                 "us_per_iteration": round(sum(v) / nit, 1)} for n, v in
                             sorted(per.items(), key=lambda kv: -sum(kv[1]))[:8]}}
import json
print(json.dumps({"thread": tid, **{f"mode{m}": v for m, v in out.items()}}, indent=1))
