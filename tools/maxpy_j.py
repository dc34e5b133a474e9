#!/usr/bin/env python3
"""Per-basis-size durations of the GMRES MDot and MAXPY + norm launches from a
rocprofv3 kernel trace of tools/config_run.py ... gmres (60 iterations = two
restart cycles, launch i has k = i % 30): median us and fraction of 8 TB/s on
the byte models 8 m (k + 2) (MDot) and 8 m (k + 3) (MAXPY)."""
import collections, csv, sys
import numpy as np
rows = list(csv.DictReader(open(sys.argv[1])))
m = int(sys.argv[2]) if len(sys.argv) > 2 else 256 ** 3
for name, extra in (("mdot_chunk", 2), ("maxpy_norm", 3)):
    ks = [r for r in rows if name in r["Kernel_Name"]]
    by = collections.defaultdict(list)
    for i, r in enumerate(ks):
        by[i % 30].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    print(f"{name}: {len(ks)} launches, grid {ks[0]['Grid_Size_X']}, VGPRs {ks[0]['VGPR_Count']}")
    tot_b = tot_t = 0.0
    for k in sorted(by):
        b, t = 8 * m * (k + extra), float(np.median(by[k]))
        tot_b += b; tot_t += t
        print(f"  k {k:2d}: {t:7.1f} us  {b / t / 1e6 / 8:.3f}")
    print(f"  all k: {tot_t:.0f} us per cycle, {tot_b / tot_t / 1e6 / 8:.3f}")
