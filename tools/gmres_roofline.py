#!/usr/bin/env python3
"""GMRES(30) per-kernel algorithmic HBM fractions from a rocprofv3 kernel
trace of tools/bench_general.py c4 (BASELINE C4, conv-diff 256^3).

Algorithmic bytes per inner step j (0-based within a restart cycle, the new
direction w = A v_j; SURVEY.md §8d's GMRES model, this build's fusions):
  MatMult (SPMV_JACOBI_S, vector Jacobi): x 8m + w 8m (+ the dictionary's
           block ids, 4 B per 128 rows); dinv comes from the per-code table
           (knob 37; 24m with the dinv vector read, knob 37 = 0)
  MDot  : w and v_0..v_j            8m (j + 2)
  MAXPY + norm (fused)             : w read + write, v_0..v_j   8m (j + 3)
The trace's kernels of each kind are summed over the whole solve and divided
into the summed bytes of the same steps.
    python tools/gmres_roofline.py TRACE_DIR its [m] [restart]"""
import csv
import glob
import json
import re
import sys

d = {}
for f in glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = re.sub(r"^void\s+", "", r["Kernel_Name"]).split("(")[0].replace("mx::", "").replace(" ", "")
        d.setdefault(k, []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
its = int(sys.argv[2])
m = int(sys.argv[3]) if len(sys.argv) > 3 else 256 ** 3
restart = int(sys.argv[4]) if len(sys.argv) > 4 else 30
# every GMRES step the bench leg runs: a 20-iteration warm-up, the converged
# solve (its) and a 60-iteration profiled solve (its standalone products use
# the plain SpMV kernel, not counted here)
steps = [j % restart for n in (20, its, 60) for j in range(n)]
mdot_b = sum(8 * m * (j + 2) for j in steps)
maxpy_b = sum(8 * m * (j + 3) for j in steps)
spmv_b = len(steps) * (16 * m + 4 * (m // 128))


def total(prefixes, lo=20.0):    # working launches (the no-ops after a stop are shorter)
    return sum(t for k, v in d.items() if k.startswith(prefixes) for t in v if t >= lo)


share = 1.0
out = {}
# MDot: mdot_kernel<NV> groups, mdot_split_kernel, mdot_chunk_kernel (knob 50);
# MatMult: the coded z-march (knob 52) or the general kernel, JACOBI_S (mode 5)
for name, prefix, b in (("MDot (mdot_*_kernel)", ("mdot_",), mdot_b),
                        ("MAXPY+norm (maxpy_norm_kernel)", ("maxpy_norm_kernel",), maxpy_b),
                        ("MatMult (JACOBI_S: spmv_pair_zmc_kernel / spmv_sell_kernel)",
                         ("spmv_pair_zmc_kernel<5,", "spmv_sell_kernel<5,"), spmv_b)):
    t_us = total(prefix) * share
    out[name] = {"alg_bytes": b, "time_us": round(t_us, 1), "TBps": round(b / t_us / 1e6, 3),
                 "frac_of_8TBps": round(b / t_us / 1e6 / 8.0, 3)}
print(json.dumps(out, indent=1))
