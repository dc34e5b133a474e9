#!/usr/bin/env python3
"""Register / spill / scratch figures of the gfx950 kernels in a built object
or library (kernel descriptor notes), filtered by a regex:

    python tools/kstats.py [path] [regex]
"""
import os, re, subprocess, sys, tempfile, pathlib
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
from test_cpu_codeobj import code_objects, LLVM  # noqa: E402

path = sys.argv[1] if len(sys.argv) > 1 else "mpi-petsc4py-example_amd/lib/libmxsolve.so"
pat = re.compile(sys.argv[2] if len(sys.argv) > 2 else ".")
d = pathlib.Path(tempfile.mkdtemp())
fb = d / "fatbin"
subprocess.check_call([os.path.join(LLVM, "llvm-objcopy"), "--dump-section", f".hip_fatbin={fb}", path, str(d / "copy")])
rows = []
for j, elf in enumerate(code_objects(fb.read_bytes())):
    co = d / f"co{j}.elf"
    co.write_bytes(elf)
    notes = subprocess.run([os.path.join(LLVM, "llvm-readelf"), "--notes", str(co)], capture_output=True, text=True,
                           check=True).stdout
    for blk in re.split(r"\n\s+- \.", notes):
        m = re.search(r"\.name:\s+(\S+)", blk)
        if not m or not pat.search(m.group(1)):
            continue
        g = lambda k: (re.search(r"\." + k + r":\s+(\d+)", blk) or [0, "0"])[1]
        rows.append((m.group(1), g("vgpr_count"), g("sgpr_count"), g("sgpr_spill_count"), g("vgpr_spill_count"),
                     g("private_segment_fixed_size")))
names = subprocess.run(["c++filt"], input="\n".join(r[0] for r in rows), capture_output=True, text=True).stdout.split("\n")
print("vgpr sgpr sspill vspill scratch  kernel")
for r, n in zip(rows, names):
    print(f"{r[1]:>4} {r[2]:>4} {r[3]:>6} {r[4]:>6} {r[5]:>7}  {n.split('(')[0]}")
