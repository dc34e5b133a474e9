"""The built library's gfx950 code objects: no hot kernel may use scratch
(private segment).  A lambda the compiler declined to inline once put a
row-pair unit's registers on the stack (432 bytes per lane) and halved the
SpMV's speed with every parity test still green; this check catches that
class of regression on the CPU, from the kernel descriptors' metadata.  The
lean row-pair MatMults (the 5/7/27-point z-march, the fp64 row-pair z-march,
the sweep form: C2-C5's hot kernels) and the Krylov vector kernels (CG's
direction / residual updates, GMRES's MDot, MAXPY and step kernels) must also
spill no SGPR or VGPR: round 2's 27-point form spilled 119 SGPRs (its 54 slot
values and lane masks) and ran VALU-bound at 0.39 of HBM peak; round 3's
chunk MDot spilled 126 SGPRs."""
import os
import re
import shutil
import struct
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "mpi-petsc4py-example_amd", "lib", "libmxsolve.so")
LLVM = "/opt/rocm/lib/llvm/bin"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"
HOT = re.compile(r"spmv_sell_kernel|spmv_pair_lean|spmv_pair_zm|cg_|mdot|maxpy|fold_kernel")
NOSPILL = re.compile(r"spmv_pair_zm|spmv_pair_lean|spmv_pair_pbw|mdot|maxpy|cg_pb|"
                     r"cg_update|cg_norms|cg_finish|gm_|fold_kernel|finish_many")


def code_objects(fatbin: bytes):
    """gfx950 ELF images of every offload bundle in a .hip_fatbin section."""
    i = fatbin.find(MAGIC)
    while i >= 0:
        n = struct.unpack_from("<Q", fatbin, i + 24)[0]
        p = i + 32
        for _ in range(n):
            off, size, tlen = struct.unpack_from("<QQQ", fatbin, p)
            triple = fatbin[p + 24:p + 24 + tlen].decode()
            p += 24 + tlen
            if "gfx950" in triple:
                yield fatbin[i + off:i + off + size]
        i = fatbin.find(MAGIC, i + 1)


def kernel_descriptors(tmp_path):
    """{kernel name: (private segment bytes, SGPR spills, VGPR spills)}."""
    fb = tmp_path / "fatbin"
    subprocess.check_call([os.path.join(LLVM, "llvm-objcopy"), "--dump-section", f".hip_fatbin={fb}", LIB,
                           str(tmp_path / "lib.copy")])
    kernels = {}
    for j, elf in enumerate(code_objects(fb.read_bytes())):
        co = tmp_path / f"co{j}.elf"
        co.write_bytes(elf)
        notes = subprocess.run([os.path.join(LLVM, "llvm-readelf"), "--notes", str(co)],
                               capture_output=True, text=True, check=True).stdout
        for blk in re.split(r"\n\s+- \.", notes):
            m = re.search(r"\.name:\s+(\S+)", blk)
            ps = re.search(r"\.private_segment_fixed_size:\s+(\d+)", blk)
            ss = re.search(r"\.sgpr_spill_count:\s+(\d+)", blk)
            vs = re.search(r"\.vgpr_spill_count:\s+(\d+)", blk)
            if m and ps:
                kernels[m.group(1)] = (int(ps.group(1)), int(ss.group(1)) if ss else 0, int(vs.group(1)) if vs else 0)
    return kernels


needs_lib = pytest.mark.skipif(not os.path.exists(LIB) or not os.path.exists(os.path.join(LLVM, "llvm-readelf")),
                               reason="library not built or no ROCm llvm tools")


@needs_lib
def test_hot_kernels_use_no_scratch(tmp_path):
    kernels = {k: v[0] for k, v in kernel_descriptors(tmp_path).items()}
    hot = {k: v for k, v in kernels.items() if HOT.search(k)}
    assert any("spmv_sell_kernel" in k for k in hot), "no SpMV kernel found in the code objects"
    bad = {k: v for k, v in hot.items() if v}
    assert not bad, f"hot kernels with scratch: {bad}"


@needs_lib
def test_zmarch_kernels_spill_nothing(tmp_path):
    zm = {k: v for k, v in kernel_descriptors(tmp_path).items() if NOSPILL.search(k)}
    assert any("zm27" in k for k in zm) and any("zmf64" in k for k in zm), sorted(zm)
    assert any("mdot_chunk" in k for k in zm) and any("cg_pb" in k for k in zm), sorted(zm)
    bad = {k: v for k, v in zm.items() if v[1] or v[2]}
    assert not bad, f"z-march kernels with register spills (scratch, SGPR, VGPR): {bad}"
