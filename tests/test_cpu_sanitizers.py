"""CPU sanitizer jobs (SURVEY.md §5 "race detection / sanitizers"):
  * the shared-memory communicator's barrier protocol
    (csrc/mx_shm_barrier.hpp, used by ShmComm) stress-tested on threads under
    ThreadSanitizer and under AddressSanitizer + UBSan -- skewed ranks running
    barrier -> collective -> barrier back to back, and mismatched collectives;
  * the CPU oracle (oracle/petsc_oracle.c) under AddressSanitizer + UBSan on
    every entry point the parity tests use.
GPU sanitizers are not available on the GPU pool; the device code is covered by
the no-scratch / code-object checks and the GPU parity suite."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "mpi-petsc4py-example_amd", "csrc")
NATIVE = os.path.join(ROOT, "tests", "native")
ORACLE = os.path.join(ROOT, "oracle")


def build_run(tmp_path, name, cmd, env=None):
    exe = str(tmp_path / name)
    try:
        subprocess.run(cmd + ["-o", exe], check=True, capture_output=True, text=True, timeout=240)
    except (subprocess.CalledProcessError, FileNotFoundError) as e:
        pytest.skip(f"sanitizer build unavailable: {getattr(e, 'stderr', e)}")
    out = subprocess.run([exe], capture_output=True, text=True, timeout=240, env=dict(os.environ, **(env or {})))
    assert out.returncode == 0, out.stdout[-2000:] + out.stderr[-4000:]
    assert out.stdout.strip().endswith("OK")


@pytest.mark.skipif(shutil.which("g++") is None, reason="no g++")
@pytest.mark.parametrize("san", ["thread", "address,undefined"])
def test_shm_barrier_protocol_sanitized(tmp_path, san):
    build_run(tmp_path, f"shm_{san.replace(',', '_')}",
              ["g++", "-std=c++17", "-O1", "-g", f"-fsanitize={san}", "-fno-sanitize-recover=all",
               "-I", CSRC, os.path.join(NATIVE, "shm_barrier_test.cpp"), "-pthread"],
              env={"TSAN_OPTIONS": "halt_on_error=1"})


@pytest.mark.skipif(shutil.which("gcc") is None, reason="no gcc")
def test_oracle_sanitized(tmp_path):
    build_run(tmp_path, "oracle_asan",
              ["gcc", "-std=c11", "-O1", "-g", "-fsanitize=address,undefined", "-fno-omit-frame-pointer",
               "-fno-sanitize-recover=all", "-fopenmp", "-ffp-contract=off", "-I", ORACLE,
               os.path.join(NATIVE, "oracle_sanitize.c"), os.path.join(ORACLE, "petsc_oracle.c"), "-lm"],
              env={"ASAN_OPTIONS": "detect_leaks=1"})
