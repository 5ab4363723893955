"""The C-ABI boundary's host code under AddressSanitizer + UndefinedBehaviorSanitizer (tests/asan/).

tests/asan/abi_host_check.c calls every entry point of include/pghip.h with the arguments the boundary must reject
(null operands, empty or inconsistent shapes, byte counts that would overflow) and the pure host functions
(pg_abi_version, pg_source_hash truncation, the exchange-buffer sizes).  tests/asan/asan_build.py compiles the library
sources with the sanitizers on the host side only and links the driver; the GPU box runs it (it links the HIP
runtime).  Each rejection must return hipErrorInvalidValue before any HIP call, with no sanitizer report.
"""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ASAN = os.path.join(ROOT, "tests", "asan")


def test_boundary_driver_compiles_against_the_header():
    """The driver is plain C over include/pghip.h (the binding a C caller writes)."""
    if shutil.which("gcc") is None:
        pytest.skip("gcc not installed")
    r = subprocess.run(["gcc", "-fsyntax-only", "-Wall", "-Werror", "-D__HIP_PLATFORM_AMD__", "-I",
                        os.path.join(ROOT, "include"), "-I", "/opt/rocm/include",
                        os.path.join(ASAN, "abi_host_check.c")], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-2000:]


@pytest.mark.gpu
def test_boundary_rejections_under_asan_and_ubsan():
    import sys
    sys.path.insert(0, ASAN)
    import asan_build
    assert asan_build.fresh(), "tests/asan/abi_host_check is missing or stale: run python tests/asan/asan_build.py"
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=0:halt_on_error=1",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    r = subprocess.run([asan_build.EXE], capture_output=True, text=True, env=env, timeout=120)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-4000:]
    assert "all boundary checks passed" in r.stdout, out[-4000:]
    assert "Sanitizer" not in out and "runtime error" not in out, out[-4000:]
