"""Build tests/asan/abi_host_check: the C-ABI library's host code under AddressSanitizer + UndefinedBehaviorSanitizer.

    python tests/asan/asan_build.py          (or __graft_entry__.build(), which calls build())

Every csrc/*.hip is compiled for gfx950 as the product is, with the sanitizers on the HOST side only (each -fsanitize
flag directly after -Xarch_host: GPU AddressSanitizer is not available on the MI355X pool, and the device code is
never run by this check), then linked with abi_host_check.c into one executable.  The executable runs on a GPU box
(tests/test_asan_host.py, marked gpu: it links the HIP runtime) and exercises the boundary's rejection paths and
pure host functions; it never launches a kernel.

Like pghip/build.py the build is keyed by content: the executable is rebuilt only when the sources, the header, this
file or the driver change (the key is stored next to it).  Objects go to a temporary directory.
"""
from __future__ import annotations

import concurrent.futures as cf
import glob
import hashlib
import os
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
CSRC = os.path.join(ROOT, "paligemma-multimodal-system_amd", "csrc")
INCLUDE = os.path.join(ROOT, "include")
DRIVER = os.path.join(HERE, "abi_host_check.c")
EXE = os.path.join(HERE, "abi_host_check")
KEY = EXE + ".key"
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
CLANG = "/opt/rocm/llvm/bin/clang"
SAN = ["-Xarch_host", "-fsanitize=address", "-Xarch_host", "-fsanitize=undefined",
       "-Xarch_host", "-fno-sanitize-recover=all", "-Xarch_host", "-fno-omit-frame-pointer"]
FLAGS = ["-O1", "--offload-arch=gfx950", "-std=c++17", "-Wno-pass-failed", "-I", CSRC, "-I", INCLUDE, *SAN]


def key() -> str:
    h = hashlib.sha256()
    for p in sorted(glob.glob(os.path.join(CSRC, "*.hip")) + glob.glob(os.path.join(CSRC, "*.h"))) + [
            os.path.join(INCLUDE, "pghip.h"), DRIVER, os.path.abspath(__file__)]:
        with open(p, "rb") as f:
            h.update(os.path.basename(p).encode() + b"\0" + f.read() + b"\0")
    return h.hexdigest()


def fresh() -> bool:
    if not os.path.exists(EXE) or not os.path.exists(KEY):
        return False
    with open(KEY) as f:
        return f.read().strip() == key()


def _run(cmd):
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"{' '.join(cmd[:3])} ... failed:\n{r.stderr[-4000:]}")


def build(force: bool = False, verbose: bool = True) -> str:
    if not force and fresh():
        return EXE
    srcs = sorted(glob.glob(os.path.join(CSRC, "*.hip")))
    sys.path.insert(0, os.path.dirname(CSRC))
    from pghip import build as product
    # the product's source hash, so pg_source_hash returns what the shipped library returns (64 hex characters)
    hash_def = f'-DPG_SOURCE_HASH="{product.source_hash()}"'
    with tempfile.TemporaryDirectory() as d:
        def obj(src):
            o = os.path.join(d, os.path.basename(src) + ".o")
            _run([HIPCC, *FLAGS, hash_def, "-c", src, "-o", o])
            return o
        jobs = max(1, min(len(srcs), int(os.environ.get("MAX_JOBS", os.cpu_count() or 4)), 16))
        with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
            objs = list(ex.map(obj, srcs))
        drv = os.path.join(d, "driver.o")
        _run([CLANG, "-x", "c", "-O1", "-g", *SAN, "-Wall", "-D__HIP_PLATFORM_AMD__", "-I", INCLUDE, "-I",
              "/opt/rocm/include", "-c", DRIVER, "-o", drv])
        tmp = EXE + ".tmp"
        _run([HIPCC, "--offload-arch=gfx950", *SAN, *objs, drv, "-o", tmp])
        os.replace(tmp, EXE)
    with open(KEY, "w") as f:
        f.write(key() + "\n")
    if verbose:
        print(f"[asan] built {EXE}")
    return EXE


if __name__ == "__main__":
    build(force="--force" in sys.argv)
