"""Build libpghip.so (gfx950 only) in-tree with hipcc.

    python -m pghip.build            (from paligemma-multimodal-system_amd/)

Each csrc/*.hip is compiled to an object in parallel, then linked into
pghip/libpghip.so next to this file (git-ignored, but it travels to the GPU box
with the snapshot).  Rebuilds only when a source or header is newer than the
library.
"""
from __future__ import annotations

import concurrent.futures as cf
import glob
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.dirname(HERE)
CSRC = os.path.join(PKG, "csrc")
INCLUDE = os.path.join(os.path.dirname(PKG), "include")
LIB = os.path.join(HERE, "libpghip.so")
OBJ_DIR = os.path.join(PKG, "build", "obj")
ARCH = os.environ.get("PGHIP_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
FLAGS = ["-O3", f"--offload-arch={ARCH}", "-fPIC", "-std=c++17", "-I", CSRC, "-I", INCLUDE,
         "-Wno-pass-failed"]


def sources():
    return sorted(glob.glob(os.path.join(CSRC, "*.hip")))


def _stale() -> bool:
    if not os.path.exists(LIB):
        return True
    t = os.path.getmtime(LIB)
    deps = sources() + glob.glob(os.path.join(CSRC, "*.h")) + glob.glob(os.path.join(INCLUDE, "*.h"))
    return any(os.path.getmtime(p) > t for p in deps)


def _compile(src: str, obj_dir: str = OBJ_DIR, defines=()) -> str:
    obj = os.path.join(obj_dir, os.path.basename(src) + ".o")
    cmd = [HIPCC, *FLAGS, *[f"-D{d}" for d in defines], "-c", src, "-o", obj]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed on {src}:\n{r.stderr}")
    return obj


def build(force: bool = False, verbose: bool = True, out: str = LIB, defines=()) -> str:
    """Build the library.  `out`/`defines` make a tuning variant (e.g. scripts/tune/*.so with -DPG_...=1);
    the product library is always the default build at pghip/libpghip.so."""
    if out == LIB and not defines and not force and not _stale():
        return LIB
    obj_dir = OBJ_DIR if out == LIB else os.path.join(OBJ_DIR, os.path.basename(out).replace(".so", ""))
    os.makedirs(obj_dir, exist_ok=True)
    srcs = sources()
    jobs = min(len(srcs), int(os.environ.get("MAX_JOBS", os.cpu_count() or 4)), 16)
    # incremental: a source is recompiled when it, or any csrc header, is newer than its object (gemm.hip alone
    # takes minutes; include/pghip.h is the C-ABI declaration, included by no source); a tuning variant (defines)
    # always compiles everything
    hdr = max([os.path.getmtime(p) for p in glob.glob(os.path.join(CSRC, "*.h"))] or [0.0])

    def obj_for(src):
        obj = os.path.join(obj_dir, os.path.basename(src) + ".o")
        if (defines or force or not os.path.exists(obj) or os.path.getmtime(obj) < max(os.path.getmtime(src), hdr)):
            return _compile(src, obj_dir, defines)
        return obj
    with cf.ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
        objs = list(ex.map(obj_for, srcs))
    tmp = out + ".tmp"
    cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", *objs, "-o", tmp]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed:\n{r.stderr}")
    os.replace(tmp, out)
    if verbose:
        print(f"[pghip] built {out} from {len(srcs)} sources for {ARCH}" + (f" {list(defines)}" if defines else ""))
    return out


if __name__ == "__main__":
    build(force="--force" in sys.argv)
