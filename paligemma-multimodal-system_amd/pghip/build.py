"""Build libpghip.so (gfx950 only) in-tree with hipcc.

    python -m pghip.build            (from paligemma-multimodal-system_amd/)

Each csrc/*.hip is compiled to an object in parallel, then linked into
pghip/libpghip.so next to this file (git-ignored, but it travels to the GPU box
with the snapshot).

Staleness is decided by content, not mtimes: source_hash() is a sha256 over
every csrc/ source and header, include/pghip.h and the compile configuration
(hipcc, flags, arch).  The hash is compiled into the library (PG_SOURCE_HASH,
read back with pg_source_hash / library_hash()), so a prebuilt library that
does not match the tree next to it is rebuilt here and refused at load time
(_lib.load(check=True)).  Objects live in a directory named after the hash of
the compile configuration, so a change of arch or flags never relinks objects
built for another target, and each object's file name carries the sha256 of its
own source text + every csrc header + that configuration (_obj_key): an object is
reused only when it was compiled from exactly these bytes, whatever the mtimes say.
"""
from __future__ import annotations

import concurrent.futures as cf
import glob
import hashlib
import os
import re
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.dirname(HERE)
CSRC = os.path.join(PKG, "csrc")
INCLUDE = os.path.join(os.path.dirname(PKG), "include")
LIB = os.path.join(HERE, "libpghip.so")
OBJ_ROOT = os.path.join(PKG, "build", "obj")
ARCH = os.environ.get("PGHIP_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
FLAGS = ["-O3", f"--offload-arch={ARCH}", "-fPIC", "-std=c++17", "-I", CSRC, "-I", INCLUDE,
         "-Wno-pass-failed"]
_MARK = b"PGHIP_SOURCE_HASH="


def sources():
    return sorted(glob.glob(os.path.join(CSRC, "*.hip")))


def _inputs():
    return sources() + sorted(glob.glob(os.path.join(CSRC, "*.h"))) + [os.path.join(INCLUDE, "pghip.h")]


def _config() -> str:
    """The compile configuration without its machine-specific include paths (the GPU box holds the tree elsewhere)."""
    flags = [f for f in FLAGS if f not in (CSRC, INCLUDE)]
    return " ".join([os.path.basename(HIPCC), *flags])


def _config_tag(defines=()) -> str:
    return hashlib.sha256(" ".join([_config(), *defines]).encode()).hexdigest()[:12]


def source_hash(defines=()) -> str:
    """sha256 over the sources, headers and compile configuration the library is built from."""
    h = hashlib.sha256()
    for p in _inputs():
        h.update(os.path.relpath(p, os.path.dirname(PKG)).encode() + b"\0")
        with open(p, "rb") as f:
            h.update(f.read())
        h.update(b"\0")
    h.update(" ".join([_config(), *defines]).encode())
    return h.hexdigest()


def library_hash(path: str = LIB):
    """The PG_SOURCE_HASH compiled into a built library (read from the file, no load), or None."""
    if not os.path.exists(path):
        return None
    with open(path, "rb") as f:
        data = f.read()
    m = re.search(re.escape(_MARK) + rb"([0-9a-f]{64}|unknown)", data)
    return m.group(1).decode() if m else None


def _stale(defines=()) -> bool:
    return library_hash() != source_hash(defines)


def _obj_key(src: str, defines=()) -> str:
    """Content key of one object: its source, every csrc header it may include, and the compile configuration."""
    h = hashlib.sha256()
    for p in [src] + sorted(glob.glob(os.path.join(CSRC, "*.h"))):
        with open(p, "rb") as f:
            h.update(os.path.basename(p).encode() + b"\0" + f.read() + b"\0")
    h.update(" ".join([_config(), *defines]).encode())
    return h.hexdigest()[:20]


def _compile(src: str, obj: str, defines=()) -> str:
    cmd = [HIPCC, *FLAGS, *[f"-D{d}" for d in defines], "-c", src, "-o", obj + ".tmp"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed on {src}:\n{r.stderr}")
    os.replace(obj + ".tmp", obj)
    return obj


def build(force: bool = False, verbose: bool = True, out: str = LIB, defines=()) -> str:
    """Build the library.  `out`/`defines` make a tuning variant (e.g. scripts/tune/*.so with -DPG_...=1);
    the product library is always the default build at pghip/libpghip.so."""
    if out == LIB and not defines and not force and not _stale():
        return LIB
    obj_dir = os.path.join(OBJ_ROOT, _config_tag(defines))
    os.makedirs(obj_dir, exist_ok=True)
    srcs = sources()
    jobs = min(len(srcs), int(os.environ.get("MAX_JOBS", os.cpu_count() or 4)), 16)
    # incremental by content: an object is reused only if its file name carries the content key of exactly this
    # source + headers + configuration (gemm.hip alone takes minutes).  misc.hip carries the source hash and is
    # always recompiled.
    shash = source_hash(defines)
    hash_def = f'PG_SOURCE_HASH="{shash}"'

    def obj_for(src):
        base = os.path.basename(src)
        if base == "misc.hip":
            return _compile(src, os.path.join(obj_dir, base + ".o"), (*defines, hash_def))
        obj = os.path.join(obj_dir, f"{base}.{_obj_key(src, defines)}.o")
        if force or not os.path.exists(obj):
            for old in glob.glob(os.path.join(obj_dir, base + ".*.o")):     # objects of other source text
                os.remove(old)
            return _compile(src, obj, defines)
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
        print(f"[pghip] built {out} from {len(srcs)} sources for {ARCH} (source hash {shash[:16]})"
              + (f" {list(defines)}" if defines else ""))
    return out


if __name__ == "__main__":
    build(force="--force" in sys.argv)
