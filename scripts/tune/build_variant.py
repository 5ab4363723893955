"""Link a tuning variant of libpghip.so: recompile ONE source with extra -D defines, reuse the product build's
other objects (paligemma-multimodal-system_amd/build/obj).

    python scripts/tune/build_variant.py out.so decode_mlp.hip PG_MLP_D_DEPTH=2 [...]
"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "paligemma-multimodal-system_amd"))
from pghip import build  # noqa: E402

out, src, defs = sys.argv[1], sys.argv[2], sys.argv[3:]
build.build()
obj_dir = os.path.join(build.OBJ_ROOT, build._config_tag())
vdir = os.path.join(obj_dir, "v_" + os.path.basename(out).replace(".so", ""))
os.makedirs(vdir, exist_ok=True)
obj = build._compile(os.path.join(build.CSRC, src), os.path.join(vdir, src + ".o"), defs)
# the product build's objects (<source>.<content key>.o; misc.hip.o) of every other source
objs = [os.path.join(obj_dir, "misc.hip.o" if os.path.basename(f) == "misc.hip"
                     else f"{os.path.basename(f)}.{build._obj_key(f, ())}.o")
        for f in build.sources() if os.path.basename(f) != src]
r = subprocess.run([build.HIPCC, f"--offload-arch={build.ARCH}", "-shared", "-fPIC", *objs, obj, "-o", out],
                   capture_output=True, text=True)
if r.returncode:
    raise SystemExit(r.stderr)
print("built", out, defs)
