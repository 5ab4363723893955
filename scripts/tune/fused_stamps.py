"""Per-workgroup timeline of the fused decode attention (pg_attn_decode; diagnostic variant built with
PG_ATTN_STAMPS=1): s_memrealtime stamps (100 MHz) at workgroup start, wave 0's blocks done, partial stored + ticket
taken, and (merging workgroup only) merge written.

    python scripts/tune/build_variant.py scripts/tune/stamps.so attn.hip PG_ATTN_STAMPS=1
    PGHIP_LIB=scripts/tune/stamps.so python scripts/tune/fused_stamps.py
"""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "paligemma-multimodal-system_amd"))
import torch  # noqa: E402
from pghip import ops, _lib  # noqa: E402

lib = _lib.load()
lib.pg_attn_stamps_read.argtypes = [C.c_void_p, C.c_int]
for name, B, L in (("pt448x16", 16, 1096), ("pt896x32", 32, 4168)):
    nh, nkv, hd = 8, 1, 256
    Smax = (L + 64 + 63) // 64 * 64
    kc = (torch.randn(4, B, Smax, hd, device="cuda") * 0.5).to(torch.bfloat16)
    vtc = (torch.randn(4, B, hd, Smax, device="cuda") * 0.5).to(torch.bfloat16)
    q = torch.randn(B, nh * hd, device="cuda").to(torch.bfloat16)
    lkv = torch.tensor([L - 1], dtype=torch.int32, device="cuda")
    kd, vd = ops.decode_cache_pack(kc.view(4 * B, Smax, hd), vtc.view(4 * B, hd, Smax), nkv)
    kd, vd = kd.view(4, B, -1), vd.view(4, B, -1)
    plan = ops.decode_plan(B, nkv, Smax)
    po = torch.empty(B * plan[0] * 16 * 256, device="cuda")
    pml = torch.empty(B * plan[0] * 16 * 2, device="cuda")
    cnt = torch.zeros(B, dtype=torch.int32, device="cuda")
    o = torch.empty(B, nh * hd, dtype=torch.bfloat16, device="cuda")
    for pipe in (False, True):
        ops.ATTN_PIPE = pipe
        for rep in range(6):
            i = rep % 4
            ops.attn_decode(q, nh * hd, o, nh * hd, kd[i], vd[i], B=B, Lkv=1, lkv_dev=lkv, Hq=nh, Hkv=nkv, D=hd,
                            scale=hd ** -0.5, kcap=Smax, part_o=po, part_ml=pml, counters=cnt, plan=plan)
            torch.cuda.synchronize()
        n = B * plan[0]
        buf = np.zeros((n, 4), dtype=np.uint64)
        assert lib.pg_attn_stamps_read(buf.ctypes.data, n) == 0
        t0 = int(buf[:, 0].min())
        t = (buf.astype(np.int64) - t0) * 10 / 1000.0     # us
        last = buf[:, 3] > 0
        q_ = lambda v: " ".join(f"{x:6.2f}" for x in np.percentile(v, [0, 10, 50, 90, 100]))  # noqa: E731
        print(f"{name} plan {plan} pipe {pipe}: {n} workgroups, {last.sum()} merging (us; p0 p10 p50 p90 p100)")
        print("  start          ", q_(t[:, 0]))
        print("  blocks         ", q_(t[:, 1] - t[:, 0]))
        print("  partial+ticket ", q_(t[:, 2] - t[:, 1]))
        print("  ticket taken at", q_(t[:, 2]))
        print("  merge          ", q_(t[last, 3] - t[last, 2]))
        print("  end            ", q_(t[last, 3]))
        # per split position (block counts differ by split)
        per = t[:, 1].reshape(B, plan[0]) - t[:, 0].reshape(B, plan[0])
        print("  blocks by split", " ".join(f"{x:5.2f}" for x in per.mean(0)))
    del kc, vtc
