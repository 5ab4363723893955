"""Per-wave timeline of the split-KV decode attention (diagnostic variant built with PG_ATTN_STAMPS=1):
s_memrealtime stamps (100 MHz) at wave start, block loads landed, compute done, partials written.

    PGHIP_LIB=scripts/tune/stamps.so python scripts/tune/attn_stamps.py
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
for name, B, L, sk in (("pt448x16", 16, 1096, 32), ("pt896x32", 32, 4168, 32),
                       ("pt224x1", 1, 328, 32)):
    nh, nkv, hd = 8, 1, 256
    Smax = (L + 64 + 63) // 64 * 64
    kc = (torch.randn(4, B, Smax, hd, device="cuda") * 0.5).to(torch.bfloat16)
    vtc = (torch.randn(4, B, hd, Smax, device="cuda") * 0.5).to(torch.bfloat16)
    q = torch.randn(B, nh * hd, device="cuda").to(torch.bfloat16)
    lkv = torch.tensor([L - 1], dtype=torch.int32, device="cuda")
    nsplit = ((Smax + sk - 1) // sk + 3) // 4 * 4
    po = torch.empty(B * nsplit * 16 * 256, device="cuda")
    pml = torch.empty(B * nsplit * 16 * 2, device="cuda")
    kd, vd = ops.decode_cache_pack(kc.view(4 * B, Smax, hd), vtc.view(4 * B, hd, Smax), nkv)
    kd, vd = kd.view(4, B, -1), vd.view(4, B, -1)
    for rep in range(6):
        i = rep % 4
        ops.attention(q, nh * hd, None, nh * hd, kc[i], Smax * hd, hd, hd, vtc[i], hd * Smax, hd * Smax, Smax,
                      B=B, Lq=1, Lkv=1, lkv_dev=lkv, Hq=nh, Hkv=nkv, D=hd, scale=hd ** -0.5, split_keys=sk,
                      nsplit=nsplit, part_o=po, part_ml=pml, kcap=Smax, kd=kd[i], vd=vd[i])
        torch.cuda.synchronize()
    n = B * nsplit
    buf = np.zeros((n, 4), dtype=np.uint64)
    assert lib.pg_attn_stamps_read(buf.ctypes.data, n) == 0
    nz = buf[:, 0] > 0
    t = (buf[nz].astype(np.int64) - int(buf[nz, 0].min())) * 10 / 1000.0     # us
    q_ = lambda v: " ".join(f"{x:6.2f}" for x in np.percentile(v, [0, 10, 50, 90, 100]))  # noqa: E731
    print(f"{name} sk{sk} waves {nz.sum()} (us; p0 p10 p50 p90 p100)")
    print("  start        ", q_(t[:, 0]))
    print("  loads landed ", q_(t[:, 1] - t[:, 0]))
    print("  compute      ", q_(t[:, 2] - t[:, 1]))
    print("  write+drain  ", q_(t[:, 3] - t[:, 2]))
    print("  end          ", q_(t[:, 3]))
    del kc, vtc
