"""Time the decode-GEMV variants of gemv_variants.hip on the decode shapes (one process, interleaved rounds).

    python scripts/tune/tune_gemv.py            (GPU box; the .so is built in this container)
"""
import ctypes as C
import os
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
lib = C.CDLL(os.path.join(HERE, "gemv_variants.so"))
lib.gemv_variant_run.argtypes = [C.c_int, C.c_void_p, C.c_int, C.c_void_p, C.c_int, C.c_int, C.c_void_p, C.c_int,
                                 C.c_int, C.c_int, C.c_void_p]
nv = lib.gemv_variant_count()
desc = []
for i in range(nv):
    d = (C.c_int * 5)()
    lib.gemv_variant_desc(i, d)
    desc.append(tuple(d))

SHAPES = {"gate_up": (32768, 2048, 1), "down": (2048, 16384, 1), "down_z2": (2048, 16384, 2),
          "down_z4": (2048, 16384, 4), "down_z8": (2048, 16384, 8), "qkv": (2560, 2048, 1), "o": (2048, 2048, 1),
          "o_z2": (2048, 2048, 2), "o_z4": (2048, 2048, 4), "lm_head": (257216, 2048, 1)}
Ms = [int(x) for x in (sys.argv[1].split(",") if len(sys.argv) > 1 else ["1", "16"])]
st = torch.cuda.current_stream().cuda_stream
res = {}
for name, (N, K, Z) in SHAPES.items():
    copies = max(1, min(8, (1 << 30) // (N * K * 2)))     # >= ~1 GiB rotated: defeats the 256 MiB MALL
    Ws = [torch.randn(N, K, device="cuda").to(torch.bfloat16) for _ in range(copies)]
    for M in Ms:
        x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
        out = torch.empty(Z, M, N, device="cuda")
        ref = (x.float() @ Ws[0].float().t())
        times = {i: [] for i in range(nv)}
        for rnd in range(5):
            for i in range(nv):
                if lib.gemv_variant_run(i, x.data_ptr(), K, Ws[0].data_ptr(), K, K, out.data_ptr(), N, M, Z, st):
                    times[i] = None
                    continue
                if rnd == 0:
                    torch.cuda.synchronize()
                    e = ((out.sum(0) - ref).abs().max() / ref.abs().max()).item()
                    if e > 1e-3:
                        print(f"  variant {i} {desc[i]} WRONG err {e}")
                        times[i] = None
                        continue
                if times[i] is None:
                    continue
                reps = 20
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for r in range(reps):
                    lib.gemv_variant_run(i, x.data_ptr(), K, Ws[r % copies].data_ptr(), K, K, out.data_ptr(), N, M, Z, st)
                e1.record()
                torch.cuda.synchronize()
                times[i].append(e0.elapsed_time(e1) / reps * 1e3)
        print(f"== {name} N={N} K={K} M={M} ({N * K * 2 / 1e6:.1f} MB)")
        rows = []
        for i in range(nv):
            if times[i]:
                t = sorted(times[i])[len(times[i]) // 2]
                rows.append((t, i))
        for t, i in sorted(rows)[:8]:
            print(f"  v{i:2d} U={desc[i][0]} D={desc[i][1]} WPT={desc[i][2]} NT={desc[i][3]} NTL={desc[i][4]}: "
                  f"{t:8.2f} us  {N * K * 2 / t / 1e3:7.0f} GB/s")
        del x, out
    del Ws
    torch.cuda.empty_cache()
