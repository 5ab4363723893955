"""Decode attention at long KV (BASELINE configs[2]: pt-448 x16, 1.03 k keys; configs[4]: pt-896 x32, 4.1 k keys) on
one library build: the split-KV attention + merge per layer, graph-replayed over the 18 layers' caches (no host in
the timing), for several keys-per-split choices, and the KV bytes / time.

    python scripts/tune/decode_attn_bench.py            (PGHIP_LIB=... for a variant build)
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "paligemma-multimodal-system_amd"))
import torch  # noqa: E402
from pghip import ops  # noqa: E402

torch.manual_seed(0)
res = {"lib": os.path.basename(os.environ.get("PGHIP_LIB", "libpghip.so"))}
for name, B, L in (("pt448x16", 16, 1096), ("pt896x32", 32, 4168), ("pt224x1", 1, 328)):
    nh, nkv, hd, layers = 8, 1, 256, 18
    Smax = (L + 64 + 63) // 64 * 64
    kvd = nkv * hd
    kc = (torch.randn(layers, B, Smax, kvd, device="cuda") * 0.5).to(torch.bfloat16)
    vtc = (torch.randn(layers, B, kvd, Smax, device="cuda") * 0.5).to(torch.bfloat16)
    q = (torch.randn(B, nh * hd, device="cuda")).to(torch.bfloat16)
    lkv = torch.tensor([L - 1], dtype=torch.int32, device="cuda")
    o = torch.empty(B, nh * hd, dtype=torch.bfloat16, device="cuda")
    packed = [ops.decode_cache_pack(kc[i], vtc[i], nkv) for i in range(layers)]
    kd, vd = [p[0] for p in packed], [p[1] for p in packed]
    dt = 256
    # the fused kernel (pg_attn_decode: attention + merge in one launch) at its default plan and neighbours
    cnt = torch.zeros(B * nkv, dtype=torch.int32, device="cuda")
    nblk = Smax // 32
    plans = [ops.decode_plan(B, nkv, Smax)]
    for nw, ns in ((2, 8), (2, 16), (4, 8), (4, 16), (4, 4), (4, 6), (4, 11), (4, 24), (4, 33), (2, 19), (4, 10),
                   (4, 5), (4, 3)):
        if nw * ns <= nblk and (ns, nw, -(-nblk // (nw * ns))) not in plans:
            plans.append((ns, nw, -(-nblk // (nw * ns))))
    for plan in plans:
        po = torch.empty(B * nkv * plan[0] * 16 * 256, device="cuda")
        pml = torch.empty(B * nkv * plan[0] * 16 * 2, device="cuda")

        def layer(i, plan=plan, po=po, pml=pml):
            ops.attn_decode(q, nh * hd, o, nh * hd, kd[i], vd[i],
                            B=B, Lkv=1, lkv_dev=lkv, Hq=nh, Hkv=nkv, D=hd, scale=hd ** -0.5, kcap=Smax, part_o=po,
                            part_ml=pml, counters=cnt, plan=plan)
        layer(0)
        torch.cuda.synchronize()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        g = torch.cuda.CUDAGraph()
        with torch.cuda.stream(s):
            with torch.cuda.graph(g, stream=s):
                for i in range(layers):
                    layer(i)
        g.replay()
        torch.cuda.synchronize()
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        ev[0].record()
        for _ in range(5):
            g.replay()
        ev[1].record()
        torch.cuda.synchronize()
        us = ev[0].elapsed_time(ev[1]) * 1000 / (5 * layers)
        kv_bytes = B * L * kvd * 2 * 2
        res[f"{name}/fused{plan}"] = round(us, 2)
        print(f"{name} fused plan {plan}: {us:7.2f} us per layer (attention + merge), "
              f"{kv_bytes / us / 1e3:7.1f} GB/s of KV", flush=True)
    if os.environ.get("PG_FUSED_ONLY"):
        del kc, vtc
        continue
    for sk in (32, 64, 128, 256, 384, 512, 768):
        nsplit = ((Smax + sk - 1) // sk + 3) // 4 * 4
        po = torch.empty(B * nkv * nsplit * 16 * dt, device="cuda")
        pml = torch.empty(B * nkv * nsplit * 16 * 2, device="cuda")

        def layer(i):
            ops.attention(q, nh * hd, None, nh * hd, kc[i], Smax * kvd, hd, kvd, vtc[i], kvd * Smax, hd * Smax, Smax,
                          B=B, Lq=1, Lkv=1, lkv_dev=lkv, Hq=nh, Hkv=nkv, D=hd, scale=hd ** -0.5, split_keys=sk,
                          nsplit=nsplit, part_o=po, part_ml=pml, kcap=Smax, kd=kd[i], vd=vd[i])
            ops.attn_combine(po, pml, o, nh * hd, B=B, Hq=nh, Hkv=nkv, D=hd, nsplit=nsplit)
        layer(0)
        torch.cuda.synchronize()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        g = torch.cuda.CUDAGraph()
        with torch.cuda.stream(s):
            with torch.cuda.graph(g, stream=s):
                for i in range(layers):
                    layer(i)
        g.replay()
        torch.cuda.synchronize()
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        ev[0].record()
        for _ in range(5):
            g.replay()
        ev[1].record()
        torch.cuda.synchronize()
        us = ev[0].elapsed_time(ev[1]) * 1000 / (5 * layers)
        kv_bytes = B * L * kvd * 2 * 2
        res[f"{name}/sk{sk}"] = round(us, 2)
        print(f"{name} sk{sk:4d} nsplit {nsplit:4d}: {us:7.2f} us per layer (attention + merge), "
              f"{kv_bytes / us / 1e3:7.1f} GB/s of KV", flush=True)
    del kc, vtc
print(json.dumps(res))
