"""Prefill attention throughput at the bench shapes (HIP events; random bf16 q/k/v).
    python scripts/tune/attn_bench.py [--only gemma448]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "paligemma-multimodal-system_amd"))
import torch  # noqa: E402
from pghip import ops  # noqa: E402

SHAPES = {  # name: (B, L, Hq, Hkv, D)
    "gemma448x16": (16, 1032, 8, 1, 256),
    "siglip448x16": (16, 1024, 16, 16, 72),
    "gemma224": (1, 264, 8, 1, 256),
    "siglip224": (1, 256, 16, 16, 72),
    "gemma896x32": (32, 4104, 8, 1, 256),
    "siglip896x32": (32, 4096, 16, 16, 72),
}
only = sys.argv[sys.argv.index("--only") + 1].split(",") if "--only" in sys.argv else list(SHAPES)
reps = int(os.environ.get("REPS", "10"))
for name in only:
    B, L, Hq, Hkv, D = SHAPES[name]
    g = torch.Generator(device="cuda").manual_seed(0)
    q = torch.randn(B * L, Hq * D, device="cuda", generator=g).to(torch.bfloat16)
    k = torch.randn(B, L, Hkv * D, device="cuda", generator=g).to(torch.bfloat16)
    vt = torch.zeros(B, Hkv * D, L + 32, device="cuda", dtype=torch.bfloat16)
    vt[:, :, :L] = torch.randn(B, Hkv * D, L, device="cuda", generator=g).to(torch.bfloat16)
    o = torch.empty(B * L, Hq * D, device="cuda", dtype=torch.bfloat16)

    def run():
        ops.attention(q, Hq * D, o, Hq * D, k, L * Hkv * D, D, Hkv * D, vt, Hkv * D * (L + 32), D * (L + 32), L + 32,
                      B=B, Lq=L, Lkv=L, Hq=Hq, Hkv=Hkv, D=D, scale=D ** -0.5)
    run()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        run()
    b.record()
    torch.cuda.synchronize()
    us = a.elapsed_time(b) * 1e3 / reps
    fl = 4.0 * B * Hq * L * L * D
    # spot check against torch on batch 0, first kv head group
    G = Hq // Hkv
    qq = q.view(B, L, Hq, D)[0, :, :G].float().permute(1, 0, 2)
    kk = k.view(B, L, Hkv, D)[0, :, 0].float()
    vv = vt.view(B, Hkv, D, L + 32)[0, 0, :, :L].float().t()
    ref = torch.softmax(qq @ kk.t() * D ** -0.5, -1) @ vv
    got = o.view(B, L, Hq, D)[0, :, :G].float().permute(1, 0, 2)
    err = ((got - ref).abs().max() / ref.abs().max()).item()
    print(name, json.dumps({"us": round(us, 1), "TFLOPs": round(fl / us / 1e6, 1), "rel_err": round(err, 5)}), flush=True)
