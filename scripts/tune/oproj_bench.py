"""Batch-1 decode o_proj GEMV with the split-KV merge prologue (PRO_ATTN_COMBINE): per-call time vs the number of
attention partials it merges (asplit) and the o split-K, graph-replayed over 18 weight copies (no MALL reuse).

    python scripts/tune/oproj_bench.py
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "paligemma-multimodal-system_amd"))
import torch  # noqa: E402
from pghip import ops  # noqa: E402

torch.manual_seed(0)
H, nh, hd, layers = 2048, 8, 256, 18
Ws = [(torch.randn(H, H, device="cuda") * 0.02).to(torch.bfloat16) for _ in range(layers)]
res = {}
for asplit in (16, 12, 8, 4):
    po = torch.randn(asplit * 16 * 256, device="cuda")
    pml = torch.randn(asplit * 16 * 2, device="cuda")
    pml.view(-1, 2)[:, 1].abs_().add_(1.0)
    for so in (1, 2, 4, 8):
        part = torch.empty(so, 1, H, device="cuda")
        fa = ops.fused_args(pro_mode=ops.PRO_ATTN_COMBINE, part_o=po, part_ml=pml, asplit=asplit, head_dim=hd,
                            dtw=256, q_per_kv=nh, kv_heads=1, akeys=32)

        def run():
            for i in range(layers):
                ops.gemm_fused(None, Ws[i], part, fa, epi=ops.EPI_F32 | ops.W_FRAG, M=1, ksplit=so)
        run()
        torch.cuda.synchronize()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        g = torch.cuda.CUDAGraph()
        with torch.cuda.stream(s):
            with torch.cuda.graph(g, stream=s):
                run()
        g.replay()
        torch.cuda.synchronize()
        best = 1e9
        for _ in range(5):
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
            ev[0].record()
            for _ in range(10):
                g.replay()
            ev[1].record()
            torch.cuda.synchronize()
            best = min(best, ev[0].elapsed_time(ev[1]) * 1000 / (10 * layers))
        res[f"asplit{asplit}/so{so}"] = round(best, 2)
        print(f"asplit {asplit:2d} split_o {so}: {best:6.2f} us per call", flush=True)
print(json.dumps(res))
