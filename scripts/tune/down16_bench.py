"""pt-448 x16 decode MLP GEMVs in isolation (M = 16, pt-224-sized Gemma weights): the finalised down GEMV (F32_FIN, the
product's split 4) against the same stream without the finalising tail (plain fp32 slabs, split 4 / 8) and the gate/up
GEMV; 18 launches per captured graph, each on the next layer's weights (no cache reuse), replay timed with HIP events.
Prints one JSON line: us per launch and the weight-stream rate."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "paligemma-multimodal-system_amd")]
import torch  # noqa: E402
from pghip import configs, ops, synthetic, weights  # noqa: E402

cfg = configs.CONFIGS["pt-224"]
w = weights.PackedWeights(cfg, synthetic.SyntheticStateDict(cfg).__getitem__)
H, I, M = w.hidden, w.inter, 16
L = w.tl
x = torch.randn(M, H, device="cuda").to(torch.bfloat16)
hx = torch.randn(M, I, device="cuda").to(torch.bfloat16)
h = torch.empty(M, I, dtype=torch.bfloat16, device="cuda")
tiles = H // 16
res = torch.randn(M, H, device="cuda")
cnt = torch.zeros(tiles, dtype=torch.int32, device="cuda")
ss = torch.empty(M, tiles, device="cuda")
xq = torch.empty(M, H, dtype=torch.bfloat16, device="cuda")
parts = {s: torch.empty(s, M, H, device="cuda") for s in (4, 8)}


def timed(fn, n=18, reps=5):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for i in range(2):
            fn(i)
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for i in range(n):
            fn(i)
    best = 1e9
    for _ in range(reps):
        g.replay()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        g.replay()
        e1.record()
        torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1) * 1e3 / n)
    return best


out = {}
fa = ops.fused_args(fin_cnt=cnt, fin_resid=res, ss_out=ss, ss_ld=tiles, fin_x=xq, norm_w=w.final_w)
out["down_fin_s4"] = timed(lambda i: ops.gemm_fused(hx, L[i % len(L)]["down_w"], parts[4], fa,
                                                    epi=ops.EPI_F32_FIN | w.wflag, M=M, ksplit=4))
for s in (4, 8):
    out[f"down_f32_s{s}"] = timed(lambda i, s=s: ops.gemm(hx, L[i % len(L)]["down_w"], parts[s], epi=ops.EPI_F32 | w.wflag,
                                                          ksplit=s))
out["gateup"] = timed(lambda i: ops.gemm(x, L[i % len(L)]["gu_w"], h, epi=ops.EPI_BF16_GELU_MUL | w.wflag))
wd, wgu = L[0]["down_w"].numel() * 2, L[0]["gu_w"].numel() * 2
out["down_w_TBs"] = {k: round(wd / v / 1e6, 2) for k, v in out.items() if k.startswith("down")}
out["gateup_w_TBs"] = round(wgu / out["gateup"] / 1e6, 2)
print(json.dumps({k: (round(v, 2) if isinstance(v, float) else v) for k, v in out.items()}), flush=True)
