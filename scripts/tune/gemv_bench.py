"""Per-kernel decode GEMV timings (pt-224 weights, M=1): N launches captured in one hipGraph (no host launch cost),
each launch on the next layer's weights (no L2/MALL reuse between launches); graph replay timed with HIP events.
Prints one JSON line (us per launch and GB/s of weights)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "paligemma-multimodal-system_amd")]
import torch  # noqa: E402
from pghip import configs, ops, synthetic, weights  # noqa: E402

cfg = configs.CONFIGS["pt-224"]
sd = synthetic.SyntheticStateDict(cfg)
w = weights.PackedWeights(cfg, sd.__getitem__)
H, I = w.hidden, w.inter
x = torch.randn(1, H, device="cuda").to(torch.bfloat16)
hx = torch.randn(1, I, device="cuda").to(torch.bfloat16)
h = torch.empty(1, I, dtype=torch.bfloat16, device="cuda")
part = torch.empty(4, 1, H, device="cuda")
part8 = torch.empty(8, 1, H, device="cuda")
logits = torch.empty(1, w.vocab_local_pad, device="cuda")
L = w.tl


def timed(fn, n):
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
    g.replay()
    torch.cuda.synchronize()
    best = 1e9
    for _ in range(5):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        g.replay()
        e1.record()
        torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1) * 1e3 / n)
    return best


res = {}
res["gateup_us"] = timed(lambda i: ops.gemm(x, L[i % 18]["gu_w"], h, epi=ops.EPI_BF16_GELU_MUL | w.wflag), 36)
res["down_s4_us"] = timed(lambda i: ops.gemm(hx, L[i % 18]["down_w"], part, epi=ops.EPI_F32 | w.wflag, ksplit=4), 36)
res["down_s8_us"] = timed(lambda i: ops.gemm(hx, L[i % 18]["down_w"], part8, epi=ops.EPI_F32 | w.wflag, ksplit=8), 36)
res["o_s2_us"] = timed(lambda i: ops.gemm(x, L[i % 18]["o_w"], part[:2], epi=ops.EPI_F32 | w.wflag, ksplit=2), 36)
res["qkv_us"] = timed(lambda i: ops.gemm(x, L[i % 18]["qkv_w"], h[:, :w.qkv_n], epi=ops.EPI_BF16 | w.wflag), 36)
res["lm_head_us"] = timed(lambda i: ops.gemm(x, w.lm_w, logits, epi=ops.EPI_F32 | w.wflag, bias=w.lm_bias), 4)
res["gateup_same_layer_us"] = timed(lambda i: ops.gemm(x, L[0]["gu_w"], h, epi=ops.EPI_BF16_GELU_MUL | w.wflag), 36)
res["down_same_layer_us"] = timed(lambda i: ops.gemm(hx, L[0]["down_w"], part, epi=ops.EPI_F32 | w.wflag, ksplit=4), 36)
res["gateup_GBs"] = L[0]["gu_w"].numel() * 2 / res["gateup_us"] / 1e3
res["down_GBs"] = L[0]["down_w"].numel() * 2 / res["down_s4_us"] / 1e3
res["lm_head_GBs"] = w.lm_w.numel() * 2 / res["lm_head_us"] / 1e3
res = {k: round(v, 2) for k, v in res.items()}
res["knobs"] = {k: os.environ[k] for k in ("PG_GEMV_CPW_OFF", "PG_GEMV_D_NT1", "PG_GEMV_D_NT2") if k in os.environ}
print(json.dumps(res), flush=True)
