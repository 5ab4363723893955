"""fp8 prefill GEMMs at the pt-896 x32 Gemma shapes (M = 32 x 4104): row-scaled A (gemm8) and the MX-row forms
(gate/up writing MX h, down reading it); HIP events, 5 launches each.   python scripts/tune/gemm8_big.py [M]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "paligemma-multimodal-system_amd"))
import torch  # noqa: E402
from pghip import ops  # noqa: E402
from pghip.weights import quant_rows_fp8  # noqa: E402

M = int(sys.argv[1]) if len(sys.argv) > 1 else 32 * 4104


def timed(fn, n=5):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(n):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1000 / n


def weights(N, K):
    W = ((torch.rand(N, K, device="cuda") * 2 - 1) / K ** 0.5).to(torch.bfloat16)
    return quant_rows_fp8(W)


K = 2048
A = (torch.rand(M, K, device="cuda") * 2 - 1).to(torch.bfloat16)
a8, sa = ops.quant_fp8(A)
del A
w8, sw = weights(32768, K)
h = torch.empty(M, 16384, dtype=torch.bfloat16, device="cuda")
res = {}
res["gateup_rows"] = timed(lambda: ops.gemm8(a8, sa, w8, sw, h, epi=ops.EPI_BF16_GELU_MUL))
del h
h8 = torch.empty(M, 16384, dtype=torch.uint8, device="cuda")
hs = torch.empty(M, 16384 // 32, dtype=torch.uint8, device="cuda")
res["gateup_mx"] = timed(lambda: ops.gemm8(a8, sa, w8, sw, h8, epi=ops.EPI_BF16_GELU_MUL, mx_out=hs))
del w8, sw
wo, so = weights(2048, K)
o = torch.empty(M, 2048, dtype=torch.float32, device="cuda")
res["o_rows"] = timed(lambda: ops.gemm8(a8, sa, wo, so, o, epi=ops.EPI_F32))
wd, sd = weights(2048, 16384)
hq, hsq = ops.quant_fp8(torch.empty(M, 16384, dtype=torch.bfloat16, device="cuda").uniform_(-1, 1))
res["down_rows"] = timed(lambda: ops.gemm8(hq, hsq, wd, sd, o, epi=ops.EPI_F32))
res["down_mx"] = timed(lambda: ops.gemm8(h8, None, wd, sd, o, epi=ops.EPI_F32, mx_in=hs))


def check(a, s_a, w, s_w, out):
    """max relative error of rows [0, 256) and the last 300 rows against fp32 over the same e4m3 bytes"""
    wf = w.view(torch.float8_e4m3fn).float() * s_w[:, None]
    errs = []
    for r0 in (0, M - 300):
        rows = slice(r0, r0 + (256 if r0 == 0 else 300))
        ref = (a[rows].view(torch.float8_e4m3fn).float() * s_a[rows, None]) @ wf.t()
        errs.append(((out[rows] - ref).abs().max() / ref.abs().max()).item())
    return max(errs)


ops.gemm8(a8, sa, wo, so, o, epi=ops.EPI_F32)
err_o = check(a8, sa, wo, so, o)
ops.gemm8(hq, hsq, wd, sd, o, epi=ops.EPI_F32)
err_d = check(hq, hsq, wd, sd, o)
print(json.dumps({"err_o": err_o, "err_down": err_d}), flush=True)
flops = {"gateup_rows": 2 * M * 32768 * K, "gateup_mx": 2 * M * 32768 * K, "o_rows": 2 * M * 2048 * K,
         "down_rows": 2 * M * 2048 * 16384, "down_mx": 2 * M * 2048 * 16384}
print(json.dumps({k: {"us": round(v, 1), "TF": round(flops[k] / v / 1e6, 1)} for k, v in res.items()}), flush=True)
