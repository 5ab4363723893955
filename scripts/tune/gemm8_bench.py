"""fp8 (PG_FP8) vs bf16 prefill GEMM throughput at the pt-448 x16 Gemma shapes and square shapes, plus the
row quantiser's bandwidth (HIP events, 10 launches each).   python scripts/tune/gemm8_bench.py"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "paligemma-multimodal-system_amd"))
import torch  # noqa: E402
from pghip import ops  # noqa: E402
from pghip.weights import frag_pack, quant_rows_fp8  # noqa: E402

SHAPES = [  # name, M, N, K, epi
    ("gemma_gu", 16512, 32768, 2048, ops.EPI_BF16_GELU_MUL),
    ("gemma_down", 16512, 2048, 16384, ops.EPI_F32),
    ("gemma_qkv_plain", 16512, 2560, 2048, ops.EPI_BF16),
    ("gemma_o", 16512, 2048, 2048, ops.EPI_F32),
    ("sq4096", 4096, 4096, 4096, ops.EPI_BF16),
    ("sq8192", 8192, 8192, 8192, ops.EPI_BF16),
]


def timed(fn, n=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(n):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1000 / n


res = {}
for name, M, N, K, epi in SHAPES:
    A = (torch.rand(M, K, device="cuda") * 2 - 1).to(torch.bfloat16)
    W = ((torch.rand(N, K, device="cuda") * 2 - 1) / K ** 0.5).to(torch.bfloat16)
    n_out = N // 2 if epi == ops.EPI_BF16_GELU_MUL else N
    dt = torch.float32 if epi == ops.EPI_F32 else torch.bfloat16
    out = torch.empty(M, n_out, dtype=dt, device="cuda")
    Wf = frag_pack(W)
    us_bf = timed(lambda: ops.gemm(A, Wf, out, epi=epi | ops.W_FRAG))
    a8, sa = ops.quant_fp8(A)
    w8, sw = quant_rows_fp8(W)
    us_8 = timed(lambda: ops.gemm8(a8, sa, w8, sw, out, epi=epi))
    us_q = timed(lambda: ops.quant_fp8(A, a8, sa))
    fl = 2 * M * N * K
    res[name] = {"bf16_us": round(us_bf, 1), "bf16_TF": round(fl / us_bf / 1e6, 1), "fp8_us": round(us_8, 1),
                 "fp8_TF": round(fl / us_8 / 1e6, 1), "quant_us": round(us_q, 1),
                 "quant_GBs": round(3 * M * K / us_q / 1e3, 1)}
    print(name, json.dumps(res[name]), flush=True)
    del A, W, Wf, a8, w8, out
    torch.cuda.empty_cache()
