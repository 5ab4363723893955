"""Prefill GEMM throughput at the pt-448 x16 shapes (HIP events, 10 launches each, random bf16 operands).
    PGHIP_LIB=... python scripts/tune/gemm_bench.py"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "paligemma-multimodal-system_amd"))
import torch  # noqa: E402
from pghip import ops  # noqa: E402
from pghip.weights import frag_pack  # noqa: E402

SHAPES = [  # name, M, N, K, epi, frag
    ("gemma_gu", 16512, 32768, 2048, ops.EPI_BF16_GELU_MUL, True),
    ("gemma_gu_nofrag", 16512, 32768, 2048, ops.EPI_BF16_GELU_MUL, False),
    ("gemma_down", 16512, 2048, 16384, ops.EPI_F32, True),
    ("gemma_down_nofrag", 16512, 2048, 16384, ops.EPI_F32, False),
    ("gemma_qkv_plain", 16512, 2560, 2048, ops.EPI_BF16, True),
    ("gemma_qkv_nofrag", 16512, 2560, 2048, ops.EPI_BF16, False),
    ("gemma_o_nofrag", 16512, 2048, 2048, ops.EPI_F32, False),
    ("gemma_o", 16512, 2048, 2048, ops.EPI_F32, True),
    ("siglip_fc1", 16384, 4304, 1152, ops.EPI_BF16_GELU, False),
    ("siglip_fc1_plain", 16384, 4304, 1152, ops.EPI_BF16, False),
    ("siglip_o", 16384, 1152, 1152, ops.EPI_F32, False),
    ("siglip_fc2", 16384, 1152, 4352, ops.EPI_F32, False),
    ("siglip_qkv", 16384, 3456, 1152, ops.EPI_BF16, False),
    ("sq4096", 4096, 4096, 4096, ops.EPI_BF16, False),
    ("sq8192", 8192, 8192, 8192, ops.EPI_BF16, False),
]
res = {}
only = sys.argv[sys.argv.index("--only") + 1].split(",") if "--only" in sys.argv else None
for name, M, N, K, epi, frag in SHAPES:
    if only and name not in only:
        continue
    A = (torch.rand(M, K, device="cuda") * 2 - 1).to(torch.bfloat16)
    W = ((torch.rand(N, K, device="cuda") * 2 - 1) / K ** 0.5).to(torch.bfloat16)
    if frag:
        W = frag_pack(W)
        epi |= ops.W_FRAG
    n_out = N // 2 if (epi & 0xFF) == ops.EPI_BF16_GELU_MUL else N
    dt = torch.float32 if (epi & 0xFF) == ops.EPI_F32 else torch.bfloat16
    ks = ops.gemm_ksplit(M, N, K) if (epi & 0xFF) == ops.EPI_F32 else 1     # the engine's split-K (fp32 slabs)
    out = torch.empty(ks, M, n_out, dtype=dt, device="cuda")
    bias = None if (epi & 0xFF) == ops.EPI_BF16_GELU_MUL else torch.zeros(N, device="cuda")
    for _ in range(3):
        ops.gemm(A, W, out, epi=epi, bias=bias, ksplit=ks)
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(10):
        ops.gemm(A, W, out, epi=epi, bias=bias, ksplit=ks)
    b.record()
    torch.cuda.synchronize()
    us = a.elapsed_time(b) * 100
    res[name] = {"us": round(us, 1), "TFLOPs": round(2 * M * N * K / us / 1e6, 1), "ksplit": ks}
    print(name, json.dumps(res[name]), flush=True)
    del A, W, out
