"""Prefill GEMMs at batch-1 row counts (pt-224: Gemma 264 rows, SigLIP 256 rows) on one library build:
device time per call (HIP events, weights rotated over copies so nothing is L2/MALL-resident) and the error
against a torch fp32 matmul.  PGHIP_LIB=scripts/tune/skinny.so python scripts/tune/skinny_bench.py"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "paligemma-multimodal-system_amd"))
import torch  # noqa: E402
from pghip import ops  # noqa: E402

torch.manual_seed(0)
dev = "cuda"
SHAPES = [  # name, M, N, K, epi, ksplits
    ("gemma_gate_up", 264, 32768, 2048, ops.EPI_BF16_GELU_MUL, [1]),
    ("gemma_down", 264, 2048, 16384, ops.EPI_F32, [8, 16]),
    ("gemma_qkv_f32", 264, 2560, 2048, ops.EPI_F32, [3, 4, 8, 12]),
    ("gemma_o", 264, 2048, 2048, ops.EPI_F32, [4, 8, 16]),
    ("siglip_qkv_f32", 256, 3456, 1152, ops.EPI_F32, [3, 6, 9]),
    ("siglip_o", 256, 1152, 1152, ops.EPI_F32, [4, 9, 18]),
    ("siglip_fc1_f32", 256, 4352, 1152, ops.EPI_F32, [2, 6, 9]),
    ("siglip_fc2", 256, 1152, 4352, ops.EPI_F32, [4, 16, 28]),
]
res = {"lib": os.path.basename(os.environ.get("PGHIP_LIB", "libpghip.so"))}
for name, M, N, K, epi, splits in SHAPES:
    ncopy = max(1, min(6, (600 << 20) // (N * K * 2)))
    Ws = [torch.randn(N, K, device=dev).div_(K ** 0.5).to(torch.bfloat16) for _ in range(ncopy)]
    A = torch.randn(M, K, device=dev).to(torch.bfloat16)
    for ks in splits:
        if epi == ops.EPI_F32:
            out = torch.empty(ks, M, N, dtype=torch.float32, device=dev)
        else:
            out = torch.empty(M, N // 2 if epi == ops.EPI_BF16_GELU_MUL else N, dtype=torch.bfloat16, device=dev)
        call = lambda W: ops.gemm(A, W, out, epi=epi, ksplit=ks)  # noqa: E731
        for i in range(3):
            call(Ws[i % ncopy])
        torch.cuda.synchronize()
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        R = 30
        ev[0].record()
        for i in range(R):
            call(Ws[i % ncopy])
        ev[1].record()
        torch.cuda.synchronize()
        us = ev[0].elapsed_time(ev[1]) * 1000 / R
        call(Ws[0])
        torch.cuda.synchronize()
        ref = A.float() @ Ws[0].float().t()
        if epi == ops.EPI_F32:
            got = out.sum(0)
        else:
            g = ref.view(M, N // 32, 2, 16)
            ref = (torch.nn.functional.gelu(g[:, :, 0], approximate="tanh") * g[:, :, 1]).reshape(M, N // 2)
            got = out.float()
        e = float((got - ref).abs().max() / ref.abs().max())
        tf = 2 * M * N * K / us / 1e6
        res[f"{name}/ks{ks}"] = [round(us, 2), round(tf, 1), f"{e:.1e}"]
        print(name, ks, f"{us:8.2f} us {tf:7.1f} TF/s err {e:.1e}", flush=True)
print(json.dumps(res))
