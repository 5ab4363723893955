"""Batch-1 prefill linears (SigLIP 256 rows, Gemma 264 rows) on one library build: per-call device time of each
(tile, split) choice, the calls replayed from a captured hipGraph over 27 / 18 distinct weight copies (no host in
the timing, no L2 reuse across calls), the split-K finalisation included for the bf16 epilogues.

    python scripts/tune/small_gemm_sweep.py            (PGHIP_LIB=... for a variant build)
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "paligemma-multimodal-system_amd"))
import torch  # noqa: E402
from pghip import ops  # noqa: E402

torch.manual_seed(0)
SHAPES = [  # name, M, N, K, epi, copies
    ("siglip_qkv", 256, 3456, 1152, ops.EPI_BF16, 27),
    ("siglip_o", 256, 1152, 1152, ops.EPI_F32, 27),
    ("siglip_fc1", 256, 4352, 1152, ops.EPI_BF16_GELU, 27),
    ("siglip_fc2", 256, 1152, 4352, ops.EPI_F32, 27),
    ("gemma_qkv", 264, 2560, 2048, ops.EPI_BF16, 18),
    ("gemma_o", 264, 2048, 2048, ops.EPI_F32, 18),
    ("gemma_gateup", 264, 32768, 2048, ops.EPI_BF16_GELU_MUL, 18),
    ("gemma_down", 264, 2048, 16384, ops.EPI_F32, 18),
]
TILES = ((0, "t64"), (ops.TILE_M1, "m1"), (ops.TILE_N64, "n64"))
# SWEEP_SHAPES / SWEEP_TILES / SWEEP_KS (comma lists) restrict the sweep; SWEEP_BLAS=0 skips the library GEMM
if os.environ.get("SWEEP_SHAPES"):
    SHAPES = [x for x in SHAPES if x[0] in os.environ["SWEEP_SHAPES"].split(",")]
if os.environ.get("SWEEP_TILES"):
    TILES = tuple(x for x in TILES if x[1] in os.environ["SWEEP_TILES"].split(","))
KS = tuple(int(k) for k in os.environ.get("SWEEP_KS", "1,2,3,4,6,9,12,18").split(","))


def run(name, M, N, K, epi, copies, flags, ks):
    Ws = [torch.randn(N, K, device="cuda").div_(K ** 0.5).to(torch.bfloat16) for _ in range(copies)]
    A = torch.randn(M, K, device="cuda").to(torch.bfloat16)
    if epi == ops.EPI_F32:
        out = torch.empty(ks, M, N, dtype=torch.float32, device="cuda")
    elif epi == ops.EPI_BF16_GELU_MUL:
        out = torch.empty(M, N // 2, dtype=torch.bfloat16, device="cuda")
    else:
        out = torch.empty(M, N, dtype=torch.bfloat16, device="cuda")
    old = ops.FINALIZE_SPLIT
    part = torch.empty(ks, M, N, dtype=torch.float32, device="cuda")

    def call(W):
        if epi == ops.EPI_F32:
            ops.gemm(A, W, out, epi=epi | flags, ksplit=ks)
        elif ks == 1:
            ops.FINALIZE_SPLIT = False
            ops.gemm(A, W, out, epi=epi | flags)
            ops.FINALIZE_SPLIT = old
        else:   # split-K fp32 slabs + the finalisation kernel, as ops.gemm does for a small grid
            ops._lib.call("pg_gemm", A.data_ptr(), K, W.data_ptr(), K, None, part.data_ptr(), N, M, N, K,
                          ops.EPI_F32 | flags, ks, None, 0, None, 0, 0, ops._s())
            ops._lib.call("pg_gemm_finalize", part.data_ptr(), ks, out.data_ptr(), out.stride(0), M, N, epi, None, 0, 0, None,
                          ops._s())
    try:
        call(Ws[0])
        torch.cuda.synchronize()
    except Exception as e:  # noqa: BLE001
        return None, str(e)[:80]
    ref = A.float() @ Ws[0].float().t()
    got = out.float().sum(0) if epi == ops.EPI_F32 else out.float()
    if epi == ops.EPI_BF16_GELU:
        ref = torch.nn.functional.gelu(ref, approximate="tanh")
    elif epi == ops.EPI_BF16_GELU_MUL:   # gate / up interleaved in 16-row groups
        r4 = ref.view(M, N // 32, 2, 16)
        ref = (torch.nn.functional.gelu(r4[:, :, 0], approximate="tanh") * r4[:, :, 1]).reshape(M, N // 2)
    e = float((got - ref).abs().max() / ref.abs().max())
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            for W in Ws:
                call(W)
    g.replay()
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ev[0].record()
    for _ in range(5):
        g.replay()
    ev[1].record()
    torch.cuda.synchronize()
    return ev[0].elapsed_time(ev[1]) * 1000 / (5 * copies), e


def blas(M, N, K, copies):
    """torch.matmul (hipBLASLt) on the same shape, plain bf16 output: the library GEMM as a yardstick."""
    Ws = [torch.randn(N, K, device="cuda").div_(K ** 0.5).to(torch.bfloat16) for _ in range(copies)]
    A = torch.randn(M, K, device="cuda").to(torch.bfloat16)
    out = torch.empty(M, N, dtype=torch.bfloat16, device="cuda")
    for W in Ws:
        torch.matmul(A, W.t(), out=out)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            for W in Ws:
                torch.matmul(A, W.t(), out=out)
    g.replay()
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ev[0].record()
    for _ in range(5):
        g.replay()
    ev[1].record()
    torch.cuda.synchronize()
    return ev[0].elapsed_time(ev[1]) * 1000 / (5 * copies)


res = {"lib": os.path.basename(os.environ.get("PGHIP_LIB", "libpghip.so"))}
for name, M, N, K, epi, copies in SHAPES:
    try:
        if os.environ.get("SWEEP_BLAS", "1") != "0":
            us = blas(M, N, K, copies)
            res[f"{name}/blas"] = round(us, 2)
            print(f"{name:11s} blas     {us:8.2f} us  {2 * M * N * K / us / 1e6:7.1f} TF/s", flush=True)
    except Exception as e:  # noqa: BLE001
        print(f"{name:11s} blas failed: {str(e)[:80]}", flush=True)
    for flags, tag in TILES:
        for ks in KS:
            if (K // 64) // ks < 2:
                continue
            us, e = run(name, M, N, K, epi, copies, flags, ks)
            if us is None:
                continue
            res[f"{name}/{tag}/ks{ks}"] = round(us, 2)
            print(f"{name:11s} {tag:3s} ks{ks:2d} {us:8.2f} us  {2 * M * N * K / us / 1e6:7.1f} TF/s  err {e:.1e}",
                  flush=True)
print(json.dumps(res))
