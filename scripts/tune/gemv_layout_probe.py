"""gate/up and down GEMV timing, row-major vs fragment-packed weights (PG_GEMV_PACKED=1 build via PGHIP_LIB).
Run under rocprofv3 --kernel-trace; phases split like mall_probe (flush marker kernels)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "paligemma-multimodal-system_amd"))
import torch  # noqa: E402
from pghip import ops  # noqa: E402

PACKED = os.environ.get("PACKED") == "1"


def pack(w):
    N, K = w.shape
    return w.view(N // 16, 16, K // 64, 4, 2, 8).permute(0, 2, 4, 3, 1, 5).contiguous().view(N, K)


dev = "cuda"
Lw = 6
gu0 = [torch.empty(32768, 2048, dtype=torch.bfloat16, device=dev).normal_() for _ in range(Lw)]
dn0 = [torch.empty(2048, 16384, dtype=torch.bfloat16, device=dev).normal_() for _ in range(Lw)]
gu = [pack(w) for w in gu0] if PACKED else gu0
dn = [pack(w) for w in dn0] if PACKED else dn0
x = torch.randn(1, 2048, device=dev).to(torch.bfloat16)
h = torch.empty(1, 16384, dtype=torch.bfloat16, device=dev)
part = torch.empty(4, 1, 2048, dtype=torch.float32, device=dev)
flush = torch.empty(256 * 1024 * 1024, dtype=torch.float32, device=dev)

# correctness of the packed addressing against the row-major build's math (torch reference)
ops.gemm(x, gu[0], h, epi=ops.EPI_BF16_GELU_MUL)
g = (x.float() @ gu0[0].float().t()).view(-1, 2, 16)
ref = (torch.nn.functional.gelu(g[:, 0], approximate="tanh") * g[:, 1]).reshape(1, -1)
err = ((h.float() - ref).abs().max() / ref.abs().max()).item()
ops.gemm(h, dn[0], part, epi=ops.EPI_F32, ksplit=4)
ref2 = h.float() @ dn0[0].float().t()
err2 = ((part.sum(0) - ref2).abs().max() / ref2.abs().max()).item()
print("packed" if PACKED else "rowmajor", "rel err gu", err, "dn", err2, flush=True)


def phase(name, body):
    torch.cuda.synchronize()
    ops.prefetch(flush, wgs=1024)
    torch.cuda.synchronize()
    time.sleep(0.005)
    body()
    torch.cuda.synchronize()
    time.sleep(0.005)


R = 12
for _ in range(2):
    phase("gu", lambda: [ops.gemm(x, gu[r % Lw], h, epi=ops.EPI_BF16_GELU_MUL) for r in range(R)])
    phase("dn", lambda: [ops.gemm(h, dn[r % Lw], part, epi=ops.EPI_F32, ksplit=4) for r in range(R)])
    phase("dn8", lambda: [ops.gemm(h, dn[r % Lw], part.new_empty(8, 1, 2048), epi=ops.EPI_F32, ksplit=8) for r in range(R)])
phase("end", lambda: None)
