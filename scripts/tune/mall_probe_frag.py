"""(fragment-packed weights, the decode layout) Does a weight stream read faster when its bytes were pulled into the Infinity Cache first?

Run under `rocprofv3 --kernel-trace`; phases are separated by host sleeps and analysed with
scripts/tune/mall_trace.py.  Phases (each cycles over 6 layers, so 6 x 134 MB > 256 MiB L3):
  gu_cold      gate/up GEMV (2x16384x2048 bf16, 134 MB) back to back
  gu_warm      [pg_prefetch(layer) -> gate/up GEMV(layer)] back to back
  dn_cold      down GEMV (2048x16384, 67 MB, split-K 4)
  dn_warm      [pg_prefetch -> down]
  chain        [3 x qkv-sized GEMV (2560x2048) -> gate/up -> down] per layer (a decode layer stand-in)
  chain_pf{W}  the same with pg_prefetch(gate/up + down of this layer, W workgroups) on a second stream
               forked at the layer start and joined before the gate/up GEMV
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "paligemma-multimodal-system_amd"))
import torch  # noqa: E402
from pghip import ops  # noqa: E402

dev = "cuda"
Lw = 6
gu = [torch.empty(32768, 2048, dtype=torch.bfloat16, device=dev).normal_() for _ in range(Lw)]
dn = [torch.empty(2048, 16384, dtype=torch.bfloat16, device=dev).normal_() for _ in range(Lw)]
qkv = [torch.empty(2560, 2048, dtype=torch.bfloat16, device=dev).normal_() for _ in range(3 * Lw)]
x = torch.randn(1, 2048, device=dev).to(torch.bfloat16)
h = torch.empty(1, 16384, dtype=torch.bfloat16, device=dev)
q_out = torch.empty(1, 2560, dtype=torch.bfloat16, device=dev)
part = torch.empty(4, 1, 2048, dtype=torch.float32, device=dev)
flush = torch.empty(256 * 1024 * 1024, dtype=torch.float32, device=dev)   # 1 GiB, read (clean) to evict L3
side = torch.cuda.Stream()


def gemv_gu(i):
    ops.gemm(x, gu[i], h, epi=ops.EPI_BF16_GELU_MUL | ops.W_FRAG)


def gemv_dn(i):
    ops.gemm(h, dn[i], part, epi=ops.EPI_F32 | ops.W_FRAG, ksplit=4)


def phase(name, body):
    torch.cuda.synchronize()
    ops.prefetch(flush, wgs=1024)          # marker + clean eviction
    torch.cuda.synchronize()
    time.sleep(0.005)
    body()
    torch.cuda.synchronize()
    time.sleep(0.005)
    print("phase", name, flush=True)


def layer(i, pf_wgs=0):
    if pf_wgs:
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            ops.prefetch(gu[i], wgs=pf_wgs)
            ops.prefetch(dn[i], wgs=pf_wgs)
    for j in range(3):
        ops.gemm(x, qkv[3 * i + j], q_out, epi=ops.EPI_BF16 | ops.W_FRAG)
    if pf_wgs:
        torch.cuda.current_stream().wait_stream(side)
    gemv_gu(i)
    gemv_dn(i)


for _ in range(2):
    gemv_gu(0); gemv_dn(0); ops.prefetch(gu[0]); layer(0); torch.cuda.synchronize()

R = 12
phase("gu_cold", lambda: [gemv_gu(r % Lw) for r in range(R)])
phase("gu_warm", lambda: [(ops.prefetch(gu[r % Lw]), gemv_gu(r % Lw)) for r in range(R)])
phase("dn_cold", lambda: [gemv_dn(r % Lw) for r in range(R)])
phase("dn_warm", lambda: [(ops.prefetch(dn[r % Lw]), gemv_dn(r % Lw)) for r in range(R)])
phase("chain", lambda: [layer(r % Lw) for r in range(R)])
for w in (32, 64, 128, 256):
    phase(f"chain_pf{w}", lambda: [layer(r % Lw, w) for r in range(R)])
phase("end", lambda: None)
