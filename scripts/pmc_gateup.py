"""Launch the roofline kernel of bench.py (the decode gate/up GEMV, 2x16384x2048 bf16, rotating the 18
layers' weights) 36 times, for a rocprofv3 --pmc pass (FETCH_SIZE and WRITE_SIZE in separate passes).

    rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/pmc_f -o run --output-format csv -- python scripts/pmc_gateup.py
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "paligemma-multimodal-system_amd")]
import torch  # noqa: E402
from pghip import configs, ops, synthetic, weights  # noqa: E402

cfg = configs.PT_224
sd = synthetic.SyntheticStateDict(cfg)
w = weights.PackedWeights(cfg, sd.__getitem__, parts=("text",))
x = torch.randn(1, w.hidden, device="cuda").to(torch.bfloat16)
h = torch.empty(1, w.inter, dtype=torch.bfloat16, device="cuda")
for i in range(36):
    ops.gemm(x, w.tl[i % len(w.tl)]["gu_w"], h, epi=ops.EPI_BF16_GELU_MUL | w.wflag)
torch.cuda.synchronize()
print("launched 36 gate/up GEMVs")
