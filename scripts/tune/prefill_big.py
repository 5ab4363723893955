"""One batched prefill of a BASELINE workload (default configs[4]: pt-896, batch 32, fp8 Gemma linears) run twice
(the second is the one to read in a kernel trace: scripts/prefill_breakdown.py picks the middle im2col segment).

    rocprofv3 --kernel-trace --stats -d <dir> -o run --output-format csv -- python scripts/tune/prefill_big.py
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "paligemma-multimodal-system_amd")]
import torch  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="pt-896")
ap.add_argument("--batch", type=int, default=32)
ap.add_argument("--bf16", action="store_true")
ap.add_argument("--reps", type=int, default=3)
a = ap.parse_args()

from pghip import configs, engine, synthetic, weights  # noqa: E402
import bench  # noqa: E402

cfg = configs.CONFIGS[a.config]
sd = synthetic.SyntheticStateDict(cfg)
eng = engine.PaliGemmaEngine(cfg, weights.PackedWeights(cfg, sd.__getitem__, fp8=not a.bf16))
ids, px = bench.synthetic_inputs(cfg, a.batch, [2, 651, 4906, 603, 476, 2121, 576, 108])
run = bench.Runner(eng, ids.cuda(), px.cuda(), 2, dict(do_sample=False))
for i in range(a.reps):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    run.prefill_run()
    torch.cuda.synchronize()
    print(f"prefill {i}: {(time.perf_counter() - t0) * 1e3:.1f} ms", flush=True)
run.request()                       # a decode step after the prefills (the breakdown's segment end)
torch.cuda.synchronize()
