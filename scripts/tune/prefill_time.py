"""Batch-1 prefill (vision + merge + Gemma + first token) of the bench workload: GPU time per prefill (HIP
events over R back-to-back prefills) and the host time to issue them, alternating engine knobs in-process.

    python scripts/tune/prefill_time.py [--config pt-224] [--reps 20] [--knob TILE_M1]

A host issue time close to the GPU time means the eager prefill is launch-bound, not kernel-bound."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "paligemma-multimodal-system_amd")]
import torch  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="pt-224")
ap.add_argument("--reps", type=int, default=20)
ap.add_argument("--knob", default="TILE_M1", help="boolean engine class attribute toggled on / off")
a = ap.parse_args()

from pghip import configs, engine, synthetic, weights  # noqa: E402
import bench  # noqa: E402

cfg = configs.CONFIGS[a.config]
sd = synthetic.SyntheticStateDict(cfg)
eng = engine.PaliGemmaEngine(cfg, weights.PackedWeights(cfg, sd.__getitem__))
ids, px = bench.synthetic_inputs(cfg, 1, [2, 651, 4906, 603, 476, 2121, 576, 108])
ids, px = ids.cuda(), px.cuda()
run = bench.Runner(eng, ids, px, 8, dict(do_sample=False))
res = {"config": a.config, "knob": a.knob}
for rnd in range(3):
    for on in (True, False):
        setattr(eng, a.knob, on)
        run.prefill_run()
        torch.cuda.synchronize()
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        ev[0].record()
        t0 = time.perf_counter()
        for _ in range(a.reps):
            run.prefill_run()
        host = (time.perf_counter() - t0) / a.reps * 1e3
        ev[1].record()
        torch.cuda.synchronize()
        gpu = ev[0].elapsed_time(ev[1]) / a.reps
        res.setdefault(f"{a.knob}={int(on)}", []).append([round(gpu, 3), round(host, 3)])
        print(f"{a.knob}={int(on)} prefill {gpu:.3f} ms (host issue {host:.3f} ms)", flush=True)
# the same prefill replayed from one captured hipGraph (bench.py --graph-prefill): no host launches in the timing
setattr(eng, a.knob, True)
g = torch.cuda.CUDAGraph()
run.prefill_run()
torch.cuda.synchronize()
with torch.cuda.graph(g):
    run.prefill_run()
torch.cuda.synchronize()
for rnd in range(3):
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ev[0].record()
    for _ in range(a.reps):
        g.replay()
    ev[1].record()
    torch.cuda.synchronize()
    gpu = ev[0].elapsed_time(ev[1]) / a.reps
    res.setdefault("graph", []).append(round(gpu, 3))
    print(f"graph prefill {gpu:.3f} ms", flush=True)
print(json.dumps(res))
