"""GPU time of one batch-1 prefill (vision + merge + Gemma + first token) of the bench workload for the library that
PGHIP_LIB selects: HIP events over R back-to-back prefills, 3 rounds; prints one JSON line (ms per prefill per round)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "paligemma-multimodal-system_amd")]
import torch  # noqa: E402
from pghip import configs, engine, synthetic, weights  # noqa: E402
import bench  # noqa: E402

cfg = configs.CONFIGS[os.environ.get("CFG", "pt-224")]
eng = engine.PaliGemmaEngine(cfg, weights.PackedWeights(cfg, synthetic.SyntheticStateDict(cfg).__getitem__))
ids, px = bench.synthetic_inputs(cfg, 1, [2, 651, 4906, 603, 476, 2121, 576, 108])
run = bench.Runner(eng, ids.cuda(), px.cuda(), 8, dict(do_sample=False))
R = int(os.environ.get("REPS", "20"))
out = []
for rnd in range(3):
    run.prefill_run()
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ev[0].record()
    for _ in range(R):
        run.prefill_run()
    ev[1].record()
    torch.cuda.synchronize()
    out.append(round(ev[0].elapsed_time(ev[1]) / R, 4))
print(json.dumps({"lib": os.path.basename(os.environ.get("PGHIP_LIB") or "product"), "prefill_ms": out}))
