"""Per-step error / margin table of the full-size pt-224 teacher-forced decode (test_pt224_full_size_teacher_forced_decode),
for comparing kernel variants: python scripts/tune/tf_errors.py"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "paligemma-multimodal-system_amd")]
import torch  # noqa: E402
from pghip import configs, engine, synthetic, weights  # noqa: E402

g = dict(np.load(os.path.join(ROOT, "tests", "golden", "pt224.npz")))
cfg = configs.PT_224
sd = synthetic.SyntheticStateDict(cfg)
eng = engine.PaliGemmaEngine(cfg, weights.PackedWeights(cfg, sd.__getitem__))
ids = torch.from_numpy(g["input_ids"]).cuda()
px = torch.from_numpy(g["pixel_values"]).cuda()
steps = len(g["greedy_ids"])
cache, feats, logits, nxt = eng.prefill_request(ids, px, torch.ones_like(ids), steps)
st = eng.decode_state(1, cache, nxt, steps)
for t in range(steps):
    if t == 0:
        lg = logits[0].cpu().numpy()
    else:
        st["ids"].fill_(int(g["greedy_ids"][t - 1]))
        lg = eng.decode_step(st, cache, feats, dict(do_sample=False))[0].cpu().numpy()
    top_ids, top_v = g["step_top64_ids"][t], g["step_top64_values"][t]
    e = float(np.abs(lg[top_ids] - top_v).max())
    print(f"step {t:2d} err {e:.4f} margin {float(g['margin'][t]):.4f} checked {g['margin'][t] > 2 * e} "
          f"top1 {int(np.argmax(lg)) == int(g['greedy_ids'][t])}", flush=True)
