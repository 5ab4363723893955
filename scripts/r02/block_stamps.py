"""Timeline of one pg_decode_attn_block launch (the last layer of a decode step) from in-kernel wall-clock stamps:
per role, when its workgroups started, finished waiting and ended (us from the launch's first start)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "paligemma-multimodal-system_amd")]
import torch  # noqa: E402
from pghip import _lib, configs, engine, synthetic, weights  # noqa: E402
import bench  # noqa: E402

cfg = configs.CONFIGS["pt-224"]
eng = engine.PaliGemmaEngine(cfg, weights.PackedWeights(cfg, synthetic.SyntheticStateDict(cfg).__getitem__))
ids, px = bench.synthetic_inputs(cfg, 1, [2, 651, 4906, 603, 476, 2121, 576, 108])
ids, px = ids.cuda(), px.cuda()
cache, feats, logits, nxt = eng.prefill_request(ids, px, torch.ones_like(ids), 40)
st = eng.decode_state(1, cache, nxt, 40)
eng.sample(logits, st, dict(do_sample=False), advance=False)
for _ in range(3):
    eng.decode_step(st, cache, feats, dict(do_sample=False))
buf = torch.zeros(256 * 4, dtype=torch.int64, device="cuda")
_lib.call("pg_decode_block_stamps", buf.data_ptr())
torch.cuda.synchronize()
eng.decode_step(st, cache, feats, dict(do_sample=False))
torch.cuda.synchronize()
_lib.call("pg_decode_block_stamps", None)
s = buf.view(256, 4).cpu().tolist()
nq, na = eng.w.qkv_n // 32, (16 + 3) // 4
rows = [r for r in s if r[0] > 0]
t0 = min(r[0] for r in rows)
us = lambda v: round((v - t0) / 100.0, 2) if v > 0 else None  # noqa: E731
roles = {"qkv": s[:nq], "attn": s[nq:nq + na], "o": s[nq + na:nq + na + 128]}
out = {}
for name, rs in roles.items():
    rs = [r for r in rs if r[0] > 0]
    col = lambda k: sorted(us(r[k]) for r in rs if r[k] > 0)  # noqa: E731
    out[name] = {k: (lambda c: [c[0], c[len(c) // 2], c[-1]] if c else None)(col(i))
                 for i, k in ((0, "start"), (1, "wait_end"), (2, "end"))}
print(json.dumps(out))
