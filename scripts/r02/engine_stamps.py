"""Timeline of one pg_decode_mlp_engine launch (the last layer of a decode step) from in-kernel wall-clock stamps:
per CU start, h published, h half gathered, down done, end -- percentiles in us from the first start."""
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
eng.MLP_ENGINE = True
ids, px = bench.synthetic_inputs(cfg, 1, [2, 651, 4906, 603, 476, 2121, 576, 108])
ids, px = ids.cuda(), px.cuda()
cache, feats, logits, nxt = eng.prefill_request(ids, px, torch.ones_like(ids), 40)
st = eng.decode_state(1, cache, nxt, 40)
eng.sample(logits, st, dict(do_sample=False), advance=False)
for _ in range(3):
    eng.decode_step(st, cache, feats, dict(do_sample=False))
for rep in range(3):
    buf = torch.zeros(256 * 8, dtype=torch.int64, device="cuda")
    _lib.call("pg_decode_mlp_engine_stamps", buf.data_ptr())
    torch.cuda.synchronize()
    eng.decode_step(st, cache, feats, dict(do_sample=False))
    torch.cuda.synchronize()
    _lib.call("pg_decode_mlp_engine_stamps", None)
    s = buf.view(256, 8).cpu().tolist()
    t0 = min(r[0] for r in s)
    pct = lambda c: [round((c[int(q * (len(c) - 1))] - t0) / 100.0, 2) for q in (0, 0.1, 0.5, 0.9, 1.0)]  # noqa
    print(json.dumps({k: pct(sorted(r[i] for r in s)) for i, k in
                      enumerate(("start", "h_pub", "gathered", "down_done", "end"))}))
eng.check()
