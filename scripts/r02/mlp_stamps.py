"""Timeline of one pg_decode_mlp_block launch (the last layer of a decode step) from in-kernel wall-clock stamps:
per workgroup start, h published, h slice ready (poll done), end -- percentiles in us from the first start."""
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
eng.MLP_BLOCK = True
ids, px = bench.synthetic_inputs(cfg, 1, [2, 651, 4906, 603, 476, 2121, 576, 108])
ids, px = ids.cuda(), px.cuda()
cache, feats, logits, nxt = eng.prefill_request(ids, px, torch.ones_like(ids), 40)
st = eng.decode_state(1, cache, nxt, 40)
eng.sample(logits, st, dict(do_sample=False), advance=False)
for _ in range(3):
    eng.decode_step(st, cache, feats, dict(do_sample=False))
G = 1024
out = []
for rep in range(3):
    buf = torch.zeros(G * 4, dtype=torch.int64, device="cuda")
    _lib.call("pg_decode_mlp_stamps", buf.data_ptr())
    torch.cuda.synchronize()
    eng.decode_step(st, cache, feats, dict(do_sample=False))
    torch.cuda.synchronize()
    _lib.call("pg_decode_mlp_stamps", None)
    s = buf.view(G, 4).cpu().tolist()
    t0 = min(r[0] for r in s)
    pct = lambda c: [round((c[int(q * (len(c) - 1))] - t0) / 100.0, 2) for q in (0, 0.1, 0.5, 0.9, 1.0)]  # noqa
    res = {k: pct(sorted(r[i] for r in s)) for i, k in enumerate(("start", "h_pub", "slice_ready", "end"))}
    # per slice: last producer's publish vs the consumers' poll end
    sl = {}
    for z in range(8):
        last_pub = max(s[p][1] for p in range(128 * z, 128 * z + 128))
        polls = sorted(s[p][2] for p in range(G) if p // 128 == z)
        sl[z] = [round((last_pub - t0) / 100.0, 2), round((polls[0] - t0) / 100.0, 2), round((polls[-1] - t0) / 100.0, 2)]
    res["slices(last_pub,first_ready,last_ready)"] = sl
    out.append(res)
    print(json.dumps(res))
eng.check()
