"""Full-size check of pg_attn_oproj (attention inside the o_proj launch) against the two-launch form:
one decode step from identical state, logits and residual compared; sync words printed.
Set AO_LAYERS to run only that many decoder layers."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "paligemma-multimodal-system_amd")]
import torch  # noqa: E402
from pghip import configs, engine, synthetic, weights  # noqa: E402
import bench  # noqa: E402

cfg = configs.CONFIGS[os.environ.get("AO_CFG", "pt-224")]
eng = engine.PaliGemmaEngine(cfg, weights.PackedWeights(cfg, synthetic.SyntheticStateDict(cfg).__getitem__))
ids, px = bench.synthetic_inputs(cfg, 1, [2, 651, 4906, 603, 476, 2121, 576, 108])
ids, px = ids.cuda(), px.cuda()
cache, feats, logits, nxt = eng.prefill_request(ids, px, torch.ones_like(ids), 16)
st0 = eng.decode_state(1, cache, nxt, 16)
eng.sample(logits, st0, dict(do_sample=False), advance=False)
k0, v0 = cache.k.clone(), cache.vt.clone()
res = {}
for fused in (False, True):
    eng.FUSE_ATTN_O = fused
    cache.k.copy_(k0)
    cache.vt.copy_(v0)
    st = {k: v.clone() for k, v in st0.items()}
    lg = eng.decode_step(st, cache, feats, dict(do_sample=False)).clone()
    torch.cuda.synchronize()
    res[fused] = (lg, eng._ws["d_res_a"].clone(), int(st["ids"][0]))
    if fused:
        print("sync", eng._ws["d_attn_sync"].tolist())
a, b = res[False], res[True]
print("ids", a[2], b[2])
print("logits max|d|", (a[0] - b[0]).abs().max().item(), "scale", a[0].abs().max().item())
print("resid max|d|", (a[1] - b[1]).abs().max().item(), "scale", a[1].abs().max().item())
