"""Diagnostic: full-size pt-224 HIP path vs the fp32 oracle and the bf16-operand-emulating oracle.
Prints scaled max errors per stage (vision out, projector, prefill last logits)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "paligemma-multimodal-system_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from oracle import paligemma_oracle as O  # noqa: E402
from pghip import configs, engine, synthetic, weights  # noqa: E402


def err(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-30))


cfg = configs.CONFIGS[sys.argv[1] if len(sys.argv) > 1 else "pt-224"]
g = dict(np.load(os.path.join(ROOT, "tests/golden/pt224.npz")))
sd = synthetic.SyntheticStateDict(cfg)
eng = engine.PaliGemmaEngine(cfg, weights.PackedWeights(cfg, sd.__getitem__))
W = {k: sd[k].float().cpu().numpy() for k in sd.keys()}
px = g["pixel_values"]
ids = g["input_ids"]
feats, hid = eng.vision(torch.from_numpy(px).cuda(), want_hidden=True)
cache, _, logits, _ = eng.prefill_request(torch.from_numpy(ids).cuda(), torch.from_numpy(px).cuda(),
                                          torch.ones(ids.shape, dtype=torch.int64).cuda(), 4, feats=feats)
hid, feats, logits = hid.cpu().numpy(), feats.cpu().numpy(), logits[0].cpu().numpy()
print("vs reference golden (fp32): vision", err(hid, g["vision_out"]), "logits", err(logits, g["prefill_last_logits"]))
for mode in ("fp32", "bf16-emul"):
    ctx = O.bf16_operands() if mode != "fp32" else open(os.devnull)
    with ctx:
        v = O.siglip_vision_model(W, cfg["vision_config"], px)[0]
        f = O.multi_modal_projector(W, v[None])[0]
        orc = O.PaliGemmaOracle(cfg, W, recompute_vision=False)
        lg = orc.forward(ids, px, np.ones_like(ids), O.KVCache(), logits_rows=slice(-1, None))["logits"][0, -1]
    top = np.argsort(-lg)[:5]
    print(f"vs oracle {mode}: vision {err(hid, v):.3e} proj {err(feats, f):.3e} logits {err(logits, lg):.3e} "
          f"top5 oracle {top.tolist()} hip {np.argsort(-logits)[:5].tolist()}")

# ---- per-layer check: oracle layer applied to the HIP layer input (no error accumulation)
vt = []
eng.vision(torch.from_numpy(px).cuda(), taps=vt)
vt = [t.cpu().numpy().reshape(1, -1, t.shape[-1]) for t in vt]
vc = cfg["vision_config"]
worst = 0.0
for i in range(vc["num_hidden_layers"]):
    lp = f"vision_tower.model.encoder.layers.{i}."
    x = vt[i]
    eps = 1e-6
    r = x
    y = O.layer_norm(x, W[lp + "layer_norm1.weight"], W[lp + "layer_norm1.bias"], eps)
    y = r + O.siglip_attention(W, lp + "self_attn.", vc, y)
    r = y
    y2 = O.layer_norm(y, W[lp + "layer_norm2.weight"], W[lp + "layer_norm2.bias"], eps)
    y = r + O.siglip_mlp(W, lp + "mlp.", y2)
    e = err(vt[i + 1] - x, y - x)
    worst = max(worst, e)
print(f"vision per-layer delta error (worst of {vc['num_hidden_layers']}): {worst:.3e}")
tt = []
resid = torch.empty(ids.size, eng.w.hidden, device="cuda")
eng.embed_merge(torch.from_numpy(ids).cuda(), feats_t if False else eng.vision(torch.from_numpy(px).cuda()), resid)
c2 = eng.new_cache(1, ids.shape[1] + 4)
eng.gemma_prefill(resid, torch.arange(1, ids.shape[1] + 1, dtype=torch.int32)[None], c2, 1, ids.shape[1], taps=tt,
                  want_logits=False)
tt = [t.cpu().numpy().reshape(1, -1, t.shape[-1]) for t in tt]
tc = cfg["text_config"]
pos = np.arange(1, ids.shape[1] + 1)[None]
mask = np.zeros((1, 1, ids.shape[1], ids.shape[1]), np.float32)
worst = 0.0
for i in range(tc["num_hidden_layers"]):
    lp = f"language_model.model.layers.{i}."
    x = tt[i]
    r = x
    y = O.rms_norm(x, W[lp + "input_layernorm.weight"])
    y = r + O.gemma_attention(W, lp + "self_attn.", tc, i, y, pos, mask, None)
    r = y
    y = r + O.gemma_mlp(W, lp + "mlp.", O.rms_norm(y, W[lp + "post_attention_layernorm.weight"]))
    e = err(tt[i + 1] - x, y - x)
    worst = max(worst, e)
print(f"gemma per-layer delta error (worst of {tc['num_hidden_layers']}): {worst:.3e}")
# intrinsic bf16 sensitivity of this synthetic model: fp32 oracle vs bf16-operand oracle
with O.bf16_operands():
    lg16 = O.PaliGemmaOracle(cfg, W, recompute_vision=False).forward(ids, px, np.ones_like(ids), O.KVCache(),
                                                                     logits_rows=slice(-1, None))["logits"][0, -1]
lg32 = O.PaliGemmaOracle(cfg, W, recompute_vision=False).forward(ids, px, np.ones_like(ids), O.KVCache(),
                                                                 logits_rows=slice(-1, None))["logits"][0, -1]
print(f"intrinsic: oracle bf16-operands vs oracle fp32 logits err {err(lg16, lg32):.3e}")
