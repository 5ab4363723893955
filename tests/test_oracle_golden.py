"""Pin the numpy oracle against golden vectors produced by the reference itself
(tests/golden/make_golden.py).  CPU only."""
import numpy as np
import pytest

from oracle import configs, synth
from oracle import paligemma_oracle as O


def close(a, b, tol=2e-5):
    """max|a-b| relative to the scale (max|b|) of the reference tensor."""
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    assert a.shape == b.shape, (a.shape, b.shape)
    err = np.abs(a - b).max() / max(np.abs(b).max(), 1e-30)
    assert err < tol, f"scaled max error {err:.3e} >= {tol:.1e}"


def _tiny_oracle(recompute=True, name="tiny"):
    cfg = configs.CONFIGS[name]
    return O.PaliGemmaOracle(cfg, synth.generate_state_dict(cfg), recompute_vision=recompute)


@pytest.mark.parametrize("name,B", [("tiny", 1), ("tiny", 2), ("tiny8", 1), ("tiny8", 16)])
def test_tiny_prefill_matches_reference(golden, name, B):
    """tiny (4 q heads) and tiny8 (8 q heads, the tensor-parallel toy: B = 16 is two images per rank at TP=8)."""
    g = golden(name)
    p = f"b{B}_"
    orc = _tiny_oracle(name=name)
    feats = orc.image_features(g[p + "pixel_values"])
    close(feats, g[p + "proj_out"])
    kv = O.KVCache()
    taps = []
    res = orc.forward(g[p + "input_ids"], g[p + "pixel_values"], np.ones_like(g[p + "input_ids"]), kv, taps=taps)
    close(res["logits"], g[p + "logits"])
    if B > 2:                   # large toy batches keep inputs, logits and projector output only
        return
    v = O.siglip_vision_model(orc.W, orc.vcfg, g[p + "pixel_values"])
    close(v, g[p + "vision_out"])
    for i, h in enumerate(taps):
        close(h, g[p + f"text_layer_{i}"])
    close(kv.k_cache[0], g[p + "k_cache0"])
    close(kv.v_cache[-1], g[p + "v_cache0"])


@pytest.mark.parametrize("name", ["tiny", "tiny8"])
def test_tiny_greedy_loop_matches_reference(golden, name):
    g = golden(name)
    orc = _tiny_oracle(name=name)
    ids, logits = O.generate(orc, g["b1_input_ids"], g["b1_pixel_values"], np.ones_like(g["b1_input_ids"]),
                             max_tokens=len(g["greedy_ids"]), record_logits=True)
    assert ids == g["greedy_ids"].tolist()
    close(np.stack(logits)[:, 0], g["greedy_logits"])


def test_tiny_no_vision_recompute_is_output_invariant(golden):
    g = golden("tiny")
    ids = O.generate(_tiny_oracle(recompute=False), g["b1_input_ids"], g["b1_pixel_values"],
                     np.ones_like(g["b1_input_ids"]), max_tokens=len(g["greedy_ids"]))
    assert ids == g["greedy_ids"].tolist()


@pytest.mark.parametrize("ci", range(4))
def test_top_p_filter_matches_reference(golden, ci):
    g = golden("topp")
    logits = g[f"c{ci}_logits"]
    probs = O.softmax_lastdim(logits / g[f"c{ci}_T"])
    ps, idx = O.top_p_filter(probs, float(g[f"c{ci}_p"]))
    keep = int((ps[0] > 0).sum())
    mine, ref = set(idx[0, :keep].tolist()), set(g[f"c{ci}_kept_ids"].tolist())
    # fp32 cumsum order differs from torch's: a token whose exact mass-before is
    # within 1e-4 of top_p may fall either side of the cut (inference.py:97-99).
    before = np.cumsum(np.sort(probs[0].astype(np.float64))[::-1]) - np.sort(probs[0])[::-1]
    rank = {int(t): r for r, t in enumerate(idx[0])}
    for t in mine ^ ref:
        assert abs(before[rank[t]] - float(g[f"c{ci}_p"])) < 1e-4, t
    n = min(keep, len(ref))
    close(ps[0, :n] * ps[0, :keep].sum() / ps[0, :n].sum(), g[f"c{ci}_kept_probs"][:n], 2e-4)


def test_inverse_cdf_sampler_distribution():
    rng = np.random.default_rng(0)
    logits = rng.standard_normal((1, 64)).astype(np.float32) * 2
    probs = O.softmax_lastdim(logits / np.float32(0.8))
    ps, idx = O.top_p_filter(probs, 0.9)
    target = np.zeros(64)
    target[idx[0]] = ps[0]
    u = rng.random(20000)
    draws = np.array([O.sample_top_p(logits, 0.8, 0.9, u[i:i + 1])[0, 0] for i in range(len(u))])
    freq = np.bincount(draws, minlength=64) / len(u)
    assert np.abs(freq - target).max() < 0.015
    assert set(np.nonzero(freq)[0]) <= set(np.nonzero(target)[0])


@pytest.mark.slow
def test_pt224_prefill_matches_reference(golden):
    """Full-size synthetic PaliGemma-3B-224: prefill logits and the first greedy
    steps of the reference's own loop."""
    g = golden("pt224")
    cfg = configs.PT_224
    orc = O.PaliGemmaOracle(cfg, synth.generate_state_dict(cfg), recompute_vision=False)
    feats = orc.image_features(g["pixel_values"])
    v = O.siglip_vision_model(orc.W, orc.vcfg, g["pixel_values"])
    close(v[0], g["vision_out"], 2e-4)
    close(feats[0, ::16], g["proj_out_rows"], 2e-4)
    ids, logits = O.generate(orc, g["input_ids"], g["pixel_values"], np.ones_like(g["input_ids"]), max_tokens=3,
                             record_logits=True)
    assert ids == g["greedy_ids"][:3].tolist()
    close(logits[0][0], g["prefill_last_logits"], 2e-4)
