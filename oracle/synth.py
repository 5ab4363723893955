"""Name-seeded synthetic PaliGemma weights (numpy side).

TEST INFRASTRUCTURE ONLY — imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg, never by the product path.

There is no checkpoint offline, so both the reference (in this
container, for the golden fixtures) and the HIP build (on the GPU box) are fed
the same synthetic weights.  Each tensor is generated from its *reference*
state-dict key (e.g. ``language_model.model.layers.3.mlp.gate_proj.weight``,
names from modeling_siglip.py:59-62,177-178,199-203,258-267,310,329 and
modeling_gemma.py:205-207,255-259,379-381,437,448,484,487;
modeling_paligemma.py:57,77,80,90) by a counter-based integer hash, so it is
reproducible bit-for-bit on any machine:

    h    = fmix32(i * 0x9E3779B1 + fmix32(crc32(name)))      (uint32 arithmetic)
    v    = ((h >> 8) * 2^-24 * 2 - 1) * a + mean              (fp32, no FMA)
    w[i] = bf16_round_nearest_even(v)                         (held as fp32 here)

with a = std * sqrt(3) (uniform distribution of the recipe's std).  The
product's HIP generator (``pghip.synthetic`` / ``pg_synth_fill``) implements
the same formula; tests/test_synth.py checks that the two agree bit-for-bit and
that their recipes agree for every key.

The default recipe is SURVEY.md §8(c)'s "measured-good" non-degenerate init (default
init makes greedy decode repeat one token): Linear W std 2/sqrt(fan_in),
embeddings/pos/conv std 0.02, Gemma RMSNorm w std 0.1, LayerNorm w 1 + std 0.1,
biases std 0.02, lm_head.bias std 1.
"""
from __future__ import annotations

import math
import zlib

import numpy as np

_GOLDEN = np.uint32(0x9E3779B1)


def fmix32(h: np.ndarray) -> np.ndarray:
    """murmur3 finalizer on a uint32 array (wrapping arithmetic)."""
    h = h ^ (h >> np.uint32(16))
    h = h * np.uint32(0x85EBCA6B)
    h = h ^ (h >> np.uint32(13))
    h = h * np.uint32(0xC2B2AE35)
    h = h ^ (h >> np.uint32(16))
    return h


def seed_of(name: str) -> int:
    s = np.array([zlib.crc32(name.encode("utf-8")) & 0xFFFFFFFF], dtype=np.uint32)
    return int(fmix32(s)[0])


def recipe(name: str, shape, linear_gain: float = 2.0) -> tuple[float, float]:
    """(std, mean) for a reference state-dict key.  Mirrors pghip.synthetic.recipe."""
    if name.endswith(("layer_norm1.weight", "layer_norm2.weight", "post_layernorm.weight")):
        return 0.1, 1.0
    if name.endswith(("input_layernorm.weight", "post_attention_layernorm.weight")) or name.endswith("model.norm.weight"):
        return 0.1, 0.0
    if name.endswith(("patch_embedding.weight", "positional_embeddings.weight", "embed_tokens.weight")):
        return 0.02, 0.0
    if name.endswith("lm_head.bias"):
        return 1.0, 0.0
    if name.endswith(".bias"):
        return 0.02, 0.0
    if len(shape) == 2:
        return linear_gain / math.sqrt(shape[1]), 0.0
    raise KeyError(f"no synthetic recipe for {name} {tuple(shape)}")


def bf16_round(x: np.ndarray) -> np.ndarray:
    """Round fp32 to the nearest bf16 (ties to even); returned as fp32."""
    u = x.astype(np.float32).view(np.uint32)
    u = (u + np.uint32(0x7FFF) + ((u >> np.uint32(16)) & np.uint32(1))) & np.uint32(0xFFFF0000)
    return u.view(np.float32)


def generate(name: str, shape, chunk: int = 1 << 24, linear_gain: float = 2.0) -> np.ndarray:
    """The synthetic tensor for ``name`` (fp32 holding bf16-exact values)."""
    std, mean = recipe(name, shape, linear_gain)
    n = int(np.prod(shape))
    a = np.float32(std * math.sqrt(3.0))
    mean32 = np.float32(mean)
    sm = np.uint32(seed_of(name))
    out = np.empty(n, dtype=np.float32)
    scale = np.float32(2.0 ** -24)
    for s in range(0, n, chunk):
        e = min(n, s + chunk)
        i = np.arange(s, e, dtype=np.uint32)
        h = fmix32(i * _GOLDEN + sm)
        v = (h >> np.uint32(8)).astype(np.float32) * scale
        v = v * np.float32(2.0) - np.float32(1.0)
        v = v * a
        if mean != 0.0:
            v = v + mean32
        out[s:e] = bf16_round(v)
    return out.reshape(shape)


# --------------------------------------------------------------------------- #
# Reference state-dict layout (key -> shape) for a HF-style PaliGemma config.
# --------------------------------------------------------------------------- #
def state_dict_shapes(cfg: dict) -> dict:
    """Key -> shape of every persistent tensor of the reference module tree.

    lm_head.weight is tied to embed_tokens.weight (modeling_gemma.py:492-499) and
    therefore not listed; lm_head.bias is (modeling_gemma.py:484).
    """
    v = cfg["vision_config"]
    t = cfg["text_config"]
    hv, iv, p, c = v["hidden_size"], v["intermediate_size"], v["patch_size"], v.get("num_channels", 3)
    npatch = (v.get("image_size", 224) // p) ** 2
    shapes = {}
    pre = "vision_tower.model."
    shapes[pre + "embeddings.patch_embedding.weight"] = (hv, c, p, p)
    shapes[pre + "embeddings.patch_embedding.bias"] = (hv,)
    shapes[pre + "embeddings.positional_embeddings.weight"] = (npatch, hv)
    for i in range(v["num_hidden_layers"]):
        lp = f"{pre}encoder.layers.{i}."
        shapes[lp + "layer_norm1.weight"] = (hv,)
        shapes[lp + "layer_norm1.bias"] = (hv,)
        for proj in ("key_proj", "value_proj", "query_proj", "out_proj"):
            shapes[lp + f"self_attn.{proj}.weight"] = (hv, hv)
            shapes[lp + f"self_attn.{proj}.bias"] = (hv,)
        shapes[lp + "mlp.fc1.weight"] = (iv, hv)
        shapes[lp + "mlp.fc1.bias"] = (iv,)
        shapes[lp + "mlp.fc2.weight"] = (hv, iv)
        shapes[lp + "mlp.fc2.bias"] = (hv,)
        shapes[lp + "layer_norm2.weight"] = (hv,)
        shapes[lp + "layer_norm2.bias"] = (hv,)
    shapes[pre + "post_layernorm.weight"] = (hv,)
    shapes[pre + "post_layernorm.bias"] = (hv,)
    proj_dim = cfg.get("projection_dim", 2048)
    shapes["multi_modal_projector.linear.weight"] = (proj_dim, hv)
    ht, it = t["hidden_size"], t["intermediate_size"]
    nh, nkv = t["num_attention_heads"], t["num_key_value_heads"]
    hd = t.get("head_dim", 256)
    vocab = t["vocab_size"]
    lm = "language_model."
    shapes[lm + "model.embed_tokens.weight"] = (vocab, ht)
    for i in range(t["num_hidden_layers"]):
        lp = f"{lm}model.layers.{i}."
        shapes[lp + "input_layernorm.weight"] = (ht,)
        shapes[lp + "self_attn.k_proj.weight"] = (nkv * hd, ht)
        shapes[lp + "self_attn.v_proj.weight"] = (nkv * hd, ht)
        shapes[lp + "self_attn.q_proj.weight"] = (nh * hd, ht)
        shapes[lp + "self_attn.o_proj.weight"] = (ht, ht)
        shapes[lp + "post_attention_layernorm.weight"] = (ht,)
        shapes[lp + "mlp.gate_proj.weight"] = (it, ht)
        shapes[lp + "mlp.up_proj.weight"] = (it, ht)
        shapes[lp + "mlp.down_proj.weight"] = (ht, it)
    shapes[lm + "model.norm.weight"] = (ht,)
    shapes[lm + "lm_head.bias"] = (vocab,)
    return shapes


def generate_state_dict(cfg: dict, linear_gain: float = 2.0) -> dict:
    """linear_gain: the 2-D Linear std is linear_gain / sqrt(fan_in).  2.0 (default) is the non-degenerate recipe
    above; 1.6 is the better-conditioned one of tests/golden/pt224wc.npz (bf16 rounding grows ~5x less through the
    45 layers, so the reference's greedy margins clear it and free-running ids can be compared exactly)."""
    return {k: generate(k, s, linear_gain=linear_gain) for k, s in state_dict_shapes(cfg).items()}
