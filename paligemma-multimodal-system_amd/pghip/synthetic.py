"""Synthetic PaliGemma weights generated on the GPU (bench / smoke / tests).

No checkpoint exists offline; the bench runs on name-seeded synthetic weights
of the real architecture.  The formula and the per-key recipe are the ones of
oracle/synth.py (kept separately so the product never imports test code);
tests/test_host.py checks the recipes agree and the GPU tests check the
generated tensors are bit-identical to the numpy ones.
"""
from __future__ import annotations

import math
import zlib

import torch

from . import ops


def _fmix32(h: int) -> int:
    h &= 0xFFFFFFFF
    h ^= h >> 16
    h = (h * 0x85EBCA6B) & 0xFFFFFFFF
    h ^= h >> 13
    h = (h * 0xC2B2AE35) & 0xFFFFFFFF
    h ^= h >> 16
    return h


def seed_of(name: str) -> int:
    return _fmix32(zlib.crc32(name.encode("utf-8")) & 0xFFFFFFFF)


def recipe(name: str, shape, linear_gain: float = 2.0) -> tuple:
    """(std, mean) per reference state-dict key (SURVEY.md §8(c) non-degenerate init)."""
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


def state_dict_shapes(cfg: dict) -> dict:
    """Reference key -> shape (modeling_siglip.py / modeling_gemma.py / modeling_paligemma.py module tree)."""
    v, t = cfg["vision_config"], cfg["text_config"]
    hv, iv, p, c = v["hidden_size"], v["intermediate_size"], v["patch_size"], v.get("num_channels", 3)
    npatch = (v.get("image_size", 224) // p) ** 2
    s = {}
    pre = "vision_tower.model."
    s[pre + "embeddings.patch_embedding.weight"] = (hv, c, p, p)
    s[pre + "embeddings.patch_embedding.bias"] = (hv,)
    s[pre + "embeddings.positional_embeddings.weight"] = (npatch, hv)
    for i in range(v["num_hidden_layers"]):
        lp = f"{pre}encoder.layers.{i}."
        s[lp + "layer_norm1.weight"] = (hv,)
        s[lp + "layer_norm1.bias"] = (hv,)
        for proj in ("key_proj", "value_proj", "query_proj", "out_proj"):
            s[lp + f"self_attn.{proj}.weight"] = (hv, hv)
            s[lp + f"self_attn.{proj}.bias"] = (hv,)
        s[lp + "mlp.fc1.weight"] = (iv, hv)
        s[lp + "mlp.fc1.bias"] = (iv,)
        s[lp + "mlp.fc2.weight"] = (hv, iv)
        s[lp + "mlp.fc2.bias"] = (hv,)
        s[lp + "layer_norm2.weight"] = (hv,)
        s[lp + "layer_norm2.bias"] = (hv,)
    s[pre + "post_layernorm.weight"] = (hv,)
    s[pre + "post_layernorm.bias"] = (hv,)
    s["multi_modal_projector.linear.weight"] = (cfg.get("projection_dim", 2048), hv)
    ht, it = t["hidden_size"], t["intermediate_size"]
    nh, nkv, hd = t["num_attention_heads"], t["num_key_value_heads"], t.get("head_dim", 256)
    lm = "language_model."
    s[lm + "model.embed_tokens.weight"] = (t["vocab_size"], ht)
    for i in range(t["num_hidden_layers"]):
        lp = f"{lm}model.layers.{i}."
        s[lp + "input_layernorm.weight"] = (ht,)
        s[lp + "self_attn.k_proj.weight"] = (nkv * hd, ht)
        s[lp + "self_attn.v_proj.weight"] = (nkv * hd, ht)
        s[lp + "self_attn.q_proj.weight"] = (nh * hd, ht)
        s[lp + "self_attn.o_proj.weight"] = (ht, ht)
        s[lp + "post_attention_layernorm.weight"] = (ht,)
        s[lp + "mlp.gate_proj.weight"] = (it, ht)
        s[lp + "mlp.up_proj.weight"] = (it, ht)
        s[lp + "mlp.down_proj.weight"] = (ht, it)
    s[lm + "model.norm.weight"] = (ht,)
    s[lm + "lm_head.bias"] = (t["vocab_size"],)
    return s


def generate(name: str, shape, device="cuda", dtype=torch.bfloat16, linear_gain: float = 2.0) -> torch.Tensor:
    std, mean = recipe(name, shape, linear_gain)
    out = torch.empty(shape, dtype=dtype, device=device)
    ops.synth_fill(out, seed_of(name), float(std * math.sqrt(3.0)), float(mean))
    return out


class SyntheticStateDict:
    """Lazy mapping key -> device tensor (bf16 for matrices, fp32 for vectors)."""

    def __init__(self, cfg: dict, device="cuda", linear_gain: float = 2.0):
        """linear_gain: 2-D Linear std = linear_gain / sqrt(fan_in) (oracle/synth.py generate_state_dict)."""
        self.shapes = state_dict_shapes(cfg)
        self.device = device
        self.linear_gain = linear_gain

    def keys(self):
        return self.shapes.keys()

    def __contains__(self, k):
        return k in self.shapes

    def __getitem__(self, k):
        shape = self.shapes[k]
        dt = torch.bfloat16 if len(shape) >= 2 else torch.float32
        return generate(k, shape, self.device, dt, self.linear_gain)
