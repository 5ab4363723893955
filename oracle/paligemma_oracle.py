"""CPU restatement (numpy, fp32) of the reference PaliGemma image->text path.

TEST INFRASTRUCTURE ONLY.  Imported by tests/, __graft_entry__.smoke() and the
``cpu_baseline`` leg of bench.py — as the checker and as the reported CPU
baseline, never as part of the product path.

Every function restates one reference symbol and cites it (file:line under the
reference repo).  The arithmetic follows the reference exactly (fp32
throughout, as the reference only runs in fp32 — SURVEY.md §7 hard part (i)),
including its quirks:

* prefill attention is fully bidirectional over the whole prefix (the additive
  mask is all zeros, modeling_paligemma.py:154-156) and position ids are
  1-based (modeling_paligemma.py:195);
* decode positions are ``cumsum(attention_mask)[:, -1]`` (modeling_paligemma.py:189);
* the vision tower is re-run on every call (modeling_paligemma.py:281) unless
  ``recompute_vision=False`` is asked for (output-invariant);
* RMSNorm computes (and returns) fp32 with weight as ``(1 + w)``
  (modeling_gemma.py:172-181);
* the tied lm_head carries its own bias (modeling_gemma.py:484,498,523).

Parity pinning: tests/test_oracle_golden.py checks this module against golden
vectors produced by the reference itself (tests/golden/make_golden.py).
"""
from __future__ import annotations

import math
from typing import Optional

import numpy as np

F32 = np.float32

# bf16-operand emulation (test aid): when on, every GEMM/attention operand is rounded to
# bf16 where the HIP path feeds bf16 to the MFMAs (activations into linears, q/k/v, RoPE'd
# q/k, softmax P).  It separates "bf16 precision" from "kernel bug" in the GPU tests.
_BF16_OPERANDS = False


class bf16_operands:
    def __enter__(self):
        global _BF16_OPERANDS
        self._old, _BF16_OPERANDS = _BF16_OPERANDS, True

    def __exit__(self, *a):
        global _BF16_OPERANDS
        _BF16_OPERANDS = self._old


# fp8-operand emulation (test aid, BASELINE configs[4]): when on, the Gemma decoder linears (q/k/v/o, gate/up/down)
# multiply e4m3 operands -- activation rows and weight output rows each scaled by max|row| / 448
# (weights.quant_rows_fp8 / pg_quant_fp8's rule) -- whenever a call has more than `min_rows` rows (the HIP path runs
# fp8 for linears of more than 16 rows: prefill, and decode at batch > 16).  The fp8 path's intrinsic sensitivity on a
# model then bounds the HIP fp8 path's distance to the fp32 reference.  The tied lm_head: the HIP path runs it in e4m3
# for 17..32-row batches (engine._lm_gemm, the fp8 GEMV) and in bf16 otherwise; lm_head=True emulates the e4m3 form
# (tests/golden/make_emu.py sets it for the batch-32 fixtures).
# mx_h=True: a down_proj call of at most 32 rows (batched decode) takes MX rows instead -- h rounded to bf16, then
# e4m3 with one power-of-two scale per 32 contiguous columns (engine.MX_H: the gate/up epilogue's mx_out rule,
# csrc/common.h mx_exp), the weights per-channel as before.  mx_norm=True: the RMSNorm-fed linears of at most 32
# rows (q|k|v, gate/up, the lm_head) take MX rows of the normalised input too (engine.MX_NORM: pg_norm_residual_mx
# quantises x*(1+w) per 32-column block and the GEMV applies rstd to its outputs -- the same block-relative e4m3
# rounding; emulated on the normalised row, so per-element bits differ where rstd is not a power of two).
# tp=W (> 1): the tensor-parallel form of the HIP path (engine.tp): the row-parallel o_proj and
# down_proj run on W equal K slices -- each rank quantises its slice of the activation row and its slice of every
# weight row with their own max/448 scales (weights.PackedWeights(tp_world=W) / pg_quant_fp8 on the local slice; MX
# blocks of 32 do not cross a slice) -- and the W partial products are summed in rank order (the xGMI exchange's
# order).  The column-parallel q|k|v, gate/up and the vocabulary-parallel lm_head quantise whole rows exactly as at
# W = 1, so they need nothing.
_FP8_MIN_ROWS = None
_FP8_LM_HEAD = False
_FP8_MX_H = False
_FP8_MX_NORM = False
_FP8_TP = 1
# mx_h_prefill=True (round 6, engine.MX_PREFILL): a down_proj call of MORE than 32 rows (the prefill) takes MX rows of
# h as well -- the fp8 gate/up tile's epilogue writes e4m3 h with one E8M0 scale per 32 columns
_FP8_MX_HP = False


class fp8_operands:
    def __init__(self, min_rows: int = 16, lm_head: bool = False, mx_h: bool = False, mx_norm: bool = False,
                 tp: int = 1, mx_h_prefill: bool = False):
        self.cfg = (min_rows, lm_head, mx_h, mx_norm, tp, mx_h_prefill)

    def __enter__(self):
        global _FP8_MIN_ROWS, _FP8_LM_HEAD, _FP8_MX_H, _FP8_MX_NORM, _FP8_TP, _FP8_MX_HP
        self._old = (_FP8_MIN_ROWS, _FP8_LM_HEAD, _FP8_MX_H, _FP8_MX_NORM, _FP8_TP, _FP8_MX_HP)
        _FP8_MIN_ROWS, _FP8_LM_HEAD, _FP8_MX_H, _FP8_MX_NORM, _FP8_TP, _FP8_MX_HP = self.cfg

    def __exit__(self, *a):
        global _FP8_MIN_ROWS, _FP8_LM_HEAD, _FP8_MX_H, _FP8_MX_NORM, _FP8_TP, _FP8_MX_HP
        _FP8_MIN_ROWS, _FP8_LM_HEAD, _FP8_MX_H, _FP8_MX_NORM, _FP8_TP, _FP8_MX_HP = self._old


def mx_exp(amax: np.ndarray) -> np.ndarray:
    """E8M0 exponent per block: the smallest e with amax <= 448 * 2^e (0 for a zero block), clamped to [-127, 127]
    (test aid mirroring csrc/common.h mx_exp: amax = f * 2^k, f in [0.5, 1) -> k - 9, or k - 8 when f * 512 > 448)."""
    f, k = np.frexp(amax.astype(F32))
    e = k - 9 + (f * F32(512.0) > F32(448.0)).astype(k.dtype)
    return np.where(amax > 0, np.clip(e, -127, 127), 0).astype(np.int32)


def mx_rows(x: np.ndarray) -> np.ndarray:
    """MX round trip (block 32 along the last axis): x ~= e4m3(x / 2^e) * 2^e, e = mx_exp(block max |x|)."""
    import torch
    x2 = np.ascontiguousarray(x, dtype=F32).reshape(-1, x.shape[-1] // 32, 32)
    sc = np.ldexp(F32(1.0), mx_exp(np.abs(x2).max(axis=2, keepdims=True))).astype(F32)
    q = torch.from_numpy(x2 / sc).to(torch.float8_e4m3fn).float().numpy()
    return (q * sc).reshape(x.shape).astype(F32)


def q8_rows(x: np.ndarray) -> np.ndarray:
    """Per-row e4m3 round trip: x ~= e4m3(x / s) * s, s = max|row| / 448 (1 for a zero row)."""
    import torch
    x2 = np.ascontiguousarray(x, dtype=F32).reshape(-1, x.shape[-1])
    amax = np.abs(x2).max(axis=1, keepdims=True)
    s = np.where(amax > 0, amax / F32(448.0), F32(1.0)).astype(F32)
    q = torch.from_numpy(np.clip(x2 / s, -448.0, 448.0)).to(torch.float8_e4m3fn).float().numpy()
    return (q * s).reshape(x.shape).astype(F32)


def q16(x: np.ndarray) -> np.ndarray:
    if not _BF16_OPERANDS:
        return x
    u = np.ascontiguousarray(x, dtype=F32).view(np.uint32)
    u = (u + np.uint32(0x7FFF) + ((u >> np.uint32(16)) & np.uint32(1))) & np.uint32(0xFFFF0000)
    return u.view(F32)


# --------------------------------------------------------------------------- #
# elementwise helpers
# --------------------------------------------------------------------------- #
def gelu_tanh(x: np.ndarray) -> np.ndarray:
    """nn.functional.gelu(x, approximate="tanh") (modeling_siglip.py:184, modeling_gemma.py:214)."""
    x = x.astype(F32, copy=False)
    k = F32(math.sqrt(2.0 / math.pi))
    return F32(0.5) * x * (F32(1.0) + np.tanh(k * (x + F32(0.044715) * x * x * x)))


def softmax_lastdim(x: np.ndarray) -> np.ndarray:
    """torch.softmax(..., dim=-1, dtype=float32) (modeling_siglip.py:122, modeling_gemma.py:329)."""
    m = x.max(axis=-1, keepdims=True)
    e = np.exp(x - m)
    return e / e.sum(axis=-1, keepdims=True)


def layer_norm(x: np.ndarray, w: np.ndarray, b: np.ndarray, eps: float) -> np.ndarray:
    """nn.LayerNorm(eps) (modeling_siglip.py:199,203,310)."""
    mean = x.mean(axis=-1, keepdims=True, dtype=np.float64)
    var = ((x - mean) ** 2).mean(axis=-1, keepdims=True)
    y = (x - mean) / np.sqrt(var + eps)
    return (y * w + b).astype(F32)


def linear(x: np.ndarray, w: np.ndarray, b: Optional[np.ndarray] = None, gemma: bool = False,
           mx: str = "", rowpar: bool = False) -> np.ndarray:
    """nn.Linear: x @ w.T + b.  (gemma: a Gemma decoder linear, for the fp8-operand emulation; mx: "h" for the
    down_proj, "x" for the RMSNorm-fed linears, whose <= 32-row calls take MX rows under fp8_operands(mx_h=True) /
    (mx_norm=True); rowpar: a row-parallel linear (o_proj, down_proj), sliced along K under fp8_operands(tp=W).)"""
    rows = x.size // x.shape[-1]
    fp8 = gemma and _FP8_MIN_ROWS is not None and rows > _FP8_MIN_ROWS

    def part(xs, ws):
        if not fp8:
            return q16(xs) @ ws.T
        if mx == "h" and ((_FP8_MX_H and rows <= 32) or (_FP8_MX_HP and rows > 32)):
            xq = mx_rows(q16(xs))
        elif mx == "x" and _FP8_MX_NORM and rows <= 32:
            xq = mx_rows(xs)
        else:
            xq = q8_rows(xs)
        return xq @ q8_rows(ws).T

    if rowpar and gemma and _FP8_MIN_ROWS is not None and _FP8_TP > 1:
        K = x.shape[-1]
        assert K % _FP8_TP == 0, (K, _FP8_TP)
        ks = K // _FP8_TP
        y = None
        for r in range(_FP8_TP):                     # each rank's partial, summed in rank order
            p = part(x[..., r * ks:(r + 1) * ks], w[:, r * ks:(r + 1) * ks]).astype(F32)
            y = p if y is None else (y + p).astype(F32)
    else:
        y = part(x, w)
    if b is not None:
        y = y + b
    return y.astype(F32, copy=False)


# --------------------------------------------------------------------------- #
# SigLIP vision tower (modeling_siglip.py)
# --------------------------------------------------------------------------- #
def siglip_embeddings(W: dict, vcfg: dict, pixel_values: np.ndarray) -> np.ndarray:
    """SiglipVisionEmbeddings.forward (modeling_siglip.py:280-299).

    Conv2d(k=s=patch, valid) == per-patch matmul over (c, kh, kw); flatten(2)
    orders patches h*nw + w; then + positional_embeddings(arange(N)).
    """
    pre = "vision_tower.model.embeddings."
    p = vcfg["patch_size"]
    B, C, H, Wd = pixel_values.shape
    nh, nw = H // p, Wd // p
    x = pixel_values[:, :, : nh * p, : nw * p].reshape(B, C, nh, p, nw, p)
    x = x.transpose(0, 2, 4, 1, 3, 5).reshape(B, nh * nw, C * p * p)
    wconv = W[pre + "patch_embedding.weight"].reshape(W[pre + "patch_embedding.weight"].shape[0], -1)
    emb = linear(x, wconv, W[pre + "patch_embedding.bias"])
    return (emb + W[pre + "positional_embeddings.weight"][None, : nh * nw]).astype(F32)


def siglip_attention(W: dict, lp: str, vcfg: dict, x: np.ndarray, weights_out: Optional[list] = None) -> np.ndarray:
    """SiglipAttention.forward (modeling_siglip.py:65-157); weights_out receives the attention weights it returns
    (:157: the scaled scores from before the softmax)."""
    B, N, E = x.shape
    nh = vcfg["num_attention_heads"]
    hd = E // nh
    scale = F32(1.0 / (hd ** 0.5))                                   # :55
    k = linear(x, W[lp + "key_proj.weight"], W[lp + "key_proj.bias"])      # :71
    q = linear(x, W[lp + "query_proj.weight"], W[lp + "query_proj.bias"])  # :73
    v = linear(x, W[lp + "value_proj.weight"], W[lp + "value_proj.bias"])  # :75
    k = q16(k).reshape(B, N, nh, hd).transpose(0, 2, 1, 3)            # :79-89
    q = q16(q).reshape(B, N, nh, hd).transpose(0, 2, 1, 3)
    v = q16(v).reshape(B, N, nh, hd).transpose(0, 2, 1, 3)
    s = (q @ k.transpose(0, 1, 3, 2)) * scale                          # :96-100
    if weights_out is not None:
        weights_out.append(s)                                           # :157 returns the pre-softmax scores
    p = softmax_lastdim(s)                                              # :122
    o = q16(p) @ v                                                      # :136
    o = o.transpose(0, 2, 1, 3).reshape(B, N, E)                        # :148-153
    return linear(o, W[lp + "out_proj.weight"], W[lp + "out_proj.bias"])   # :156


def siglip_mlp(W: dict, lp: str, x: np.ndarray) -> np.ndarray:
    """SiglipMLP.forward (modeling_siglip.py:181-186)."""
    h = gelu_tanh(linear(x, W[lp + "fc1.weight"], W[lp + "fc1.bias"]))
    return linear(h, W[lp + "fc2.weight"], W[lp + "fc2.bias"])


def siglip_vision_model(W: dict, vcfg: dict, pixel_values: np.ndarray) -> np.ndarray:
    """SiglipVisionModel.forward -> SiglipTransformer.forward (modeling_siglip.py:312-334)."""
    eps = vcfg.get("layer_norm_eps", 1e-6)
    x = siglip_embeddings(W, vcfg, pixel_values.astype(F32))
    for i in range(vcfg["num_hidden_layers"]):                          # SiglipEncoder :234-239
        lp = f"vision_tower.model.encoder.layers.{i}."
        r = x                                                           # SiglipEncoderLayer :206-221
        x = layer_norm(x, W[lp + "layer_norm1.weight"], W[lp + "layer_norm1.bias"], eps)
        x = r + siglip_attention(W, lp + "self_attn.", vcfg, x)
        r = x
        x = layer_norm(x, W[lp + "layer_norm2.weight"], W[lp + "layer_norm2.bias"], eps)
        x = r + siglip_mlp(W, lp + "mlp.", x)
    pre = "vision_tower.model.post_layernorm."
    return layer_norm(x, W[pre + "weight"], W[pre + "bias"], eps)      # :319


def multi_modal_projector(W: dict, x: np.ndarray) -> np.ndarray:
    """PaliGemmaMultiModalProjector.forward: Linear, no bias (modeling_paligemma.py:57,60-65)."""
    return linear(x, W["multi_modal_projector.linear.weight"])


# --------------------------------------------------------------------------- #
# Gemma decoder (modeling_gemma.py)
# --------------------------------------------------------------------------- #
class KVCache:
    """KVCache (modeling_gemma.py:8-64): per-layer list, concat on dim -2."""

    def __init__(self):
        self.k_cache: list = []
        self.v_cache: list = []

    def update(self, k: np.ndarray, v: np.ndarray, layer_idx: int):
        if layer_idx >= len(self.k_cache):                              # :33-40
            self.k_cache.append(k)
            self.v_cache.append(v)
        else:                                                           # :54-55
            self.k_cache[layer_idx] = np.concatenate([self.k_cache[layer_idx], k], axis=-2)
            self.v_cache[layer_idx] = np.concatenate([self.v_cache[layer_idx], v], axis=-2)
        return self.k_cache[layer_idx], self.v_cache[layer_idx]

    def num_items(self) -> int:                                          # :59-64
        return 0 if not self.k_cache else self.k_cache[0].shape[-2]


def rope_inv_freq(dim: int, base: float = 10000.0) -> np.ndarray:
    """GemmaRotaryEmbedding.__init__ (modeling_gemma.py:112)."""
    return (F32(1.0) / (F32(base) ** (np.arange(0, dim, 2, dtype=np.int64).astype(F32) / F32(dim)))).astype(F32)


def rope_cos_sin(dim: int, position_ids: np.ndarray, base: float = 10000.0):
    """GemmaRotaryEmbedding.forward (modeling_gemma.py:116-135): fp32 freqs, emb = cat(f, f)."""
    inv = rope_inv_freq(dim, base)
    pos = np.asarray(position_ids, dtype=F32)                           # (B, L)
    freqs = inv[None, None, :] * pos[:, :, None]                        # :129 (K=1 matmul)
    emb = np.concatenate([freqs, freqs], axis=-1)                       # :131
    return np.cos(emb).astype(F32), np.sin(emb).astype(F32)


def rotate_half(x: np.ndarray) -> np.ndarray:
    """rotate_half (modeling_gemma.py:138-142): cat(-x2, x1)."""
    h = x.shape[-1] // 2
    return np.concatenate([-x[..., h:], x[..., :h]], axis=-1)


def apply_rotary_pos_emb(q, k, cos, sin):
    """apply_rotary_pos_emb (modeling_gemma.py:145-151), head dim unsqueezed at 1."""
    cos = cos[:, None]
    sin = sin[:, None]
    return q * cos + rotate_half(q) * sin, k * cos + rotate_half(k) * sin


def rms_norm(x: np.ndarray, w: np.ndarray, eps: float = 1e-6) -> np.ndarray:
    """GemmaRMSNorm.forward (modeling_gemma.py:165-182); returns fp32."""
    x = x.astype(F32)
    t = np.reciprocal(np.sqrt((x * x).mean(axis=-1, keepdims=True) + F32(eps)))
    return (x * t * (F32(1.0) + w.astype(F32))).astype(F32)


def gemma_attention(W: dict, lp: str, tcfg: dict, layer_idx: int, x: np.ndarray,
                    position_ids: np.ndarray, mask: np.ndarray, kv_cache: Optional[KVCache],
                    weights_out: Optional[list] = None):
    """GemmaAttention.forward (modeling_gemma.py:264-358); weights_out receives the attention weights it returns
    (:358)."""
    B, L, _ = x.shape
    nh, nkv = tcfg["num_attention_heads"], tcfg["num_key_value_heads"]
    hd = tcfg.get("head_dim", 256)
    k = linear(x, W[lp + "k_proj.weight"], gemma=True, mx="x")                      # :274
    v = linear(x, W[lp + "v_proj.weight"], gemma=True, mx="x")                      # :276
    q = linear(x, W[lp + "q_proj.weight"], gemma=True, mx="x")                      # :278
    k = q16(k).reshape(B, L, nkv, hd).transpose(0, 2, 1, 3)             # :285-287
    v = q16(v).reshape(B, L, nkv, hd).transpose(0, 2, 1, 3)
    q = q16(q).reshape(B, L, nh, hd).transpose(0, 2, 1, 3)
    cos, sin = rope_cos_sin(hd, position_ids, tcfg.get("rope_theta", 10000.0))  # :293
    q, k = apply_rotary_pos_emb(q, k, cos, sin)                         # :295
    q, k = q16(q), q16(k)
    if kv_cache is not None:                                            # :301-302
        k, v = kv_cache.update(k, v, layer_idx)
    g = nh // nkv                                                       # repeat_kv :185-196
    if g > 1:
        k = np.repeat(k, g, axis=1)
        v = np.repeat(v, g, axis=1)
    s = (q @ k.transpose(0, 1, 3, 2)) / F32(math.sqrt(hd))              # :314
    assert mask is not None, "Attention Mask needss to be provided"    # :325
    s = s + mask                                                        # :326
    p = softmax_lastdim(s)                                              # :329
    if weights_out is not None:
        weights_out.append(p)
    o = q16(p) @ v                                                      # :339
    if o.shape != (B, nh, L, hd):                                       # :341-345
        raise ValueError("Size Mismatch")
    o = o.transpose(0, 2, 1, 3).reshape(B, L, -1)                       # :354-355
    return linear(o, W[lp + "o_proj.weight"], gemma=True, rowpar=True)              # :356


def gemma_mlp(W: dict, lp: str, x: np.ndarray) -> np.ndarray:
    """GemmaMLP.forward (modeling_gemma.py:210-218)."""
    y = gelu_tanh(linear(x, W[lp + "gate_proj.weight"], gemma=True, mx="x"))
    u = linear(x, W[lp + "up_proj.weight"], gemma=True, mx="x")
    return linear(y * u, W[lp + "down_proj.weight"], gemma=True, mx="h", rowpar=True)


def gemma_model(W: dict, tcfg: dict, input_embeds: np.ndarray, position_ids, mask, kv_cache,
                taps: Optional[list] = None) -> np.ndarray:
    """GemmaModel.forward (modeling_gemma.py:453-472) with DecoderLayer.forward (:385-418)."""
    h = input_embeds
    for i in range(tcfg["num_hidden_layers"]):
        lp = f"language_model.model.layers.{i}."
        r = h
        x = rms_norm(h, W[lp + "input_layernorm.weight"])
        h = r + gemma_attention(W, lp + "self_attn.", tcfg, i, x, position_ids, mask, kv_cache)
        r = h
        x = rms_norm(h, W[lp + "post_attention_layernorm.weight"])
        h = r + gemma_mlp(W, lp + "mlp.", x)
        if taps is not None:
            taps.append(h)
    return rms_norm(h, W["language_model.model.norm.weight"])          # :470


def gemma_for_causal_lm(W: dict, tcfg: dict, input_embeds, position_ids, mask, kv_cache,
                        logits_rows: Optional[slice] = None, taps: Optional[list] = None) -> np.ndarray:
    """GemmaForCausalLM.forward (modeling_gemma.py:501-534).

    ``logits_rows`` (output-invariant option) restricts the lm_head to some
    positions; the reference computes all of them (:523).
    """
    x = input_embeds * F32(tcfg["hidden_size"] ** 0.5)                 # :510-511
    h = gemma_model(W, tcfg, x, position_ids, mask, kv_cache, taps)
    if logits_rows is not None:
        h = h[:, logits_rows]
    emb = W["language_model.model.embed_tokens.weight"]                 # tied (:492-499)
    return linear(h, emb, W["language_model.lm_head.bias"], gemma=_FP8_LM_HEAD, mx="x")   # :523-525


# --------------------------------------------------------------------------- #
# PaliGemma composition (modeling_paligemma.py)
# --------------------------------------------------------------------------- #
def merge_input_ids_with_image_features(cfg: dict, input_ids: np.ndarray, input_embeds: np.ndarray,
                                        image_features: np.ndarray) -> np.ndarray:
    """_get_masks + _create_final_embedding (modeling_paligemma.py:93-128).

    text rows <- token embeddings; image rows <- projector output * proj_dim^-0.5,
    filled in flattened (B, L) order (masked_scatter); pad rows <- 0.
    """
    pad = cfg.get("pad_token_id")
    pad = -1 if pad is None else pad                                    # :84
    img = cfg["image_token_index"]
    pad_m = input_ids == pad
    img_m = input_ids == img
    txt_m = (input_ids != img) & (input_ids != pad)
    out = np.zeros(input_embeds.shape, dtype=F32)
    out[txt_m] = input_embeds[txt_m]                                    # :111
    scaled = image_features * F32(cfg.get("projection_dim", 2048) ** -0.5)   # :116-117
    n_img = int(img_m.sum())
    flat = scaled.reshape(-1, scaled.shape[-1])
    out[img_m] = flat[:n_img]                                           # masked_scatter :121-122
    out[pad_m] = 0.0                                                    # :125-127
    return out


def causal_mask_and_position_ids(kv_len_before: int, attention_mask: np.ndarray, q_len: int):
    """_get_causal_mask_and_position_ids (modeling_paligemma.py:130-198)."""
    B = attention_mask.shape[0]
    if kv_len_before == 0:                                              # prefill :149-156
        mask = np.zeros((B, 1, q_len, q_len), dtype=F32)
        cs = np.cumsum(attention_mask, axis=-1)
        pos = np.where(attention_mask == 0, 1, cs)                      # :195
    else:                                                               # decode :158-169
        assert q_len == 1, "Generation Phase more than one token CAN'T be input"
        mask = np.zeros((B, 1, q_len, kv_len_before + q_len), dtype=F32)
        pos = np.cumsum(attention_mask, axis=-1)[:, -1]                 # :189
        pos = pos.reshape(-1, 1) if B > 1 else pos[None, :]             # (fixed (1,B) quirk -> (B,1))
    return mask, pos


class PaliGemmaOracle:
    """PaliGemmaForConditionalGeneration (modeling_paligemma.py:69-308) on numpy."""

    def __init__(self, cfg: dict, weights: dict, recompute_vision: bool = True):
        self.cfg = cfg
        self.W = weights
        self.vcfg = cfg["vision_config"]
        self.tcfg = cfg["text_config"]
        self.recompute_vision = recompute_vision
        self._img_feat = None

    def image_features(self, pixel_values: np.ndarray) -> np.ndarray:
        v = siglip_vision_model(self.W, self.vcfg, pixel_values)        # :281
        return multi_modal_projector(self.W, v)                         # :282

    def forward(self, input_ids, pixel_values, attention_mask, kv_cache: KVCache,
                logits_rows: Optional[slice] = None, taps: Optional[list] = None):
        """forward (modeling_paligemma.py:257-308) -> {"logits", "kv_cache"}."""
        if self.recompute_vision or self._img_feat is None or kv_cache.num_items() == 0:
            self._img_feat = self.image_features(pixel_values)
        emb = self.W["language_model.model.embed_tokens.weight"][input_ids]   # :288
        x = merge_input_ids_with_image_features(self.cfg, input_ids, emb, self._img_feat)
        mask, pos = causal_mask_and_position_ids(kv_cache.num_items(), attention_mask, input_ids.shape[1])
        logits = gemma_for_causal_lm(self.W, self.tcfg, x, pos, mask, kv_cache, logits_rows, taps)
        return {"logits": logits, "kv_cache": kv_cache}


# --------------------------------------------------------------------------- #
# generation loop and sampling (inference.py)
# --------------------------------------------------------------------------- #
def top_p_filter(probs: np.ndarray, p: float):
    """_sample_top_p's filtering (inference.py:90-102): sort desc, cumsum, mask, renorm.

    Returns (probs_sort, probs_idx) as the reference holds them right before
    torch.multinomial (:104).
    """
    idx = np.argsort(-probs, axis=-1, kind="stable")
    ps = np.take_along_axis(probs, idx, axis=-1).astype(F32)
    cs = np.cumsum(ps, axis=-1, dtype=F32)
    ps[(cs - ps) > F32(p)] = 0.0
    ps = ps / ps.sum(axis=-1, keepdims=True)
    return ps, idx


def sample_top_p(logits: np.ndarray, temperature: float, top_p: float, u: np.ndarray) -> np.ndarray:
    """softmax(logits/T) (inference.py:65) + top-p filter (:90-102), then an
    explicit-uniform inverse-CDF draw in vocabulary order over the filtered,
    renormalised distribution (the build's sampler contract, SURVEY.md §7 (ix):
    same distribution as torch.multinomial (:104), reproducible)."""
    probs = softmax_lastdim((logits / F32(temperature)).astype(F32))
    ps, idx = top_p_filter(probs, top_p)
    out = np.empty((logits.shape[0], 1), dtype=np.int64)
    for b in range(logits.shape[0]):
        q = np.zeros(probs.shape[-1], dtype=np.float64)
        q[idx[b]] = ps[b]
        c = np.cumsum(q)
        t = float(u[b]) * c[-1]
        j = int(np.searchsorted(c, t, side="right"))
        out[b, 0] = min(j, int(np.nonzero(q)[0].max()))
    return out


def generate(oracle: PaliGemmaOracle, input_ids: np.ndarray, pixel_values: np.ndarray,
             attention_mask: np.ndarray, max_tokens: int, do_sample: bool = False,
             temperature: float = 0.8, top_p: float = 0.9, uniforms: Optional[np.ndarray] = None,
             stop_token: Optional[int] = 1, teacher: Optional[np.ndarray] = None,
             record_logits: bool = False):
    """test_inference's token loop (inference.py:45-82) for one sequence.

    ``teacher`` forces the fed-back ids (teacher forcing) while still
    recording what greedy would have produced.
    """
    kv = KVCache()
    ids = input_ids
    mask = attention_mask.astype(np.int64)
    out, logits_hist = [], []
    for t in range(max_tokens):
        res = oracle.forward(ids, pixel_values, mask, kv, logits_rows=slice(-1, None))
        last = res["logits"][:, -1, :]                                  # :59
        if record_logits:
            logits_hist.append(last.copy())
        if do_sample:
            nxt = sample_top_p(last, temperature, top_p, uniforms[t])
        else:
            nxt = np.argmax(last, axis=-1)[:, None]                     # :68
        out.append(int(nxt[0, 0]))
        if stop_token is not None and int(nxt[0, 0]) == stop_token:     # :73-74
            break
        fed = nxt if teacher is None else np.array([[teacher[t]]], dtype=np.int64)
        ids = fed                                                       # :76
        mask = np.concatenate([mask, np.ones((mask.shape[0], 1), dtype=mask.dtype)], axis=-1)  # :77-79
    return (out, logits_hist) if record_logits else out
