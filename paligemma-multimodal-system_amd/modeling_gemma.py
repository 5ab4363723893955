"""Gemma-2B decoder — drop-in for the reference's ``modeling_gemma`` module, computed by libpghip.

Same importable names, constructor arguments, forward signatures, module tree and
state-dict keys as the reference (modeling_gemma.py:8-534), so checkpoints and
calling code move over unchanged.  Parameters stay in the reference layout (fp32 by
default, like the reference); the first forward on the HIP device packs them into the
kernel layouts (bf16, fused q|k|v, interleaved gate/up) and caches the pack until the
parameters change.  Every forward requires CUDA(HIP) tensors: there is no CPU path.

Deliberate, output-invariant differences:
  * ``GemmaAttention.forward`` returns ``(attn_output, None)`` unless ``module.return_attn_weights``
    (or PG_ATTN_WEIGHTS=1) asks for the softmax weights (:358; pg_attn_probs forms them): the flash
    kernels never materialise them, and no reference caller uses them (:398-403).
  * ``KVCache`` keeps the reference API (``update`` / ``num_items`` / ``k_cache`` /
    ``v_cache``) on top of a static, in-place HBM buffer (no torch.cat per step, :54-55).
  * batch > 1 decode works (the reference builds (1, B) position ids and fails, :189-191).
"""
from __future__ import annotations

import math
from typing import List, Optional, Tuple

import torch
import torch.nn as nn

from pghip import ops
from pghip.engine import KVStore, rope_tables
from pghip.weights import rope_row_perm


def _require_hip(t: torch.Tensor, what: str):
    if not t.is_cuda:
        raise RuntimeError(f"{what}: the pghip path runs on the HIP device only (got {t.device}); "
                           "move the model and inputs with .to('cuda')")


def _rup(x: int, m: int) -> int:
    return (x + m - 1) // m * m


# --------------------------------------------------------------------------------------------
class KVCache:
    """Per-layer K/V cache with the reference API (modeling_gemma.py:8-64).

    Storage is static: K [B][Smax][kv_heads*head_dim] (RoPE applied) and V^T
    [B][kv_heads*head_dim][Smax] per layer, grown by doubling when full.  ``k_cache`` /
    ``v_cache`` expose (B, kv_heads, len, head_dim) views like the reference's lists.
    """

    def __init__(self):
        self._store: Optional[KVStore] = None
        self._len: List[int] = []          # items per layer
        self.image_features = None         # projector output of the current request (vision runs once)
        self.layers = 0

    # -- storage management (used by the pghip modules and the engine)
    def _ensure(self, layers: int, B: int, kv_heads: int, head_dim: int, need: int, device):
        st = self._store
        if st is not None and (st.B != B or st.kv_dim != kv_heads * head_dim):
            raise ValueError("KVCache: batch / kv geometry changed inside one cache")
        if st is None:
            self._store = KVStore(layers, B, _rup(max(need, 64), 64), kv_heads * head_dim, device, kv_heads=kv_heads)
            self._len = [0] * layers
            self.layers = layers
            self._kv_heads, self._head_dim = kv_heads, head_dim
            return self._store
        if need > st.Smax or layers > st.k.shape[0]:
            nl = max(layers, st.k.shape[0])
            new = KVStore(nl, B, _rup(max(need, 2 * st.Smax if need > st.Smax else st.Smax), 64), st.kv_dim,
                          st.k.device, kv_heads=st.kv_heads)
            n = max(self._len) if self._len else 0
            new.copy_prefix_from(st, n)
            self._store = new
            self._len += [0] * (nl - len(self._len))
            self.layers = nl
        return self._store

    def adopt(self, store: KVStore, length: int, kv_heads: int, head_dim: int):
        """Take over an engine-filled static store (prefill) with `length` items in every layer."""
        self._store = store
        self.layers = store.k.shape[0]
        self._len = [length] * self.layers
        self._kv_heads, self._head_dim = kv_heads, head_dim

    # -- reference API
    def update(self, key_states: torch.Tensor, value_states: torch.Tensor,
               layer_idx: int) -> Tuple[torch.Tensor, torch.Tensor]:
        """Append (B, kv_heads, L, head_dim) states for ``layer_idx``; return the full K, V (:18-57)."""
        B, nkv, L, hd = key_states.shape
        layers = max(layer_idx + 1, self.layers)
        cur = self._len[layer_idx] if layer_idx < len(self._len) else 0
        st = self._ensure(layers, B, nkv, hd, cur + L, key_states.device)
        if len(self._len) < layers:
            self._len += [0] * (layers - len(self._len))
        k = key_states.transpose(1, 2).reshape(B, L, nkv * hd)
        st.k[layer_idx, :, cur:cur + L] = k.to(st.k.dtype)
        st.vt[layer_idx, :, :, cur:cur + L] = value_states.transpose(1, 2).reshape(B, L, nkv * hd).transpose(1, 2).to(
            st.vt.dtype)
        if hd % 16 == 0:                          # the decode-order copies the engine's decode kernels read
            # repack only the 32-key blocks holding the appended positions [cur, cur + L) (the layout is
            # block-local, attn_common.h dec_koff / dec_voff), not the whole cache on every call
            b0, b1 = cur // 32 * 32, _rup(cur + L, 32)
            kd, vd = ops.decode_cache_pack(st.k[layer_idx, :, b0:b1], st.vt[layer_idx, :, :, b0:b1], nkv)
            st.kd[layer_idx].view(B, nkv, st.Smax, hd)[:, :, b0:b1] = kd
            st.vd[layer_idx].view(B, nkv, st.Smax, hd)[:, :, b0:b1] = vd
        self._len[layer_idx] = cur + L
        return self._views(layer_idx)

    def num_items(self) -> int:
        """Number of cached positions (the reference reads layer 0, :59-64)."""
        return self._len[0] if self._len else 0

    def _views(self, i: int):
        st, n = self._store, self._len[i]
        B, nkv, hd = st.B, self._kv_heads, self._head_dim
        k = st.k[i, :, :n].view(B, n, nkv, hd).transpose(1, 2)
        v = st.vt[i, :, :, :n].view(B, nkv, hd, n).transpose(-1, -2)
        return k, v

    @property
    def k_cache(self) -> list:
        return [self._views(i)[0] for i in range(len(self._len))] if self._store is not None else []

    @property
    def v_cache(self) -> list:
        return [self._views(i)[1] for i in range(len(self._len))] if self._store is not None else []


# --------------------------------------------------------------------------------------------
class GemmaConfig:
    """Text-model hyper-parameters (modeling_gemma.py:68-99); unknown keys are accepted and ignored."""

    def __init__(self, rope_theta: float = 10000.0, max_position_encodings: int = 8192, rms_norm_eps: float = None,
                 hidden_size: int = None, num_hidden_layers: int = None, num_attention_heads: int = None,
                 num_key_value_heads: int = None, head_dim: int = 256, intermediate_size: int = None,
                 attention_bias: bool = False, attention_dropout: float = 0.0, pad_token_id: int = None,
                 vocab_size: int = None, **kwargs):
        self.rope_theta = rope_theta
        self.max_position_encodings = max_position_encodings
        self.rms_norm_eps = rms_norm_eps
        self.hidden_size = hidden_size
        self.num_hidden_layers = num_hidden_layers
        self.num_attention_heads = num_attention_heads
        self.num_key_value_heads = num_key_value_heads
        self.head_dim = head_dim
        self.intermediate_size = intermediate_size
        self.attention_bias = attention_bias
        self.attention_dropout = attention_dropout
        self.pad_token_id = pad_token_id
        self.vocab_size = vocab_size
        for k, v in kwargs.items():
            setattr(self, k, v)


class GemmaRotaryEmbedding(nn.Module):
    """cos/sin of the rotary embedding (modeling_gemma.py:103-135); half-split layout, fp32."""

    def __init__(self, dim, max_position_embeddings=2048, base=10000, device=None):
        super().__init__()
        self.dim, self.max_position_embeddings, self.base = dim, max_position_embeddings, base
        inv_freq = 1.0 / (base ** (torch.arange(0, dim, 2, dtype=torch.int64).float() / dim))
        self.register_buffer("inv_freq", tensor=inv_freq, persistent=False)
        self._tables = None

    def tables(self, n_pos: int, device):
        """[n_pos][dim/2] fp32 cos/sin tables indexed by the integer position (kernel input)."""
        t = self._tables
        if t is None or t[0].shape[0] < n_pos or t[0].device != torch.device(device):
            n = _rup(max(n_pos, 1024), 1024)
            self._tables = rope_tables(self.dim, n, float(self.base), device)
        return self._tables

    @torch.no_grad()
    def forward(self, x, position_ids, seq_len=None):
        cos_t, sin_t = self.tables(int(position_ids.max().item()) + 1, x.device)
        p = position_ids.long()
        cos = torch.cat([cos_t[p], cos_t[p]], dim=-1)
        sin = torch.cat([sin_t[p], sin_t[p]], dim=-1)
        return cos.to(dtype=x.dtype), sin.to(dtype=x.dtype)


def rotate_half(x):
    """cat(-x2, x1) over the last dim (modeling_gemma.py:138-142)."""
    h = x.shape[-1] // 2
    return torch.cat((-x[..., h:], x[..., :h]), dim=-1)


def apply_rotary_pos_emb(q, k, cos, sin, unsqueeze_dim=1):
    """q*cos + rotate_half(q)*sin (modeling_gemma.py:145-151).  Host utility kept for API parity;
    the pghip path applies RoPE inside the fused q|k|v GEMM epilogue."""
    cos, sin = cos.unsqueeze(unsqueeze_dim), sin.unsqueeze(unsqueeze_dim)
    return q * cos + rotate_half(q) * sin, k * cos + rotate_half(k) * sin


def repeat_kv(x: torch.Tensor, group_size: int):
    """Expand kv heads (modeling_gemma.py:185-196).  API parity only: the kernels read one kv head
    for all the q heads sharing it."""
    if group_size == 1:
        return x
    b, h, s, d = x.shape
    return x[:, :, None].expand(b, h, group_size, s, d).reshape(b, h * group_size, s, d)


# --------------------------------------------------------------------------------------------
class _PackCache:
    """Packed bf16 copies of a module's parameters, rebuilt when any parameter changes."""

    def __init__(self):
        self.key = None
        self.val = None

    def get(self, params, build):
        key = tuple((p.data_ptr(), p._version, p.device) for p in params)
        if key != self.key:
            self.val = build()
            self.key = key
        return self.val


def _bf(t):
    return t.detach().to(torch.bfloat16).contiguous()


def _rows(x: torch.Tensor):
    """(…, H) float -> (M, H) fp32 contiguous working copy."""
    return x.reshape(-1, x.shape[-1]).to(torch.float32).contiguous()


class GemmaRMSNorm(nn.Module):
    """x * rsqrt(mean(x^2) + eps) * (1 + w), computed and returned in fp32 (modeling_gemma.py:157-182)."""

    def __init__(self, dim: int, eps: float = 1e-6):
        super().__init__()
        self.dim, self.eps = dim, eps
        self.weight = nn.Parameter(torch.zeros(dim))

    def forward(self, x):
        _require_hip(x, "GemmaRMSNorm")
        r = _rows(x)
        out = torch.empty_like(r)
        ops.norm_residual(r, self.weight.detach().float().contiguous(), mode=ops.NORM_RMS, eps=self.eps, out_f32=out,
                          write_resid=False)
        return out.view(x.shape)


class GemmaMLP(nn.Module):
    """down(gelu_tanh(gate(x)) * up(x)) (modeling_gemma.py:198-218): one GEMM with the GELU*mul epilogue
    over interleaved gate/up rows, then the down GEMM."""

    def __init__(self, config: GemmaConfig):
        super().__init__()
        self.intermediate_size, self.hidden_size = config.intermediate_size, config.hidden_size
        self.gate_proj = nn.Linear(self.hidden_size, self.intermediate_size, bias=False)
        self.up_proj = nn.Linear(self.hidden_size, self.intermediate_size, bias=False)
        self.down_proj = nn.Linear(self.intermediate_size, self.hidden_size, bias=False)
        self._pk = _PackCache()

    def packed(self):
        def build():
            I, H = self.intermediate_size, self.hidden_size
            g = _bf(self.gate_proj.weight).view(I // 16, 16, H)
            u = _bf(self.up_proj.weight).view(I // 16, 16, H)
            return torch.stack([g, u], 1).reshape(2 * I, H).contiguous(), _bf(self.down_proj.weight)
        return self._pk.get([self.gate_proj.weight, self.up_proj.weight, self.down_proj.weight], build)

    def forward(self, x):
        _require_hip(x, "GemmaMLP")
        gu, down = self.packed()
        xb = x.reshape(-1, x.shape[-1]).to(torch.bfloat16).contiguous()
        M = xb.shape[0]
        h = torch.empty(M, self.intermediate_size, dtype=torch.bfloat16, device=x.device)
        ops.gemm(xb, gu, h, epi=ops.EPI_BF16_GELU_MUL)
        out = torch.empty(M, self.hidden_size, dtype=torch.float32, device=x.device)
        ops.gemm(h, down, out, epi=ops.EPI_F32)
        return out.view(*x.shape[:-1], self.hidden_size)


class GemmaAttention(nn.Module):
    """Multi-query attention with RoPE and the KV cache (modeling_gemma.py:221-358).

    q|k|v projection, RoPE and the cache append run as ONE GEMM (rope-permuted weight rows,
    fused epilogue); the attention is the flash kernel over the cached keys (MQA by row stacking,
    no repeat_kv); o_proj is the last GEMM.  Returns (attn_output fp32, None).
    """

    def __init__(self, config: GemmaConfig, layer_idx: int):
        super().__init__()
        self.config, self.layer_idx = config, layer_idx
        self.hidden_size, self.head_dim = config.hidden_size, config.head_dim
        self.attention_dropout = config.attention_dropout
        self.rms_norm_eps = config.rms_norm_eps
        self.max_position_embeddings = config.max_position_encodings
        self.rope_theta = config.rope_theta
        self.is_causal = True
        self.rotary_emb = GemmaRotaryEmbedding(self.head_dim, max_position_embeddings=self.max_position_embeddings,
                                               base=self.rope_theta)
        self.num_heads, self.num_key_value_heads = config.num_attention_heads, config.num_key_value_heads
        assert self.num_heads % self.num_key_value_heads == 0, \
            "number of Key/Value heads donot divide Number of Query Heads"
        self.key_value_groups = self.num_heads // self.num_key_value_heads
        kvd = self.num_key_value_heads * self.head_dim
        self.k_proj = nn.Linear(self.hidden_size, kvd, bias=config.attention_bias)
        self.v_proj = nn.Linear(self.hidden_size, kvd, bias=config.attention_bias)
        self.q_proj = nn.Linear(self.hidden_size, self.num_heads * self.head_dim, bias=config.attention_bias)
        self.o_proj = nn.Linear(self.hidden_size, self.hidden_size, bias=config.attention_bias)
        self._pk = _PackCache()
        self.return_attn_weights = ops.ATTN_WEIGHTS

    def packed(self):
        def build():
            nblk = self.num_heads + 2 * self.num_key_value_heads
            w = torch.cat([_bf(self.q_proj.weight), _bf(self.k_proj.weight), _bf(self.v_proj.weight)], 0)
            perm = rope_row_perm(self.head_dim).to(w.device)
            w = w.view(nblk, self.head_dim, -1)[:, perm, :].reshape(nblk * self.head_dim, -1).contiguous()
            b = None
            if self.q_proj.bias is not None:
                b = torch.cat([self.q_proj.bias, self.k_proj.bias, self.v_proj.bias]).detach().float()
                b = b.view(nblk, self.head_dim)[:, perm.cpu() if b.device.type == "cpu" else perm].reshape(-1)
                b = b.contiguous()
            ob = self.o_proj.bias.detach().float().contiguous() if self.o_proj.bias is not None else None
            return w, b, _bf(self.o_proj.weight), ob
        ps = [self.q_proj.weight, self.k_proj.weight, self.v_proj.weight, self.o_proj.weight]
        return self._pk.get(ps, build)

    def forward(self, hidden_states: torch.Tensor, position_ids: torch.Tensor, kv_cache: Optional[KVCache] = None,
                attention_mask: Optional[torch.Tensor] = None, **kwargs):
        _require_hip(hidden_states, "GemmaAttention")
        assert attention_mask is not None, "Attention Mask needss to be provided"     # :325
        B, L, _ = hidden_states.shape
        nh, nkv, hd = self.num_heads, self.num_key_value_heads, self.head_dim
        wqkv, bqkv, wo, bo = self.packed()
        dev = hidden_states.device
        cache = kv_cache if kv_cache is not None else KVCache()
        layers = max(self.layer_idx + 1, cache.layers)
        past = cache._len[self.layer_idx] if self.layer_idx < len(cache._len) else 0
        st = cache._ensure(layers, B, nkv, hd, past + L, dev)
        if len(cache._len) < layers:
            cache._len += [0] * (layers - len(cache._len))
        pos = position_ids.reshape(B, -1).to(device=dev, dtype=torch.int32)
        if pos.shape[1] != L:                                   # decode: one position per row
            pos = pos.reshape(B, 1).expand(B, L)
        pos = pos.contiguous()
        cos_t, sin_t = self.rotary_emb.tables(int(pos.max().item()) + 2, dev)
        xb = hidden_states.reshape(B * L, -1).to(torch.bfloat16).contiguous()
        q = torch.empty(B * L, nh * hd, dtype=torch.bfloat16, device=dev)
        fa = ops.fused_args(head_dim=hd, cos_t=cos_t, sin_t=sin_t, pos=pos, rows_per_batch=L, slot_base=past,
                            kc=st.k[self.layer_idx], vtc=st.vt[self.layer_idx], smax=st.Smax, q_heads=nh,
                            kv_heads=nkv, kd=st.kd[self.layer_idx], vd=st.vd[self.layer_idx])
        ops.gemm_fused(xb, wqkv, q, fa, epi=ops.EPI_QKV_ROPE, M=B * L, bias=bqkv)
        cache._len[self.layer_idx] = past + L
        Lkv = past + L
        mask = attention_mask
        if mask.dim() == 4:
            mask = mask[:, 0]
        mask = mask.to(device=dev, dtype=torch.float32).expand(B, L, Lkv).contiguous()
        o = torch.empty(B * L, nh * hd, dtype=torch.bfloat16, device=dev)
        kvd = nkv * hd
        ops.attention(q, nh * hd, o, nh * hd, st.k[self.layer_idx], st.Smax * kvd, hd, kvd, st.vt[self.layer_idx],
                      kvd * st.Smax, hd * st.Smax, st.Smax, B=B, Lq=L, Lkv=Lkv, Hq=nh, Hkv=nkv, D=hd,
                      scale=1.0 / math.sqrt(hd), mask=mask, mask_bs=L * Lkv, mask_rs=Lkv)
        out = torch.empty(B * L, self.hidden_size, dtype=torch.float32, device=dev)
        ops.gemm(o, wo, out, epi=ops.EPI_F32, bias=bo)
        weights = None
        if self.return_attn_weights:        # the softmax matrix the reference returns (:358), formed on request only
            weights = ops.attn_probs(q, nh * hd, st.k[self.layer_idx], st.Smax * kvd, hd, kvd, B=B, Lq=L, Lkv=Lkv,
                                     Hq=nh, Hkv=nkv, D=hd, scale=1.0 / math.sqrt(hd), mask=mask, mask_bs=L * Lkv,
                                     mask_rs=Lkv)
        return out.view(B, L, self.hidden_size), weights


class DecoderLayer(nn.Module):
    """x + attn(RMSNorm(x)), then x + mlp(RMSNorm(x)) (modeling_gemma.py:364-418); fp32 residual."""

    def __init__(self, config: GemmaConfig, layer_idx: Optional[int] = None):
        super().__init__()
        self.layer_idx = layer_idx
        self.input_layernorm = GemmaRMSNorm(dim=config.hidden_size)
        self.self_attn = GemmaAttention(config, layer_idx)
        self.post_attention_layernorm = GemmaRMSNorm(dim=config.hidden_size)
        self.mlp = GemmaMLP(config)

    def forward(self, hidden_states: torch.Tensor, position_ids: Optional[torch.LongTensor] = None,
                attention_mask: Optional[torch.Tensor] = None, kv_cache: Optional[KVCache] = None):
        h = hidden_states.to(torch.float32)
        a, _ = self.self_attn(hidden_states=self.input_layernorm(h), position_ids=position_ids,
                              attention_mask=attention_mask, kv_cache=kv_cache)
        h = h + a
        return h + self.mlp(self.post_attention_layernorm(h))


class GemmaModel(nn.Module):
    """Embedding table + decoder stack + final RMSNorm (modeling_gemma.py:424-472)."""

    def __init__(self, config: GemmaConfig):
        super().__init__()
        self.vocab_size, self.hidden_size = config.vocab_size, config.hidden_size
        self.pad_token_id = config.pad_token_id
        self.num_hidden_layers = config.num_hidden_layers
        self.embed_tokens = nn.Embedding(self.vocab_size, self.hidden_size, padding_idx=self.pad_token_id)
        self.layers = nn.ModuleList([DecoderLayer(config, i) for i in range(self.num_hidden_layers)])
        self.rms_norm_eps = config.rms_norm_eps
        self.norm = GemmaRMSNorm(dim=self.hidden_size)

    def tie_weights(self):
        return self.embed_tokens

    def forward(self, input_embeds: Optional[torch.FloatTensor] = None,
                position_ids: Optional[torch.LongTensor] = None, attention_mask: Optional[torch.Tensor] = None,
                kv_cache: Optional[KVCache] = None):
        h = input_embeds
        for layer in self.layers:
            h = layer(hidden_states=h, position_ids=position_ids, attention_mask=attention_mask, kv_cache=kv_cache)
        return self.norm(h)


class GemmaForCausalLM(nn.Module):
    """GemmaModel + tied lm_head with its own bias (modeling_gemma.py:474-534); logits in fp32."""

    def __init__(self, config: GemmaConfig):
        super().__init__()
        self.vocab_size, self.hidden_size = config.vocab_size, config.hidden_size
        self.lm_head = nn.Linear(self.hidden_size, self.vocab_size)
        self.text_config = config
        self.model = GemmaModel(self.text_config)
        self._pk = _PackCache()

    def get_input_embeddings(self):
        return self.model.embed_tokens

    def tie_weights(self):
        self.lm_head.weight = self.model.embed_tokens.weight

    def _head(self):
        return self._pk.get([self.lm_head.weight, self.lm_head.bias],
                            lambda: (_bf(self.lm_head.weight), self.lm_head.bias.detach().float().contiguous()))

    def forward(self, input_embeds: Optional[torch.FloatTensor] = None,
                position_ids: Optional[torch.LongTensor] = None, attention_mask: Optional[torch.Tensor] = None,
                kv_cache: Optional[KVCache] = None):
        _require_hip(input_embeds, "GemmaForCausalLM")
        x = input_embeds * torch.tensor(self.hidden_size ** 0.5, dtype=input_embeds.dtype, device=input_embeds.device)
        h = self.model(attention_mask=attention_mask, kv_cache=kv_cache, position_ids=position_ids, input_embeds=x)
        w, b = self._head()
        hb = h.reshape(-1, self.hidden_size).to(torch.bfloat16).contiguous()
        logits = torch.empty(hb.shape[0], self.vocab_size, dtype=torch.float32, device=hb.device)
        ops.gemm(hb, w, logits, epi=ops.EPI_F32, bias=b)
        out = {"logits": logits.view(*h.shape[:-1], self.vocab_size)}
        if kv_cache is not None:
            out["kv_cache"] = kv_cache
        return out
