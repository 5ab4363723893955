"""PaliGemma composition — drop-in for the reference's ``modeling_paligemma`` module (libpghip).

Same names, constructor arguments, module tree / state-dict keys and forward signature as
the reference (modeling_paligemma.py:14-308).  ``forward`` keeps the reference's contract:
prefill when the cache is empty (bidirectional prefix attention, 1-based positions from
``attention_mask``), otherwise one-token decode with position ``sum(attention_mask)``; it
returns ``{"logits": fp32 (B, L, V), "kv_cache": kv_cache}``.

Output-invariant differences: the vision tower runs once per request (its
projected features are kept in the ``KVCache``) instead of on every call (:281); the cache is
the static in-place store of ``modeling_gemma.KVCache``; ``logits_to_keep=1`` (opt-in) limits
the lm_head to the last position.  HIP tensors only.
"""
from __future__ import annotations

import copy
from typing import Optional

import torch
import torch.nn as nn

from modeling_gemma import GemmaConfig, GemmaForCausalLM, KVCache
from modeling_siglip import SiglipVisionConfig, SiglipVisionModel
from pghip import ops
from pghip.engine import PaliGemmaEngine
from pghip.weights import PackedWeights


class PaliGemmaConfig:
    """Top-level config (modeling_paligemma.py:14-45) built from a HF-style config.json dict."""

    def __init__(self, vision_config=None, text_config=None, projection_dim=2048, ignore_index=-100,
                 image_token_index=256000, pad_token_id=None, vocab_size=257152, hidden_size=2048, **kwargs):
        self._raw = copy.deepcopy(dict(vision_config=vision_config, text_config=text_config,
                                       projection_dim=projection_dim, ignore_index=ignore_index,
                                       image_token_index=image_token_index, pad_token_id=pad_token_id,
                                       vocab_size=vocab_size, hidden_size=hidden_size, **kwargs))
        self.projection_dim, self.ignore_index = projection_dim, ignore_index
        self.image_token_index, self.pad_token_id = image_token_index, pad_token_id
        self.hidden_size = hidden_size
        self.vision_config = SiglipVisionConfig(**vision_config)
        self.text_config = GemmaConfig(**text_config, pad_token_id=self.pad_token_id)
        self.vocab_size = self.text_config.vocab_size
        self.text_config.num_image_tokens = (self.vision_config.image_size // self.vision_config.patch_size) ** 2
        self.vision_config.projection_dim = projection_dim

    def as_dict(self) -> dict:
        return copy.deepcopy(self._raw)


class PaliGemmaMultiModalProjector(nn.Module):
    """Linear vision->text projection, no bias (modeling_paligemma.py:52-65)."""

    def __init__(self, config: PaliGemmaConfig):
        super().__init__()
        self.projection_dim = config.projection_dim
        self.image_emb = config.vision_config.hidden_size
        self.linear = nn.Linear(self.image_emb, self.projection_dim, bias=False)

    def forward(self, pixel_values: torch.FloatTensor):
        if not pixel_values.is_cuda:
            raise RuntimeError("PaliGemmaMultiModalProjector: HIP device only")
        x = pixel_values.reshape(-1, pixel_values.shape[-1]).to(torch.bfloat16).contiguous()
        out = torch.empty(x.shape[0], self.projection_dim, dtype=torch.float32, device=x.device)
        ops.gemm(x, self.linear.weight.detach().to(torch.bfloat16).contiguous(), out, epi=ops.EPI_F32)
        return out.view(*pixel_values.shape[:-1], self.projection_dim)


class PaliGemmaForConditionalGeneration(nn.Module):
    """SigLIP -> projector -> token/image merge -> Gemma (modeling_paligemma.py:69-308)."""

    def __init__(self, config: PaliGemmaConfig):
        super().__init__()
        self.config = config
        self.vision_config = self.config.vision_config
        self.vision_tower = SiglipVisionModel(self.vision_config)
        self.text_config = self.config.text_config
        self.language_model = GemmaForCausalLM(self.text_config)
        self.pad_token_id = self.config.pad_token_id if self.config.pad_token_id is not None else -1
        self.dummy_image_token_id = self.config.image_token_index
        self.multi_modal_projector = PaliGemmaMultiModalProjector(self.config)
        self._eng_key = None
        self._eng = None

    def tie_weights(self):
        return self.language_model.tie_weights()

    # ---- the packed engine (rebuilt when parameters change)
    def engine(self, device=None) -> PaliGemmaEngine:
        params = list(self.parameters())
        device = torch.device(device) if device is not None else params[0].device
        key = tuple((p.data_ptr(), p._version) for p in params) + (device,)
        if key != self._eng_key:
            sd = self.state_dict()
            if "language_model.lm_head.weight" not in sd:
                sd["language_model.lm_head.weight"] = sd["language_model.model.embed_tokens.weight"]
            self._eng = None
            cfg = self.config.as_dict()
            self._eng = PaliGemmaEngine(cfg, PackedWeights(cfg, sd.__getitem__, device=device), device=device)
            self._eng_key = key
        return self._eng

    # ---- reference helpers (host logic; same semantics)
    def _get_masks(self, input_ids):
        """(pad, text, image) token masks (modeling_paligemma.py:93-97)."""
        pad = input_ids == self.pad_token_id
        img = input_ids == self.dummy_image_token_id
        return pad, (~img) & (~pad), img

    def _get_causal_mask_and_position_ids(self, kv_cache: Optional[KVCache] = None,
                                          attention_mask: torch.Tensor = None, input_embeds: torch.Tensor = None):
        """All-zero additive mask + positions (modeling_paligemma.py:130-198): prefill 1-based cumsum,
        decode sum(mask) per row (the reference's (1, B) batch quirk is fixed to (B, 1))."""
        B, q_len = input_embeds.shape[0], input_embeds.shape[1]
        dev, dt = input_embeds.device, input_embeds.dtype
        if kv_cache is None or kv_cache.num_items() == 0:
            mask = torch.zeros(B, 1, q_len, q_len, dtype=dt, device=dev)
            pos = attention_mask.cumsum(-1).masked_fill(attention_mask == 0, 1).to(dev)
        else:
            assert q_len == 1, "Generation Phase more than one token CAN'T be input"
            kv_len = kv_cache.num_items() + q_len
            mask = torch.zeros(B, 1, q_len, kv_len, dtype=dt, device=dev)
            pos = attention_mask.cumsum(-1)[:, -1].reshape(B, 1)
        return mask, pos

    def _merge_input_ids_with_image_features(self, input_ids, input_embeds, attention_mask, kv_cache,
                                             projected_image_features):
        """Text rows <- embeddings, image rows <- projected features * proj_dim^-0.5 (masked_scatter
        order), pad rows <- 0 (modeling_paligemma.py:201-251).  Runs the pghip merge kernel on the
        embedding table and returns (final_embedding fp32, causal_mask, position_ids).  (The
        ``input_embeds`` argument is accepted for API parity; the kernel gathers the rows itself.)"""
        eng = self.engine(input_ids.device)
        B, L = input_ids.shape
        out = torch.empty(B * L, eng.w.hidden, dtype=torch.float32, device=input_ids.device)
        feats = projected_image_features.reshape(-1, projected_image_features.shape[-1]).float().contiguous()
        eng.embed_merge(input_ids.contiguous(), feats, out)
        x = (out / (eng.w.hidden ** 0.5)).view(B, L, -1)          # merge kernel applies the *sqrt(H) of :510
        mask, pos = self._get_causal_mask_and_position_ids(kv_cache, attention_mask, x)
        return x, mask, pos

    # ---- forward
    def forward(self, input_ids: torch.LongTensor = None, pixel_values: torch.FloatTensor = None,
                attention_mask: Optional[torch.Tensor] = None, kv_cache: Optional[KVCache] = None,
                logits_to_keep: Optional[int] = None):
        if not input_ids.is_cuda:
            raise RuntimeError("PaliGemmaForConditionalGeneration: the pghip path runs on the HIP device only")
        eng = self.engine(input_ids.device)
        w = eng.w
        cache = kv_cache if kv_cache is not None else KVCache()
        B, L = input_ids.shape
        dev = input_ids.device
        if attention_mask is None:
            attention_mask = torch.ones(B, L, dtype=torch.int64, device=dev)
        attention_mask = attention_mask.to(dev)
        if cache.num_items() == 0:
            feats = eng.vision(pixel_values.to(dev))
            cache.image_features = feats
            store = eng.new_cache(B, L + 128)
            resid = torch.empty(B * L, w.hidden, dtype=torch.float32, device=dev)
            eng.embed_merge(input_ids.contiguous(), feats, resid)
            pos = attention_mask.cumsum(-1).masked_fill(attention_mask == 0, 1)
            rows = None
            if logits_to_keep:
                k = int(logits_to_keep)
                rows = (torch.arange(B, device=dev, dtype=torch.int32)[:, None] * L
                        + torch.arange(L - k, L, device=dev, dtype=torch.int32)[None]).reshape(-1).contiguous()
            logits, _ = eng.gemma_prefill(resid, pos, store, B, L, logits_rows=rows)
            cache.adopt(store, L, w.kv_heads, w.head_dim)
            logits = logits.reshape(B, -1, w.vocab)
        else:
            assert L == 1, "Generation Phase more than one token CAN'T be input"
            feats = cache.image_features
            if feats is None and pixel_values is not None:
                feats = cache.image_features = eng.vision(pixel_values.to(dev))
            n = cache.num_items()
            store = cache._ensure(w.t_layers, B, w.kv_heads, w.head_dim, n + 1, dev)
            st = {"ids": input_ids.reshape(B).contiguous(),
                  "pos": attention_mask.sum(-1).to(torch.int32).reshape(B).contiguous(),
                  "kv_len": torch.full((1,), n, dtype=torch.int32, device=dev)}
            logits = eng.decode_step(st, store, feats, sampler=None).reshape(B, 1, w.vocab).clone()
            cache._len = [n + 1] * len(cache._len)
        return {"logits": logits, "kv_cache": cache}

    @torch.no_grad()
    def generate(self, input_ids, pixel_values, attention_mask=None, max_new_tokens: int = 100,
                 do_sample: bool = False, temperature: float = 0.8, top_p: float = 0.9, uniforms=None,
                 stop_token: Optional[int] = 1):
        """The token loop of inference.py:45-82 on the engine (vision once, hipGraph-replayed decode steps)."""
        eng = self.engine(input_ids.device)
        if attention_mask is None:
            attention_mask = torch.ones_like(input_ids)
        return eng.generate(input_ids, pixel_values, attention_mask, max_new_tokens, do_sample=do_sample,
                            temperature=temperature, top_p=top_p, uniforms=uniforms, stop_token=stop_token)
