"""Checkpoint + tokenizer loader — drop-in for the reference's ``utils.load_hf_model`` (utils.py:9-38).

Reads ``config.json`` and every ``*.safetensors`` of a local model directory, builds the pghip
``PaliGemmaForConditionalGeneration`` (same module tree and key names as the reference), loads
the tensors with ``strict=False`` and ties lm_head to the embedding, exactly like the reference.

What the reference does silently is reported here (SURVEY.md §5 checkpoint row, §8(f) row 1):
  * missing and unexpected keys are counted and named in a ``LoadReport`` (returned on request) and in one
    warning: with HF PaliGemma names the reference loads no SigLIP weight at all (``vision_model`` /
    ``position_embedding`` / ``q_proj`` vs its ``model`` / ``positional_embeddings`` / ``query_proj``);
  * an HF projector bias (``multi_modal_projector.linear.bias``; the reference's projector has ``bias=False``,
    modeling_paligemma.py:57) is dropped by default, as the reference does, with a warning;
    ``projector_bias="refuse"`` raises instead;
  * ``language_model.lm_head.bias`` (the reference's lm_head is an ``nn.Linear`` with its default bias,
    modeling_gemma.py:484) is left at its random init when the checkpoint has none, as the reference does, with a
    warning; ``zero_missing_lm_head_bias=True`` zeroes it (the HF model has no such bias).
``remap_hf_keys=True`` (opt-in) maps HF key names onto the reference's first: the SigLIP names above, and the
``model.*`` / top-level ``lm_head`` layout of newer transformers exports.  ``strict=True`` raises on any
missing (other than the tied lm_head weight) or unexpected key.
"""
from __future__ import annotations

import glob
import json
import os
import re
import warnings
from dataclasses import dataclass, field
from typing import List, Tuple

from modeling_paligemma import PaliGemmaConfig, PaliGemmaForConditionalGeneration

_SIGLIP_HF_TO_REF = [
    (r"^vision_tower\.vision_model\.", "vision_tower.model."),
    (r"embeddings\.position_embedding\.", "embeddings.positional_embeddings."),
    (r"self_attn\.q_proj\.(weight|bias)$", r"self_attn.query_proj.\1"),
    (r"self_attn\.k_proj\.(weight|bias)$", r"self_attn.key_proj.\1"),
    (r"self_attn\.v_proj\.(weight|bias)$", r"self_attn.value_proj.\1"),
]
# newer transformers exports nest everything under "model." and keep lm_head at the top level
_LAYOUT_HF_TO_REF = [
    (r"^model\.vision_tower\.", "vision_tower."),
    (r"^model\.multi_modal_projector\.", "multi_modal_projector."),
    (r"^model\.language_model\.", "language_model.model."),
    (r"^lm_head\.", "language_model.lm_head."),
]
PROJECTOR_BIAS = "multi_modal_projector.linear.bias"
LM_HEAD_BIAS = "language_model.lm_head.bias"
TIED = "language_model.lm_head.weight"


def remap_hf_key(key: str) -> str:
    """An HF PaliGemma state-dict key -> the reference's name for the same tensor (unchanged if it already is)."""
    for pat, rep in _LAYOUT_HF_TO_REF:
        key = re.sub(pat, rep, key)
    if key.startswith("vision_tower.vision_model."):
        for pat, rep in _SIGLIP_HF_TO_REF:
            key = re.sub(pat, rep, key)
    return key


@dataclass
class LoadReport:
    """What load_state_dict(strict=False) did with a checkpoint (the reference discards this, utils.py:33)."""
    missing: List[str] = field(default_factory=list)      # model keys the checkpoint did not provide
    unexpected: List[str] = field(default_factory=list)   # checkpoint keys the model has no place for
    dropped: List[str] = field(default_factory=list)      # checkpoint keys deliberately not loaded
    remapped: int = 0                                      # keys renamed by remap_hf_keys

    def summary(self) -> str:
        def few(ks):
            return ", ".join(ks[:4]) + (f" ... (+{len(ks) - 4})" if len(ks) > 4 else "")
        parts = []
        if self.missing:
            parts.append(f"{len(self.missing)} missing (left at init): {few(self.missing)}")
        if self.unexpected:
            parts.append(f"{len(self.unexpected)} unexpected (ignored): {few(self.unexpected)}")
        if self.dropped:
            parts.append(f"dropped: {few(self.dropped)}")
        return "; ".join(parts)


def load_state_dict_reported(model, tensors: dict, projector_bias: str = "drop", strict: bool = False,
                             zero_missing_lm_head_bias: bool = False) -> LoadReport:
    """model.load_state_dict(tensors, strict=False) + tie_weights() as the reference (utils.py:33-36), reporting
    missing / unexpected keys and applying the projector-bias and lm_head-bias policies of the module docstring."""
    import torch
    if projector_bias not in ("drop", "refuse"):
        raise ValueError("projector_bias must be 'drop' (the reference's behaviour) or 'refuse'")
    rep = LoadReport()
    tensors = dict(tensors)
    if PROJECTOR_BIAS in tensors:
        if projector_bias == "refuse":
            raise ValueError(f"checkpoint has {PROJECTOR_BIAS}, but the reference projector has no bias "
                             "(modeling_paligemma.py:57); load with projector_bias='drop' to discard it")
        tensors.pop(PROJECTOR_BIAS)
        rep.dropped.append(PROJECTOR_BIAS + " (reference projector has bias=False)")
    res = model.load_state_dict(tensors, strict=False)
    rep.missing = sorted(k for k in res.missing_keys if k != TIED)
    rep.unexpected = sorted(res.unexpected_keys)
    if LM_HEAD_BIAS in rep.missing and zero_missing_lm_head_bias:
        with torch.no_grad():
            model.language_model.lm_head.bias.zero_()
        rep.missing.remove(LM_HEAD_BIAS)
        rep.dropped.append(LM_HEAD_BIAS + " zeroed (not in the checkpoint)")
    if strict and (rep.missing or rep.unexpected):
        raise KeyError("state dict does not match the reference module tree: " + rep.summary())
    model.tie_weights()
    return rep


def load_hf_model(model_path: str, device: str, remap_hf_keys: bool = False, projector_bias: str = "drop",
                  strict: bool = False, zero_missing_lm_head_bias: bool = False, return_report: bool = False
                  ) -> Tuple[PaliGemmaForConditionalGeneration, object]:
    """(model, tokenizer) from a local directory, as utils.py:9-38; see the module docstring for the options.
    return_report=True returns (model, tokenizer, LoadReport)."""
    from safetensors import safe_open
    from transformers import AutoTokenizer

    tokenizer = AutoTokenizer.from_pretrained(model_path, padding_side="right")
    assert tokenizer.padding_side == "right"
    tensors, renamed = {}, 0
    for fn in sorted(glob.glob(os.path.join(model_path, "*.safetensors"))):
        with safe_open(fn, framework="pt", device="cpu") as f:
            for key in f.keys():
                k = remap_hf_key(key) if remap_hf_keys else key
                renamed += k != key
                tensors[k] = f.get_tensor(key)
    with open(os.path.join(model_path, "config.json"), "r") as f:
        config = PaliGemmaConfig(**json.load(f))
    model = PaliGemmaForConditionalGeneration(config).to(device)
    rep = load_state_dict_reported(model, tensors, projector_bias=projector_bias, strict=strict,
                                   zero_missing_lm_head_bias=zero_missing_lm_head_bias)
    rep.remapped = renamed
    if rep.missing or rep.unexpected or rep.dropped:
        warnings.warn(f"load_hf_model({model_path}): {rep.summary()}", stacklevel=2)
    if return_report:
        return model, tokenizer, rep
    return model, tokenizer
