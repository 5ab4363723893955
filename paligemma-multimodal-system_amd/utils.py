"""Checkpoint + tokenizer loader — drop-in for the reference's ``utils.load_hf_model`` (utils.py:9-38).

Reads ``config.json`` and every ``*.safetensors`` of a local model directory, builds the pghip
``PaliGemmaForConditionalGeneration`` (same module tree and key names as the reference), loads
the tensors with ``strict=False`` and ties lm_head to the embedding, exactly like the reference.
With ``remap_hf_keys=True`` (opt-in) HF PaliGemma key names
(``vision_tower.vision_model.*``, ``position_embedding``, ``q_proj``/``k_proj``/``v_proj``) are
mapped onto the reference names first, so the SigLIP tower is actually loaded.
"""
from __future__ import annotations

import glob
import json
import os
import re
from typing import Tuple

from modeling_paligemma import PaliGemmaConfig, PaliGemmaForConditionalGeneration

_HF_TO_REF = [
    (r"^vision_tower\.vision_model\.", "vision_tower.model."),
    (r"embeddings\.position_embedding\.", "embeddings.positional_embeddings."),
    (r"self_attn\.q_proj\.(weight|bias)$", r"self_attn.query_proj.\1"),
    (r"self_attn\.k_proj\.(weight|bias)$", r"self_attn.key_proj.\1"),
    (r"self_attn\.v_proj\.(weight|bias)$", r"self_attn.value_proj.\1"),
    (r"self_attn\.out_proj\.", "self_attn.out_proj."),
]


def remap_hf_key(key: str) -> str:
    if not key.startswith("vision_tower.vision_model."):
        return key
    for pat, rep in _HF_TO_REF:
        key = re.sub(pat, rep, key)
    return key


def load_hf_model(model_path: str, device: str, remap_hf_keys: bool = False) -> Tuple[PaliGemmaForConditionalGeneration, object]:
    from safetensors import safe_open
    from transformers import AutoTokenizer

    tokenizer = AutoTokenizer.from_pretrained(model_path, padding_side="right")
    assert tokenizer.padding_side == "right"
    tensors = {}
    for fn in glob.glob(os.path.join(model_path, "*.safetensors")):
        with safe_open(fn, framework="pt", device="cpu") as f:
            for key in f.keys():
                tensors[remap_hf_key(key) if remap_hf_keys else key] = f.get_tensor(key)
    with open(os.path.join(model_path, "config.json"), "r") as f:
        config = PaliGemmaConfig(**json.load(f))
    model = PaliGemmaForConditionalGeneration(config).to(device)
    model.load_state_dict(tensors, strict=False)
    model.tie_weights()
    return model, tokenizer
