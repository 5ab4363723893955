"""The model directory and image of BASELINE configs[0] ("single-image greedy decode via inference.py"), shared by
tests/golden/make_golden.py (which runs the REFERENCE's inference.main on them, in the development container) and
tests/test_dropin_gpu.py (which runs the drop-in's inference.main on the same files on the GPU box).  Test
infrastructure: the weights come from oracle/synth.py, the tokenizer is the offline one in tests/golden/tokenizer.

The directory is what the reference's utils.load_hf_model reads (utils.py:9-38): config.json, *.safetensors in the
reference's key names, and the tokenizer files.  The config is TINY's (300-id vocabulary) with <image> at the id the
PaliGemmaProcessor gives it on this tokenizer (after the base words; <seg> and <loc> follow, processing_paligemma.py:
129-145), so every id the model can emit decodes.  The image is an RGBA PNG shaped like the reference's
test_images/pic1.png (1004 x 444).  IMAGE_SEED and MAX_TOKENS were chosen (seed search with the oracle)
so that the reference's top1-top2 margin stays >= 0.05 logits over the 12 greedy steps, 4x the bf16-operand emulation's
logit error (0.012): free-running greedy ids can then be compared exactly.
"""
from __future__ import annotations

import copy
import json
import os
import shutil

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
TOKENIZER_DIR = os.path.join(HERE, "golden", "tokenizer")
PROMPT = "caption en"
IMAGE_SEED = 39
IMAGE_HW = (444, 1004)
MAX_TOKENS = 12


def tokenizer_ids():
    """(tokenizer length after the processor's additions, the <image> id) of the offline tokenizer."""
    from transformers import AutoTokenizer
    tok = AutoTokenizer.from_pretrained(TOKENIZER_DIR)
    base = len(tok)
    return base + 1 + 128 + 1024, base


def main_config() -> dict:
    import sys
    sys.path.insert(0, os.path.dirname(HERE))
    from oracle import configs
    n_tok, image_id = tokenizer_ids()
    cfg = copy.deepcopy(configs.TINY)
    assert image_id < cfg["text_config"]["vocab_size"] <= n_tok
    n = (cfg["vision_config"]["image_size"] // cfg["vision_config"]["patch_size"]) ** 2
    cfg["image_token_index"] = image_id
    cfg["text_config"]["num_image_tokens"] = n
    cfg["vision_config"]["num_image_tokens"] = n        # read by inference.main (inference.py:132)
    return cfg


def write_model_dir(path: str) -> dict:
    """config.json + model.safetensors (fp32, reference keys; the tied lm_head weight omitted as in HF checkpoints)
    + tokenizer files.  Returns the config."""
    import sys
    sys.path.insert(0, os.path.dirname(HERE))
    from oracle import synth
    from safetensors.numpy import save_file
    cfg = main_config()
    os.makedirs(path, exist_ok=True)
    with open(os.path.join(path, "config.json"), "w") as f:
        json.dump(cfg, f)
    sd = synth.generate_state_dict(cfg)
    sd.pop("language_model.lm_head.weight", None)
    save_file({k: np.ascontiguousarray(v, dtype=np.float32) for k, v in sd.items()},
              os.path.join(path, "model.safetensors"))
    for fn in os.listdir(TOKENIZER_DIR):
        shutil.copy(os.path.join(TOKENIZER_DIR, fn), os.path.join(path, fn))
    return cfg


def write_image(path: str) -> str:
    """An RGBA PNG with a varying alpha channel (PIL premultiplies alpha while resizing, then the processor drops it:
    processing_paligemma.py:17,52)."""
    from PIL import Image
    rng = np.random.default_rng(IMAGE_SEED)
    h, w = IMAGE_HW
    rgb = rng.integers(0, 256, (h, w, 3), dtype=np.uint8)
    alpha = (np.linspace(40, 255, w)[None, :] * np.ones((h, 1))).astype(np.uint8)
    Image.fromarray(np.dstack([rgb, alpha])).save(path)       # (h, w, 4) uint8: mode RGBA
    return path
