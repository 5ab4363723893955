"""HF-style config.json dicts for the PaliGemma-3B variants and a tiny test config.

TEST INFRASTRUCTURE ONLY (the product carries its own copy in
``pghip/configs.py``; tests/test_configs.py checks they agree).

The pt-224 dict is the published ``google/paligemma-3b-pt-224`` config.json as
consumed by ``PaliGemmaConfig(**config)`` (modeling_paligemma.py:14-45,
utils.py:25-27).  pt-448 / pt-896 differ only in image size and image-token
count.  ``tiny`` keeps every structural feature (MQA, head_dim not a multiple
of 32 in the vision tower, sizes that need padding) at toy width.
"""
import copy

PT_224 = {
    "bos_token_id": 2,
    "eos_token_id": 1,
    "hidden_size": 2048,
    "ignore_index": -100,
    "image_token_index": 257152,
    "model_type": "paligemma",
    "pad_token_id": 0,
    "projection_dim": 2048,
    "text_config": {
        "hidden_size": 2048,
        "intermediate_size": 16384,
        "model_type": "gemma",
        "num_attention_heads": 8,
        "num_hidden_layers": 18,
        "num_image_tokens": 256,
        "num_key_value_heads": 1,
        "torch_dtype": "float32",
        "vocab_size": 257216,
    },
    "vision_config": {
        "hidden_size": 1152,
        "intermediate_size": 4304,
        "model_type": "siglip_vision_model",
        "num_attention_heads": 16,
        "num_hidden_layers": 27,
        "num_image_tokens": 256,
        "patch_size": 14,
        "projection_dim": 2048,
        "projector_hidden_act": "gelu_fast",
        "vision_use_head": False,
    },
}


def _sized(image_size: int) -> dict:
    c = copy.deepcopy(PT_224)
    n = (image_size // 14) ** 2
    c["vision_config"]["image_size"] = image_size
    c["vision_config"]["num_image_tokens"] = n
    c["text_config"]["num_image_tokens"] = n
    return c


PT_448 = _sized(448)
PT_896 = _sized(896)

# Toy config: vision head_dim 24 (not a multiple of 32, like SigLIP's 72), hidden sizes that are
# multiples of 64 (as the real ones),
# intermediate sizes that are not multiples of 64, MQA (4 q heads : 1 kv head),
# a small vocab that still holds the special ids (pad 0, eos 1, bos 2, image 299).
TINY = {
    "bos_token_id": 2,
    "eos_token_id": 1,
    "hidden_size": 128,
    "ignore_index": -100,
    "image_token_index": 299,
    "pad_token_id": 0,
    "projection_dim": 128,
    "text_config": {
        "hidden_size": 128,
        "intermediate_size": 320,
        "num_attention_heads": 4,
        "num_hidden_layers": 2,
        "num_key_value_heads": 1,
        "head_dim": 32,
        "vocab_size": 300,
    },
    "vision_config": {
        "hidden_size": 192,
        "intermediate_size": 200,
        "image_size": 56,
        "num_attention_heads": 8,
        "num_hidden_layers": 2,
        "patch_size": 14,
    },
}

# Toy config for tensor parallelism up to 8 ranks (BASELINE configs[4] runs Gemma at TP=8): 8 q heads : 1 kv head
# (one q head per rank at TP=8, as the real model), head_dim 128 and hidden 1024 = 8 x 128 (the reference's o_proj
# is hidden -> hidden, modeling_gemma.py:259; every rank's q|k|v and o slices stay fragment-packable and fp8-able),
# intermediate 640 (80 per rank at TP=8, zero-padded to the GEMM K step), vocab 304 (38 rows per rank at TP=8,
# padded to 48).  The vision tower is TINY's, projected to 1024.
TINY8 = copy.deepcopy(TINY)
TINY8.update(hidden_size=1024, projection_dim=1024)
TINY8["text_config"].update(hidden_size=1024, intermediate_size=640, num_attention_heads=8, head_dim=128,
                            vocab_size=304)

CONFIGS = {"pt-224": PT_224, "mix-224": PT_224, "pt-448": PT_448, "pt-896": PT_896, "tiny": TINY, "tiny8": TINY8}  # mix = pt shapes


def num_image_tokens(cfg: dict) -> int:
    v = cfg["vision_config"]
    return (v.get("image_size", 224) // v["patch_size"]) ** 2
