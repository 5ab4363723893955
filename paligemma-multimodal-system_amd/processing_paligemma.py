"""Image/prompt pre-processing — drop-in for the reference's ``processing_paligemma`` (host side).

Behaviour of processing_paligemma.py:13-212: PIL bicubic resize to (image_size, image_size),
RGB, x/255 in fp32, (x - 0.5)/0.5, HWC -> CHW, batch stack; the "gemma string"
``<image>*N + <bos> + prompt + "\\n"`` tokenised with the image token and 128 <seg> / 1024
<loc> tokens added to the tokenizer.  As in the reference, ``__call__`` passes the LIST of
prompts to the string builder, so the prompt text is the list's repr (e.g. ``['caption en']``,
SURVEY.md §8(c)) — kept for output parity.  Batch size 1, as the reference asserts.
Host-only code (PIL / numpy / tokenizer); the image tensor it returns is what the HIP path consumes.
"""
from __future__ import annotations

from typing import List, Optional, Sequence, Union

import numpy as np
import torch

IMAGENET_STANDARD_MEAN = [0.5, 0.5, 0.5]
IMAGENET_STANDARD_STD = [0.5, 0.5, 0.5]


def resize(image, resampling, image_size: int, reducing_gap: Optional[int] = None):
    return image.resize((image_size, image_size), resample=resampling, reducing_gap=reducing_gap)


def rescale(image: np.ndarray, scale_factor: float, dtype=np.float32) -> np.ndarray:
    return (image * scale_factor).astype(dtype)


def normalise(image: np.ndarray, mean: Union[float, Sequence[float]], std: Union[float, Sequence[float]]):
    return (image - np.asarray(mean, dtype=image.dtype)) / np.asarray(std, dtype=image.dtype)


def process_images(images: List, image_size: int, scale_factor: float, resampling=None,
                   reducing_gap: Optional[int] = None) -> List[np.ndarray]:
    """resize -> RGB -> rescale -> normalise -> CHW, per image (processing_paligemma.py:38-73)."""
    out = []
    for im in images:
        arr = np.array(resize(im, resampling, image_size, reducing_gap).convert("RGB"))
        arr = normalise(rescale(arr, scale_factor), IMAGENET_STANDARD_MEAN, IMAGENET_STANDARD_STD)
        out.append(arr.transpose(2, 0, 1))
    return out


def create_gemma_string(prefix_prompt, image_seq_len: int, image_token: str, bos_token: str) -> str:
    """<image>*N <bos> prompt \\n (processing_paligemma.py:77-89)."""
    return f"{image_token * image_seq_len}{bos_token}{prefix_prompt}\n"


class PaliGemmaProcessor:
    """Tokenizer + image pipeline (processing_paligemma.py:94-212)."""

    IMAGE_TOKEN = "<image>"

    def __init__(self, tokenizer, num_image_tokens: int, image_size: int, device=None):
        """device: when a HIP device is given, RGB images are resized/normalised there (pghip.image,
        bit-exact with the host path below); None keeps the reference's host (PIL + numpy) path."""
        self.device = device
        self.tokenizer = tokenizer
        self.image_seq_len = num_image_tokens
        self.image_size = image_size
        tokenizer.add_special_tokens({"additional_special_tokens": [self.IMAGE_TOKEN]})
        extra = [f"<seg{i:03d}>" for i in range(128)] + [f"<loc{i:04d}>" for i in range(1024)]
        tokenizer.add_tokens(extra)
        tokenizer.image_token_id = tokenizer.convert_tokens_to_ids(self.IMAGE_TOKEN)
        tokenizer.add_eos_token = False
        tokenizer.add_bos_token = False

    def __call__(self, images: List, text: List[str], padding: str = "longest", truncation: bool = True):
        assert len(images) == 1 and len(text) == 1, \
            "Working with only 1 image and prompt, to test, got more than one"
        from PIL import Image
        if self.device is not None and all(getattr(im, "mode", None) == "RGB" for im in images):
            from pghip import image as gpu_image
            pixel_values = gpu_image.preprocess(images, self.image_size, self.device)
        else:
            pixel_values = torch.tensor(np.stack(process_images(images, self.image_size, scale_factor=1 / 255.0,
                                                                resampling=Image.Resampling.BICUBIC), axis=0))
        s = create_gemma_string(prefix_prompt=text, image_seq_len=self.image_seq_len, image_token=self.IMAGE_TOKEN,
                                bos_token=self.tokenizer.bos_token)
        toks = self.tokenizer(s, return_tensors="pt", truncation=truncation, padding=padding)
        return {"pixel_values": pixel_values, **toks}
