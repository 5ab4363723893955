"""Image->text generation entry point — drop-in for the reference's ``inference.py``.

Same functions and CLI flags as inference.py:11-154 (``main``, ``test_inference``,
``_sample_top_p``, ``get_model_inputs``, ``move_inputs_to_device``); flags are parsed with
argparse in fire's ``--name value`` form (fire is not installed offline).  The token loop
keeps the reference's semantics — one model call per generated token, greedy argmax or
softmax(logits/T) + top-p sampling, stop at the tokenizer's EOS, print ``prompt + decoded`` —
but runs on the HIP engine: vision once, graph-replayed decode steps, sampling on the device.
There is no CPU path: ``--only_cpu True`` is rejected (the reference forces CPU at :127).
"""
from __future__ import annotations

import argparse
import sys

import torch

from modeling_gemma import KVCache  # noqa: F401  (re-exported like the reference's import)
from modeling_paligemma import PaliGemmaForConditionalGeneration
from pghip import ops
from processing_paligemma import PaliGemmaProcessor
from utils import load_hf_model


def move_inputs_to_device(model_inputs: dict, device: str):
    return {k: v.to(device) for k, v in model_inputs.items()}


def get_model_inputs(processor: PaliGemmaProcessor, prompt: str, image_file_path: str, device: str):
    from PIL import Image
    image = Image.open(image_file_path)
    return move_inputs_to_device(processor(text=[prompt], images=[image]), device)


def _sample_top_p(probs: torch.Tensor, p: float):
    """Top-p draw from a probability matrix (B, V) -> (B, 1) token ids (inference.py:90-106).

    Same filter (sorted-descending mass before a token <= p, renormalised) on the device; the
    draw is an inverse CDF with a fresh uniform per row (torch.multinomial's stream is not
    reproducible across devices anyway)."""
    if not probs.is_cuda:
        raise RuntimeError("_sample_top_p: HIP device only")
    B = probs.shape[0]
    logits = torch.log(probs.float().clamp_min(1e-38)).contiguous()
    out = torch.empty(B, dtype=torch.int64, device=probs.device)
    u = torch.rand(1, B, device=probs.device)
    ops.topp_sample(logits, out, u, temperature=1.0, top_p=float(p))
    return out.view(B, 1)


def test_inference(model: PaliGemmaForConditionalGeneration, processor: PaliGemmaProcessor, device: str,
                   prompt: str, image_file_path: str, max_tokens_to_generate: int, temperature: float,
                   top_p: float, do_sample: bool):
    """Generate until EOS or max_tokens_to_generate, then print prompt + decoded (inference.py:29-87)."""
    inputs = get_model_inputs(processor, prompt, image_file_path, device)
    ids = model.generate(inputs["input_ids"], inputs["pixel_values"], inputs["attention_mask"],
                         max_new_tokens=max_tokens_to_generate, do_sample=do_sample, temperature=temperature,
                         top_p=top_p, stop_token=processor.tokenizer.eos_token_id)
    decoded = processor.tokenizer.decode(ids[0], skip_special_tokens=True)
    print(prompt + decoded)
    return ids


def main(model_path: str = None, prompt: str = None, image_file_path: str = None, max_tokens_to_generate: int = 100,
         temperature: float = 0.8, top_p: float = 0.9, do_sample: bool = False, only_cpu: bool = False):
    if only_cpu:
        raise RuntimeError("this build has no CPU path (HIP kernels only); drop --only_cpu")
    if not torch.cuda.is_available():
        raise RuntimeError("no HIP device visible")
    device = "cuda"
    print("Device in use: ", device)
    print("Loading model")
    model, tokenizer = load_hf_model(model_path, device)
    model = model.to(device).eval()
    processor = PaliGemmaProcessor(tokenizer, model.config.vision_config.num_image_tokens or
                                   model.config.text_config.num_image_tokens, model.config.vision_config.image_size,
                                   device=device)        # resize + normalise on the device (bit-exact with PIL)
    print("Running inference")
    with torch.no_grad():
        test_inference(model, processor, device, prompt, image_file_path, max_tokens_to_generate, temperature,
                       top_p, do_sample)


def _bool(s) -> bool:
    if isinstance(s, bool):
        return s
    return str(s).strip().lower() in ("1", "true", "yes", "y", "t")


def _cli(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--model_path")
    ap.add_argument("--prompt")
    ap.add_argument("--image_file_path")
    ap.add_argument("--max_tokens_to_generate", type=int, default=100)
    ap.add_argument("--temperature", type=float, default=0.8)
    ap.add_argument("--top_p", type=float, default=0.9)
    ap.add_argument("--do_sample", type=_bool, default=False)
    ap.add_argument("--only_cpu", type=_bool, default=False)
    a = ap.parse_args(argv)
    main(**vars(a))


if __name__ == "__main__":
    _cli(sys.argv[1:])
