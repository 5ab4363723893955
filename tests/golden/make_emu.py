"""Operand-rounding emulation fixtures from the numpy ORACLE (not the reference): the fp32 oracle run with the HIP
fp8 path's operand rounding -- bf16 operands everywhere, e4m3 Gemma linears and tied lm_head with per-row /
per-channel scales (oracle.paligemma_oracle.fp8_operands; min_rows=0: prefill and batch > 16 decode both run fp8;
mx_h / mx_norm: the decode down_proj and the RMSNorm-fed decode linears on MX rows, engine.MX_H / MX_NORM) -- on a reference
golden's requests, teacher-forced with the reference's own greedy ids.  Stored per image and step: the emulated
logits at the reference's top-64 ids, the emulated argmax and top1-top2 margin.  tests/test_large_gpu.py bounds the
HIP fp8 path's distance to the reference by 1.5x this intrinsic distance (the bf16 tests do the same with
oracle.bf16_operands live).

--tp W (round 6): the tensor-parallel form (oracle fp8_operands(tp=W): the row-parallel o_proj / down_proj quantised
per rank on their K slices and summed in rank order) -> <golden>_fp8emu_tp<W>.npz, the bound of the TP=W GPU test
(tests/test_tp_gpu.py::test_tp8_pt896_fp8_batch32).

Runs on the CPU in the development container (minutes per pt-896 request):
    python tests/golden/make_emu.py [pt896wc] [--tp 8]
"""
from __future__ import annotations

import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from oracle import configs, synth  # noqa: E402
from oracle import paligemma_oracle as O  # noqa: E402


def pixels(seed: int, size: int) -> np.ndarray:
    from PIL import Image
    sys.path.insert(0, os.path.join(ROOT, "paligemma-multimodal-system_amd"))
    from processing_paligemma import process_images
    img = np.random.default_rng(seed).integers(0, 256, (1, size, size, 3), dtype=np.uint8)
    return np.stack(process_images([Image.fromarray(img[0])], size, 1 / 255.0, Image.Resampling.BICUBIC)).astype(
        np.float32)


def make(name: str, cfg: dict, tp: int = 1):
    g = dict(np.load(os.path.join(HERE, f"{name}.npz")))
    gain = float(g.get("linear_gain", 2.0))
    W = synth.generate_state_dict(cfg, gain)
    size = cfg["vision_config"]["image_size"]
    out = {"linear_gain": np.float32(gain), "tp": np.int32(tp),
           "mode": np.array("bf16 operands + e4m3 Gemma linears and lm_head (min_rows=0), MX decode rows (down_proj h, "
                            "RMSNorm-fed q|k|v, gate/up, lm_head), MX prefill h (round 6)"
                            + (f"; TP={tp}: o_proj / down_proj per-rank K slices, rank-order sums" if tp > 1 else ""))}
    for j, seed in enumerate(g["seeds"]):
        p = f"i{j}_"
        pv = pixels(int(seed), size)
        assert np.array_equal(pv.reshape(-1)[::9973], g[p + "pixel_sample"])
        ids = g[p + "input_ids"]
        ref = g[p + "greedy_ids"]
        top_ids = g[p + "step_top_ids"]
        steps = len(ref)
        orc = O.PaliGemmaOracle(cfg, W, recompute_vision=False)
        kv = O.KVCache()
        mask = np.ones_like(ids)
        cur = ids
        vals, am, mg = [], [], []
        with O.bf16_operands(), O.fp8_operands(min_rows=0, lm_head=True, mx_h=True, mx_norm=True, tp=tp,
                                                       mx_h_prefill=True):
            for t in range(steps):
                lg = orc.forward(cur, pv, mask, kv, logits_rows=slice(-1, None))["logits"][0, -1]
                vals.append(lg[top_ids[t]])
                s = np.sort(lg)
                am.append(int(np.argmax(lg)))
                mg.append(float(s[-1] - s[-2]))
                cur = np.array([[ref[t]]], dtype=np.int64)
                mask = np.concatenate([mask, np.ones((1, 1), mask.dtype)], -1)
                print(f"{name} image {seed} step {t}: emu top-64 err "
                      f"{np.abs(vals[-1] - g[p + 'step_top_values'][t]).max():.4f}, argmax {am[-1]} ref {ref[t]}",
                      flush=True)
        out[p + "emu_top_values"] = np.stack(vals).astype(np.float32)
        out[p + "emu_argmax"] = np.array(am, np.int64)
        out[p + "emu_margin"] = np.array(mg, np.float32)
    np.savez_compressed(os.path.join(HERE, f"{name}_fp8emu" + (f"_tp{tp}" if tp > 1 else "") + ".npz"), **out)


if __name__ == "__main__":
    import torch
    torch.set_num_threads(os.cpu_count())
    args = sys.argv[1:]
    tp = 1
    if "--tp" in args:
        i = args.index("--tp")
        tp = int(args[i + 1])
        del args[i:i + 2]
    for name in args or ["pt896wc"]:
        make(name, {"pt896wc": configs.PT_896, "pt896": configs.PT_896, "pt448wc": configs.PT_448}[name], tp)
