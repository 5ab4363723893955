"""GPU image pre-processing: the reference's process_images (processing_paligemma.py:38-73) for RGB
uint8 images as two HIP passes (pg_resize_h_u8, pg_resize_v_norm).

The resize is PIL's ``Image.resize(..., BICUBIC)`` (Pillow 12.2.0, libImaging/Resample.c — a
third-party algorithm the reference calls, not in /root/reference): separable convolution with the
a = -0.5 cubic kernel widened by the downscale factor, double coefficients normalised per output
pixel and rounded to 22-bit fixed point, a horizontal pass over the rows the vertical pass needs
(rounded and clipped to uint8), then the vertical pass.  The coefficient tables below restate
Pillow's precompute_coeffs / normalize_coeffs_8bpc in the same double arithmetic; the kernels do the
integer accumulation.  The rescale+normalise of the reference (uint8 * (1/255.0) in float64 -> float32,
then (x - 0.5) / 0.5 in float32) is a 256-entry table, so the whole pipeline is bit-exact with the
reference's host path (tests/test_host.py, tests/test_kernels_gpu.py).
"""
from __future__ import annotations

import math
from typing import List, Sequence

import numpy as np
import torch

from . import ops

PRECISION_BITS = 32 - 8 - 2


def _bicubic(x: float) -> float:
    a = -0.5
    if x < 0.0:
        x = -x
    if x < 1.0:
        return ((a + 2.0) * x - (a + 3.0)) * x * x + 1
    if x < 2.0:
        return (((x - 5) * x + 8) * x - 4) * a
    return 0.0


def resample_coeffs(in_size: int, out_size: int):
    """(bounds int32 [out][2] = (first input index, count), fixed-point taps int32 [out][ksize], ksize)."""
    scale = in_size / out_size
    filterscale = max(scale, 1.0)
    support = 2.0 * filterscale
    ksize = int(math.ceil(support)) * 2 + 1
    bounds = np.zeros((out_size, 2), np.int32)
    kk = np.zeros((out_size, ksize), np.int32)
    ss = 1.0 / filterscale
    for xx in range(out_size):
        center = (xx + 0.5) * scale
        xmin = max(int(center - support + 0.5), 0)
        xmax = min(int(center + support + 0.5), in_size) - xmin
        w = [_bicubic((x + xmin - center + 0.5) * ss) for x in range(xmax)]
        ww = 0.0
        for v in w:
            ww += v
        if ww != 0.0:
            w = [v / ww for v in w]
        for x, v in enumerate(w):
            kk[xx, x] = int(-0.5 + v * (1 << PRECISION_BITS)) if v < 0 else int(0.5 + v * (1 << PRECISION_BITS))
        bounds[xx] = (xmin, xmax)
    return bounds, kk, ksize


def normalise_lut(scale_factor: float = 1 / 255.0, mean: float = 0.5, std: float = 0.5) -> np.ndarray:
    """float32 [256]: the reference's rescale ((u8 * scale) in float64 -> float32) then normalise in float32."""
    x = (np.arange(256, dtype=np.uint8) * scale_factor).astype(np.float32)
    return (x - np.float32(mean)) / np.float32(std)


_coeff_cache: dict = {}


def _coeffs_dev(in_size, out_size, device):
    key = (in_size, out_size, str(device))
    if key not in _coeff_cache:
        b, k, ks = resample_coeffs(in_size, out_size)
        _coeff_cache[key] = (torch.from_numpy(b).to(device), torch.from_numpy(k).to(device), ks, b)
    return _coeff_cache[key]


def preprocess(images: Sequence, image_size: int, device="cuda") -> torch.Tensor:
    """RGB uint8 images (PIL images in mode RGB, or HxWx3 uint8 arrays / tensors) -> float32
    [B, 3, S, S] pixel_values on the HIP device, equal to the reference's process_images + stack."""
    dev = torch.device(device)
    lut = torch.from_numpy(normalise_lut()).to(dev)
    S = int(image_size)
    out = torch.empty(len(images), 3, S, S, dtype=torch.float32, device=dev)
    for i, im in enumerate(images):
        if hasattr(im, "mode"):
            if im.mode != "RGB":
                raise ValueError(f"pghip.image.preprocess: RGB images only (got mode {im.mode})")
            arr = torch.from_numpy(np.asarray(im, dtype=np.uint8).copy())
        else:
            arr = torch.as_tensor(im)
        if arr.dtype != torch.uint8 or arr.dim() != 3 or arr.shape[2] != 3:
            raise ValueError("pghip.image.preprocess: expected HxWx3 uint8")
        src = arr.to(dev).contiguous()
        H, W = src.shape[0], src.shape[1]
        hb = hk = None
        hks = 0
        rows, y0 = H, 0
        vb, vk, vks, vb_host = _coeffs_dev(H, S, dev)
        need_h, need_v = W != S, H != S
        if need_h:
            hb, hk, hks, _ = _coeffs_dev(W, S, dev)
            if need_v:                      # only the source rows the vertical pass reads (Resample.c)
                y0 = int(vb_host[0, 0])
                rows = int(vb_host[-1, 0] + vb_host[-1, 1]) - y0
        tmp = torch.empty(rows, S if need_h else W, 3, dtype=torch.uint8, device=dev) if need_h else None
        ops.image_preprocess(src, H, W, S, hb, hk, hks, vb if need_v else None, vk if need_v else None,
                             vks if need_v else 0, y0, rows, lut, tmp, out[i])
    return out
