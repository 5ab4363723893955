"""numpy restatement of Pillow 12.2.0's 8-bit BICUBIC resample (libImaging/Resample.c: precompute_coeffs,
normalize_coeffs_8bpc, ImagingResampleHorizontal_8bpc / Vertical_8bpc, clip8) — the third-party algorithm
behind the reference's resize (processing_paligemma.py:13-19), absent from /root/reference.

TEST INFRASTRUCTURE ONLY (checker for pghip.image / pg_resize_*).  Pinned bit-exactly against PIL
itself in tests/test_host.py.  The fixed-point coefficient tables come from pghip.image.resample_coeffs
(the host half of the product path), so this file checks the integer passes and pins the tables."""
import numpy as np

PRECISION_BITS = 22


def clip8(acc: np.ndarray) -> np.ndarray:
    return np.clip(acc >> PRECISION_BITS, 0, 255).astype(np.uint8)


def resize_u8(img: np.ndarray, size: int, coeffs) -> np.ndarray:
    """img uint8 [H][W][C] -> [size][size][C] like Image.resize((size, size), BICUBIC)."""
    H, W, C = img.shape
    if H == size and W == size:
        return img.copy()
    vb, vk, _ = coeffs(H, size)
    x = img.astype(np.int64)
    if W != size:
        hb, hk, _ = coeffs(W, size)
        y0, y1 = (int(vb[0, 0]), int(vb[-1, 0] + vb[-1, 1])) if H != size else (0, H)
        rows = x[y0:y1]
        acc = np.full((y1 - y0, size, C), 1 << (PRECISION_BITS - 1), np.int64)
        for xx in range(size):
            s, n = hb[xx]
            acc[:, xx, :] += (rows[:, s:s + n, :] * hk[xx, :n][None, :, None]).sum(1)
        x = clip8(acc).astype(np.int64)
        vb = vb.copy()
        if H != size:
            vb[:, 0] -= y0
    if H != size:
        acc = np.full((size, x.shape[1], C), 1 << (PRECISION_BITS - 1), np.int64)
        for yy in range(size):
            s, n = vb[yy]
            acc[yy] += (x[s:s + n] * vk[yy, :n][:, None, None]).sum(0)
        x = clip8(acc).astype(np.int64)
    return x.astype(np.uint8)
