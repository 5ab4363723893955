"""Tensor-level wrappers over the C-ABI (include/pghip.h).

Every function takes CUDA(HIP) torch tensors, checks dtype/shape/contiguity on
the host (so no kernel is launched with a shape it does not handle), and
enqueues on torch's current stream.  torch is used only for memory and streams.
"""
from __future__ import annotations

import math
import os
from typing import Optional

import torch

from . import _lib

EPI_BF16, EPI_BF16_GELU, EPI_BF16_GELU_MUL, EPI_F32, EPI_F32_POS, EPI_BF16_VT, EPI_QKV_ROPE, EPI_F32_FIN, \
    EPI_F32_ADD, EPI_FX_ADD, EPI_F32_RES = range(11)
FX_SCALE = 2.0 ** 32   # PG_EPI_FX_ADD: the int64 accumulator holds round(value * 2^32)
PRO_NONE, PRO_RMSNORM, PRO_ATTN_COMBINE, PRO_RMSNORM_FIN, PRO_X_RSTD = range(5)
NORM_LAYER, NORM_RMS = 0, 1
W_FRAG = 0x100   # OR into epi: W is fragment-packed (weights.frag_pack, include/pghip.h PG_W_FRAG)
TILE_M1 = 0x400  # OR into epi: all 256..288 rows in one row tile (batch-1 prefill, include/pghip.h PG_TILE_M1)
TILE_N64 = 0x800  # OR into epi: 64 x 64 output tiles (small-M prefill GEMMs, include/pghip.h PG_TILE_N64)


def _p(t: Optional[torch.Tensor]):
    return None if t is None else t.data_ptr()


def _s() -> int:
    return torch.cuda.current_stream().cuda_stream


def _chk(t: torch.Tensor, dtype, name: str):
    if not t.is_cuda:
        raise RuntimeError(f"pghip: {name} must be on the HIP device (got {t.device}); no CPU path")
    if t.dtype != dtype:
        raise TypeError(f"pghip: {name} must be {dtype}, got {t.dtype}")


def _chk_frag(W: torch.Tensor, epi: int):
    if epi & W_FRAG and (W.shape[0] % 16 or W.shape[1] % 64 or W.stride(0) != W.shape[1]):
        raise ValueError(f"pghip: a fragment-packed W must be [N%16][K%64] and contiguous, got {tuple(W.shape)}")


def gemm(A: torch.Tensor, W: torch.Tensor, out: torch.Tensor, *, epi: int = EPI_BF16,
         bias: Optional[torch.Tensor] = None, ksplit: int = 1, N: Optional[int] = None,
         aux: Optional[torch.Tensor] = None, aux_rows: int = 0, aux_out: Optional[torch.Tensor] = None,
         aux_ld: int = 0, aux_n: int = 0, M: Optional[int] = None, split_m: Optional[int] = None) -> torch.Tensor:
    """out = epilogue(A[M][K] . W[N][K]^T).  K = W.shape[1] (zero-padded), A.shape[1] >= K.
    epi may carry W_FRAG (W fragment-packed, weights.frag_pack).  split_m: choose the small-M split-K of a bf16
    epilogue as for that many rows (a data-parallel rank slice then sums in the same order as the whole batch)."""
    _chk(A, torch.bfloat16, "A")
    _chk(W, torch.bfloat16, "W")
    _chk_frag(W, epi)
    flags, epi = epi, epi & 0xFF
    if A.stride(1) != 1 or W.stride(1) != 1 or out.stride(-1) != 1:
        raise ValueError("pghip.gemm: inner dims must be contiguous")
    M = A.shape[0] if M is None else M
    N = W.shape[0] if N is None else N
    K = W.shape[1]
    if A.shape[1] < K:
        raise ValueError(f"pghip.gemm: A has {A.shape[1]} cols < K={K}")
    if bias is not None:
        _chk(bias, torch.float32, "bias")
    ldc = out.stride(-2) if out.dim() >= 2 else out.shape[-1]
    if epi in (EPI_F32, EPI_F32_RES):
        _chk(out, torch.float32, "out")
        need = (ksplit * M - 1) * ldc + N                                # last element touched, in elements
        if out.storage_offset() + need > out.untyped_storage().nbytes() // out.element_size():
            raise ValueError("pghip.gemm: partial output too small")
        if epi == EPI_F32_RES and (ksplit != 1 or M <= 16):
            raise ValueError("pghip.gemm: EPI_F32_RES (out += acc + bias) is a one-split tile epilogue (M > 16)")
    elif epi == EPI_F32_POS:
        _chk(out, torch.float32, "out")
    else:
        _chk(out, torch.bfloat16, "out")
    if M > 16 and K % 64:
        raise ValueError("pghip.gemm: K must be a multiple of 64 for M > 16")
    s = finalize_split(split_m or M, N, K) if ksplit == 1 and epi in _FIN_EPIS else 1
    if s > 1:   # small-M prefill: split K into fp32 slabs, then the epilogue in pg_gemm_finalize
        part = torch.empty(s, M, N, dtype=torch.float32, device=out.device)
        _lib.call("pg_gemm", _p(A), A.stride(0), _p(W), W.stride(0), _p(bias), _p(part), N, M, N, K,
                  (flags & ~0xFF) | EPI_F32, s, None, 0, None, 0, 0, _s())
        _lib.call("pg_gemm_finalize", _p(part), s, _p(out), ldc, M, N, epi, _p(aux_out), aux_ld, aux_n, None, _s())
        return out
    _lib.call("pg_gemm", _p(A), A.stride(0), _p(W), W.stride(0), _p(bias), _p(out), ldc, M, N, K, flags, ksplit,
              _p(aux), aux_rows, _p(aux_out), aux_ld, aux_n, _s())
    return out


EPI_FP8 = 0x200   # PG_FP8: A and W fp8 e4m3 with row scales (include/pghip.h)


def quant_fp8(x: torch.Tensor, q: Optional[torch.Tensor] = None, scale: Optional[torch.Tensor] = None,
              M: Optional[int] = None):
    """Row quantisation bf16 [M][K] -> (fp8 e4m3 bytes [M][K] as uint8, fp32 scale [M]) (pg_quant_fp8)."""
    _chk(x, torch.bfloat16, "x")
    M = x.shape[0] if M is None else M
    K = x.shape[1]
    if q is None:
        q = torch.empty(M, K, dtype=torch.uint8, device=x.device)
    if scale is None:
        scale = torch.empty(M, dtype=torch.float32, device=x.device)
    if q.dtype != torch.uint8 or q.stride(1) != 1 or x.stride(1) != 1 or q.shape[1] < K or scale.numel() < M:
        raise ValueError("pghip.quant_fp8: bad output buffers")
    _lib.call("pg_quant_fp8", _p(x), x.stride(0), M, K, _p(q), q.stride(0), _p(scale), _s())
    return q, scale


def gemm8(A8: torch.Tensor, a_scale: Optional[torch.Tensor], W8: torch.Tensor, w_scale: torch.Tensor,
          out: torch.Tensor, *, epi: int = EPI_BF16, M: Optional[int] = None, bias: Optional[torch.Tensor] = None,
          ksplit: int = 1, fa=None, frag: bool = False, mx_in: Optional[torch.Tensor] = None,
          mx_out: Optional[torch.Tensor] = None, ss_in: Optional[torch.Tensor] = None,
          eps: float = 1e-6) -> torch.Tensor:
    """fp8 GEMM: out = epilogue((A8 . W8^T) * a_scale[m] * w_scale[n]) (PG_FP8, pg_gemm_fused).  A8, W8 are
    uint8 tensors of e4m3 bytes; `fa` (fused_args) carries the RoPE/KV epilogue arguments for EPI_QKV_ROPE.
    frag: W8 is fp8 fragment-packed (weights.frag_pack8) -> the weight-streaming fp8 GEMV, M <= 32.
    MX rows: mx_in = A8's E8M0 block scales (EPI_F32; a_scale None), mx_out = the scales a gelu*up launch writes
    beside its e4m3 h (out uint8 [M][N/2]).  Layout: frag (decode GEMV) [M][4][K/128]; tile (M > 32, the prefill, ABI
    12) [M][K/32], block b of row m at m*K/32 + b.  ss_in (frag, with mx_in, rows from norm_residual_mx): the outputs
    are multiplied by each row's RMSNorm rstd."""
    for t, n in ((A8, "A8"), (W8, "W8")):
        if t.dtype != torch.uint8 or not t.is_cuda or t.stride(1) != 1:
            raise ValueError(f"pghip.gemm8: {n} must be a row-major uint8 (e4m3) HIP tensor")
    if mx_in is None:
        _chk(a_scale, torch.float32, "a_scale")
    _chk(w_scale, torch.float32, "w_scale")
    M = A8.shape[0] if M is None else M
    N, K = W8.shape
    fa = fused_args() if fa is None else fa
    fa.a_scale = a_scale.data_ptr() if a_scale is not None else None
    fa.w_scale = w_scale.data_ptr()
    for t, n, numel in ((mx_in, "mx_in", M * K // 32), (mx_out, "mx_out", M * N // 64)):
        if t is None:
            continue
        if (t.dtype != torch.uint8 or not t.is_cuda or not t.is_contiguous() or t.numel() < numel
                or (not frag and M <= 32)):
            raise ValueError(f"pghip.gemm8: {n} must be a contiguous uint8 HIP tensor of >= {numel} E8M0 scales "
                             "(the fp8 GEMV, or the tile GEMM at M > 32)")
        setattr(fa, n, t.data_ptr())
    if ss_in is not None:
        _chk(ss_in, torch.float32, "ss_in")
        if mx_in is None or ss_in.stride(-1) != 1 or K % 1024 or not 0 < K // 1024 <= 4 or ss_in.shape[-1] < K // 1024:
            raise ValueError("pghip.gemm8: ss_in needs mx_in and fp32 [M][K/1024] sums of squares (K <= 4096)")
        fa.ss_in, fa.ss_ld, fa.ss_n, fa.eps = ss_in.data_ptr(), ss_in.stride(-2), K // 1024, float(eps)
    e = epi & 0xFF
    ldc = out.stride(-2) if out.dim() >= 2 else out.shape[-1]
    if frag:
        if M > 32:
            raise ValueError("pghip.gemm8: the fp8 GEMV takes at most 32 rows")
        _lib.call("pg_gemm_fused", _p(A8), A8.stride(0), _p(W8), W8.stride(0), _p(bias), _p(out), ldc, M, N, K,
                  e | EPI_FP8 | W_FRAG, ksplit, _lib.C.byref(fa), _s())
        return out
    s = finalize_split(M, N, K // 2) if ksplit == 1 and e in _FIN_EPIS and mx_out is None else 1
    if s > 1:   # small M: fp32 slabs, then the epilogue (scales already applied inside the slabs)
        part = torch.empty(s, M, N, dtype=torch.float32, device=out.device)
        _lib.call("pg_gemm_fused", _p(A8), A8.stride(0), _p(W8), W8.stride(0), _p(bias), _p(part), N, M, N, K,
                  EPI_F32 | EPI_FP8, s, _lib.C.byref(fa), _s())
        _lib.call("pg_gemm_finalize", _p(part), s, _p(out), ldc, M, N, e, None, 0, 0, _lib.C.byref(fa), _s())
        return out
    _lib.call("pg_gemm_fused", _p(A8), A8.stride(0), _p(W8), W8.stride(0), _p(bias), _p(out), ldc, M, N, K,
              e | EPI_FP8, ksplit, _lib.C.byref(fa), _s())
    return out


def gemm8_hx(H: torch.Tensor, amax: torch.Tensor, amax_ld: int, W8: torch.Tensor, w_scale: torch.Tensor,
             out: torch.Tensor, *, M: int, ksplit: int, bias: Optional[torch.Tensor] = None) -> torch.Tensor:
    """The fp8 GEMV (fragment-packed W8, EPI_F32 slabs) on bf16 rows H quantised in its prologue (pro_mode 5):
    row m's scale is amax[m * amax_ld] (float bits of max |H[m]|, max-ed by a gemm8 gelu*up launch with
    amax_out) / 448 -- the bytes and scale quant_fp8(H) would give, without its launch.  K / 128 / ksplit must be
    8 or 16."""
    _chk(H, torch.bfloat16, "H")
    _chk(w_scale, torch.float32, "w_scale")
    if W8.dtype != torch.uint8 or not W8.is_cuda or amax.dtype != torch.int32 or not amax.is_cuda:
        raise ValueError("pghip.gemm8_hx: W8 uint8 (fragment-packed e4m3) and amax int32 HIP tensors")
    N, K = W8.shape
    if M > 32 or (K // 128) % ksplit or (K // 128 // ksplit) not in (8, 16) or amax.numel() < M * amax_ld:
        raise ValueError("pghip.gemm8_hx: M <= 32, K / 128 / ksplit in (8, 16), amax [M * amax_ld]")
    fa = fused_args(pro_mode=5, amax_in=amax, amax_ld=amax_ld, w_scale=w_scale)
    ldc = out.stride(-2) if out.dim() >= 2 else out.shape[-1]
    _lib.call("pg_gemm_fused", _p(H), H.stride(0), _p(W8), W8.stride(0), _p(bias), _p(out), ldc, M, N, K,
              EPI_F32 | EPI_FP8 | W_FRAG, ksplit, _lib.C.byref(fa), _s())
    return out


def fused_args(**kw) -> "_lib.PgFusedArgs":
    """Build a PgFusedArgs; tensors are passed as their data pointers."""
    fa = _lib.PgFusedArgs()
    for k, v in kw.items():
        setattr(fa, k, v.data_ptr() if isinstance(v, torch.Tensor) else v)
    return fa


def gemm_fused(A: Optional[torch.Tensor], W: torch.Tensor, out: torch.Tensor, fa, *, epi: int = EPI_BF16,
               M: int, bias: Optional[torch.Tensor] = None, ksplit: int = 1, N: Optional[int] = None,
               ldc: Optional[int] = None, keep=None) -> torch.Tensor:
    """pg_gemm_fused: the GEMM with a fused prologue (x produced in-kernel) and/or RoPE/KV epilogue.
    `fa` is a PgFusedArgs (see fused_args); `keep` holds tensors it points to alive for the call."""
    _chk(W, torch.bfloat16, "W")
    _chk_frag(W, epi)
    if (epi & 0xFF) == EPI_FX_ADD:
        _chk(out, torch.int64, "out (the fixed-point accumulator)")
    N = W.shape[0] if N is None else N
    K = W.shape[1]
    if ldc is None:
        ldc = out.stride(-2) if out.dim() >= 2 else out.shape[-1]
    lda = A.stride(0) if A is not None else K
    s = finalize_split(M, N, K) if (fa.pro_mode == 0 and A is not None and ksplit == 1 and
                                    (epi & 0xFF) in _FIN_EPIS) else 1
    if s > 1:   # small-M prefill: split K into fp32 slabs, then the (RoPE / KV-append) epilogue
        part = torch.empty(s, M, N, dtype=torch.float32, device=out.device)
        _lib.call("pg_gemm", _p(A), lda, _p(W), W.stride(0), _p(bias), _p(part), N, M, N, K,
                  (epi & ~0xFF) | EPI_F32, s, None, 0, None, 0, 0, _s())
        _lib.call("pg_gemm_finalize", _p(part), s, _p(out), ldc, M, N, epi & 0xFF, None, 0, 0,
                  _lib.C.byref(fa), _s())
        return out
    _lib.call("pg_gemm_fused", _p(A), lda, _p(W), W.stride(0), _p(bias), _p(out), ldc, M, N, K, epi, ksplit,
              _lib.C.byref(fa), _s())
    return out


def norm_residual(resid: torch.Tensor, w: torch.Tensor, *, b: Optional[torch.Tensor] = None,
                  mode: int = NORM_RMS, eps: float = 1e-6, partials: Optional[torch.Tensor] = None,
                  nsplit: int = 0, out: Optional[torch.Tensor] = None, out_f32: Optional[torch.Tensor] = None,
                  row_map: Optional[torch.Tensor] = None, write_resid: bool = True):
    _chk(resid, torch.float32, "resid")
    M, H = resid.shape[-2], resid.shape[-1]
    M_out = row_map.numel() if row_map is not None else M
    ldo = out.stride(-2) if out is not None else H
    _lib.call("pg_norm_residual", _p(resid), _p(partials), nsplit, M, _p(w), _p(b), _p(out), ldo, _p(out_f32),
              _p(row_map), M_out, H, mode, float(eps), int(write_resid), _s())


def norm_residual_fp8(resid: torch.Tensor, w: torch.Tensor, q: torch.Tensor, scale: torch.Tensor, *,
                      b: Optional[torch.Tensor] = None, mode: int = NORM_RMS, eps: float = 1e-6,
                      partials: Optional[torch.Tensor] = None, nsplit: int = 0, write_resid: bool = True):
    """norm_residual with the output quantised to fp8 e4m3 rows (q uint8 [M][H], scale fp32 [M]) for a
    PG_FP8 GEMM; the bytes equal quant_fp8 of the bf16 output (pg_norm_residual_fp8)."""
    _chk(resid, torch.float32, "resid")
    M, H = resid.shape[-2], resid.shape[-1]
    if q.dtype != torch.uint8 or q.stride(-1) != 1 or q.shape[-1] < H or scale.numel() < M:
        raise ValueError("pghip.norm_residual_fp8: bad output buffers")
    _lib.call("pg_norm_residual_fp8", _p(resid), _p(partials), nsplit, M, _p(w), _p(b), _p(q), q.stride(-2),
              _p(scale), None, M, H, mode, float(eps), int(write_resid), _s())
    return q, scale


def norm_residual_mx(resid: torch.Tensor, w: torch.Tensor, q: torch.Tensor, qs: torch.Tensor, ss: torch.Tensor, *,
                     partials: Optional[torch.Tensor] = None, nsplit: int = 0, write_resid: bool = True):
    """Gemma RMSNorm feeding an MX fp8 GEMV (pg_norm_residual_mx): resid += sum of the partials' first nsplit slabs,
    q uint8 [M][H] = e4m3 of resid*(1+w) with E8M0 block scales qs uint8 [M*H/32] ([M][4][H/128]), ss fp32
    [M][H/1024] sums of squares; gemm8(..., mx_in=qs, ss_in=ss) applies rstd.  Returns (q, qs, ss)."""
    _chk(resid, torch.float32, "resid")
    _chk(w, torch.float32, "w")
    M, H = resid.shape[-2], resid.shape[-1]
    if (q.dtype != torch.uint8 or q.stride(-1) != 1 or q.shape[-1] < H or q.shape[0] < M or qs.dtype != torch.uint8
            or not qs.is_contiguous() or qs.numel() < M * H // 32 or ss.dtype != torch.float32
            or ss.stride(-1) != 1 or ss.shape[-1] < H // 1024 or ss.shape[0] < M or H % 1024):
        raise ValueError("pghip.norm_residual_mx: bad output buffers (q uint8 [M][H], qs uint8 [M*H/32], "
                         "ss fp32 [M][H/1024], H % 1024 == 0)")
    if nsplit and (partials is None or partials.dtype != torch.float32):
        raise ValueError("pghip.norm_residual_mx: fp32 partials needed for nsplit > 0")
    _lib.call("pg_norm_residual_mx", _p(resid), _p(partials), nsplit, M, _p(w), _p(q), q.stride(-2), _p(qs), _p(ss),
              ss.stride(-2), M, H, int(write_resid), _s())
    return q, qs, ss


def attention(q, q_rs, o, o_rs, k, k_bs, k_hs, k_rs, vt, vt_bs, vt_hs, vt_ds, *, B, Lq, Lkv, Hq, Hkv, D,
              scale, mask=None, mask_bs=0, mask_rs=0, lkv_dev=None, split_keys=0, nsplit=0, part_o=None,
              part_ml=None, kcap=0, kd=None, vd=None):
    """q/k/vt/o are base tensors (bf16) with explicit element strides (see include/pghip.h).  kcap (decode): the
    static cache's row capacity Smax, so each split's first K/V block is loaded before the kv length arrives; the
    decode kernels then read K and V from the decode-order copies kd / vd (decode_cache_pack)."""
    _lib.call("pg_attention", _p(q), q_rs, _p(o), o_rs, _p(k), k_bs, k_hs, k_rs, _p(vt), vt_bs, vt_hs, vt_ds,
              _p(mask), mask_bs, mask_rs, B, Lq, Lkv, _p(lkv_dev), Hq, Hkv, D, float(scale), split_keys, nsplit,
              _p(part_o), _p(part_ml), int(kcap), _p(kd), _p(vd), _s())


def decode_cache_pack(k: torch.Tensor, vt: torch.Tensor, Hkv: int):
    """The decode-order copies (kd, vd) [B][Hkv][Smax][D] of a canonical cache (k [B][Smax][Hkv*D], vt [B][Hkv*D][Smax])
    -- what the QKV epilogue writes beside the canonical cache (csrc/attn_common.h dec_koff / dec_voff); for tests
    and benchmarks that build a cache by hand.  Smax % 32 == 0, D % 16 == 0."""
    B, S, KV = k.shape
    D = KV // Hkv
    nb = S // 32
    # K: key 32 blk + 8 q + 4 h + j  <->  [blk][h][D/8 chunk][row 4q + j][8]
    kd = (k.reshape(B, nb, 4, 2, 4, Hkv, D // 8, 8).permute(0, 5, 1, 3, 6, 2, 4, 7)
          .reshape(B, Hkv, S, D).contiguous())
    # V: key 32 blk + 8 g + e, dim 16 t + c  <->  [blk][t][g][c][e]
    vd = (vt.reshape(B, Hkv, D // 16, 16, nb, 4, 8).permute(0, 1, 4, 2, 5, 3, 6)
          .reshape(B, Hkv, S, D).contiguous())
    return kd, vd


PF_KEYSPLIT = os.environ.get("PG_PF_KEYSPLIT", "1") != "0"


def prefill_key_splits(B: int, Lq: int, Lkv: int, Hq: int, Hkv: int) -> int:
    """Key splits for an unmasked prefill attention whose grid of 64-row workgroups leaves most CUs idle (batch 1:
    pt-224 Gemma 33 workgroups, SigLIP 64): as many splits (<= 8, >= one 64-key block each) as keep the split grid
    within one round; 1 = unsplit.  Each split writes (O, m, l) partials that pg_attention merges itself."""
    wgs = math.ceil(Lq * (Hq // Hkv) / 64) * Hkv * B
    if not PF_KEYSPLIT or wgs >= 128:
        return 1
    return max(1, min(8, 256 // wgs, math.ceil(Lkv / 64)))


def prefill_split_workspace(B: int, Lq: int, Hq: int, Hkv: int, D: int, nks: int):
    """(part_o, part_ml) sizes in fp32 elements for prefill_key_splits' nks splits."""
    rows = B * Hkv * nks * Lq * (Hq // Hkv)
    return rows * ((D + 15) // 16 * 16), rows * 2


def attn_combine(part_o, part_ml, o, o_rs, *, B, Hq, Hkv, D, nsplit):
    _lib.call("pg_attn_combine", _p(part_o), _p(part_ml), B, Hq, Hkv, D, nsplit, _p(o), o_rs, _s())


# the module API's attention weights (modeling_*.py: SiglipAttention / GemmaAttention return them when asked): off by
# default -- the flash kernels never form the softmax matrix, which at pt-896 x32 is 34 GB per layer
ATTN_WEIGHTS = os.environ.get("PG_ATTN_WEIGHTS", "0") == "1"


def attn_probs(q, q_rs, k, k_bs, k_hs, k_rs, *, B, Lq, Lkv, Hq, Hkv, D, scale, mask=None, mask_bs=0, mask_rs=0,
               probs=True, out=None) -> torch.Tensor:
    """The attention weights [B][Hq][Lq][Lkv] fp32 with pg_attention's addressing (pg_attn_probs): the softmax
    probabilities (probs, GemmaAttention's second output) or the scaled scores before the softmax (SiglipAttention's),
    on request only."""
    if out is None:
        out = torch.empty(B, Hq, Lq, Lkv, dtype=torch.float32, device=q.device)
    if mask is not None:
        _chk(mask, torch.float32, "mask")
    _lib.call("pg_attn_probs", _p(q), q_rs, _p(k), k_bs, k_hs, k_rs, _p(mask), mask_bs, mask_rs, B, Lq, Lkv, Hq, Hkv,
              D, float(scale), int(bool(probs)), _p(out), _s())
    return out


DECODE_MAX_SPLITS = int(os.environ.get("PG_DECODE_MAX_SPLITS", "8"))


def decode_plan(B: int, Hkv: int, kcap: int):
    """(nsplit, nw, nb) of pg_attn_decode for a batch of B rows over a static cache of kcap keys: 4 waves per split
    and at most 8 splits per (row, kv head), the rounds following from the cache length.  The last split's workgroup
    merges every partial alone (8 KB each), so fewer splits win while the rounds stay few: measured per layer
    (attention + merge, profiles/r03_decode_attn_plans.txt) pt-448 x16 8 x 4 x 2 12.7 us vs 16 x 2 x 2 13.9 and
    5 x 4 x 2 13.1; pt-896 x32 8 x 4 x 5 31.9 vs 6 x 4 x 6 30.9, 16 x 4 x 3 37.8, 16 x 2 x 5 35.4."""
    nblk = kcap // 32
    nw = 4 if nblk >= 4 else 2
    nsplit = max(1, min(DECODE_MAX_SPLITS, nblk // nw))
    nb = -(-nblk // (nw * nsplit))
    return nsplit, nw, nb


# the staggered form of pg_attn_decode (PG_ATTN_PIPE flag on nw; head_dim 256, 4-wave splits, >= 2 rounds): the
# next block's K / V are issued between the current block's score and P.V phases
ATTN_PIPE = os.environ.get("PG_ATTN_PIPE", "1") != "0"
_ATTN_PIPE_FLAG = 0x100


def attn_decode(q, q_rs, o, o_rs, kd, vd, *, B, Lkv, lkv_dev, Hq, Hkv, D, scale, kcap, part_o, part_ml, counters,
                plan=None, q8=None, q8_scale=None):
    """Batched decode attention with the split merge in the same launch (pg_attn_decode): o[b][hq*D + d] bf16 from
    q (one position per row) over the decode-order cache copies kd / vd; part_o / part_ml / counters are workspaces
    (counters int32 [B*Hkv], zeroed once).  q8 uint8 [B][>= Hq*D] / q8_scale f32 [B] (optional, one kv head and a
    4-wave plan, see attn_decode_q8_ok): also the rows as fp8 e4m3, byte-identical to quant_fp8(o)."""
    nsplit, nw, nb = plan or decode_plan(B, Hkv, kcap)
    if q8 is not None:
        _chk(q8, torch.uint8, "q8")
        _chk(q8_scale, torch.float32, "q8_scale")
        if not attn_decode_q8_ok(Hq, Hkv, D, nw) or q8.shape[0] < B or q8_scale.numel() < B:
            raise ValueError("pghip.attn_decode: fp8 row copy needs one kv head, Hq*D/8 <= 64*nw and B rows")
    if part_o.numel() < B * Hkv * nsplit * 16 * D or part_ml.numel() < B * Hkv * nsplit * 16 * 2:
        raise ValueError("pghip.attn_decode: partial workspace too small")
    if counters.dtype != torch.int32 or counters.numel() < B * Hkv:
        raise ValueError("pghip.attn_decode: counters must be int32 [B*Hkv]")
    _lib.call("pg_attn_decode", _p(q), q_rs, _p(o), o_rs, _p(kd), _p(vd), B, Lkv, _p(lkv_dev), Hq, Hkv, D,
              float(scale), kcap, nsplit, nw | (_ATTN_PIPE_FLAG if ATTN_PIPE else 0), nb, _p(part_o), _p(part_ml), _p(counters), _p(q8), _p(q8_scale),
              q8.stride(0) if q8 is not None else 0, _s())


def attn_decode_q8_ok(Hq: int, Hkv: int, D: int, nw: int) -> bool:
    """Whether pg_attn_decode can also write the fp8 row copy: the merging workgroup must hold the whole row."""
    return Hkv == 1 and Hq * (D // 8) <= 64 * nw


def rope_kv_write(qkv, pos, cos_t, sin_t, kc, vtc, *, T, L, Hq, Hkv, D, Smax, slot_base=0, slot_dev=None):
    _chk(qkv, torch.bfloat16, "qkv")
    _chk(pos, torch.int32, "pos")
    _lib.call("pg_rope_kv_write", _p(qkv), qkv.stride(0), _p(pos), T, L, Hq, Hkv, D, _p(cos_t), _p(sin_t), _p(kc),
              _p(vtc), Smax, slot_base, _p(slot_dev), _s())


def patch_im2col(px: torch.Tensor, patch: int, out: torch.Tensor):
    _chk(px, torch.float32, "pixel_values")
    px = px.contiguous()
    B, C, H, W = px.shape
    _lib.call("pg_patch_im2col", _p(px), B, C, H, W, patch, _p(out), out.stride(0), _s())


def image_rank(ids: torch.Tensor, image_id: int, rank: torch.Tensor):
    _chk(ids, torch.int64, "input_ids")
    _lib.call("pg_image_rank", _p(ids), ids.numel(), int(image_id), _p(rank), _s())


def embed_merge(ids, rank, embed, feat, n_feat, out, *, image_id, pad_id, img_scale, normalizer):
    _chk(ids, torch.int64, "input_ids")
    V, H = embed.shape
    _lib.call("pg_embed_merge", _p(ids), _p(rank), ids.numel(), _p(embed), V, _p(feat), n_feat, H, int(image_id),
              int(pad_id), float(img_scale), float(normalizer), _p(out), _s())


def _rows(t: Optional[torch.Tensor], B: int) -> int:
    """Steps a [steps][B] decode-state buffer holds (its step-indexed writes/reads are bounded by this)."""
    return 0 if t is None else t.numel() // B


def argmax(logits, out_ids, workspace, *, hist=None, step=None, pos=None, kv_len=None):
    _chk(logits, torch.float32, "logits")
    B, V = logits.shape
    _lib.call("pg_argmax", _p(logits), logits.stride(0), B, V, _p(workspace), _p(out_ids), _p(hist), _rows(hist, B),
              _p(step), _p(pos), _p(kv_len), _s())


def argmax_embed(logits, out_ids, workspace, embed, feat, n_feat, res, *, image_id, pad_id, img_scale, normalizer,
                 hist=None, step=None, pos=None, kv_len=None):
    """argmax + the next step's input rows res[b] = embed_merge(winner_b) (one launch fewer per decode step)."""
    _chk(logits, torch.float32, "logits")
    _chk(res, torch.float32, "res")
    B, V = logits.shape
    Ve, H = embed.shape
    assert res.is_contiguous() and res.numel() >= B * H
    _lib.call("pg_argmax_embed", _p(logits), logits.stride(0), B, V, _p(workspace), _p(out_ids), _p(hist),
              _rows(hist, B), _p(step), _p(pos), _p(kv_len), _p(embed), Ve, _p(feat), int(n_feat), H, int(image_id),
              int(pad_id), float(img_scale), float(normalizer), _p(res), _s())


def argmax_pairs(logits, workspace, pairs, *, vocab_offset: int):
    _chk(logits, torch.float32, "logits")
    B, V = logits.shape
    _lib.call("pg_argmax_pairs", _p(logits), logits.stride(0), B, V, int(vocab_offset), _p(workspace), _p(pairs), _s())


def argmax_merge(pairs, out_ids, *, world: int, hist=None, step=None, pos=None, kv_len=None):
    B = out_ids.numel()
    _lib.call("pg_argmax_merge", _p(pairs), int(world), B, _p(out_ids), _p(hist), _rows(hist, B), _p(step), _p(pos),
              _p(kv_len), _s())


def topp_sample(logits, out_ids, uniforms, *, temperature, top_p, hist=None, step=None, pos=None, kv_len=None,
                probs_out=None):
    _chk(logits, torch.float32, "logits")
    B, V = logits.shape
    rows = _rows(uniforms, B) if hist is None else min(_rows(uniforms, B), _rows(hist, B))
    _lib.call("pg_topp_sample", _p(logits), logits.stride(0), B, V, float(temperature), float(top_p), _p(uniforms),
              _p(out_ids), _p(hist), rows, _p(step), _p(pos), _p(kv_len), _p(probs_out), _s())


def image_preprocess(src, H, W, S, hb, hk, hks, vb, vk, vks, y0, rows, lut, tmp, out):
    _chk(src, torch.uint8, "image")
    _chk(out, torch.float32, "pixel_values")
    _lib.call("pg_image_preprocess", _p(src), H, W, S, _p(hb), _p(hk), hks, _p(vb), _p(vk), vks, y0, rows, _p(lut),
              _p(tmp), _p(out), _s())


def synth_fill(out: torch.Tensor, seedmix: int, a: float, mean: float):
    kind = 0 if out.dtype == torch.bfloat16 else 1
    if kind == 1:
        _chk(out, torch.float32, "out")
    _lib.call("pg_synth_fill", _p(out), out.numel(), seedmix & 0xFFFFFFFF, float(a), float(mean), kind, _s())


_FIN_EPIS = (EPI_BF16, EPI_BF16_GELU, EPI_BF16_GELU_MUL, EPI_BF16_VT, EPI_QKV_ROPE)
FINALIZE_SPLIT = True   # tuning switch (scripts/tune): small-M bf16-epilogue GEMMs split K + pg_gemm_finalize


def finalize_split(M: int, N: int, K: int) -> int:
    """K split for a prefill GEMM whose epilogue needs full sums (bf16 / gelu / RoPE ...): used when its
    full-K tile grid (64x128 tiles, csrc/gemm.hip launch_tile) leaves most CUs idle, as at batch 1; the fp32
    slabs are then reduced by pg_gemm_finalize.  1 = one launch with the fused epilogue."""
    if not FINALIZE_SPLIT or M <= 16 or K % 64:
        return 1
    if math.ceil(M / 256) * math.ceil(N / 256) >= CUS:
        return 1
    tiles = math.ceil(M / 64) * math.ceil(N / 128)
    # measured per call, graph-replayed with the finalisation included (scripts/tune/small_gemm_sweep.py,
    # profiles/r03_small_gemm_sweep.txt): SigLIP q|k|v (108 tiles) 13.6 us unsplit vs 19.2 at split 3, fc1 (136)
    # 14.9 vs 21.9 at split 2 -- the finalisation launch and the fp32 slabs cost more than the idle CUs; Gemma
    # q|k|v (100 tiles) 17.2 at split 2 vs 20.9 unsplit / 21.7 at split 3
    if tiles > 100:
        return 1
    s = min(2, math.ceil(CUS / tiles), (K // 64) // 6)
    return s if s >= 2 else 1


def slab_sum(part: torch.Tensor, out: torch.Tensor) -> torch.Tensor:
    """out[M][N] (fp32, row stride out.stride(0)) = sum over the slabs of part[s][M][N] (pg_gemm_finalize, PG_EPI_F32)."""
    _chk(part, torch.float32, "part")
    _chk(out, torch.float32, "out")
    S, M, N = part.shape
    if not part.is_contiguous() or out.shape != (M, N) or out.stride(1) != 1:
        raise ValueError("pghip.slab_sum: part must be contiguous [S][M][N] and out [M][N] with unit column stride")
    _lib.call("pg_gemm_finalize", _p(part), S, _p(out), out.stride(0), M, N, EPI_F32, None, 0, 0, None, _s())
    return out


def split_for(tiles: int, k_steps: int, target: int = 256, max_split: int = 4) -> int:
    """split-K factor: the most splits with tiles * split <= target (one round of workgroups), keeping >= 2
    k-steps per split.  (Rounding up to fill every CU measured worse: the Gemma o projection at batch 1, 80 tiles,
    10.3 us at split 3 vs 14.9 at split 4 -- the fourth split starts a second round; profiles/r03_tile_sweep.txt.)"""
    s = max(1, min(max_split, target // max(tiles, 1), k_steps // 2))
    return s


CUS = 256   # MI355X compute units


def gemm_ksplit(M: int, N: int, K: int) -> int:
    """split-K factor for an fp32-partial (EPI_F32) prefill GEMM, mirroring libpghip's tile choice.
    Large M (a 256x256 grid of >= 256 tiles, csrc/gemm.hip gemm256_kernel): the split that best fills the
    last round of one-workgroup-per-CU tiles, each extra split charged its partial-slab round trip
    (2*M*N*4 B at ~5 TB/s against 2*M*N*K flop at ~1 PF/s, i.e. 800/K of the GEMM per split).
    Smaller M: as many splits of the 64x128 tiles as keep one round of workgroups (split_for)."""
    t256 = math.ceil(M / 256) * math.ceil(N / 256)
    if t256 >= CUS:
        kt = K // 64
        best, best_s = -1.0, 1
        for s in (1, 2, 3, 4):
            if s > 1 and kt // s < 8:
                break
            u = t256 * s
            eff = u / (math.ceil(u / CUS) * CUS) - 800.0 / K * (s - 1)
            if eff > best + 1e-9:
                best, best_s = eff, s
        return best_s
    # few 256x256 tiles (prefill at batch 1): a K split deep enough to give every CU one 256-row tile, when
    # each slice keeps >= 8 k-tiles (W then streams once instead of once per 64-row tile)
    s256 = math.ceil(CUS / t256)
    if s256 <= min(16, (K // 64) // 8):
        return s256
    # up to 6 splits: SigLIP o / fc2 at batch 1 (36 tiles) 6.1 / 11.4 us at split 6 vs 6.8 / 13.6 at 4, slower again
    # at 9 (profiles/r03_small_gemm_sweep.txt)
    return split_for(math.ceil(M / 64) * math.ceil(N / 128), K // 64, max_split=6)
