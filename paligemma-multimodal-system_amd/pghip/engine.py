"""PaliGemma image->text engine on libpghip (one process per GPU).

Restates PaliGemmaForConditionalGeneration.forward (modeling_paligemma.py:257-308)
and the test_inference token loop (inference.py:45-82) as a fixed sequence of
HIP kernels:

  vision (once per request)  im2col -> patch GEMM(+bias+pos) -> 27 x [LN -> QKV GEMM(+bias, V^T)
                             -> attention -> out GEMM(split-K partials) -> LN(+partials) -> fc1 GEMM(+gelu)
                             -> fc2 GEMM(partials)] -> post-LN -> projector GEMM
  prefill                    rank scan -> embed merge -> 18 x [RMSNorm(+partials) -> QKV GEMM -> RoPE+KV write
                             -> attention -> o GEMM(partials) -> RMSNorm -> gate/up GEMM(gelu*mul) -> down GEMM
                             (partials)] -> final RMSNorm -> lm_head GEMM(+bias)
  decode step                the same per token with the GEMV kernels, split-KV attention, argmax / top-p;
                             every per-step scalar (kv length, positions, step) lives in device memory,
                             so one step is captured once as a hipGraph and replayed.

Output-invariant deviations from the reference: the vision
tower runs once per request instead of on every call (modeling_paligemma.py:281);
the KV cache is a static in-place buffer instead of torch.cat (modeling_gemma.py:54-55);
the generation loop computes only last-position logits.

Tensor parallelism (PackedWeights(tp_rank, tp_world) + a TPComm): every rank runs the same
kernel sequence on its head / intermediate / vocabulary slice.  The partial sums of o_proj and
down_proj are completed by one SUM all-reduce of ONE fp32 slab per sub-block (a rank's split-K
slabs are summed locally first); at prefill sizes the rows are cut into chunks and each chunk's
all-reduce runs on the communication stream while the next chunk's GEMM runs (_row_parallel).
Greedy decoding all-gathers per-rank (max, index) pairs, full logits are all-gathered by
vocabulary slice, and with at least one image per rank the SigLIP tower runs data-parallel over
the images, its features all-gathered.
"""
from __future__ import annotations

import math
import os
from typing import Optional

import torch

from . import ops
from .tp import CaptureUnsupported, SoloComm
from .weights import PackedWeights


def _rup(x: int, m: int) -> int:
    return (x + m - 1) // m * m


def rope_tables(dim: int, n_pos: int, base: float, device):
    """cos/sin [n_pos][dim/2] exactly as GemmaRotaryEmbedding (modeling_gemma.py:112,121-135):
    inv_freq = 1/base^(arange(0,dim,2)/dim) in fp32, freqs = inv_freq * pos (fp32), cos/sin in fp32.
    Computed with torch on the CPU (the reference's own arithmetic), then uploaded."""
    inv = 1.0 / (base ** (torch.arange(0, dim, 2, dtype=torch.int64).float() / dim))
    pos = torch.arange(n_pos, dtype=torch.int64).float()
    freqs = inv[None, :] * pos[:, None]
    return freqs.cos().to(device).contiguous(), freqs.sin().to(device).contiguous()


class KVStore:
    """Static KV cache: K [layers][B][Smax][nkv*hd] (roped), V^T [layers][B][nkv*hd][Smax], bf16, plus the
    decode-order copies kd / vd [layers][B][nkv][Smax][hd] that the QKV epilogue writes beside them and the decode
    attention kernels read (csrc/attn_common.h dec_koff / dec_voff: one contiguous KiB per load instruction)."""

    def __init__(self, layers: int, B: int, Smax: int, kv_dim: int, device, kv_heads: int = 1):
        if kv_dim % kv_heads:
            raise ValueError(f"kv_dim {kv_dim} does not split into {kv_heads} kv heads")
        self.B, self.Smax, self.kv_dim, self.kv_heads = B, Smax, kv_dim, kv_heads
        self.k = torch.zeros(layers, B, Smax, kv_dim, dtype=torch.bfloat16, device=device)
        self.vt = torch.zeros(layers, B, kv_dim, Smax, dtype=torch.bfloat16, device=device)
        self.kd = torch.zeros(layers, B * Smax * kv_dim, dtype=torch.bfloat16, device=device)
        self.vd = torch.zeros(layers, B * Smax * kv_dim, dtype=torch.bfloat16, device=device)
        self.length = 0

    def copy_prefix_from(self, old: "KVStore", n: int):
        """Grow: the first n positions of every layer of a smaller store (canonical and decode-order copies)."""
        nl = old.k.shape[0]
        self.k[:nl, :, :n] = old.k[:, :, :n]
        self.vt[:nl, :, :, :n] = old.vt[:, :, :, :n]
        if (old.B, old.kv_dim, old.kv_heads) != (self.B, self.kv_dim, self.kv_heads):
            raise ValueError("copy_prefix_from: the stores differ in batch or kv-head layout")
        nb = -(-n // 32) * 32                     # decode-order copies hold whole 32-key blocks per (row, kv head)
        hk, hd = self.kv_heads, self.kv_dim // self.kv_heads
        for t_new, t_old in ((self.kd, old.kd), (self.vd, old.vd)):   # [layers][B][Hkv][Smax][hd] (dec_koff / voff)
            t_new.view(-1, self.B, hk, self.Smax, hd)[:nl, :, :, :nb] = t_old.view(nl, old.B, hk, old.Smax, hd)[:, :, :, :nb]


class PaliGemmaEngine:
    DECODE_SPLIT_O = 2      # split-K of o_proj at decode (B > FUSE_MAX_B: more workgroups for the batched GEMV)
    DECODE_SPLIT_O_SMALL = 2  # ... at B <= FUSE_MAX_B: split 2 (256 workgroups, tile finalised by the second arriver).
                              # Unsplit won earlier this round (1.120-1.122 vs 1.123-1.127 ms/token); with the q|k|v
                              # weights Infinity-Cache resident split 2 wins 7 of 8 interleaved pairs, -3.7 us mean
                              # (scripts/r02/gpu_s3r.sh)
    # 5..16 rows on the in-kernel-finalised path (F32_FIN): o_proj unsplit and down_proj split 4 (pt-448 x16: 1.391 vs
    # 1.405 ms/step at 2 / 8, profiles/r05_decode_splits_pt448x16.jsonl); PG_SPLIT_O / PG_SPLIT_DOWN override
    DECODE_SPLIT_O_FIN16, DECODE_SPLIT_DOWN_FIN16 = 1, 4
    DECODE_SPLIT_DOWN = 8   # split-K of down_proj at decode (8 vs 4: -4..6 us per pt-224 step, scripts/r02/gpu_t.sh)
    DECODE_SPLIT_KEYS = 32  # keys per wave in split-KV decode attention (one MFMA block)
    # keys per split at B <= FUSE_MAX_B: every o_proj workgroup merges all active splits in its prologue, so
    # fewer, longer splits (one wave per 32 keys, merged in LDS by attn_decode_wg_kernel) cut that re-read
    DECODE_SPLIT_KEYS_SMALL = int(os.environ.get("PG_SK_SMALL", "32"))
    # prefill GEMMs of at least this many rows read the row-major weight copies (weights.prefill_rowmajor)
    PREFILL_ROWMAJOR_MIN_M = int(os.environ.get("PG_ROWMAJOR_MIN_M", "256"))
    ROW_BLOCKS = os.environ.get("PG_ROW_BLOCKS", "1") != "0"   # ragged fp32-slab GEMMs as head + tail launches
    TAIL_SPLIT = os.environ.get("PG_TAIL_SPLIT", "1") != "0"   # ... the tail with its own deeper split-K
    HEAD_KSPLIT = os.environ.get("PG_HEAD_KSPLIT", "1") != "0"  # ... and the split-K chosen for the head
    ROW_BLOCKS_GU = os.environ.get("PG_ROW_BLOCKS_GU", "1") != "0"  # gate/up (bf16 gelu*up) as row blocks too
    # ragged-N SigLIP GEMMs as head + tail launches: measured neutral at pt-448 x16 and pt-896 x32 (the small-tile
    # tail costs what the saved round gave back; scripts/tune/run_s4_p.sh), so off
    COL_BLOCKS = os.environ.get("PG_COL_BLOCKS", "0") == "1"
    # batch-1 prefill (256 <= rows <= 288): these Gemma linears run as ONE row tile per 128 columns (PG_TILE_M1),
    # with this split-K -- each weight tile streams once instead of once per 256-row tile.  Per call at 264 rows
    # (scripts/tune/skinny_bench.py, profiles/r02_skinny_gemm_*.txt): gate/up 60.8 -> 52.8 us, down 38.9 -> 33.5,
    # o 15.2 -> 14.1.  The q|k|v / SigLIP epilogues cannot split K, so their one-tile grids would idle most CUs.
    TILE_M1 = os.environ.get("PG_TILE_M1", "1") != "0"
    # (o left the table: 64-row tiles at split 3 take 10.3 us against 12.7-13.5 for one row tile at split 8-12,
    # and leave 3 slabs instead of 8 for the RMSNorm; profiles/r03_tile_sweep.txt)
    TILE_M1_SPLIT = {"gu": 1, "down": int(os.environ.get("PG_M1_DOWN", "16"))}
    FUSE_MAX_B = 2          # decode batches up to this size fuse RMSNorm / attention merge into the GEMVs
    DECODE_SPLIT_TARGET = 1024  # B > FUSE_MAX_B: aim for about this many decode-attention splits (waves)
    # long KV x batch: splits of several 32-key rounds per wave sized to one round of workgroups (_split_keys).
    # Measured level with the 128-key splits (pt-896 x32: 51.8 vs 51.1 us per layer, attention + merge, same box;
    # profiles/r03_decode_attn_bench.txt), so off
    DECODE_ONE_ROUND = os.environ.get("PG_DECODE_ONE_ROUND", "0") == "1"
    FIN_MIN_B = 5           # FIN_MIN_B <= B <= 16: in-kernel finalisation with the merge as its own kernel
    USE_FIN = True          # single rank: split-K slabs finalised in-kernel (see _decode_layers_fin)
    # tensor parallel: SigLIP data-parallel over the images when every rank gets at least one (else replicated)
    VISION_DP = os.environ.get("PG_VISION_DP", "1") != "0"
    # tensor-parallel prefill: rows per all-reduce chunk (each chunk's all-reduce overlaps the next chunk's GEMM)
    AR_CHUNK_ROWS = int(os.environ.get("PG_AR_CHUNK_ROWS", "4096"))
    # chained greedy decode (single rank): the argmax's final launch also writes the next step's input rows
    # (pg_argmax_embed), so a decode step starts at layer 0 with no embed launch (decode_state(sampler=...))
    CHAIN_EMBED = os.environ.get("PG_CHAIN_EMBED", "1") != "0"
    # 17..32-row fp8 decode: the down GEMV quantises h itself from the row maxima the gate/up epilogue collects
    # (ops.gemm8_hx) instead of the pg_quant_fp8 launch between them.  Same bytes either way; measured slower at
    # pt-896 x32 (r4 timelines: down 10.0 -> 15.7 us with 16 slabs, 18.0 with 8; gate/up +1.2 us for the
    # atomics; the quantiser it removes costs 7.3 us), so off
    HQ_FUSED = os.environ.get("PG_HQ_FUSED", "0") != "0"

    # 17..32-row fp8 decode MLP on MX rows: the gate/up epilogue writes h as e4m3 with one E8M0 scale per 32
    # columns (PgFusedArgs.mx_out) and the down GEMV reads those block scales into its MFMAs (mx_in) -- no
    # quantiser launch and no cross-workgroup row maximum (the block max stays inside one workgroup)
    MX_H = os.environ.get("PG_MX_H", "1") != "0"
    # ... and the RMSNorms in front of the q|k|v, gate/up and lm_head GEMVs write MX rows of x*(1+w) with per-1024-column
    # sums of squares (pg_norm_residual_mx: one workgroup per 1024 columns and row, no row-wide reduction); the GEMV applies
    # rstd to its outputs.  Replaces the norm + per-row quantiser pair
    MX_NORM = os.environ.get("PG_MX_NORM", "1") != "0"
    # fp8 prefill MLP on MX h too (ABI 12): the 128 x 128 fp8 gate/up tile writes h as e4m3 + one E8M0 scale per 32
    # columns (each wave owns one block per row) and the 256 x 256 fp8 down GEMM stages the block scales beside h --
    # the row quantiser launch between them (and half of h's bytes) is gone
    MX_PREFILL = os.environ.get("PG_MX_PREFILL", "1") != "0"
    # prefill linears that end a residual branch (SigLIP o / fc2, Gemma o / down) with ONE split on one rank add into
    # the residual in their epilogue (PG_EPI_F32_RES, ABI 13): the next norm reads the residual alone, 4 B per element
    # less than a slab write + slab read + residual rewrite; bit-identical (the same one fp32 add)
    PREFILL_RES = os.environ.get("PG_PREFILL_RES", "1") != "0"
    # ... from this many rows on: pt-896 x32 prefill 672-675 -> 665-667 ms; at pt-448 x16 (16 k rows) level to 0.5%
    # slower (85.4-85.6 vs 84.9-85.1 ms; profiles/r06_prefill_res_ab.jsonl), so off there
    PREFILL_RES_MIN_M = int(os.environ.get("PG_PREFILL_RES_MIN_M", "65536"))

    AMAX_LD = 32                     # one 128-B line per row maximum (the gate/up atomics of 32 rows spread out)
    # 128-k chunks of h per down workgroup (8 or 16): bf16 h costs twice fp8's bytes per workgroup, so the split
    # doubles instead (pt-896: 16 slabs of 8 chunks, as many x bytes per workgroup as the 8-slab fp8 route)
    HQ_CHUNKS = int(os.environ.get("PG_HQ_CHUNKS", "8"))
    # B > FUSE_MAX_B: split-KV attention and its merge in one launch (pg_attn_decode; 0 = split kernel + combine)
    DECODE_FUSED_ATTN = os.environ.get("PG_DECODE_FUSED", "1") != "0"
    FUSED_MIN_ROUNDS = int(os.environ.get("PG_FUSED_MIN_ROUNDS", "2"))   # ... used from this many rounds per split on
    # fp8 decode (> 16 rows): the one-launch attention also writes its rows as e4m3 for the fp8 o_proj (no
    # pg_quant_fp8 launch; same bytes)
    ATTN_FP8_OUT = os.environ.get("PG_ATTN_FP8_OUT", "1") != "0"
    # B <= FUSE_MAX_B single rank: row-parallel decode linears that add their split-K partials straight into the
    # residual instead of finalising slabs in-kernel (F32_FIN's slab store -> ticket -> slab load tail); the next GEMV
    # then normalises the residual itself (PRO_RMSNORM).  "fx" (default): o_proj and down_proj add into a fixed-point
    # int64 accumulator with integer atomics (PG_EPI_FX_ADD) -- the sum is exact, so decode is bit-reproducible run to
    # run; "both": the same with float atomics into the fp32 residual (unordered: ~1 ulp run-to-run drift); "down":
    # down_proj only, float atomics; "0": off (F32_FIN, deterministic).  The last layer's down_proj always finalises
    # (F32_FIN), its x' and sums of squares feeding the lm_head
    DECODE_ADD = os.environ.get("PG_DECODE_ADD", "fx")
    # fp8 linears of 17..32 rows (batched decode, the lm_head of a 17..32-row batch) on the weight-streaming fp8 GEMV
    # (fragment-packed e4m3 weights, csrc/gemm.hip gemv8_kernel) instead of the LDS-staged fp8 tile GEMM
    FP8_GEMV = os.environ.get("PG_FP8_GEMV", "1") != "0"
    DECODE_ADD_B32 = os.environ.get("PG_DECODE_ADD_B32", "0") == "1"   # (see _decode_layers_unfused)

    def __init__(self, cfg: dict, weights: PackedWeights, device="cuda", comm=None):
        self.cfg = cfg
        self.w = weights
        self.comm = comm if comm is not None else SoloComm()
        self.fp8 = bool(getattr(weights, "fp8", False))
        self.tp = getattr(weights, "tp_world", 1)
        if self.comm.world != self.tp:
            raise ValueError(f"weights packed for tp_world={self.tp}, communicator has world {self.comm.world}")
        self.split_o = self.DECODE_SPLIT_O if self.tp == 1 else 1        # smaller all-reduce messages under TP
        if os.environ.get("PG_SPLIT_O"):                                   # tuning overrides
            self.split_o = int(os.environ["PG_SPLIT_O"])
        self.split_down = self.DECODE_SPLIT_DOWN if self.tp == 1 else max(1, self.DECODE_SPLIT_DOWN // self.tp)
        if os.environ.get("PG_SPLIT_DOWN"):
            self.split_down = int(os.environ["PG_SPLIT_DOWN"])
        self._validate_splits()
        self.device = torch.device(device)
        self.image_token_id = cfg.get("image_token_index", 256000)
        pad = cfg.get("pad_token_id")
        self.pad_id = -1 if pad is None else pad
        self.n_img = weights.n_img
        self._rope = None
        self._rope_n = 0
        self._ws = {}
        self.graphs = {}

    # ------------------------------------------------------------------ helpers
    def _validate_splits(self):
        """Refuse split-K settings (tuning knobs included) that a kernel would reject at launch time, before any
        launch: the decode o / down GEMVs finalise in-kernel (PG_EPI_F32_FIN) with at most 8 splits."""
        w = self.w
        if not hasattr(w, "heads"):                     # vision-only pack (modeling_siglip.SiglipVisionModel)
            return
        checks = [("o_proj (PG_SPLIT_O)", self.split_o, w.heads * w.head_dim, 8),
                  ("o_proj at batch <= 2", self.DECODE_SPLIT_O_SMALL, w.heads * w.head_dim, 8),
                  ("down_proj (PG_SPLIT_DOWN)", self.split_down, w.inter, 8)]
        if self.TILE_M1:    # (a model too narrow for this split just skips the row-tile path, _tile_m1)
            checks.append(("batch-1 prefill down_proj (PG_M1_DOWN)", self.TILE_M1_SPLIT["down"], 64 * 64, 64))
        if self.HQ_CHUNKS not in (8, 16):
            raise ValueError(f"PG_HQ_CHUNKS {self.HQ_CHUNKS}: the bf16-h down GEMV stages 8 or 16 chunks")
        for what, ks, K, hi in checks:          # (a split past K's 64-wide chunks just computes a zero slab)
            if not 1 <= ks <= hi:
                raise ValueError(f"split-K {ks} for {what}: needs 1 <= split <= {hi} (K = {K})")

    def _buf(self, name, shape, dtype):
        t = self._ws.get(name)
        n = math.prod(shape)
        if t is None or t.numel() < n or t.dtype != dtype:
            t = torch.empty(max(n, 1), dtype=dtype, device=self.device)
            self._ws[name] = t
        return t[:n].view(*shape)

    def rope(self, n_pos: int):
        if self._rope is None or self._rope_n < n_pos:
            n = _rup(max(n_pos, 1024), 1024)
            self._rope = rope_tables(self.w.head_dim, n, self.w.rope_theta, self.device)
            self._rope_n = n
        return self._rope

    def new_cache(self, B: int, Smax: int) -> KVStore:
        w = self.w
        return KVStore(w.t_layers, B, _rup(Smax, 64), w.kv_heads * w.head_dim, self.device, kv_heads=w.kv_heads)

    # ------------------------------------------------------------------ vision tower
    def vision(self, pixel_values: torch.Tensor, want_hidden: bool = False, taps: Optional[list] = None,
               _split_batch: Optional[int] = None):
        """SiglipVisionModel.forward + projector (modeling_siglip.py:312-334, modeling_paligemma.py:60-65).
        Returns image features fp32 [B*N][P] (projector output, unscaled) and optionally the
        post-LN vision output fp32 [B*N][hv].  _split_batch (the data-parallel call of a rank's slice): choose the
        split-K and attention key splits as for a batch of that many images, so that each image's features are
        bit-identical to the single-rank run over the whole batch."""
        w = self.w
        px = pixel_values.to(device=self.device, dtype=torch.float32).contiguous()
        B = px.shape[0]
        if (_split_batch is None and self.tp > 1 and self.VISION_DP and B >= self.tp and B % self.tp == 0
                and not want_hidden and taps is None and w.proj_w is not None):
            # data-parallel over the images (output-invariant): this rank encodes its B/W images,
            # then the projected features [B*N][P] are all-gathered in rank order = image order.  The rank-local
            # call takes the whole batch's split choices, so the features equal the replicated run's bit for bit
            Bl = B // self.tp
            mine = self.vision(px[self.comm.rank * Bl:(self.comm.rank + 1) * Bl], _split_batch=B)
            feats = torch.empty(B * w.n_img, w.proj_dim, dtype=torch.float32, device=self.device)
            self.comm.all_gather(feats, mine)
            return feats
        N, hv, nh, hd = w.n_img, w.v_hidden, w.v_heads, w.v_head_dim
        M = B * N
        patches = self._buf("v_patches", (M, w.patch_k), torch.bfloat16)
        ops.patch_im2col(px, w.patch, patches)
        resid = self._buf("v_resid", (M, hv), torch.float32)
        ops.gemm(patches, w.patch_w, resid, epi=ops.EPI_F32_POS, bias=w.patch_b, aux=w.pos_emb, aux_rows=N)
        if taps is not None:
            taps.append(resid.clone())
        xn = self._buf("v_xn", (M, hv), torch.bfloat16)
        qkv = self._buf("v_qkv", (M, 3 * hv), torch.bfloat16)
        vt = self._buf("v_vt", (hv, M + 32), torch.bfloat16)            # rows padded: attention reads 32-key blocks
        attn = self._buf("v_attn", (M, hv), torch.bfloat16)
        h = self._buf("v_h", (M, w.v_inter), torch.bfloat16)
        Bs = _split_batch or B                                            # the batch the splits are chosen for
        s_o = ops.gemm_ksplit(Bs * N, hv, hv)
        s_2 = ops.gemm_ksplit(Bs * N, hv, w.v_inter)
        ks_v = self._key_split_args("v", Bs, N, N, nh, nh, hd)
        part = self._buf("v_part", (max(s_o, s_2), M, hv), torch.float32)
        res = self.PREFILL_RES and M >= max(17, self.PREFILL_RES_MIN_M)
        res_o, res_2 = res and s_o == 1, res and s_2 == 1
        ns = 0
        for L in w.vl:
            ops.norm_residual(resid, L["ln1_w"], b=L["ln1_b"], mode=ops.NORM_LAYER, eps=w.v_eps, partials=part,
                              nsplit=ns, out=xn, write_resid=ns > 0)
            ops.gemm(xn, L["qkv_w"], qkv, epi=ops.EPI_BF16_VT, bias=L["qkv_b"], aux_out=vt, aux_ld=M + 32,
                     aux_n=2 * hv, split_m=Bs * N)
            ops.attention(qkv, 3 * hv, attn, hv, qkv[:, hv:], N * 3 * hv, hd, 3 * hv, vt, N, hd * (M + 32), M + 32,
                          B=B, Lq=N, Lkv=N, Hq=nh, Hkv=nh, D=hd, scale=1.0 / (hd ** 0.5), **ks_v)
            if res_o:
                self._gemm_cols(attn, L["o_w"], resid, epi=ops.EPI_F32_RES, bias=L["o_b"])
            else:
                self._gemm_cols(attn, L["o_w"], part, epi=ops.EPI_F32, bias=L["o_b"], ksplit=s_o)
            ops.norm_residual(resid, L["ln2_w"], b=L["ln2_b"], mode=ops.NORM_LAYER, eps=w.v_eps, partials=part,
                              nsplit=0 if res_o else s_o, out=xn, write_resid=not res_o)
            self._gemm_cols(xn, L["fc1_w"], h, epi=ops.EPI_BF16_GELU, bias=L["fc1_b"], split_m=Bs * N)
            if res_2:
                self._gemm_cols(h, L["fc2_w"], resid, epi=ops.EPI_F32_RES, bias=L["fc2_b"])
                ns = 0
            else:
                self._gemm_cols(h, L["fc2_w"], part, epi=ops.EPI_F32, bias=L["fc2_b"], ksplit=s_2)
                ns = s_2
            if taps is not None:                                          # debug: residual after the layer
                taps.append((resid + part[:ns].sum(0)).clone())
        hid = torch.empty(M, hv, dtype=torch.float32, device=self.device) if want_hidden else None
        ops.norm_residual(resid, w.post_w, b=w.post_b, mode=ops.NORM_LAYER, eps=w.v_eps, partials=part, nsplit=ns,
                          out=xn, out_f32=hid)
        feats = torch.empty(M, max(w.proj_dim, 1), dtype=torch.float32, device=self.device)
        if w.proj_w is None:                                              # vision-only pack
            return (None, hid) if want_hidden else None
        ops.gemm(xn, w.proj_w, feats, epi=ops.EPI_F32)
        return (feats, hid) if want_hidden else feats

    # ------------------------------------------------------------------ Gemma stack (prefill, T = B*L rows)
    def embed_merge(self, input_ids: torch.Tensor, feats: torch.Tensor, out: torch.Tensor, rank=None):
        w = self.w
        ids = input_ids.reshape(-1)
        n = ids.numel()
        if rank is None and n > 64:
            rank = self._buf("rank", (n,), torch.int32)
            ops.image_rank(ids, self.image_token_id, rank)
        ops.embed_merge(ids, rank, w.embed, feats, feats.shape[0] if feats is not None else 0, out,
                        image_id=self.image_token_id, pad_id=self.pad_id,
                        img_scale=float(w.proj_dim ** -0.5), normalizer=float(w.hidden ** 0.5))

    def gemma_prefill(self, x_resid: torch.Tensor, positions: torch.Tensor, cache: KVStore, B: int, L: int,
                      logits_rows: Optional[torch.Tensor] = None, mask: Optional[torch.Tensor] = None,
                      want_hidden: bool = False, want_logits: bool = True, taps: Optional[list] = None):
        """GemmaForCausalLM.forward after the *sqrt(H) (modeling_gemma.py:510-534) on resid fp32 [B*L][H]
        (already scaled).  Fills cache slots [0, L).  logits_rows: int32 rows to emit logits for (None = all)."""
        w = self.w
        T = B * L
        H, I, nh, nkv, hd = w.hidden, w.inter, w.heads, w.kv_heads, w.head_dim
        cos_t, sin_t = self.rope(L + 2)
        xn = self._buf("t_xn", (T, H), torch.bfloat16)
        qb = self._buf("t_q", (T, nh * hd), torch.bfloat16)
        attn = self._buf("t_attn", (T, nh * hd), torch.bfloat16)
        h = self._buf("t_h", (T, I), torch.bfloat16)
        s_o = self._ksplit(T, H, nh * hd) if T > 16 else self.DECODE_SPLIT_O
        s_d = self._ksplit(T, H, I) if T > 16 else self.DECODE_SPLIT_DOWN
        part = self._buf("t_part", (max(s_o, s_d), T, H), torch.float32)
        pos = positions.to(device=self.device, dtype=torch.int32).reshape(-1).contiguous()
        ks_t = self._key_split_args("t", B, L, L, nh, nkv, hd) if mask is None else {}
        ns = 0
        if taps is not None:
            taps.append(x_resid.clone())
        kvd = nkv * hd
        for i, Lw in enumerate(w.tl):
            xin = self._norm(x_resid, Lw["in_w"], part, ns, xn, T)
            # q|k|v projection + RoPE + KV-cache append in one GEMM (modeling_gemma.py:274-302)
            fa = ops.fused_args(head_dim=hd, cos_t=cos_t, sin_t=sin_t, pos=pos, rows_per_batch=L, slot_base=0,
                                kc=cache.k[i], vtc=cache.vt[i], smax=cache.Smax, q_heads=nh, kv_heads=nkv,
                                kd=cache.kd[i], vd=cache.vd[i])
            self._lin(xin, Lw, "qkv", qb, ops.EPI_QKV_ROPE, T, fa=fa)
            ops.attention(qb, nh * hd, attn, attn.stride(0), cache.k[i], cache.Smax * kvd, hd, kvd,
                          cache.vt[i], kvd * cache.Smax, hd * cache.Smax, cache.Smax,
                          B=B, Lq=L, Lkv=L, Hq=nh, Hkv=nkv, D=hd, scale=1.0 / math.sqrt(hd),
                          mask=mask, mask_bs=(mask.stride(0) if mask is not None else 0),
                          mask_rs=(mask.stride(-2) if mask is not None else 0), **ks_t)
            n_o = self._row_parallel(attn, Lw, "o", part, T, s_o, resid=x_resid)
            xin = self._norm(x_resid, Lw["post_w"], part, n_o, xn, T)
            if self._mx_prefill(T):
                # MX h: e4m3 rows + block scales from the gate/up epilogue, straight into the down GEMM
                h8 = self._buf("t_h8", (T, I), torch.uint8)
                hs = self._buf("t_hs", (T, I // 32), torch.uint8)
                x8, xs = xin
                ops.gemm8(x8, xs, Lw["gu_w8"], Lw["gu_s8"], h8, epi=ops.EPI_BF16_GELU_MUL, M=T, mx_out=hs)
                ns = self._row_parallel(("mx", h8, hs), Lw, "down", part, T, s_d, resid=x_resid)
            else:
                self._lin(xin, Lw, "gu", h, ops.EPI_BF16_GELU_MUL, T)
                ns = self._row_parallel(h, Lw, "down", part, T, s_d, resid=x_resid)
            if taps is not None:
                taps.append((x_resid + part[:ns].sum(0)).clone())
        cache.length = L
        rows = logits_rows.numel() if logits_rows is not None else T
        xf = self._buf("t_xf", (rows, H), torch.bfloat16)
        hid = torch.empty(rows, H, dtype=torch.float32, device=self.device) if want_hidden else None
        ops.norm_residual(x_resid, w.final_w, mode=ops.NORM_RMS, partials=part, nsplit=ns, out=xf, out_f32=hid,
                          row_map=logits_rows, write_resid=False)
        logits = self.lm_head(xf, rows, fresh=True) if want_logits else None
        return logits, hid

    def _key_split_args(self, tag: str, B: int, Lq: int, Lkv: int, Hq: int, Hkv: int, D: int) -> dict:
        """pg_attention keyword arguments for a key-split prefill attention (ops.prefill_key_splits; {} = unsplit):
        the split count and its (O, m, l) workspace."""
        nks = ops.prefill_key_splits(B, Lq, Lkv, Hq, Hkv)
        if nks <= 1:
            return {}
        no, nml = ops.prefill_split_workspace(B, Lq, Hq, Hkv, D, nks)
        return dict(nsplit=nks, part_o=self._buf(f"pf_po_{tag}", (no,), torch.float32),
                    part_ml=self._buf(f"pf_pml_{tag}", (nml,), torch.float32))

    def _fp8_rows(self, M: int) -> bool:
        return self.fp8 and M > 16

    def _mx_prefill(self, M: int) -> bool:
        """The fp8 prefill MLP on MX h (MX_PREFILL): the tile GEMMs (more than 32 rows) with row-major fp8 weights."""
        L0 = self.w.tl[0]
        # (under TP the down projection may run as row chunks (_row_parallel): each must keep > 32 rows)
        chunks_ok = self.tp == 1 or M < 2 * self.AR_CHUNK_ROWS or self.AR_CHUNK_ROWS >= 64
        return (self.MX_PREFILL and self._fp8_rows(M) and M > 32 and "gu_w8" in L0 and "down_w8" in L0
                and self.w.inter % 128 == 0 and chunks_ok)

    def _mx_decode(self, B: int) -> tuple:
        """(MX h, MX norms) for a B-row decode step: the 17..32-row fp8 GEMV path with the packed fp8 weights"""
        w = self.w
        L0 = w.tl[0]
        base = (self.FP8_GEMV and self._fp8_rows(B) and B <= 32 and not self.HQ_FUSED and
                not (self.tp == 1 and self.DECODE_ADD_B32))
        mx_h = (base and self.MX_H and "gu_w8f" in L0 and "down_w8f" in L0 and w.inter % 128 == 0
                and w.hidden <= 4096)
        mx_n = (mx_h and self.MX_NORM and "qkv_w8f" in L0 and w.hidden % 1024 == 0
                and getattr(w, "lm_w8f", None) is not None)
        return mx_h, mx_n

    def _ksplit(self, M: int, N: int, K: int) -> int:
        """split-K of an fp32-partial GEMM (fp8 operands: the kernels count K in byte pairs).  A GEMM that will
        run as row blocks (_lin / _row_head) takes the split that suits its whole-tile head: the pt-448 x16
        down projection then runs 512 full-K tiles in 2 rounds instead of 1536 third-K tiles in 6, and two
        fewer fp32 slabs are written and re-read by the next RMSNorm."""
        if self._fp8_rows(M):
            return ops.gemm_ksplit(M, N, K // 2)
        m1 = self._tile_m1(M, "down" if K == self.w.inter else "o")
        if m1:
            return m1
        Mh = M // 256 * 256
        if self.ROW_BLOCKS and self.HEAD_KSPLIT and 0 < Mh < M:
            s = ops.gemm_ksplit(Mh, N, K)
            if self._row_head(M, N, s):
                return s
        return ops.gemm_ksplit(M, N, K)

    def _tile_m1(self, M: int, name: str) -> int:
        """split-K of a batch-1 prefill linear run as one row tile (PG_TILE_M1), 0 when it does not apply."""
        if (not self.TILE_M1 or self.fp8 or self.tp != 1 or not 256 <= M <= 288
                or M < self.PREFILL_ROWMAJOR_MIN_M):
            return 0
        ks = self.TILE_M1_SPLIT.get(name, 0)
        K = self.w.inter if name == "down" else self.w.hidden
        return ks if ks * 64 <= K else 0

    def _lin(self, x: torch.Tensor, Lw: dict, name: str, out: torch.Tensor, epi: int, M: int, ksplit: int = 1,
             fa=None):
        """One Gemma linear: bf16 (fragment-packed W) or, with fp8 weights and M > 16, the activation rows
        quantised to e4m3 (pg_quant_fp8) feeding the PG_FP8 GEMM with the per-channel weight scales."""
        w = self.w
        if isinstance(x, tuple) and x[0] == "mx":  # MX rows (e4m3 + [M][K/32] block scales): the tile GEMM
            return ops.gemm8(x[1], None, Lw[name + "_w8"], Lw[name + "_s8"], out, epi=epi, M=M, ksplit=ksplit, fa=fa,
                             mx_in=x[2])
        if not isinstance(x, tuple) and self._fp8_rows(M):
            K = x.shape[1]
            x8 = self._buf(f"x8_{K}", (M, K), torch.uint8)
            xs = self._buf(f"xs_{K}", (M,), torch.float32)
            ops.quant_fp8(x, x8, xs, M=M)
            x = (x8, xs)
        if isinstance(x, tuple):        # fp8 rows (quantised here, by _norm, or by the attention kernel)
            x8, xs = x
            if self.FP8_GEMV and M <= 32 and name + "_w8f" in Lw:
                return ops.gemm8(x8, xs, Lw[name + "_w8f"], Lw[name + "_s8"], out, epi=epi, M=M, ksplit=ksplit,
                                 fa=fa, frag=True)
            return ops.gemm8(x8, xs, Lw[name + "_w8"], Lw[name + "_s8"], out, epi=epi, M=M, ksplit=ksplit, fa=fa)
        W, flag = Lw[name + "_w"], w.wflag
        if M >= self.PREFILL_ROWMAJOR_MIN_M and name + "_wr" in Lw:
            W, flag = Lw[name + "_wr"], 0
            if fa is None and self._tile_m1(M, name) == ksplit:
                return ops.gemm(x, W, out, epi=epi | ops.TILE_M1, ksplit=ksplit)
        if fa is None and epi == ops.EPI_F32 and self.ROW_BLOCKS:
            Mh = self._row_head(M, W.shape[0], ksplit)
            if Mh:
                # the 256-row tiles of the first Mh rows fill whole rounds of CUs; the ragged last rows
                # (pt-448 x16: 128 of 16512) run as a small GEMM instead of one more mostly idle round.
                # Both write the same [ksplit][M][N] slabs (PgFusedArgs.slab_rows)
                fr = ops.fused_args(slab_rows=M)
                ops.gemm_fused(x[:Mh], W, out, fr, epi=epi | flag, M=Mh, ksplit=ksplit, ldc=out.stride(-2))
                N, K, Mt = W.shape[0], W.shape[1], M - Mh
                st = max(ksplit, ops.split_for(math.ceil(Mt / 64) * math.ceil(N / 128), K // 64, max_split=8))
                if st > ksplit and self.TAIL_SPLIT:
                    # the tail's own deeper split (its 64x128 tiles alone leave most CUs idle), summed into
                    # slab 0's tail rows; the other slabs' tail rows are zeroed (the head never writes them)
                    tp = self._buf("row_tail", (st, Mt, N), torch.float32)
                    ops.gemm(x[Mh:M], W, tp, epi=epi | flag, ksplit=st)
                    ops.slab_sum(tp, out[0, Mh:M])
                    if ksplit > 1:
                        out[1:ksplit, Mh:M].zero_()
                    return out
                tail = out.view(-1)[Mh * out.stride(-2):]
                return ops.gemm_fused(x[Mh:M], W, tail, fr, epi=epi | flag, M=Mt, ksplit=ksplit,
                                      ldc=out.stride(-2))
        if fa is None and epi == ops.EPI_BF16_GELU_MUL and self.ROW_BLOCKS and self.ROW_BLOCKS_GU:
            Mh = self._row_head(M, W.shape[0], 1)
            if Mh:      # gate/up at pt-448 x16: 8192 whole tiles (32 rounds) + a 128-row tail, not 33 rounds
                ops.gemm(x[:Mh], W, out[:Mh], epi=epi | flag)
                return ops.gemm(x[Mh:M], W, out[Mh:M], epi=epi | flag)
        if fa is not None:
            return ops.gemm_fused(x, W, out, fa, epi=epi | flag, M=M)
        return ops.gemm(x, W, out, epi=epi | flag, ksplit=ksplit)

    def _gemm_cols(self, A: torch.Tensor, W: torch.Tensor, out: torch.Tensor, *, epi: int, bias=None, ksplit: int = 1,
                   split_m: Optional[int] = None):
        """ops.gemm; or, when the last 256-column tile is ragged and dropping it saves a round of CUs, the whole
        256-column tiles and the remaining columns as two GEMMs into the same output (column views: same ldc
        and slab stride).  SigLIP o / fc1 / fc2 at pt-448 x16: 320 -> 256, 1088 -> 1024, 640 -> 512 tiles."""
        Nh = self._col_head(A.shape[0], W.shape[0], ksplit) if self.COL_BLOCKS else 0
        if not Nh:
            return ops.gemm(A, W, out, epi=epi, bias=bias, ksplit=ksplit, split_m=split_m)
        ops.gemm(A, W[:Nh], out[..., :Nh], epi=epi, bias=None if bias is None else bias[:Nh], ksplit=ksplit,
                 split_m=split_m)
        return ops.gemm(A, W[Nh:], out[..., Nh:], epi=epi, bias=None if bias is None else bias[Nh:], ksplit=ksplit,
                        split_m=split_m)

    @staticmethod
    def _col_head(M: int, N: int, ksplit: int, cus: int = ops.CUS) -> int:
        """Columns to issue as whole 256-column tiles (0: one launch), in the one-tile-per-CU regime."""
        Nh = N // 256 * 256
        tm = (M + 255) // 256
        if Nh == N or Nh == 0 or tm * ((N + 255) // 256) * ksplit < cus:
            return 0
        rounds = lambda tiles: (tiles + cus - 1) // cus  # noqa: E731
        return Nh if rounds(tm * (Nh // 256) * ksplit) < rounds(tm * ((N + 255) // 256) * ksplit) else 0

    @staticmethod
    def _row_head(M: int, N: int, ksplit: int, cus: int = ops.CUS) -> int:
        """Rows of an fp32-slab prefill GEMM to issue as whole 256-row tiles, 0 to keep it one launch: only
        in the one-tile-per-CU regime (>= `cus` 256x256 tiles) and when dropping the ragged last row tile
        saves a round of CUs (Gemma o / down at pt-448 x16: 2.03 -> 2 and 6.1 -> 6 rounds)."""
        Mh = M // 256 * 256
        tn = (N + 255) // 256
        if Mh == M or Mh == 0 or (M + 255) // 256 * tn * ksplit < cus:
            return 0
        rounds = lambda tiles: (tiles + cus - 1) // cus  # noqa: E731
        return Mh if rounds(Mh // 256 * tn * ksplit) < rounds((M + 255) // 256 * tn * ksplit) else 0

    def _norm(self, resid: torch.Tensor, norm_w: torch.Tensor, part, nsplit: int, xn: torch.Tensor, M: int):
        """Gemma RMSNorm of the residual (+ split-K partials) feeding a linear: bf16 rows, or fp8 rows with
        their scales (one launch, pg_norm_residual_fp8) when that linear runs on the fp8 path."""
        if self._fp8_rows(M):
            H = resid.shape[-1]
            x8 = self._buf(f"x8_{H}", (M, H), torch.uint8)
            xs = self._buf(f"xs_{H}", (M,), torch.float32)
            return ops.norm_residual_fp8(resid, norm_w, x8, xs, mode=ops.NORM_RMS, partials=part, nsplit=nsplit,
                                         write_resid=nsplit > 0)
        ops.norm_residual(resid, norm_w, mode=ops.NORM_RMS, partials=part, nsplit=nsplit, out=xn,
                          write_resid=nsplit > 0)
        return xn

    def _allreduce_slabs(self, part: torch.Tensor, ns: int) -> int:
        """Complete a row-parallel linear's partial sums: one rank keeps its ns split-K slabs (the next norm adds
        them); under TP the rank's slabs are summed into slab 0 on the way into ONE all-reduce of [rows][H] fp32
        (xGMI: inside the exchange kernel; RCCL / gloo: a slab-sum launch first).  Returns the slab count the
        next norm must add."""
        if self.tp == 1:
            return ns
        return self.comm.all_reduce_slabs(part[:ns], ns)

    def _row_parallel(self, x: torch.Tensor, Lw: dict, name: str, part: torch.Tensor, T: int, ks: int,
                      resid: Optional[torch.Tensor] = None) -> int:
        """A row-parallel prefill linear (o_proj / down_proj) into fp32 partial slabs; returns how many slabs the
        next norm must add.  One rank: `ks` split-K slabs.  Tensor parallel: ONE slab, completed by a SUM all-reduce
        -- a rank's split-K slabs are summed locally first (slab_sum), so every sub-block moves T*H*4 bytes instead
        of ks times that.  From 2 * AR_CHUNK_ROWS rows on, the rows run as chunks with one split each: chunk c's
        all-reduce is issued asynchronously (comm stream) and overlaps chunk c+1's GEMM."""
        if self.tp == 1:
            # (not where the bf16 GEMM runs as row blocks: its ragged tail takes a deeper split of its own, which a
            # one-split epilogue cannot -- pt-448 x16 prefill 82.9 -> 86.6 ms with it)
            row_blocks = (not self._fp8_rows(T) and self.ROW_BLOCKS and
                          self._row_head(T, self.w.hidden, 1) > 0)
            if (resid is not None and self.PREFILL_RES and ks == 1 and T >= max(17, self.PREFILL_RES_MIN_M)
                    and not row_blocks):
                self._lin(x, Lw, name, resid, ops.EPI_F32_RES, T)     # the residual add in the epilogue
                return 0
            self._lin(x, Lw, name, part, ops.EPI_F32, T, ksplit=ks)
            return ks
        # at most AR_CHUNK_ROWS rows per chunk (4096 x 2048 fp32 = the xGMI exchange's 2^23 cap: no chunk spills to
        # the process group)
        C = -(-T // self.AR_CHUNK_ROWS) if T >= 2 * self.AR_CHUNK_ROWS else 1
        if C <= 1:
            self._lin(x, Lw, name, part, ops.EPI_F32, T, ksplit=ks)
            return self.comm.all_reduce_slabs(part[:ks], ks)
        bounds = [T * c // C for c in range(C + 1)]
        works = []
        for r0, r1 in zip(bounds[:-1], bounds[1:]):
            xc = ("mx", x[1][r0:r1], x[2][r0:r1]) if isinstance(x, tuple) else x[r0:r1]
            self._lin(xc, Lw, name, part[0, r0:r1], ops.EPI_F32, r1 - r0, ksplit=1)
            works.append(self.comm.all_reduce_async(part[0, r0:r1]))
        for wk in works:
            wk.wait()
        return 1

    def lm_head(self, xf: torch.Tensor, rows: int, fresh: bool = False, name: str = "lm"):
        """Full-vocabulary logits fp32 [rows][V] from normalised bf16 rows (modeling_gemma.py:530-534).
        Under TP each rank computes its vocabulary slice and an all-gather assembles the rows (each slice
        crosses the links once; the zero-padded SUM of round 2 moved W times the bytes)."""
        w = self.w
        alloc = (lambda shape: torch.empty(*shape, dtype=torch.float32, device=self.device)) if fresh else \
            (lambda shape: self._buf(name, shape, torch.float32))
        if self.tp == 1:
            logits = alloc((rows, w.vocab_local_pad))      # lm_w rows padded to 16 (fragment packing)
            self._lm_gemm(xf, rows, logits)
            return logits[:, :w.vocab]
        vl, vlp = w.vocab_local, w.vocab_local_pad
        loc = self._buf(name + "_loc", (rows, vlp), torch.float32)
        self._lm_gemm(xf, rows, loc)
        g = self._buf(name + "_gather", (self.tp, rows, vlp), torch.float32)
        self.comm.all_gather(g, loc)                                      # [rank][rows][vocab slice]
        out = alloc((rows, w.vocab))
        out.view(rows, self.tp, vl).copy_(g[:, :, :vl].permute(1, 0, 2))
        return out

    def _lm_gemm(self, xf: torch.Tensor, rows: int, out: torch.Tensor):
        """This rank's lm_head rows [rows][vocab_local_pad] fp32 (+ bias) from normalised bf16 rows: bf16 GEMV / GEMM,
        or with fp8 weights at 17..32 rows the e4m3 rows through the fp8 GEMV (half the 1.05 GB of bf16 weights)."""
        w = self.w
        if isinstance(xf, tuple):                   # ("mx", e4m3 rows, block scales, sums of squares)
            _, x8, xs, ss = xf
            return ops.gemm8(x8, None, w.lm_w8f, w.lm_s8, out, epi=ops.EPI_F32, M=rows, bias=w.lm_bias, frag=True,
                             mx_in=xs, ss_in=ss)
        if self.FP8_GEMV and self._fp8_rows(rows) and rows <= 32 and getattr(w, "lm_w8f", None) is not None:
            H = xf.shape[1]
            x8 = self._buf(f"x8_{H}", (rows, H), torch.uint8)
            xs = self._buf(f"xs_{H}", (rows,), torch.float32)
            ops.quant_fp8(xf, x8, xs, M=rows)
            return ops.gemm8(x8, xs, w.lm_w8f, w.lm_s8, out, epi=ops.EPI_F32, M=rows, bias=w.lm_bias, frag=True)
        return ops.gemm(xf, w.lm_w, out, epi=ops.EPI_F32 | w.wflag, bias=w.lm_bias)

    # ------------------------------------------------------------------ decode step (graph-capturable)
    def _chain_ok(self, sampler) -> bool:
        return self.CHAIN_EMBED and self.tp == 1 and sampler is not None and not sampler.get("do_sample")

    def decode_state(self, B: int, cache: KVStore, positions_next: torch.Tensor, max_steps: int, sampler=None):
        """Device-resident decode state: ids, positions, kv length, step counter, token history.

        With the loop's sampler given (generate / bench) and greedy single-rank decoding, the state is
        *chained*: every sample() also writes the embedding of the sampled ids into the decode input buffer,
        and decode_step skips its embed launch.  A caller that writes st["ids"] itself (teacher forcing)
        builds the state without a sampler."""
        st = {
            "ids": torch.zeros(B, dtype=torch.int64, device=self.device),
            "pos": positions_next.to(device=self.device, dtype=torch.int32).reshape(B).contiguous().clone(),
            "kv_len": torch.full((1,), cache.length, dtype=torch.int32, device=self.device),
            "step": torch.zeros(1, dtype=torch.int32, device=self.device),
            "hist": torch.zeros(max_steps + 1, B, dtype=torch.int64, device=self.device),
            "ws": torch.empty(B * 64 * 2, dtype=torch.float32, device=self.device),
            "chain": self._chain_ok(sampler),
        }
        return st

    def decode_step(self, st: dict, cache: KVStore, feats: Optional[torch.Tensor], sampler: dict):
        """One token for B rows: embed(ids) -> 18 layers -> lm_head -> argmax/top-p (advances the state).

        Per layer 5 launches: [RMSNorm + q|k|v GEMV + RoPE + KV append] -> split-KV attention ->
        [attention merge + o GEMV (split-K partials)] -> [RMSNorm + gate/up GEMV + gelu*mul] ->
        down GEMV (split-K partials).  The residual stream ping-pongs between two fp32 buffers; the
        RMSNorm prologues add the previous GEMV's split-K partials (deterministic order)."""
        w = self.w
        B = st["ids"].numel()
        H, I, nh, nkv, hd = w.hidden, w.inter, w.heads, w.kv_heads, w.head_dim
        kvd = nkv * hd
        cos_t, sin_t = self.rope(cache.Smax + 2)
        res_a = self._buf("d_res_a", (B, H), torch.float32)
        res_b = self._buf("d_res_b", (B, H), torch.float32)
        xn = self._buf("d_xn", (B, H), torch.bfloat16)
        qb = self._buf("d_q", (B, nh * hd), torch.bfloat16)
        h = self._buf("d_h", (B, I), torch.bfloat16)
        so, sd = self._split_o(B), self.split_down
        part = self._buf("d_part", (max(so, sd, 16), B, H), torch.float32)     # (16: the gemm8_hx down path)
        SK = self._split_keys(B, cache.Smax)
        nsplit = _rup((cache.Smax + SK - 1) // SK, 4)
        dt = (hd + 15) // 16 * 16
        ns_ws = max(nsplit, ops.decode_plan(B, nkv, cache.Smax)[0]) if B > self.FUSE_MAX_B else nsplit
        part_o = self._buf("d_po", (B * nkv * ns_ws * 16 * dt,), torch.float32)
        part_ml = self._buf("d_pml", (B * nkv * ns_ws * 16 * 2,), torch.float32)
        chain = bool(st.get("chain")) and self._chain_ok(sampler)
        if not chain:                               # chained: the previous sample() wrote res_a already
            ops.embed_merge(st["ids"], None, w.embed, feats, feats.shape[0] if feats is not None else 0, res_a,
                            image_id=self.image_token_id, pad_id=self.pad_id, img_scale=float(w.proj_dim ** -0.5),
                            normalizer=float(w.hidden ** 0.5))
        ns = 0
        fin = self.tp == 1 and self.USE_FIN and (B <= self.FUSE_MAX_B or self.FIN_MIN_B <= B <= 16) and \
            not self._fp8_rows(B)
        if B > self.FUSE_MAX_B and not fin:
            ns = self._decode_layers_unfused(st, cache, res_a, xn, qb, h, part, part_o, part_ml, nsplit, dt, cos_t,
                                             sin_t, SK)
        if fin:
            xq, ss, tiles, n_ss = self._decode_layers_fin(st, cache, res_a, qb, h, part, part_o, part_ml, nsplit, dt,
                                                          cos_t, sin_t, SK)
            # final RMSNorm folded into the lm_head GEMV: x' = resid*(1+w) from the last down_proj, rstd on the outputs
            logits = self._buf("d_logits", (B, w.vocab_local_pad), torch.float32)
            fa = ops.fused_args(pro_mode=ops.PRO_X_RSTD, ss_in=ss, ss_ld=tiles, ss_n=n_ss, eps=1e-6)
            ops.gemm_fused(xq, w.lm_w, logits, fa, epi=ops.EPI_F32 | w.wflag, M=B, bias=w.lm_bias)
            logits = logits[:, :w.vocab]
            if sampler is not None:
                self.sample(logits, st, sampler, advance=True, feats=feats)
            return logits
        for i, Lw in enumerate(w.tl if B <= self.FUSE_MAX_B else ()):      # (TP / USE_FIN off, B <= FUSE_MAX_B)
            fa = ops.fused_args(pro_mode=ops.PRO_RMSNORM, resid_in=res_a, resid_out=res_b, partials=part, nsplit=ns,
                                norm_w=Lw["in_w"], eps=1e-6, head_dim=hd, cos_t=cos_t, sin_t=sin_t, pos=st["pos"],
                                rows_per_batch=1, slot_dev=st["kv_len"], slot_base=0, kc=cache.k[i],
                                vtc=cache.vt[i], smax=cache.Smax, q_heads=nh, kv_heads=nkv, kd=cache.kd[i],
                                vd=cache.vd[i])
            ops.gemm_fused(None, Lw["qkv_w"], qb, fa, epi=ops.EPI_QKV_ROPE | w.wflag, M=B)
            ops.attention(qb, nh * hd, None, nh * hd, cache.k[i], cache.Smax * kvd, hd, kvd,
                          cache.vt[i], kvd * cache.Smax, hd * cache.Smax, cache.Smax,
                          B=B, Lq=1, Lkv=1, lkv_dev=st["kv_len"], Hq=nh, Hkv=nkv, D=hd,
                          scale=1.0 / math.sqrt(hd), split_keys=SK, nsplit=nsplit, part_o=part_o, part_ml=part_ml,
                          kcap=cache.Smax, kd=cache.kd[i], vd=cache.vd[i])
            fa = ops.fused_args(pro_mode=ops.PRO_ATTN_COMBINE, part_o=part_o, part_ml=part_ml, asplit=nsplit,
                                head_dim=hd, dtw=dt, q_per_kv=nh // nkv, kv_heads=nkv, slot_dev=st["kv_len"],
                                akeys=SK)
            ops.gemm_fused(None, Lw["o_w"], part, fa, epi=ops.EPI_F32 | w.wflag, M=B, ksplit=so)
            n_o = self._allreduce_slabs(part, so)
            fa = ops.fused_args(pro_mode=ops.PRO_RMSNORM, resid_in=res_b, resid_out=res_a, partials=part, nsplit=n_o,
                                norm_w=Lw["post_w"], eps=1e-6)
            ops.gemm_fused(None, Lw["gu_w"], h, fa, epi=ops.EPI_BF16_GELU_MUL | w.wflag, M=B)
            ops.gemm(h, Lw["down_w"], part, epi=ops.EPI_F32 | w.wflag, ksplit=sd)
            ns = self._allreduce_slabs(part, sd)
        if B > self.FUSE_MAX_B and self._mx_decode(B)[1]:   # MX rows for the fp8 lm_head (it applies rstd)
            H = w.hidden
            xn = ("mx",) + ops.norm_residual_mx(res_a, w.final_w, self._buf("d_x8n", (B, H), torch.uint8),
                                                self._buf("d_xsn", (B * H // 32,), torch.uint8),
                                                self._buf("d_ssn", (B, H // 1024), torch.float32), partials=part,
                                                nsplit=ns, write_resid=False)
        else:
            ops.norm_residual(res_a, w.final_w, mode=ops.NORM_RMS, partials=part, nsplit=ns, out=xn,
                              write_resid=False)
        if self.tp > 1 and sampler is not None and not sampler.get("do_sample"):
            # vocabulary-parallel greedy: local (max, index) pairs -> all-reduce of the zeroed slots -> merge
            loc = self._buf("d_logits_loc", (B, w.vocab_local_pad), torch.float32)
            self._lm_gemm(xn, B, loc)
            loc = loc[:, :w.vocab_local]
            Bp = B + (B & 1)                    # whole 16-byte exchange units (pairs of rows)
            mine = self._buf("d_pairs_loc", (Bp, 2), torch.float32)
            ops.argmax_pairs(loc, st["ws"], mine, vocab_offset=w.vocab_offset)
            pairs = self._buf("d_pairs", (self.tp, Bp, 2), torch.float32)
            self.comm.all_gather(pairs, mine)
            if Bp != B:
                pairs = self._buf("d_pairs_b", (self.tp, B, 2), torch.float32).copy_(pairs[:, :B])
            ops.argmax_merge(pairs, st["ids"], world=self.tp, hist=st["hist"], step=st["step"], pos=st["pos"],
                             kv_len=st["kv_len"])
            return loc
        logits = self.lm_head(xn, B, name="d_logits")
        if sampler is not None:
            self.sample(logits, st, sampler, advance=True, feats=feats)
        return logits

    def _decode_attn_merged(self, i, st, cache, qb, attn, part_o, part_ml, SK, nsplit, want_fp8=False):
        """Split-KV decode attention of layer i for B > FUSE_MAX_B rows, merged into attn bf16 [B][nh*hd]: one
        pg_attn_decode launch (DECODE_FUSED_ATTN), else the split kernel + pg_attn_combine.  want_fp8: return the
        rows also as (e4m3, row scales) when the one-launch kernel can write them (the fp8 o_proj's input, no
        quantiser launch), else None."""
        w = self.w
        B = qb.shape[0]
        nh, nkv, hd = w.heads, w.kv_heads, w.head_dim
        kvd = nkv * hd
        # the one-launch kernel where the cache needs several rounds of waves (pt-896 x32: 34.3 vs 43.3 us per layer,
        # attention + merge); with one round its last split's serial merge of every partial costs more than the
        # combine launch (pt-224 x16 1.374 vs 1.350 ms/step, round 4).  Since round 5's cheaper merge tail (8 partials
        # per round trip, the four waves storing the split's partial) two rounds win too: pt-448 x16 1.348-1.351 vs
        # 1.391-1.392 ms/step (profiles/r05_fused_attn_pt448_ab.jsonl; round 4 measured 1.429 vs 1.412)
        plan = ops.decode_plan(B, nkv, cache.Smax)
        if self.DECODE_FUSED_ATTN and hd in (32, 256) and cache.Smax >= 64 and plan[2] >= self.FUSED_MIN_ROUNDS:
            x8 = None
            if want_fp8 and self.ATTN_FP8_OUT and ops.attn_decode_q8_ok(nh, nkv, hd, plan[1]):
                x8 = (self._buf(f"x8_{nh * hd}", (B, nh * hd), torch.uint8), self._buf(f"xs_{nh * hd}", (B,),
                                                                                     torch.float32))
            ops.attn_decode(qb, nh * hd, attn, nh * hd, cache.kd[i], cache.vd[i],
                            B=B, Lkv=1, lkv_dev=st["kv_len"], Hq=nh, Hkv=nkv, D=hd, scale=1.0 / math.sqrt(hd),
                            kcap=cache.Smax, part_o=part_o, part_ml=part_ml,
                            counters=self._zeros("d_dec_cnt", (B * nkv,), torch.int32), plan=plan,
                            q8=x8[0] if x8 else None, q8_scale=x8[1] if x8 else None)
            return x8
        ops.attention(qb, nh * hd, None, nh * hd, cache.k[i], cache.Smax * kvd, hd, kvd,
                      cache.vt[i], kvd * cache.Smax, hd * cache.Smax, cache.Smax,
                      B=B, Lq=1, Lkv=1, lkv_dev=st["kv_len"], Hq=nh, Hkv=nkv, D=hd,
                      scale=1.0 / math.sqrt(hd), split_keys=SK, nsplit=nsplit, part_o=part_o,
                      part_ml=part_ml, kcap=cache.Smax, kd=cache.kd[i], vd=cache.vd[i])
        ops.attn_combine(part_o, part_ml, attn, nh * hd, B=B, Hq=nh, Hkv=nkv, D=hd, nsplit=nsplit)
        return None

    def _split_o(self, B: int) -> int:
        if self.tp == 1 and B <= self.FUSE_MAX_B and not os.environ.get("PG_SPLIT_O"):
            return self.DECODE_SPLIT_O_SMALL
        return self.split_o

    def fx_status(self) -> torch.Tensor:
        """The fixed-point residual's status word (PgFusedArgs.status): an FX_ADD launch sets it when a value is
        non-finite or beyond the accumulator's +-2^31 range (saturated, so the step's results are invalid)."""
        return self._zeros("d_fx_status", (1,), torch.int32)

    def check_numerics(self):
        """Raise if a decode step's fixed-point residual overflowed or received a NaN / Inf (one host read)."""
        t = self._ws.get("d_fx_status")
        if t is not None and int(t.item()):
            t.zero_()
            raise FloatingPointError("decode residual: a non-finite or out-of-range (|v| >= 2^31) value reached the "
                                     "fixed-point accumulator; the generated tokens are invalid")

    def _zeros(self, name, shape, dtype):
        """Persistent zero-initialised buffer (e.g. self-resetting arrival tickets)."""
        t = self._ws.get(name)
        if t is None or tuple(t.shape) != tuple(shape) or t.dtype != dtype:
            t = torch.zeros(*shape, dtype=dtype, device=self.device)
            self._ws[name] = t
        return t

    def _decode_layers_fin(self, st, cache, res, qb, h, part, part_o, part_ml, nsplit, dt, cos_t, sin_t, SK=None):
        """Decode layers (single rank, B <= FUSE_MAX_B) in 5 launches with in-kernel split-K finalisation:
        o_proj and down_proj add their split-K slabs into the residual in place (the last-arriving split of
        each 16-column tile), and write x' = bf16(resid*(1+w_next)) plus per-tile sums of squares; the next
        GEMV (gate/up, the next layer's qkv, finally the lm_head) reads x' like a plain activation and
        scales its outputs by rstd (RMSNorm: W.(x*rstd*(1+w)) = rstd * W.(x*(1+w))).
        At B > FUSE_MAX_B (up to 16 rows) the split-KV merge runs as its own kernel (folded into every o_proj
        workgroup it would be recomputed per workgroup) and the GEMVs run two 16-row tiles per workgroup, so
        the sums of squares come one per tile pair.
        Returns (x', sums of squares, their row stride, entries per row) of the final norm for the lm_head."""
        w = self.w
        B = st["ids"].numel()
        H, nh, nkv, hd = w.hidden, w.heads, w.kv_heads, w.head_dim
        kvd = nkv * hd
        so, sd = self._split_o(B), self.split_down
        if B > self.FUSE_MAX_B and self.tp == 1:
            if not os.environ.get("PG_SPLIT_O"):
                so = self.DECODE_SPLIT_O_FIN16
            if not os.environ.get("PG_SPLIT_DOWN"):
                sd = self.DECODE_SPLIT_DOWN_FIN16
        tiles = (H + 15) // 16
        n_ss = tiles if B <= 4 else (tiles + 1) // 2         # one entry per GEMV workgroup (M > 4: tile pairs)
        merge_in_gemv = B <= self.FUSE_MAX_B
        attn = None if merge_in_gemv else self._buf("d_attn", (B, nh * hd), torch.bfloat16)
        cnt = self._zeros("d_fin_cnt", (tiles,), torch.int32)
        ss_o = self._buf("d_ss_o", (B, tiles), torch.float32)
        ss_d = self._buf("d_ss_d", (B, tiles), torch.float32)
        xq = self._buf("d_xq", (B, H), torch.bfloat16)
        SK = SK or self.DECODE_SPLIT_KEYS
        nl = len(w.tl)
        add_down = merge_in_gemv and self.DECODE_ADD in ("down", "both", "fx")
        add_o = merge_in_gemv and self.DECODE_ADD in ("both", "fx")
        # "fx": the partials go to the fixed-point accumulator (zero between steps: the last layer's F32_FIN clears it);
        # layer 0's o_proj also folds the embedding rows in, so from there on it holds the whole residual
        fx = self._zeros("d_fx", (B, H), torch.int64) if merge_in_gemv and self.DECODE_ADD == "fx" else None
        fx_st = self.fx_status() if fx is not None else None      # set by an FX_ADD launch given an unholdable value
        add_epi, add_dst = (ops.EPI_FX_ADD, fx) if fx is not None else (ops.EPI_F32_ADD, res)
        for i, Lw in enumerate(w.tl):
            rope = dict(head_dim=hd, cos_t=cos_t, sin_t=sin_t, pos=st["pos"], rows_per_batch=1,
                        slot_dev=st["kv_len"], slot_base=0, kc=cache.k[i], vtc=cache.vt[i], smax=cache.Smax,
                        q_heads=nh, kv_heads=nkv, kd=cache.kd[i], vd=cache.vd[i])
            if i == 0 or add_down:  # the residual rows are final (embedding, or atomically added): RMSNorm prologue
                # (fx mode: layer 0 reads the embedding rows; from layer 0's o_proj on the accumulator holds the whole
                # residual -- that launch folds res in -- and the consumers read it alone)
                fa = ops.fused_args(pro_mode=ops.PRO_RMSNORM, resid_in=res if (i == 0 or fx is None) else None,
                                    fx=fx if i > 0 else None, nsplit=0, norm_w=Lw["in_w"], eps=1e-6, **rope)
                if i == 0 and fx is not None:
                    # the step starts from a zero accumulator whatever an earlier (interrupted) step left in it: layer 0's
                    # q|k|v GEMV does not read it and clears it before layer 0's o_proj adds into it
                    fa.amax_zero, fa.amax_zero_n = fx.data_ptr(), fx.numel() * 2
                ops.gemm_fused(None, Lw["qkv_w"], qb, fa, epi=ops.EPI_QKV_ROPE | w.wflag, M=B)
            else:
                fa = ops.fused_args(pro_mode=ops.PRO_X_RSTD, ss_in=ss_d, ss_ld=tiles, ss_n=n_ss, eps=1e-6, **rope)
                ops.gemm_fused(xq, Lw["qkv_w"], qb, fa, epi=ops.EPI_QKV_ROPE | w.wflag, M=B)
            if merge_in_gemv:
                ops.attention(qb, nh * hd, None, nh * hd, cache.k[i], cache.Smax * kvd, hd, kvd,
                              cache.vt[i], kvd * cache.Smax, hd * cache.Smax, cache.Smax,
                              B=B, Lq=1, Lkv=1, lkv_dev=st["kv_len"], Hq=nh, Hkv=nkv, D=hd,
                              scale=1.0 / math.sqrt(hd), split_keys=SK, nsplit=nsplit, part_o=part_o,
                              part_ml=part_ml, kcap=cache.Smax, kd=cache.kd[i], vd=cache.vd[i])
                if add_o:
                    fa = ops.fused_args(pro_mode=ops.PRO_ATTN_COMBINE, part_o=part_o, part_ml=part_ml, asplit=nsplit,
                                        head_dim=hd, dtw=dt, q_per_kv=nh // nkv, kv_heads=nkv, slot_dev=st["kv_len"],
                                        akeys=SK, resid_in=res if (fx is not None and i == 0) else None,
                                        status=fx_st)
                    ops.gemm_fused(None, Lw["o_w"], add_dst, fa, epi=add_epi | w.wflag, M=B, ksplit=so)
                else:
                    fa = ops.fused_args(pro_mode=ops.PRO_ATTN_COMBINE, part_o=part_o, part_ml=part_ml, asplit=nsplit,
                                        head_dim=hd, dtw=dt, q_per_kv=nh // nkv, kv_heads=nkv, slot_dev=st["kv_len"],
                                        akeys=SK, fin_cnt=cnt, fin_resid=res, ss_out=ss_o, ss_ld=tiles, fin_x=xq,
                                        norm_w=Lw["post_w"])
                    ops.gemm_fused(None, Lw["o_w"], part, fa, epi=ops.EPI_F32_FIN | w.wflag, M=B, ksplit=so)
            else:
                self._decode_attn_merged(i, st, cache, qb, attn, part_o, part_ml, SK, nsplit)
                fa = ops.fused_args(fin_cnt=cnt, fin_resid=res, ss_out=ss_o, ss_ld=tiles, fin_x=xq,
                                    norm_w=Lw["post_w"])
                ops.gemm_fused(attn, Lw["o_w"], part, fa, epi=ops.EPI_F32_FIN | w.wflag, M=B, ksplit=so)
            nxt_w = w.tl[i + 1]["in_w"] if i + 1 < nl else w.final_w
            self._mlp_fin(Lw, xq, ss_o, tiles, n_ss, h, part, cnt, res, ss_d, nxt_w, B, sd,
                          add=add_down and i + 1 < nl, gu_rms=add_o, fx=fx, fx_st=fx_st)
        return xq, ss_d, tiles, n_ss

    def _mlp_fin(self, Lw, xq, ss_o, tiles, n_ss, h, part, cnt, res, ss_d, nxt_w, B, sd, add=False, gu_rms=False,
                 fx=None, fx_st=None):
        """gate/up + down of a _decode_layers_fin layer: x' = xq with rstd from ss_o -> h -> down, finalised into res
        (x' of the next norm -> xq, its sums of squares -> ss_d).  add: down adds its partials into res with float
        atomics (EPI_F32_ADD), or into the fixed-point accumulator fx (EPI_FX_ADD); the next GEMV normalises res (+ fx)
        itself.  gu_rms: o_proj did so, gate/up normalises res (+ fx).  The finalising form adds fx and clears it."""
        w = self.w
        if gu_rms:
            fa = ops.fused_args(pro_mode=ops.PRO_RMSNORM, resid_in=res if fx is None else None, fx=fx, nsplit=0,
                                norm_w=Lw["post_w"], eps=1e-6)
            ops.gemm_fused(None, Lw["gu_w"], h, fa, epi=ops.EPI_BF16_GELU_MUL | w.wflag, M=B)
        else:
            fa = ops.fused_args(pro_mode=ops.PRO_X_RSTD, ss_in=ss_o, ss_ld=tiles, ss_n=n_ss, eps=1e-6)
            ops.gemm_fused(xq, Lw["gu_w"], h, fa, epi=ops.EPI_BF16_GELU_MUL | w.wflag, M=B)
        if add:
            if fx is not None:
                ops.gemm_fused(h, Lw["down_w"], fx, ops.fused_args(status=fx_st), epi=ops.EPI_FX_ADD | w.wflag, M=B,
                               ksplit=sd)
            else:
                ops.gemm_fused(h, Lw["down_w"], res, ops.fused_args(), epi=ops.EPI_F32_ADD | w.wflag, M=B, ksplit=sd)
            return
        fa = ops.fused_args(fin_cnt=cnt, fin_resid=res, ss_out=ss_d, ss_ld=tiles, fin_x=xq, norm_w=nxt_w, fx=fx)
        ops.gemm_fused(h, Lw["down_w"], part, fa, epi=ops.EPI_F32_FIN | w.wflag, M=B, ksplit=sd)

    def _split_keys(self, B: int, Smax: int) -> int:
        """Keys per decode-attention split: 32 (one MFMA block) at small batch; at B > FUSE_MAX_B (separate
        merge kernel) whole multiples of 32 such that B * splits stays near DECODE_SPLIT_TARGET -- fewer (O, m, l)
        partials to write and merge once the batch alone fills the chip."""
        SK = self.DECODE_SPLIT_KEYS
        if B <= self.FUSE_MAX_B:
            return self.DECODE_SPLIT_KEYS_SMALL
        blocks = (Smax + SK - 1) // SK
        if self.DECODE_ONE_ROUND and B * blocks >= 2048:
            # long KV x batch: 4-wave splits of several 32-key rounds per wave, about 512 workgroups in all (two
            # resident per CU: one round) -- pt-896 x32: 12 splits of 384 keys instead of 36 of 128 (2.25 rounds)
            per_batch = max(4, (512 // B) // 4 * 4)
            return 128 * (-(-Smax // (128 * per_batch)))
        mult = max(1, min(8, (B * blocks) // self.DECODE_SPLIT_TARGET))
        # a power of two: 2 / 4 / 8-block splits run one wave per block, merged in LDS (attn_decode_wg_kernel)
        return SK * (1 << (mult.bit_length() - 1))

    def _decode_layers_unfused(self, st, cache, res, xn, qb, h, part, part_o, part_ml, nsplit, dt, cos_t, sin_t,
                               SK=None):
        """Decode layers for B > FUSE_MAX_B: the RMSNorm and the split-KV merge run once as their own
        kernels (fused into every GEMV workgroup they would be recomputed B-fold per workgroup)."""
        w = self.w
        B = st["ids"].numel()
        nh, nkv, hd = w.heads, w.kv_heads, w.head_dim
        kvd = nkv * hd
        so, sd = self.split_o, self.split_down
        attn = self._buf("d_attn", (B, nh * hd), torch.bfloat16)
        # 17..32 rows on the fp8 GEMV, one rank: o_proj / down_proj may add their partials into the residual with
        # float atomics (no slabs for the next norm to re-read), as the batch-1 path does.  Measured slower at pt-896
        # x32 (down 11.5 -> 14.9 us: the MFMA output layout scatters each atomic instruction over 16 rows), so off
        add = (self.tp == 1 and self.DECODE_ADD_B32 and self.FP8_GEMV and self._fp8_rows(B) and B <= 32
               and "o_w8f" in w.tl[0] and "down_w8f" in w.tl[0])
        # 17..32 rows on the fp8 GEMVs: the gate/up epilogue max-es each row's |h| (amax_out) and the down GEMV
        # quantises h while staging it (ops.gemm8_hx) -- no quantiser launch; the QKV GEMV clears the maxima
        ich = h.shape[1] // 128
        sdh = ich // self.HQ_CHUNKS                # the down GEMV's splits on this path (x chunk per workgroup)
        hq = (self.HQ_FUSED and self.FP8_GEMV and self._fp8_rows(B) and B <= 32 and not add
              and all(k in w.tl[0] for k in ("qkv_w8f", "gu_w8f", "down_w8f"))
              and ich % self.HQ_CHUNKS == 0 and part.shape[0] >= sdh)
        I, H = h.shape[1], w.hidden
        mx, mxn = self._mx_decode(B)
        mx, mxn = mx and not hq and not add, mxn and not hq and not add
        if mx:
            h8 = self._buf("d_h8", (B, I), torch.uint8)
            hs = self._buf("d_hs", (B * I // 32,), torch.uint8)
        if mxn:
            x8n = self._buf("d_x8n", (B, H), torch.uint8)
            xsn = self._buf("d_xsn", (B * H // 32,), torch.uint8)
            ssn = self._buf("d_ssn", (B, H // 1024), torch.float32)
        if hq:
            amax = self._buf("d_hamax", (B * self.AMAX_LD,), torch.int32)
            fa_gu = ops.fused_args(amax_out=amax, amax_ld=self.AMAX_LD)
        ns = 0
        for i, Lw in enumerate(w.tl):
            fa = ops.fused_args(head_dim=hd, cos_t=cos_t, sin_t=sin_t, pos=st["pos"], rows_per_batch=1,
                                slot_dev=st["kv_len"], slot_base=0, kc=cache.k[i], vtc=cache.vt[i], smax=cache.Smax,
                                q_heads=nh, kv_heads=nkv, kd=cache.kd[i], vd=cache.vd[i])
            if mxn:                                 # MX rows of x*(1+w); the q|k|v GEMV applies rstd
                ops.norm_residual_mx(res, Lw["in_w"], x8n, xsn, ssn, partials=part, nsplit=ns)
                ops.gemm8(x8n, None, Lw["qkv_w8f"], Lw["qkv_s8"], qb, epi=ops.EPI_QKV_ROPE, M=B, fa=fa, frag=True,
                          mx_in=xsn, ss_in=ssn)
            else:
                xin = self._norm(res, Lw["in_w"], part, ns, xn, B)
                if hq:
                    fa.amax_zero, fa.amax_zero_n = amax.data_ptr(), B * self.AMAX_LD
                self._lin(xin, Lw, "qkv", qb, ops.EPI_QKV_ROPE, B, fa=fa)
            a8 = self._decode_attn_merged(i, st, cache, qb, attn, part_o, part_ml, SK or self.DECODE_SPLIT_KEYS,
                                          nsplit, want_fp8=self._fp8_rows(B))
            if add:
                self._lin(a8 or attn, Lw, "o", res, ops.EPI_F32_ADD, B, ksplit=so)
                n_o = 0
            else:
                self._lin(a8 or attn, Lw, "o", part, ops.EPI_F32, B, ksplit=so)
                n_o = self._allreduce_slabs(part, so)
            if mxn:                                 # MX norm -> gate/up (rstd, MX h) -> down (MX rows)
                ops.norm_residual_mx(res, Lw["post_w"], x8n, xsn, ssn, partials=part, nsplit=n_o)
                ops.gemm8(x8n, None, Lw["gu_w8f"], Lw["gu_s8"], h8, epi=ops.EPI_BF16_GELU_MUL, M=B, frag=True,
                          mx_in=xsn, ss_in=ssn, mx_out=hs)
                ops.gemm8(h8, None, Lw["down_w8f"], Lw["down_s8"], part, epi=ops.EPI_F32, M=B, ksplit=sd, frag=True,
                          mx_in=hs)
                ns = self._allreduce_slabs(part, sd)
                continue
            xin = self._norm(res, Lw["post_w"], part, n_o, xn, B)
            if hq:
                self._lin(xin, Lw, "gu", h, ops.EPI_BF16_GELU_MUL, B, fa=fa_gu)
                ops.gemm8_hx(h, amax, self.AMAX_LD, Lw["down_w8f"], Lw["down_s8"], part, M=B, ksplit=sdh)
                ns = self._allreduce_slabs(part, sdh)
                continue
            if mx:                                  # MX h: e4m3 + block scales straight from gate/up into down
                x8, xs = xin
                ops.gemm8(x8, xs, Lw["gu_w8f"], Lw["gu_s8"], h8, epi=ops.EPI_BF16_GELU_MUL, M=B, frag=True, mx_out=hs)
                ops.gemm8(h8, None, Lw["down_w8f"], Lw["down_s8"], part, epi=ops.EPI_F32, M=B, ksplit=sd, frag=True,
                          mx_in=hs)
                ns = self._allreduce_slabs(part, sd)
                continue
            self._lin(xin, Lw, "gu", h, ops.EPI_BF16_GELU_MUL, B)
            if add:
                self._lin(h, Lw, "down", res, ops.EPI_F32_ADD, B, ksplit=sd)
                ns = 0
            else:
                self._lin(h, Lw, "down", part, ops.EPI_F32, B, ksplit=sd)
                ns = self._allreduce_slabs(part, sd)
        return ns

    def sample(self, logits: torch.Tensor, st: dict, sampler: dict, advance: bool,
               feats: Optional[torch.Tensor] = None):
        """Next ids from logits [B][V] (greedy or top-p); advance=True also moves pos / kv_len on.  A chained
        state (decode_state) also gets the next step's input rows: pass the request's image features."""
        kw = dict(hist=st["hist"], step=st["step"])
        if advance:
            kw.update(pos=st["pos"], kv_len=st["kv_len"])
        if st.get("chain") and self._chain_ok(sampler):
            w = self.w
            B = st["ids"].numel()
            ops.argmax_embed(logits, st["ids"], st["ws"], w.embed, feats, feats.shape[0] if feats is not None else 0,
                             self._buf("d_res_a", (B, w.hidden), torch.float32), image_id=self.image_token_id,
                             pad_id=self.pad_id, img_scale=float(w.proj_dim ** -0.5),
                             normalizer=float(w.hidden ** 0.5), **kw)
        elif sampler.get("do_sample"):
            ops.topp_sample(logits, st["ids"], sampler["uniforms"], temperature=sampler["temperature"],
                            top_p=sampler["top_p"], **kw)
        else:
            ops.argmax(logits, st["ids"], st["ws"], **kw)

    # ------------------------------------------------------------------ full request
    def prefill_request(self, input_ids: torch.Tensor, pixel_values: torch.Tensor, attention_mask: torch.Tensor,
                        max_new_tokens: int, feats: Optional[torch.Tensor] = None):
        """Vision + merge + Gemma prefill; returns (cache, feats, last-position logits [B][V], next positions)."""
        B, L = input_ids.shape
        if feats is None:
            feats = self.vision(pixel_values)
        cache = self.new_cache(B, L + max_new_tokens + 1)
        resid = self._buf("p_resid", (B * L, self.w.hidden), torch.float32)
        self.embed_merge(input_ids.to(self.device), feats, resid)
        am = attention_mask.to(self.device)
        pos = am.cumsum(-1).masked_fill(am == 0, 1)                       # modeling_paligemma.py:195
        rows = (torch.arange(B, device=self.device, dtype=torch.int32) * L + (L - 1)).contiguous()
        logits, _ = self.gemma_prefill(resid, pos, cache, B, L, logits_rows=rows)
        nxt = am.sum(-1).to(torch.int32) + 1                              # modeling_paligemma.py:189
        return cache, feats, logits, nxt

    def generate(self, input_ids, pixel_values, attention_mask, max_new_tokens: int, do_sample=False,
                 temperature=0.8, top_p=0.9, uniforms=None, stop_token: Optional[int] = 1, use_graph=True,
                 check_every: Optional[int] = None, pad_token: int = 0, return_list: bool = False):
        """test_inference's loop (inference.py:45-82) for B >= 1 rows.

        B = 1: ids [1][n], stopping after EOS like the reference.  B > 1 (the reference asserts B = 1,
        SURVEY §8(f2)): every row decodes in the same static-shape graph until ALL rows have produced
        `stop_token` (checked every `check_every` steps, default 8, one host sync each) or max_new_tokens;
        a row's tokens after its EOS are replaced by `pad_token` in the [B][n] result, or dropped when
        return_list=True (a list of per-row id lists, each ending at its EOS)."""
        B = input_ids.shape[0]
        if check_every is None:
            check_every = 1 if B == 1 else 8
        cache, feats, logits, nxt = self.prefill_request(input_ids, pixel_values, attention_mask, max_new_tokens)
        sampler = dict(do_sample=do_sample, temperature=temperature, top_p=top_p)
        st = self.decode_state(B, cache, nxt, max_new_tokens, sampler=sampler)
        if do_sample:
            if uniforms is None:
                uniforms = torch.rand(max_new_tokens + 1, B)
            sampler["uniforms"] = uniforms.to(device=self.device, dtype=torch.float32).contiguous()
        self.sample(logits, st, sampler, advance=False, feats=feats)     # token 1 from the prefill logits
        n = 1
        step_fn = None
        if use_graph and self.comm.capturable:
            try:
                step_fn = self._graph_step(st, cache, feats, sampler)
            except CaptureUnsupported:
                # a collective that cannot be captured (an all-reduce larger than the xGMI exchange buffer):
                # _graph_step restored the state before capturing and a failed capture runs nothing, so the
                # eager steps start from the same state.  Any other error propagates.
                torch.cuda.synchronize()
                step_fn = None
        if step_fn is None:
            step_fn = lambda: self.decode_step(st, cache, feats, sampler)  # noqa: E731
        while n < max_new_tokens:
            if stop_token is not None and n % check_every == 0:
                if B == 1:
                    if int(st["ids"][0]) == stop_token:                   # inference.py:73-74
                        break
                elif bool((st["hist"][:n] == stop_token).any(0).all()):   # every row has finished
                    break
            step_fn()
            n += 1
        hist = st["hist"][:n].t().contiguous().cpu()
        self.check_numerics()
        if hasattr(self.comm, "check"):
            self.comm.check()              # an xGMI exchange that timed out leaves meaningless sums: raise
        if stop_token is None:
            return [r.tolist() for r in hist] if return_list else hist
        rows = []
        for r in hist.tolist():
            rows.append(r[: r.index(stop_token) + 1] if stop_token in r else r)
        if return_list:
            return rows
        if B == 1:
            return torch.tensor(rows, dtype=torch.int64)
        out = torch.full((B, max(len(r) for r in rows)), pad_token, dtype=torch.int64)
        for b, r in enumerate(rows):
            out[b, : len(r)] = torch.tensor(r, dtype=torch.int64)
        return out

    def _graph_step(self, st, cache, feats, sampler):
        """Capture one decode step into a hipGraph (warm-up run first, on a side stream)."""
        torch.cuda.synchronize()
        # warm-up pass to allocate every workspace outside capture, then undo its state advance
        snap = {k: st[k].clone() for k in ("ids", "pos", "kv_len", "step")}
        hist0 = st["hist"].clone()
        res0 = self._ws["d_res_a"][: st["ids"].numel() * self.w.hidden].clone() if st.get("chain") else None
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        try:
            with torch.cuda.stream(s):
                self.decode_step(st, cache, feats, sampler)
            torch.cuda.current_stream().wait_stream(s)
        finally:                                    # restored even when the warm-up step raises
            torch.cuda.synchronize()
            for k, v in snap.items():
                st[k].copy_(v)
            st["hist"].copy_(hist0)
            if res0 is not None:                    # the chained input rows the warm-up step overwrote
                self._ws["d_res_a"][: res0.numel()].copy_(res0)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            self.decode_step(st, cache, feats, sampler)
        torch.cuda.synchronize()
        self.graphs["decode"] = g
        return g.replay
