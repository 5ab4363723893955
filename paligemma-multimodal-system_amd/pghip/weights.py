"""Pack reference-layout weights into the kernel layouts held in HBM.

Input: any mapping from the reference's state-dict keys (modeling_siglip.py /
modeling_gemma.py / modeling_paligemma.py module tree) to
tensors of any float dtype on any device.  Output, on the HIP device:

  SigLIP   patch W [hv][Kp] bf16 (Conv2d weight flattened (c, kh, kw), K padded to 64)
           per layer: qkv W [3hv][hv] (query | key | value rows) + fp32 bias, out W, fc1 W
           [Ip][hv] (N padded to 64, zero rows), fc2 W [hv][Ip] (K padded), fp32 LN params
  proj     W [P][hv] bf16
  Gemma    embed [V][H] bf16 (gather AND tied lm_head, modeling_gemma.py:492-499), lm_head bias fp32,
           per layer: qkv W [(nh+2nkv)*hd][H] (q | k | v, rows of every head block in rope_row_perm
           order for the fused RoPE/KV-append epilogue), o W, gate/up W [2I][H] interleaved in
           16-row blocks (gate 16u..16u+15, then up 16u..16u+15) for the fused GELU*mul epilogue,
           down W [H][I], fp32 RMSNorm weights (the kernel applies 1 + w).

Padding rows/columns are zero so padded outputs are exactly 0 (gelu(0) = 0).

The Gemma linear weights (q|k|v, o, gate/up, down and the lm_head copy of the embedding) are then
stored fragment-packed (frag_pack; `frag` = True): the decode GEMVs stream them as 1 KiB lane-linear
wave-instructions (gate/up 28.7 -> 23.0 us on MI355X) and the prefill tile GEMM stages them with the
same per-lane address arithmetic.  The embedding used by the gather stays row-major.

Tensor parallelism (tp_world > 1): rank r keeps the q heads
[r*nh/W, (r+1)*nh/W) and every (replicated) k/v head, the matching o_proj input columns,
the gate/up rows and down input columns of its slice [r*I/W, (r+1)*I/W) of the
intermediate dimension, and the lm_head rows (= embedding rows) of its vocabulary slice
[r*V/W, (r+1)*V/W).  o_proj and down then produce partial sums that one all-reduce
completes; the embedding gather, RMSNorm weights and the vision tower stay replicated.
"""
from __future__ import annotations

import torch


def _rup(x: int, m: int) -> int:
    return (x + m - 1) // m * m


def frag_pack(w: torch.Tensor) -> torch.Tensor:
    """Row-major W[N][K] (N % 16 == 0, K % 64 == 0) -> the fragment-packed layout of include/pghip.h
    PG_W_FRAG: W[16t + r][64c + 16g + 8s + e] at ((((t*K/64 + c)*2 + s)*64 + 16g + r)*8 + e), so that
    every GEMV wave-instruction (lane 16g + r, piece s) reads 1 KiB contiguous.  Same shape [N][K]."""
    N, K = w.shape
    if N % 16 or K % 64:
        raise ValueError(f"frag_pack needs N % 16 == 0 and K % 64 == 0, got {tuple(w.shape)}")
    return w.reshape(N // 16, 16, K // 64, 4, 2, 8).permute(0, 2, 4, 3, 1, 5).contiguous().view(N, K)


def frag_unpack(p: torch.Tensor) -> torch.Tensor:
    """Inverse of frag_pack."""
    N, K = p.shape
    return p.reshape(N // 16, K // 64, 2, 4, 16, 8).permute(0, 4, 1, 3, 2, 5).contiguous().view(N, K)


def frag_pack8(w8: torch.Tensor) -> torch.Tensor:
    """Row-major e4m3 bytes W8[N][K] (uint8, N % 16 == 0, K % 128 == 0) -> the fp8 fragment-packed layout of
    include/pghip.h (PG_FP8 | PG_W_FRAG, the fp8 decode GEMV): W8[16t + r][128c + 64s + 16g + e] at byte
    ((t*K/128 + c)*2 + s)*1024 + (16g + r)*16 + e, so each (16-row x 128-k chunk, piece s) is one 1-KiB lane-linear
    wave load.  Same shape [N][K]."""
    N, K = w8.shape
    if N % 16 or K % 128 or w8.dtype != torch.uint8:
        raise ValueError(f"frag_pack8 needs uint8 [N][K] with N % 16 == 0 and K % 128 == 0, got {tuple(w8.shape)}")
    return w8.reshape(N // 16, 16, K // 128, 2, 4, 16).permute(0, 2, 3, 4, 1, 5).contiguous().view(N, K)


def frag_unpack8(p: torch.Tensor) -> torch.Tensor:
    """Inverse of frag_pack8."""
    N, K = p.shape
    return p.reshape(N // 16, K // 128, 2, 4, 16, 16).permute(0, 4, 1, 2, 3, 5).contiguous().view(N, K)


def rope_row_perm(D: int) -> torch.Tensor:
    """Row order inside one D-wide head block for the fused RoPE epilogue: 16-row tile t holds
    dims 8t..8t+7 then D/2+8t..D/2+8t+7, so each lane's rotate_half partner is lane ^ 32."""
    idx = []
    for t in range(D // 16):
        idx += [8 * t + j for j in range(8)] + [D // 2 + 8 * t + j for j in range(8)]
    return torch.tensor(idx, dtype=torch.long)


def quant_rows_fp8(w: torch.Tensor):
    """Per-row (output channel) fp8 e4m3 quantisation of a row-major matrix: (uint8 e4m3 bytes, fp32 scales),
    w ~= q * scale[:, None], scale = max|row| / 448 (1 for a zero row).  Same rule as pg_quant_fp8."""
    wf = w.float()
    amax = wf.abs().amax(1)
    # tensor / tensor: a correctly rounded division, as in pg_quant_fp8 (torch turns "/ 448.0" into a multiply)
    scale = torch.where(amax > 0, amax / torch.full_like(amax, 448.0), torch.ones_like(amax))
    q = (wf / scale[:, None]).clamp_(-448.0, 448.0).to(torch.float8_e4m3fn)
    return q.view(torch.uint8).contiguous(), scale.contiguous()


class PackedWeights:
    def __init__(self, cfg: dict, get, device="cuda", parts=("vision", "proj", "text"), tp_rank: int = 0,
                 tp_world: int = 1, fp8: bool = False, prefill_rowmajor: bool = True):
        """fp8: also hold the Gemma decoder linears as fp8 e4m3 with per-output-channel scales (`<name>8`,
        `<name>_s8` in each layer dict) for the PG_FP8 GEMMs of prefill and batch > 16 decode (BASELINE
        configs[4]); the bf16 copies stay for the weight-streaming GEMV path (batch <= 16 decode)."""
        self.cfg = cfg
        self.fp8 = bool(fp8)
        self.prefill_rowmajor = bool(prefill_rowmajor)   # keep row-major Gemma linears beside the packed ones
        self.tp_rank, self.tp_world = int(tp_rank), int(tp_world)
        if not 0 <= self.tp_rank < self.tp_world:
            raise ValueError(f"tp_rank {tp_rank} outside tp_world {tp_world}")
        self.device = torch.device(device)
        self.parts = tuple(parts)
        v, t = cfg["vision_config"], cfg.get("text_config")
        dev = self.device

        def bf(x):
            return x.detach().to(device=dev, dtype=torch.bfloat16).contiguous()

        def f32(x):
            return x.detach().to(device=dev, dtype=torch.float32).contiguous()

        self.vl, self.tl = [], []
        self.proj_w, self.proj_dim = None, 0
        if "vision" in self.parts:
            self._pack_vision(v, get, dev, bf, f32)
        if "text" in self.parts:
            self._pack_text(t, get, dev, bf, f32)

    def _pack_vision(self, v, get, dev, bf, f32):
        # ---------------- SigLIP
        hv, iv = v["hidden_size"], v["intermediate_size"]
        self.v_hidden, self.v_heads = hv, v["num_attention_heads"]
        self.v_head_dim = hv // self.v_heads
        self.v_layers = v["num_hidden_layers"]
        self.v_eps = v.get("layer_norm_eps", 1e-6)
        self.patch = v["patch_size"]
        self.channels = v.get("num_channels", 3)
        self.image_size = v.get("image_size", 224)
        self.n_img = (self.image_size // self.patch) ** 2
        pre = "vision_tower.model."
        kraw = self.channels * self.patch * self.patch
        self.patch_k = _rup(kraw, 64)
        pw = torch.zeros(hv, self.patch_k, dtype=torch.bfloat16, device=dev)
        pw[:, :kraw] = bf(get(pre + "embeddings.patch_embedding.weight").reshape(hv, kraw))
        self.patch_w = pw
        self.patch_b = f32(get(pre + "embeddings.patch_embedding.bias"))
        self.pos_emb = f32(get(pre + "embeddings.positional_embeddings.weight"))
        self.v_inter = _rup(iv, 64)
        self.vl = []
        for i in range(self.v_layers):
            lp = f"{pre}encoder.layers.{i}."
            a = lp + "self_attn."
            qkv_w = torch.cat([bf(get(a + "query_proj.weight")), bf(get(a + "key_proj.weight")),
                               bf(get(a + "value_proj.weight"))], 0).contiguous()
            qkv_b = torch.cat([f32(get(a + "query_proj.bias")), f32(get(a + "key_proj.bias")),
                               f32(get(a + "value_proj.bias"))], 0).contiguous()
            fc1_w = torch.zeros(self.v_inter, hv, dtype=torch.bfloat16, device=dev)
            fc1_w[:iv] = bf(get(lp + "mlp.fc1.weight"))
            fc1_b = torch.zeros(self.v_inter, dtype=torch.float32, device=dev)
            fc1_b[:iv] = f32(get(lp + "mlp.fc1.bias"))
            fc2_w = torch.zeros(hv, self.v_inter, dtype=torch.bfloat16, device=dev)
            fc2_w[:, :iv] = bf(get(lp + "mlp.fc2.weight"))
            self.vl.append(dict(
                ln1_w=f32(get(lp + "layer_norm1.weight")), ln1_b=f32(get(lp + "layer_norm1.bias")),
                qkv_w=qkv_w, qkv_b=qkv_b,
                o_w=bf(get(a + "out_proj.weight")), o_b=f32(get(a + "out_proj.bias")),
                ln2_w=f32(get(lp + "layer_norm2.weight")), ln2_b=f32(get(lp + "layer_norm2.bias")),
                fc1_w=fc1_w, fc1_b=fc1_b, fc2_w=fc2_w, fc2_b=f32(get(lp + "mlp.fc2.bias"))))
        self.post_w = f32(get(pre + "post_layernorm.weight"))
        self.post_b = f32(get(pre + "post_layernorm.bias"))
        self.proj_w = bf(get("multi_modal_projector.linear.weight")) if "proj" in self.parts else None
        self.proj_dim = self.proj_w.shape[0] if self.proj_w is not None else 0

    def _pack_text(self, t, get, dev, bf, f32):
        # ---------------- Gemma
        R, W = self.tp_rank, self.tp_world
        self.hidden = t["hidden_size"]
        self.heads_total = t["num_attention_heads"]
        self.kv_heads = t["num_key_value_heads"]
        self.head_dim = t.get("head_dim", 256)
        self.inter_total = t["intermediate_size"]
        self.t_layers = t["num_hidden_layers"]
        self.vocab = t["vocab_size"]
        self.rope_theta = t.get("rope_theta", 10000.0)
        if self.heads_total % W or (self.heads_total // W) % self.kv_heads:
            raise ValueError(f"{self.heads_total} q heads do not split over {W} ranks x {self.kv_heads} kv heads")
        if self.inter_total % (16 * W):
            raise ValueError("intermediate_size / tp_world must be a multiple of 16 for the gate/up interleave")
        if self.vocab % W:
            raise ValueError(f"vocab_size {self.vocab} does not split over {W} ranks")
        if self.head_dim % 16:
            raise ValueError("head_dim must be a multiple of 16 for the fused RoPE epilogue")
        if t.get("attention_bias"):
            # GemmaAttention creates q/k/v/o biases when attention_bias is set (modeling_gemma.py:255-259) and
            # the reference adds them; the HIP q|k|v and o epilogues carry none, so refuse rather than diverge
            raise NotImplementedError("attention_bias=True is not supported by the HIP Gemma path")
        self.heads = self.heads_total // W                    # q heads held by this rank
        self.inter_real = self.inter_total // W               # intermediate slice held by this rank
        self.inter = _rup(self.inter_real, 128 if self.fp8 else 64)   # kernel width: zero-padded to the GEMM K step
        self.vocab_local = self.vocab // W
        self.vocab_offset = R * self.vocab_local
        hd, H, I = self.head_dim, self.hidden, self.inter
        q_lo, q_hi = R * self.heads * hd, (R + 1) * self.heads * hd
        Ir = self.inter_real
        i_lo, i_hi = R * Ir, (R + 1) * Ir
        perm = rope_row_perm(hd).to(dev)
        nblk = self.heads + 2 * self.kv_heads
        lm = "language_model."
        self.embed = bf(get(lm + "model.embed_tokens.weight"))
        # tied lm_head rows of this rank's vocabulary slice (a view of the embedding when no padding is
        # needed; the GEMM wants N % 4 == 0, so an odd-sized slice gets a zero-padded copy)
        vo, vl = self.vocab_offset, self.vocab_local
        bias = f32(get(lm + "lm_head.bias"))[vo:vo + vl]
        # every Gemma matrix must be packable (N % 16, K % 64), else all stay row-major (toy TP shards)
        self.frag = (self.hidden % 64 == 0 and (self.heads * self.head_dim) % 64 == 0 and
                     ((self.heads + 2 * self.kv_heads) * self.head_dim) % 16 == 0)
        pad_to = 16 if self.frag else 4
        self.vocab_local_pad = _rup(vl, pad_to)
        if self.vocab_local_pad == vl and not self.frag:
            self.lm_w, self.lm_bias = self.embed[vo:vo + vl], bias.contiguous()
        else:
            lm_w = torch.zeros(self.vocab_local_pad, self.hidden, dtype=torch.bfloat16, device=dev)
            lm_w[:vl] = self.embed[vo:vo + vl]
            self.lm_w = frag_pack(lm_w) if self.frag else lm_w
            del lm_w
            self.lm_bias = torch.zeros(self.vocab_local_pad, dtype=torch.float32, device=dev)
            self.lm_bias[:vl] = bias
        self.tl = []
        for i in range(self.t_layers):
            lp = f"{lm}model.layers.{i}."
            a = lp + "self_attn."
            for nm in ("q_proj.bias", "k_proj.bias", "v_proj.bias", "o_proj.bias"):
                try:
                    b = get(a + nm)
                except LookupError:         # KeyError / IndexError of a mapping-style loader: the key is absent
                    continue
                if b is not None:
                    raise NotImplementedError(f"{a + nm}: Gemma attention biases are not supported by the HIP path")
            qkv_w = torch.cat([bf(get(a + "q_proj.weight")[q_lo:q_hi]), bf(get(a + "k_proj.weight")),
                               bf(get(a + "v_proj.weight"))], 0)
            qkv_w = qkv_w.view(nblk, hd, H)[:, perm, :].reshape(nblk * hd, H).contiguous()
            g = torch.zeros(I, H, dtype=torch.bfloat16, device=dev)      # padded rows: gelu(0) * 0 = 0
            u = torch.zeros(I, H, dtype=torch.bfloat16, device=dev)
            g[:Ir] = bf(get(lp + "mlp.gate_proj.weight")[i_lo:i_hi])
            u[:Ir] = bf(get(lp + "mlp.up_proj.weight")[i_lo:i_hi])
            gu = torch.stack([g.view(I // 16, 16, H), u.view(I // 16, 16, H)], dim=1).reshape(2 * I, H).contiguous()
            down = torch.zeros(H, I, dtype=torch.bfloat16, device=dev)
            down[:, :Ir] = bf(get(lp + "mlp.down_proj.weight")[:, i_lo:i_hi])
            o_w = bf(get(a + "o_proj.weight")[:, q_lo:q_hi])
            pk = frag_pack if self.frag else (lambda x: x)
            layer = dict(
                in_w=f32(get(lp + "input_layernorm.weight")), qkv_w=pk(qkv_w), o_w=pk(o_w),
                post_w=f32(get(lp + "post_attention_layernorm.weight")), gu_w=pk(gu), down_w=pk(down))
            if self.frag and self.prefill_rowmajor and not self.fp8:
                # row-major copies for the large-M prefill GEMMs: gemm256's LDS-DMA tile loads run 7-11%
                # faster on them than on the fragment-packed image (scripts/tune/gemm_bench.py), and
                # 3.96 GB more of the 288 GB HBM is cheap
                layer.update(qkv_wr=qkv_w, o_wr=o_w, gu_wr=gu, down_wr=down)
            if self.fp8:
                if H % 128 or (self.heads * hd) % 128:
                    raise ValueError("fp8 weights need hidden and heads*head_dim multiples of 128")
                for name, m in (("qkv", qkv_w), ("o", o_w), ("gu", gu), ("down", down)):
                    layer[name + "_w8"], layer[name + "_s8"] = quant_rows_fp8(m)
                    if m.shape[0] % 16 == 0 and m.shape[1] % 128 == 0:
                        # fragment-packed copy for the fp8 decode GEMV (17..32 rows; the tile GEMMs read _w8)
                        layer[name + "_w8f"] = frag_pack8(layer[name + "_w8"])
            self.tl.append(layer)
            del qkv_w, o_w, gu, down
            del g, u
        self.lm_w8f = self.lm_s8 = None
        if self.fp8 and self.hidden % 128 == 0 and self.vocab_local_pad % 16 == 0:
            # the tied lm_head as fp8 rows too (per-row scales, fragment-packed) for the batch > 16 decode GEMV
            lmr = frag_unpack(self.lm_w) if self.frag else self.lm_w
            w8, self.lm_s8 = quant_rows_fp8(lmr)
            self.lm_w8f = frag_pack8(w8)
            del lmr, w8
        self.final_w = f32(get(lm + "model.norm.weight"))
        self.wflag = 0x100 if self.frag else 0            # ops.W_FRAG for every Gemma linear
        self.qkv_n = (self.heads + 2 * self.kv_heads) * hd

    def nbytes(self) -> int:
        n = 0
        for k, x in vars(self).items():
            if isinstance(x, torch.Tensor):
                n += x.numel() * x.element_size()
        for lst in (self.vl, self.tl):
            for d in lst:
                n += sum(x.numel() * x.element_size() for x in d.values())
        return n

    def decode_weight_bytes(self) -> int:
        """HBM bytes of weights one decode step streams (Gemma linears + tied lm_head)."""
        n = sum(sum(d[k].numel() * 2 for k in ("qkv_w", "o_w", "gu_w", "down_w")) for d in self.tl)
        return n + self.lm_w.numel() * 2

    def decode_weight_bytes_fp8(self) -> int:
        """The same for the fp8 path (batch > 16 decode): e4m3 linears + scales, e4m3 lm_head + scales (bf16 when
        no fp8 copy was packed)."""
        n = sum(sum(d[k + "_w8"].numel() + d[k + "_s8"].numel() * 4 for k in ("qkv", "o", "gu", "down"))
                for d in self.tl)
        if self.lm_w8f is not None:
            return n + self.lm_w8f.numel() + self.lm_s8.numel() * 4
        return n + self.lm_w.numel() * 2
