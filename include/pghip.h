/* libpghip — MI355X (gfx950) kernels for the PaliGemma image->text path.
 *
 * Drop-in boundary.  The reference has no FFI: its interface is the Python module API
 * (SURVEY.md §8(b)).  The Python drop-in modules in paligemma-multimodal-system_amd/
 * (modeling_siglip.py, modeling_gemma.py, modeling_paligemma.py, inference.py) keep
 * that API and call ONLY these entry points (through ctypes, pghip/_lib.py).  Each
 * entry point replaces the torch ops at the reference call sites cited below.
 *
 * Conventions: plain device pointers + sizes; every call enqueues on `stream`
 * (hipStream_t; pass torch.cuda.current_stream().cuda_stream), never allocates,
 * never synchronises, and returns 0 or a hipError_t code (hipErrorInvalidValue, before
 * any HIP call, for a rejected shape or a null required operand).  bf16 = IEEE bfloat16
 * bits in uint16; "f32" = float.
 * Buffers are owned by the caller (PyTorch's caching allocator).
 */
#ifndef PGHIP_H
#define PGHIP_H
#include <stdint.h>
#include <hip/hip_runtime_api.h>

#ifdef __cplusplus
extern "C" {
#endif

int pg_abi_version(void);   /* 13: PG_EPI_F32_RES (the prefill residual add in the producing tile GEMM), pg_attn_probs
                              (the modules' attention weights); 12: PgFusedArgs.status (FX_ADD range check), amax_zero on the bf16 GEMV, the xGMI
                              reduce-scatter + all-gather (pg_allreduce_xgmi_rs) and err diagnostics; 11: PgFusedArgs mx_out / mx_in (MX block-scaled fp8 decode MLP rows); 10: PG_EPI_FX_ADD + PgFusedArgs.fx (bit-reproducible decode residual); 9: PgFusedArgs amax_out / amax_in (pro_mode 5) / amax_zero, PG_ATTN_PIPE; 8: pg_allreduce_xgmi_slabs, PG_EPI_F32_ADD; 7: pg_attn_decode's optional fp8 row copy (q8 / q8_scale / q8_ld); 6: decode-order KV copies (PgFusedArgs.kd / vd; pg_attention, pg_attn_decode read
                              them); 5: pg_attn_decode; 4: the measured-slower decode variants removed */
/* sha256 (hex, 64 chars + NUL) of the csrc/ sources, include/pghip.h and the compile flags this library was built
 * from (pghip/build.py).  The Python loader refuses a library whose hash differs from the tree it runs from.
 * Returns hipErrorInvalidValue (truncated) when n < 65. */
int pg_source_hash(char* out, int n);

/* Epilogues of pg_gemm */
enum {
  PG_EPI_BF16 = 0,          /* C bf16 = acc + bias                                              */
  PG_EPI_BF16_GELU = 1,     /* C bf16 = gelu_tanh(acc + bias)          SiglipMLP fc1 (siglip:183-184) */
  PG_EPI_BF16_GELU_MUL = 2, /* C bf16 [M][N/2] = gelu(gate)*up, W rows interleaved 16 gate/16 up
                               GemmaMLP gate/up (gemma:212-217)                                  */
  PG_EPI_F32 = 3,           /* C f32 [ksplit][M][ldc] partial slabs (+bias on slab 0)          */
  PG_EPI_F32_POS = 4,       /* C f32 = acc + bias + aux[(m % aux_rows)*ldc + n]   patch+pos emb  */
  PG_EPI_BF16_VT = 5,       /* cols < aux_n -> C bf16; cols >= aux_n -> aux_out[(n-aux_n)*aux_ld + m] */
  PG_EPI_QKV_ROPE = 6,      /* fused q|k|v (rope-permuted W rows): RoPE(q) -> C, RoPE(k) -> K cache, v -> V^T
                               cache (gemma.py:274-302 + KVCache.update :18-57); pg_gemm_fused only          */
  PG_EPI_F32_FIN = 7,       /* M <= 4: F32 slabs, then the last split of each 16-column tile adds them into
                               fin_resid and writes ss_out (the residual add of gemma.py:401,416 + the next
                               RMSNorm's sum of squares); pg_gemm_fused only                                  */
  PG_EPI_F32_ADD = 8,       /* (ABI 8) M <= 16, pro_mode 0 or 2: C f32 [M][ldc] += acc (+ bias by split 0) by
                               hardware float atomic adds in any split order (the residual add of gemma.py:401,416
                               with no slab or ticket; the next GEMV normalises with pro_mode 1, nsplit 0)       */
  PG_EPI_FX_ADD = 9,        /* (ABI 10) M <= 16, bf16, pro_mode 0 or 2: C int64 [M][ldc] += round(acc * 2^32) (+ bias by
                               split 0) by 64-bit integer atomics -- F32_ADD's residual add, but the fixed-point sum is
                               exact and so the same bits in any split order (bit-reproducible decode).  C is the
                               PgFusedArgs.fx accumulator that pro_mode 1 and PG_EPI_F32_FIN consumers read      */
  PG_EPI_F32_RES = 10       /* (ABI 13) tile GEMMs (M > 16), ksplit 1, pro_mode 0: C f32 [M][ldc] += acc + bias -- the
                               prefill residual add (siglip:203-221, gemma.py:401,416) done by the producing GEMM, one
                               workgroup per output, so the next norm reads the residual alone (nsplit 0)        */
};

/* Fused-operation arguments of pg_gemm_fused (M <= 16 for the prologues). */
typedef struct PgFusedArgs {
  int pro_mode;             /* 0: x = A ; 1: x = RMSNorm(resid_in + sum partials)*(1+norm_w) (gemma.py:172-181) ;
                               2: x = merge of split-KV attention partials (pg_attn_combine folded in) ;
                               3: x = resid_in*(1+norm_w), rstd from ss_in applied to the outputs (RMSNorm of a
                                  residual finalised by a PG_EPI_F32_FIN producer) ;
                               4: x = A (the producer's fin_x = bf16(resid*(1+norm_w))), rstd from ss_in applied
                                  to the outputs (M <= 2)                                                     */
  const float* resid_in;
  float* resid_out;         /* written once: resid_in + sum partials (ping-pong residual stream; may be NULL) */
  const float* partials;    /* [nsplit][M][K] */
  int nsplit;
  const float* norm_w;
  float eps;
  const float* part_o;      /* [B][Hkv][asplit][16][dtw] from pg_attention (split mode) */
  const float* part_ml;     /* [B][Hkv][asplit][16][2] */
  int asplit, head_dim, dtw, q_per_kv, kv_heads;
  const float* cos_t;       /* [P][head_dim/2] */
  const float* sin_t;
  const int* pos;           /* rotary position per output row */
  int rows_per_batch;       /* row m -> batch m / L, cache slot slot_base + *slot_dev + m % L */
  const int* slot_dev;
  int slot_base;
  void* kc;                 /* bf16 [B][smax][kv_heads*head_dim] */
  void* vtc;                /* bf16 [B][kv_heads*head_dim][smax] */
  int smax;
  int q_heads;
  int* fin_cnt;             /* PG_EPI_F32_FIN: per-output-tile arrival tickets, zero-initialised, self-resetting */
  float* fin_resid;         /* PG_EPI_F32_FIN: residual [M][N] the split-K slabs are added into              */
  float* ss_out;            /* PG_EPI_F32_FIN: per-16-column-tile sum of squares [M][ss_ld]                   */
  const float* ss_in;       /* pro_mode 3: producer's per-tile sums of squares [M][ss_ld], ss_n tiles          */
  int ss_ld, ss_n;
  void* fin_x;              /* PG_EPI_F32_FIN (optional): bf16 [M][N] x' = resid*(1+norm_w) for a pro_mode 4 consumer */
  int akeys;                /* pro_mode 2: keys per attention split; with slot_dev (kv length before this token)
                               only the non-empty splits are merged                                            */
  const float* a_scale;     /* PG_FP8: [M] row scales of A (dequantised A = q * a_scale[m])                      */
  const float* w_scale;     /* PG_FP8: [N] row scales of W, in W's row order                                   */
  int slab_rows;            /* PG_EPI_F32 split-K: rows between slabs (slab z of row m at C + (z*slab_rows + m)*ldc);
                               0 = M.  Lets a GEMM be issued as row blocks that write into one [ksplit][rows][N]
                               partial tensor (C pointing at the block's first row)                            */
  void* kd;                 /* PG_EPI_QKV_ROPE (ABI 6, may be null): decode-order copies of the cache, [B][Hkv][Smax][D]
                               each, written beside kc / vtc (element offsets: csrc/attn_common.h dec_koff / dec_voff) */
  void* vd;
  /* ABI 9 -- the batched fp8 decode MLP without a quantiser launch (BASELINE configs[4]):                         */
  unsigned* amax_out;       /* PG_EPI_BF16_GELU_MUL with PG_FP8|PG_W_FRAG (optional): max |bf16 output| of row m is
                               atomically max-ed into amax_out[m * amax_ld] (float bits; zero beforehand)          */
  const unsigned* amax_in;  /* pro_mode 5 (PG_FP8|PG_W_FRAG, PG_EPI_F32, M <= 32): A is bf16 [M][lda elements],
                               quantised to e4m3 while staged, row scale s[m] = amax_in[m * amax_ld] / 448 (1 when
                               zero) -- pg_quant_fp8's bytes and scale; a_scale is not read                          */
  int amax_ld;
  unsigned* amax_zero;      /* optional, any PG_FP8|PG_W_FRAG launch: amax_zero[0 .. amax_zero_n) set to 0 (n <= 4096);
                               (ABI 12) any bf16 PG_W_FRAG GEMV (M <= 16): the same after its weight stream, n <= 16384,
                               n % 4 == 0, 16-B aligned (the batch-1 decode's first GEMV clears the fx accumulator)  */
  int amax_zero_n;
  /* ABI 10: */
  int64_t* fx;              /* fixed-point residual accumulator [M][K] (value = q * 2^-32, |value| < 2^31) written by
                               PG_EPI_FX_ADD producers; a PG_EPI_FX_ADD launch with resid_in set also adds those fp32
                               rows (split 0), after which fx holds the whole residual.  pro_mode 1: x =
                               RMSNorm(resid_in (may be NULL) + fx + sum partials) ; PG_EPI_F32_FIN (pro_mode != 1):
                               the finalised residual is fx + slabs (written to fin_resid, whose old rows are not
                               read), and the launch leaves fx zero (each tile's finalising workgroup clears its
                               entries)                                                                           */
  /* ABI 11 -- MX (OCP microscaling) rows for the batched fp8 decode MLP: one E8M0 scale per 32 k, no quantiser launch */
  uint8_t* mx_out;          /* (ABI 12: also PG_FP8 without PG_W_FRAG at M > 32 -- the prefill 128 x 128 tile -- with the
                               scales in natural order [M][N/64], block kb of row m at m*(N/64) + kb; N % 128 == 0)
                               PG_EPI_BF16_GELU_MUL with PG_FP8|PG_W_FRAG, M <= 32, ksplit 1, (N/2) % 128 == 0: C is
                               written as e4m3 bytes [M][ldc bytes] of h = bf16(gelu(gate)*up) / 2^e, and mx_out
                               [M][4][N/256] the E8M0 byte e + 127 of each 32-column block kb at [m][kb % 4][kb / 4],
                               e = the smallest exponent with max|h| of the block <= 448 * 2^e (0 for a zero block),
                               clamped to [-127, 127] (e4m3 RNE of h / 2^e)                                          */
  const uint8_t* mx_in;     /* (ABI 12: also PG_FP8 without PG_W_FRAG, PG_EPI_F32, M > 32 -- the prefill down projection on
                               the 256 x 256 kernel -- with the scales in natural order [M][K/32], 4-B aligned)
                               PG_FP8|PG_W_FRAG (any epilogue but F32_ADD), M <= 32, pro_mode 0: A is e4m3 [M][lda]
                               with mx_out's block scales [M][4][K/128] (x = q * 2^(s - 127) per 32-k block); a_scale
                               is not read.  With ss_in (rows from pg_norm_residual_mx: sums of squares per 1024
                               columns, ss_n = K / 1024 <= 4, eps) the outputs are multiplied by the row's
                               rstd = rsqrt(sum ss_in[m*ss_ld + i] / K + eps)                                       */
  /* ABI 12: */
  int* status;              /* PG_EPI_FX_ADD (optional): set to 1 when an added value is non-finite or |v| >= 2^31; the
                               value is then saturated (+-2^30 as the accumulator's value, NaN as 0), so a caller that
                               finds *status set must treat the launch's results as invalid                           */
} PgFusedArgs;

/* Weight layout flag, OR-ed into `epi` of pg_gemm / pg_gemm_fused.  PG_W_FRAG: W is fragment-packed,
 * the HBM layout of the Gemma decoder weights (pghip/weights.py frag_pack): for 16-row block t and 64-wide
 * k chunk c, W[16t + r][64c + 16g + 8s + e] (r < 16, g < 4, s < 2, e < 8) is stored at element
 * ((((t * K/64 + c) * 2 + s) * 64 + 16g + r) * 8 + e): each GEMV wave-instruction then reads 1 KiB
 * contiguous, lane-linear.  Requires N % 16 == 0 and K % 64 == 0; ldw must equal K. */
#define PG_W_FRAG 0x100
/* PG_FP8 (pg_gemm_fused only, BASELINE configs[4]): A [M][K] and W [N][K] are fp8 e4m3 (OCP, one byte per
 * element, lda / ldw in bytes) with per-row scales PgFusedArgs.a_scale / w_scale; the fp32 accumulator of
 * C[m][n] is multiplied by a_scale[m] * w_scale[n] before the epilogue (bias, gelu*mul, RoPE/KV, fp32 slabs).
 * 16x16x128 block-scaled MFMA with unit block scales (2x the bf16 rate).  M > 16, K % 128 == 0, lda and ldw
 * multiples of 16, no prologue, epi in {BF16, BF16_GELU_MUL, F32, QKV_ROPE}. */
/* With PG_W_FRAG the fp8 W is packed per 16-row block t and 128-wide k chunk c as W[16t + r][128c + 64s + 16g + e]
 * (r, e < 16, g < 4, s < 2) at byte ((((t * K/128 + c) * 2 + s) * 4 + g) * 16 + r) * 16 + e (pghip/weights.py
 * frag_pack8): the 16x16x128 MFMA's own k order. */
#define PG_FP8 0x200
/* PG_TILE_M1 (bf16 tile GEMMs, 256 <= M <= 288: batch-1 prefill, 256 image rows + the prompt): all M rows
 * in ONE row tile per 128 output columns, so each weight tile streams from HBM once (the 256x256 tiling
 * spends a second row tile -- and a second weight read -- on the last M - 256 rows).  Measured on the
 * pt-224 Gemma gate/up (ks 1), down (ks 16) and o (ks 8) shapes. */
#define PG_TILE_M1 0x400
/* PG_TILE_N64 (tile GEMMs, M > 16, bf16 or fp8): 64 x 64 output tiles instead of 64 x 128 (or larger), twice
 * the workgroups without a K split, for small-M GEMMs whose 64 x 128 grid leaves CUs idle. */
#define PG_TILE_N64 0x800

/* C = A[M][K] . W[N][K]^T with fused epilogue.  nn.Linear call sites: siglip.py:59-62,71-75,156,177-178,
 * 183-185; paligemma.py:57,64; gemma.py:205-207,212-218,255-259,274-278,356,484,523.  K % 32 == 0
 * (% 64 when M > 16), N % 4 == 0.  M <= 16 takes the weight-streaming GEMV path. */
int pg_gemm(const void* A, int lda, const void* W, int ldw, const float* bias, void* C, int ldc,
            int M, int N, int K, int epi, int ksplit, const float* aux, int aux_rows, void* aux_out,
            int aux_ld, int aux_n, hipStream_t stream);

/* Split-K finalisation: C = epilogue(sum_z part[z]) for a GEMM first run with PG_EPI_F32 into nsplit fp32 slabs
 * [z][M][N] (bias in slab 0).  epi: PG_EPI_BF16 / _GELU / _GELU_MUL / _VT (aux_out, aux_ld, aux_n) / _QKV_ROPE
 * (fused).  Lets a small-M prefill GEMM with a non-linear epilogue split K across CUs. */
int pg_gemm_finalize(const float* part, int nsplit, void* C, int ldc, int M, int N, int epi, void* aux_out,
                     int aux_ld, int aux_n, const PgFusedArgs* fused, hipStream_t stream);

/* pg_gemm + fused prologue / RoPE-KV epilogue (decode layer in 5 launches). */
int pg_gemm_fused(const void* A, int lda, const void* W, int ldw, const float* bias, void* C, int ldc,
                  int M, int N, int K, int epi, int ksplit, const PgFusedArgs* fused, hipStream_t stream);

/* resid[row] += sum_s partials[s][row]; y = LayerNorm (mode 0, w, b) | Gemma RMSNorm (mode 1, (1+w)).
 * siglip.py:199,203,210,218,310,319 ; gemma.py:157-182,395,412,470.  y -> out bf16 (ldo) and/or out_f32. */
int pg_norm_residual(float* resid, const float* partials, int nsplit, int M_part, const float* w,
                     const float* b, void* out, int ldo, float* out_f32, const int* row_map, int M_out,
                     int H, int mode, float eps, int write_resid, hipStream_t stream);

/* Flash attention (bidirectional unless an additive mask is given; MQA/GQA by row stacking).
 * siglip.py:96-136 ; gemma.py:307-339 (repeat_kv :185-196 eliminated).  split_keys > 0: decode
 * split-KV partials, merge with pg_attn_combine; kcap > 0 = readable cache rows (Smax, multiple of 32): each split's
 * first block is loaded before the kv length is read (ABI 2), and (D a multiple of 32) K and V are read from the
 * decode-order copies kd / vd the QKV epilogue writes (PgFusedArgs.kd / vd, ABI 6; null otherwise). */
int pg_attention(const void* q, long q_rs, void* o, long o_rs, const void* k, long k_bs, long k_hs,
                 long k_rs, const void* vt, long vt_bs, long vt_hs, long vt_ds, const float* mask,
                 long mask_bs, long mask_rs, int B, int Lq, int Lkv, const int* lkv_dev, int Hq, int Hkv,
                 int D, float scale, int split_keys, int nsplit, float* part_o, float* part_ml,
                 int kcap, const void* kd, const void* vd, hipStream_t stream);
int pg_attn_combine(const float* part_o, const float* part_ml, int B, int Hq, int Hkv, int D, int nsplit,
                    void* o, long o_rs, hipStream_t stream);

/* The attention weights the reference's modules return, out fp32 [B][Hq][Lq][Lkv] with pg_attention's q / k / mask
 * addressing: probs = 1 softmax(q . k^T * scale + mask) (gemma.py:358), probs = 0 the scaled scores + mask before the
 * softmax (siglip.py:157 returns those).  The module API's opt-in (the flash kernels never form this matrix; at
 * pt-896 x32 it is 34 GB per layer). */
int pg_attn_probs(const void* q, long q_rs, const void* k, long k_bs, long k_hs, long k_rs, const float* mask,
                  long mask_bs, long mask_rs, int B, int Lq, int Lkv, int Hq, int Hkv, int D, float scale,
                  int probs, float* out, hipStream_t stream);

/* Batched split-KV decode attention with the split merge in the same launch (gemma.py:307-339 for one new position
 * per row; replaces pg_attention(split) + pg_attn_combine for B > 2, ABI 5).  The kcap/32 cache blocks of a
 * (batch, kv head) are cut into nsplit contiguous ranges for splits of nw (2 or 4) waves, nb rounds each (nw*nsplit <=
 * kcap/32 <= nw*nsplit*nb); the last-arriving split (one agent-scope ticket in counters[b*Hkv + kvh], left zero)
 * merges the partials and writes o[b][hq][0..D) bf16.  D = 32 or 256.  The cache must hold finite values in every
 * row below kcap (masked keys get weight 0 but their V is not zeroed).  q8 (optional, ABI 7; Hkv == 1 and
 * Hq*D/8 <= nw*64): the merging workgroup also writes the row as fp8 e4m3, q8[b*q8_ld + hq*D + d], with
 * q8_scale[b] -- the bytes pg_quant_fp8 makes from o, so the fp8 o_proj needs no quantiser launch.
 * nw | PG_ATTN_PIPE (D == 256, nw == 4, nb >= 2; ignored otherwise): the double-buffered form, one round's K/V in
 * flight while the previous round is computed (one wave per SIMD: for grids of at most one workgroup per CU). */
#define PG_ATTN_PIPE 0x100
int pg_attn_decode(const void* q, long q_rs, void* o, long o_rs, const void* kd, const void* vd, int B, int Lkv,
                   const int* lkv_dev, int Hq, int Hkv, int D, float scale, int kcap, int nsplit, int nw, int nb,
                   float* part_o, float* part_ml, int* counters, void* q8, float* q8_scale, long q8_ld,
                   hipStream_t stream);

/* RoPE (gemma.py:112-151) on q in place and k; k -> cache rows, v -> transposed cache (KVCache.update
 * gemma.py:18-57 as a static in-place append). */
int pg_rope_kv_write(void* qkv, int ldq, const int* pos, int T, int L, int Hq, int Hkv, int D,
                     const float* cosT, const float* sinT, void* kc, void* vtc, int Smax, int slot_base,
                     const int* slot_dev, hipStream_t stream);

/* Conv2d(k=s=patch, valid) input rows (siglip.py:258-263,285). */
int pg_patch_im2col(const float* px, int B, int C, int H, int W, int p, void* out, int ldk, hipStream_t stream);

/* masked_scatter order of image tokens (paligemma.py:121-122): exclusive count. */
int pg_image_rank(const int64_t* ids, int n, long image_id, int* rank, hipStream_t stream);

/* embed gather + merge + pad zero + *sqrt(H)  (paligemma.py:99-128,288 ; gemma.py:510-511). */
int pg_embed_merge(const int64_t* ids, const int* rank, int n, const void* embed, int V, const float* feat,
                   int n_feat, int H, long image_id, long pad_id, float img_scale, float normalizer,
                   float* out, hipStream_t stream);

/* greedy next token (inference.py:59,68), first index on ties; optional decode-state advance:
 * hist[*step][b] = token (only while *step < hist_rows), pos[b] += 1, *kv_len += 1, *step += 1. */
int pg_argmax(const float* logits, long ld, int B, int V, void* workspace, int64_t* out_ids,
              int64_t* hist, int hist_rows, int* step, int* pos, int* kv_len, hipStream_t stream);
/* pg_argmax, then the next decode step's input rows res[b] = pg_embed_merge of the winners (rank = nullptr:
 * image-token rank = count of earlier rows whose winner is the image token), in the same final launch;
 * the chained greedy loop of inference.py:59-80 then needs no separate embed launch per step.  B <= 1024. */
int pg_argmax_embed(const float* logits, long ld, int B, int V, void* workspace, int64_t* out_ids,
                    int64_t* hist, int hist_rows, int* step, int* pos, int* kv_len, const void* embed, int V_embed,
                    const float* feat, int n_feat, int H, long image_id, long pad_id, float img_scale,
                    float normalizer, float* res, hipStream_t stream);

/* vocabulary-parallel greedy for tensor parallelism: local (max, first global index) pairs [B][2] of a
 * vocab shard starting at vocab_offset; after an all-gather, pg_argmax_merge takes the global winner
 * (lowest index on ties, as torch.argmax) and advances the decode state like pg_argmax. */
int pg_argmax_pairs(const float* logits, long ld, int B, int V, int vocab_offset, void* workspace,
                    float* pairs, hipStream_t stream);
int pg_argmax_merge(const float* pairs, int world, int B, int64_t* out_ids, int64_t* hist, int hist_rows,
                    int* step, int* pos, int* kv_len, hipStream_t stream);

/* softmax(logits/T) + top-p filter (inference.py:65,90-102) + explicit-uniform inverse-CDF draw.
 * uniforms [hist_rows][B] indexed by min(*step, hist_rows - 1); hist as pg_argmax. */
int pg_topp_sample(const float* logits, long ld, int B, int V, float temperature, float top_p,
                   const float* uniforms, int64_t* out_ids, int64_t* hist, int hist_rows, int* step, int* pos,
                   int* kv_len, float* probs_out, hipStream_t stream);

/* Reference image pre-processing (processing_paligemma.py:13-73) on the device: PIL BICUBIC resize of an RGB
 * uint8 image [H][W][3] to S x S (Pillow Resample.c fixed-point passes; tables hb/hk (horizontal, rows
 * [y0, y0+rows) of the source) and vb/vk (vertical) from pghip/image.py; null = no pass on that axis),
 * then out[c][y][x] = lut[u8] (rescale 1/255 + normalise).  tmp: uint8 [rows][S][3]. */
int pg_image_preprocess(const uint8_t* src, int H, int W, int S, const int* hb, const int* hk, int hks,
                        const int* vb, const int* vk, int vks, int y0, int rows, const float* lut, uint8_t* tmp,
                        float* out, hipStream_t stream);

/* name-seeded synthetic weights, bit-identical to oracle/synth.py (out_kind 0 bf16, 1 f32). */
int pg_synth_fill(void* out, long n, unsigned int seedmix, float a, float mean, int out_kind,
                  hipStream_t stream);

/* fp8 row quantisation feeding PG_FP8 GEMMs: q[m][k] = e4m3(x[m][k] / scale[m]), scale[m] = max|x[m][:]| / 448
 * (1 for an all-zero row).  x bf16 (row stride ldx), q bytes (row stride ldq).  K, ldx, ldq multiples of 8. */
int pg_quant_fp8(const void* x, int ldx, int M, int K, void* q, int ldq, float* scale, hipStream_t stream);
/* pg_norm_residual with y quantised as pg_quant_fp8 of its bf16 value: q uint8 [M_out][ldq], scale [M_out]
 * (one launch feeding a PG_FP8 GEMM; GemmaRMSNorm modeling_gemma.py:165-182 / nn.LayerNorm). */
int pg_norm_residual_fp8(float* resid, const float* partials, int nsplit, int M_part, const float* w,
                         const float* b, void* q, int ldq, float* scale, const int* row_map, int M_out,
                         int H, int mode, float eps, int write_resid, hipStream_t stream);
/* (ABI 11) Gemma RMSNorm for MX fp8 consumers (GemmaRMSNorm modeling_gemma.py:165-182 split at rstd): x = resid +
 * sum_s partials[s] (slab order; written back when write_resid), q uint8 [M][ldq] = e4m3 of y = x*(1+w) with one
 * E8M0 scale per 32 columns in qs [M][4][H/128] (the PgFusedArgs.mx_out rule), ss [M][ss_ld] = sum of x^2 per 1024
 * columns.  The consumer (an fp8 GEMV with mx_in = qs, ss_in = ss, ss_n = H/1024, eps) applies rstd to its outputs.
 * H % 1024 == 0; resid, partials, w 16-B aligned. */
int pg_norm_residual_mx(float* resid, const float* partials, int nsplit, int M_part, const float* w, void* q,
                        int ldq, void* qs, float* ss, int ss_ld, int M, int H, int write_resid, hipStream_t stream);

/* ---- one-shot all-reduce over xGMI (the reference is single-device, so this
 * replaces nothing there -- it is the tensor-parallel exchange of the Gemma decoder's o_proj / down_proj
 * partial sums -- o_proj at modeling_gemma.py:356 and down_proj at modeling_gemma.py:218, split across ranks).
 * Setup: each rank allocates one exchange buffer of pg_xgmi_buffer_bytes(world, cap) bytes with
 * pg_xgmi_alloc (uncached device memory), exports it with pg_xgmi_ipc_handle (64-byte handle), and maps
 * every peer's handle with pg_xgmi_ipc_open.  peers[r] = rank r's buffer as mapped in this process. */
int pg_xgmi_buffer_bytes(int world, long cap, long* bytes);
int pg_xgmi_alloc(long bytes, void** out);
int pg_xgmi_free(void* p);
int pg_xgmi_ipc_handle(void* p, void* handle64);
int pg_xgmi_ipc_open(const void* handle64, void** out);
int pg_xgmi_ipc_close(void* p);
/* In-place SUM of data[0, n) fp32 over `world` ranks (<= 8): every rank stores its data into slot `rank`
 * of every peer's buffer, raises a per-workgroup flag there, waits for the peers' flags in its own buffer
 * and sums the slots in rank order 0..world-1 (bit-identical result on every rank).  epochs: 64 local
 * zero-initialised u32 words owned by the communicator; err: 8 local ints (ABI 12), err[0] set to 1 if a peer did
 * not arrive within 20 s, and the first timeout's diagnostics in err[1..6]: kind (1 one-shot, 2 reduce-scatter,
 * 3 all-gather phase of pg_allreduce_xgmi_rs), workgroup, peer rank waited for, epoch expected, flag value seen, this
 * rank.  Once err[0] is set later calls skip their waits (results invalid).  n % 4 == 0, n <= cap, data 16-byte
 * aligned.  Device-side state only, so the call can be captured into a hipGraph; every rank must issue the same
 * sequence of calls. */
int pg_allreduce_xgmi(float* data, long n, int rank, int world, void* const* peers, long cap,
                      unsigned* epochs, int* err, hipStream_t stream);
/* (ABI 8) The same SUM where each rank contributes the sum of its nslab (1..64) split-K slabs
 * data[s * slab_stride + i], s = 0..nslab-1 in order (slab_stride >= n, a multiple of 4): the result is written
 * to data[0, n).  A row-parallel o_proj / down_proj then moves one slab over xGMI, with no slab-sum launch. */
int pg_allreduce_xgmi_slabs(float* data, long n, int nslab, long slab_stride, int rank, int world,
                            void* const* peers, long cap, unsigned* epochs, int* err, hipStream_t stream);
/* All-gather in rank order over the same exchange: out[r*n + i] = rank r's in[i] (the vocabulary-parallel
 * lm_head logits; replaces the zero-padded SUM that moved W x the bytes).  in != out, both
 * 16-byte aligned; otherwise as pg_allreduce_xgmi, whose buffer and epochs it shares (calls may interleave). */
int pg_allgather_xgmi(const float* in, long n, float* out, int rank, int world, void* const* peers, long cap,
                      unsigned* epochs, int* err, hipStream_t stream);
/* (ABI 12) Large messages (the prefill's row-chunk all-reduces after o_proj / down_proj, modeling_gemma.py:356 and
 * :218 split across ranks; up to 32 MB): reduce-scatter + all-gather over a second buffer per rank of
 * pg_xgmi_rs_buffer_bytes(world, rs_cap) bytes (allocated, exported and mapped like the exchange buffer).  Chunks of
 * world x 1024 floats; rank p sums sub-piece p of every chunk in rank order (the same bits as pg_allreduce_xgmi_slabs)
 * and stores it into every rank's gather slot.  2(W-1)/W * n floats leave each rank instead of (W-1) * n.
 * nslab / slab_stride as pg_allreduce_xgmi_slabs; nwg (1..256) workgroups, the same on every rank and call (a workgroup
 * waits only for the same workgroup of its peers: no grid-wide co-residency needed); epochs: 256 local zero-initialised
 * u32 words owned by this RS buffer; err as above.  n % 4 == 0, n <= rs_cap, data 16-byte aligned. */
int pg_xgmi_rs_buffer_bytes(int world, long rs_cap, long* bytes);
int pg_allreduce_xgmi_rs(float* data, long n, int nslab, long slab_stride, int rank, int world, void* const* peers,
                         long rs_cap, int nwg, unsigned* epochs, int* err, hipStream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* PGHIP_H */
