// bf16 MFMA GEMMs with fused epilogues:  C[m][n] = sum_k A[m][k] * W[n][k]  (+ epilogue)
//
// A: activations, bf16 row-major (lda).  W: nn.Linear weight layout [N][K] (ldw),
// bf16, K zero-padded to a multiple of 64 at pack time.  fp32 accumulation.
//
// Two kernels:
//  * gemm_tile_kernel : 128x128x64 tiles, 4 waves (2x2, 64x64 each), A and W tiles
//    staged HBM->LDS by global_load_lds (16 B/lane) into a double-buffered,
//    XOR-swizzled LDS image; mfma_f32_16x16x32_bf16 with the operands swapped
//    (MFMA-A = W, MFMA-B = A) so each lane ends with 4 consecutive n of one m —
//    8/16-byte epilogue stores.  Used for prefill (M = tokens).
//  * gemv_kernel      : M <= 16 (decode).  Weight streaming: each wave reads
//    16 rows of W with 16U-byte contiguous loads per lane straight
//    into VGPRs (no LDS round trip), the k order inside an MFMA step is permuted
//    identically for both operands so a lane's bytes are contiguous; 4 waves per
//    workgroup split K and reduce through LDS; an optional second level of
//    split-K writes fp32 partial slabs that the next norm kernel reduces.
//
// Replaces the nn.Linear call sites of modeling_siglip.py:59-62,177-178,
// modeling_paligemma.py:57, modeling_gemma.py:205-207,255-259,484.
//
// Translation units (compiled in parallel; this header holds what they share -- the fused arguments and the
// epilogues): gemm_tile.hip (prefill tile GEMMs, split-K finalisation), gemm_gemv.hip (bf16 decode GEMV),
// gemm_gemv8.hip (fp8 decode GEMV), gemm.hip (argument checks and the C-ABI entry points).
#pragma once
#include <cstdlib>
#include <type_traits>

#include "attn_common.h"

#ifndef PG_G256_STAGGER
#define PG_G256_STAGGER 1       // gemm256: wave groups one barrier apart (MFMA of one || LDS reads of the other); +4-14%
#endif
#ifndef PG_G256_F8_BUF
#define PG_G256_F8_BUF 1        // gemm256 fp8: operand pieces through buffer resources (two lane offsets, no spills)
#endif
#ifndef PG_G256_PREFETCH
#define PG_G256_PREFETCH 1      // gemm256: LDS reads one phase ahead of the MFMAs
#endif

enum {
  PG_EPI_BF16 = 0,          // C bf16 = acc + bias
  PG_EPI_BF16_GELU = 1,     // C bf16 = gelu_tanh(acc + bias)
  PG_EPI_BF16_GELU_MUL = 2, // W rows interleaved in 16-row blocks (gate, up); C bf16 [M][N/2] = gelu(g)*u
  PG_EPI_F32 = 3,           // C f32 [z][M][ldc] = acc (+ bias on split 0)
  PG_EPI_F32_POS = 4,       // C f32 = acc + bias + aux[(m % aux_rows) * ldc + n]  (patch + position emb)
  PG_EPI_BF16_VT = 5,       // n < aux_n: C bf16 = acc + bias ; n >= aux_n: aux_out bf16 [(n-aux_n)][m] (ld aux_ld)
  PG_EPI_QKV_ROPE = 6,      // fused q|k|v projection (rope-permuted W rows): RoPE on q -> C, RoPE on k -> K cache,
                            // v -> V^T cache (GemmaAttention.forward :274-302 + KVCache.update)
  PG_EPI_F32_FIN = 7,       // GEMV (M <= 16) split-K slabs as PG_EPI_F32, then the last-arriving split of each
                            // output tile adds the slabs into fin_resid and writes the tile's sum of squares
                            // (ss_out): the residual add + RMSNorm statistics of the NEXT norm, done in-kernel
  PG_EPI_F32_ADD = 8,       // GEMV (M <= 16): C f32 [M][ldc] += acc (+ bias by split 0) with hardware float atomic
                            // adds, any split count (the residual add of a row-parallel decode linear, no slabs)
  PG_EPI_FX_ADD = 9,        // GEMV (M <= 16, bf16): C int64 [M][ldc] += rn(acc * 2^32) (+ bias by split 0) with
                            // 64-bit integer atomics: F32_ADD's one-round-trip tail, but the sum is exact and so
                            // independent of the split order -- bit-reproducible decode (PgFusedArgs.fx)
  PG_EPI_F32_RES = 10,      // tile GEMMs (M > 16), ksplit 1: C f32 [M][ldc] += acc + bias -- the residual add of the
                            // next norm done by the producer (each output has ONE producing workgroup: plain RMW)
};

// the fixed-point residual accumulator (PG_EPI_FX_ADD, PgFusedArgs.fx): value = q * 2^-32, |value| < 2^31
#define PG_FX_SCALE 0x1p32f
#define PG_FX_INV 0x1p-32f
// rn(v * 2^32) as int64 without __float2ll_rn's emulation: integer part t (exact), the fraction scaled by 2^32 and
// rounded (exact, |r| <= 2^32), r split into 16-bit halves (exact) -- equal to llrintf(v * 2^32) for |v| < 2^31
// (checked on the host over 14 M values and the edge cases)
__device__ __forceinline__ long long fx_from_f32(float v) {
  const float t = truncf(v);
  const int hi = (int)t;
  const float r = rintf((v - t) * PG_FX_SCALE);
  const float rh = truncf(r * 0x1p-16f);
  const float rl = fmaf(rh, -65536.f, r);
  return (long long)((unsigned long long)(long long)hi << 32) + ((long long)(int)rh << 16) + (long long)(int)rl;
}
// (consumers convert every entry of a row in every workgroup, so this is 3 VALU ops instead of __ll2float_rn's 12:
// q = hi * 2^32 + lo with hi = q >> 32 (arithmetic), lo the unsigned low word; value = hi + lo * 2^-32, rounded twice --
// a fixed function of q's bits, so every reader gets the same float)
// The range-checked form the FX_ADD epilogue uses: a value the accumulator cannot hold (|v| >= 2^31, or NaN / Inf) is
// saturated to +-2^62 (NaN: 0) -- far outside any residual, without the int conversion's undefined behaviour -- and
// reported through *status (PgFusedArgs.status, may be null)
__device__ __forceinline__ long long fx_from_f32_checked(float v, int* status) {
  if (__builtin_expect(!(fabsf(v) < 0x1p31f), 0)) {
    if (status) atomicOr(status, 1);
    return v > 0.f ? (1LL << 62) : (v < 0.f ? -(1LL << 62) : 0LL);
  }
  return fx_from_f32(v);
}
__device__ __forceinline__ float fx_to_f32(long long q) {
  return fmaf((float)(unsigned)(unsigned long long)q, PG_FX_INV, (float)(int)(q >> 32));
}
typedef long long i64x2 __attribute__((ext_vector_type(2)));
// 4 consecutive accumulator entries as fp32 (two 16-B loads)
__device__ __forceinline__ f32x4 fx_load4(const long long* p) {
  const i64x2 a = *(const i64x2*)p, b = *(const i64x2*)(p + 2);
  return f32x4{fx_to_f32(a[0]), fx_to_f32(a[1]), fx_to_f32(b[0]), fx_to_f32(b[1])};
}

// Extra arguments of the fused entry point pg_gemm_fused (mirrors PgFusedArgs in include/pghip.h).
struct PgFusedArgs {
  // prologue: 0 = x read from A (bf16), 1 = x = RMSNorm(resid_in + sum partials) * (1 + norm_w),
  //           2 = x = merge of split-KV attention partials (pg_attn_combine folded into the GEMV)
  int pro_mode;
  const float* resid_in;
  float* resid_out;          // written once (workgroup 0) with resid_in + sum partials (may be null)
  const float* partials;     // [nsplit][M][K]
  int nsplit;
  const float* norm_w;
  float eps;
  const float* part_o;       // attention partials [B][Hkv][asplit][16][dtw]
  const float* part_ml;      // [B][Hkv][asplit][16][2]
  int asplit, head_dim, dtw, q_per_kv, kv_heads;
  // RoPE / KV-cache epilogue (PG_EPI_QKV_ROPE)
  const float* cos_t;
  const float* sin_t;
  const int* pos;            // rotary position per output row m
  int rows_per_batch;        // L (row m -> batch m / L, in-batch index m % L)
  const int* slot_dev;       // cache slot base from device memory (may be null)
  int slot_base;
  bf16_t* kc;                // [B][Smax][Hkv*D]
  bf16_t* vtc;               // [B][Hkv*D][Smax]
  int smax;
  int q_heads;
  // in-kernel split-K finalisation (PG_EPI_F32_FIN) and the prologue that consumes it (pro_mode 3:
  // x = resid_in * (1 + norm_w), rstd from ss_in applied to the accumulators: W.(x*rstd) = rstd*(W.x))
  int* fin_cnt;              // [gridDim.x] arrival tickets, zero between launches (the last arriver resets)
  float* fin_resid;          // [M][N] residual the slabs are added into
  float* ss_out;             // [M][ss_ld] per-tile sum of squares of the finalised residual
  const float* ss_in;        // [M][ss_ld] (consumer side), ss_n tiles per row
  int ss_ld, ss_n;
  bf16_t* fin_x;             // PG_EPI_F32_FIN (optional): x' = bf16(resid * (1 + norm_w)) [M][N] for a pro_mode 4
                             // consumer (x' read like A, rstd from ss_in applied to its outputs)
  int akeys;                 // pro_mode 2: keys per attention split; with slot_dev (= kv length before this
                             // token) only the ceil((*slot_dev + 1) / akeys) non-empty splits are merged
  // PG_FP8: A and W are fp8 e4m3 with per-row scales (dequantised value = q * scale): the accumulator of
  // C[m][n] is multiplied by a_scale[m] * w_scale[n] before the epilogue
  const float* a_scale;      // [M]
  const float* w_scale;      // [N] (in W's row order, e.g. the packed q|k|v or interleaved gate/up rows)
  int slab_rows;             // PG_EPI_F32 split-K: rows between slabs (0 = M); lets a GEMM run as row blocks
  // PG_EPI_QKV_ROPE (optional, ABI 6): the decode-order copies of the cache (kd / vd, attn_common.h dec_koff /
  // dec_voff), [B][Hkv][Smax][D] each: every appended k / v is also written there
  bf16_t* kd;
  bf16_t* vd;
  // ABI 9: the batched fp8 decode MLP without a quantiser launch -- the gate/up epilogue max-es each row's |h| into
  // amax_out (float bits); pro_mode 5 (down) stages bf16 h quantised with amax_in / 448; amax_zero is cleared by
  // the first workgroup of any fp8 GEMV launch (the QKV GEMV of the same layer)
  unsigned* amax_out;
  const unsigned* amax_in;
  int amax_ld;
  unsigned* amax_zero;
  int amax_zero_n;
  // ABI 10: the fixed-point residual accumulator [M][K] int64 (value q * 2^-32) that PG_EPI_FX_ADD producers add
  // into (with resid_in set, split 0 of an FX_ADD launch also adds those fp32 rows: the accumulator then holds the
  // whole residual).  pro_mode 1 normalises resid_in (optional with fx) + fx (+ partials); PG_EPI_F32_FIN finalises
  // fx + slabs (fin_resid is written, not read) and clears the fx entries it finalised (the accumulator is zero again
  // once the FIN launch ends)
  long long* fx;
  // ABI 11, MX (OCP microscaling) fp8 rows for the 17..32-row fp8 decode MLP: E8M0 scales, one per 32 consecutive k of
  // a row, stored [M][4][K/128] (row m's block g of 128-k chunk c at m*K/32 + g*K/128 + c: a lane's scales for the
  // chunks of its K split are consecutive bytes).  mx_out (gate/up: PG_EPI_BF16_GELU_MUL with PG_FP8|PG_W_FRAG): C is
  // the e4m3 h [M][ldc] bytes and mx_out its scales -- x = q * 2^(s - 127); mx_in (a PG_FP8|PG_W_FRAG consumer, the
  // down projection): A holds such rows and mx_in their scales, fed to the MFMA as its per-lane block scales (a_scale
  // is not read)
  uint8_t* mx_out;
  const uint8_t* mx_in;
  // ABI 12: PG_EPI_FX_ADD status word (optional): set to 1 when an added value is non-finite or |v| >= 2^31 -- it is
  // then saturated (the accumulator cannot hold it), so the caller must treat the step's results as invalid
  int* status;
};

// 4 consecutive fp32 values at p[n0..n0+3] (one 16-B load when fully inside [0, N), else guarded)
__device__ __forceinline__ f32x4 load4_guard(const float* __restrict__ p, int n0, int N) {
  if (n0 + 3 < N) return *(const f32x4*)(p + n0);
  f32x4 v = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int j = 0; j < 4; ++j) if (n0 + j < N) v[j] = p[n0 + j];
  return v;
}

#define PG_W_FRAG 0x100   // weight layout flag OR-ed into epi (include/pghip.h)
#define PG_TILE_M1 0x400  // one row tile of all M (256..288) rows (include/pghip.h)
#define PG_TILE_N64 0x800 // 64 x 64 tiles (include/pghip.h)
#define PG_FP8 0x200      // A and W fp8 e4m3 with row scales (PgFusedArgs a_scale / w_scale), M > 16

// fp8 GEMV: the wide form (x once per workgroup in LDS, waves split N), gemm_gemv8.hip; gemm.hip checks against it
#ifndef PG_GEMV8_WIDE
#define PG_GEMV8_WIDE 1
#endif

#define TBN 128   // tile GEMM: output columns per tile
#define TBK 64    // ... k per stage

struct EpiArgs {
  const float* bias;
  void* C;
  int ldc;
  int M, N;
  const float* aux;
  int aux_rows;
  bf16_t* aux_out;
  int aux_ld;
  int aux_n;
  PgFusedArgs f;
};

// fp8 dequantisation of one accumulator fragment: C[m][n0..n0+3] *= a_scale[m] * w_scale[n0..n0+3]
__device__ __forceinline__ void scale_acc(const EpiArgs& e, int m, int n0, f32x4& v) {
  if (m >= e.M || n0 >= e.N) return;
  v *= (e.f.mx_in ? 1.0f : e.f.a_scale[m]) * load4_guard(e.f.w_scale, n0, e.N);   // (MX rows: scaled in the MFMA)
}

// The fp8 GEMVs' row factor: a_scale[m]; MX rows (mx_in): 1, or with ss_in (rows from pg_norm_residual_mx: x*(1+w)
// quantised without its RMS) the RMSNorm's rstd = rsqrt(sum_i ss_in[m*ss_ld + i] / (1024*ss_n) + eps)
// Two halves so a kernel can issue the loads ahead of its weight stream and reduce them in the epilogue: every load
// is issued before any is used (ss_n <= 4, host-checked), one memory round trip
struct Fp8RowLoads {
  float v[4];
};
__device__ __forceinline__ Fp8RowLoads fp8_row_load(const EpiArgs& e, int m) {
  Fp8RowLoads r;
  m = min(m, e.M - 1);
  if (!e.f.mx_in) {
    r.v[0] = e.f.a_scale[m];
  } else if (e.f.ss_in) {
    const float* p = e.f.ss_in + (size_t)m * e.f.ss_ld;
#pragma unroll
    for (int i = 0; i < 4; ++i) r.v[i] = p[min(i, e.f.ss_n - 1)];
  }
  return r;
}
__device__ __forceinline__ float fp8_row_finish(const EpiArgs& e, const Fp8RowLoads& r) {
  if (!e.f.mx_in) return r.v[0];
  if (!e.f.ss_in) return 1.0f;
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < 4; ++i) s += i < e.f.ss_n ? r.v[i] : 0.f;
  return rsqrtf(s / (1024.0f * (float)e.f.ss_n) + e.f.eps);
}
__device__ __forceinline__ float fp8_row_factor(const EpiArgs& e, int m) { return fp8_row_finish(e, fp8_row_load(e, m)); }
// C[m][n0..n0+3] *= rf * w_scale[n0..n0+3] (rf = fp8_row_factor)
__device__ __forceinline__ void scale_acc_rf(const EpiArgs& e, int m, int n0, f32x4& v, float rf) {
  if (m >= e.M || n0 >= e.N) return;
  v *= rf * load4_guard(e.f.w_scale, n0, e.N);
}

// RoPE + KV append for 4 consecutive permuted columns n0..n0+3 of row m.  The q|k|v weight rows are
// packed so that 16-column tile t of every D-wide head block holds dims 8t..8t+7 then D/2+8t..D/2+8t+7:
// the rotate_half partner of a lane's 4 values sits in lane ^ 32.  ALL lanes must call (shuffle).
// v: columns n0..n0+3 (bias added), pr: the same four of the rotate_half partner columns (n0 ^ 8)
// index in [0, D/2) of column n0's rotary frequency, and whether n0 is in a q or k block (RoPE'd)
__device__ __forceinline__ int rope_freq_index(const PgFusedArgs& f, int n0, bool* roped) {
  const int D = f.head_dim, within = n0 % D, jj0 = within & 15;
  *roped = n0 / D < f.q_heads + f.kv_heads;
  return 8 * (within >> 4) + (jj0 & 7);
}
// the epilogue with the rotary cos/sin of its 4 columns and the cache slot base already loaded
__device__ __forceinline__ void epi_qkv_rope4_core(const EpiArgs& e, int m, int n0, f32x4 v, f32x4 pr, f32x4 cs,
                                                   f32x4 sn, int slot0) {
  if (m >= e.M || n0 >= e.N) return;
  const PgFusedArgs& f = e.f;
  const int D = f.head_dim, half = D >> 1;
  const int blk = n0 / D, within = n0 % D;
  const int t = within >> 4, jj0 = within & 15;
  const bool second = jj0 >= 8;
  const int ii = 8 * t + (jj0 & 7);                   // index in [0, D/2) of element 0
  const int d0 = second ? half + ii : ii;             // original dim of element 0
  const int b = m / f.rows_per_batch, i = m % f.rows_per_batch;
  const int slot = slot0 + i;
  const bool in_cache = slot < f.smax;                // a token past the static cache is not appended
  const int Hq = f.q_heads, Hkv = f.kv_heads;
  const int KV = Hkv * D;
  if (blk < Hq + Hkv) {
    f32x4 y;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      // q*cos + rotate_half(q)*sin, rotate_half(x) = cat(-x2, x1)  (modeling_gemma.py:138-151)
      y[j] = second ? v[j] * cs[j] + pr[j] * sn[j] : v[j] * cs[j] - pr[j] * sn[j];
    }
    u32x2 pk;
    pk[0] = pack_bf2(y[0], y[1]);
    pk[1] = pack_bf2(y[2], y[3]);
    if (blk < Hq) {
      *(u32x2*)((bf16_t*)e.C + (size_t)m * e.ldc + blk * D + d0) = pk;
    } else if (in_cache) {
      *(u32x2*)(f.kc + ((size_t)b * f.smax + slot) * KV + (blk - Hq) * D + d0) = pk;
      if (f.kd)     // 4 dims of one key: 8 contiguous bytes of one 16-B chunk
        *(u32x2*)(f.kd + ((size_t)b * Hkv + (blk - Hq)) * f.smax * D + dec_koff(slot, d0, D)) = pk;
    }
  } else {
    const int c0 = (blk - Hq - Hkv) * D + d0;
    if (in_cache) {
#pragma unroll
      for (int j = 0; j < 4; ++j) f.vtc[((size_t)b * KV + c0 + j) * f.smax + slot] = f2bf(v[j]);
      if (f.vd) {
        bf16_t* vd = f.vd + ((size_t)b * Hkv + (blk - Hq - Hkv)) * f.smax * D;
#pragma unroll
        for (int j = 0; j < 4; ++j) vd[dec_voff(slot, d0 + j, D)] = f2bf(v[j]);
      }
    }
  }
}

__device__ __forceinline__ void epi_qkv_rope4_pr(const EpiArgs& e, int m, int n0, f32x4 v, f32x4 pr) {
  if (m >= e.M || n0 >= e.N) return;
  const PgFusedArgs& f = e.f;
  bool roped;
  const int ii = rope_freq_index(f, n0, &roped);
  f32x4 cs = {1.f, 1.f, 1.f, 1.f}, sn = {0.f, 0.f, 0.f, 0.f};
  if (roped) {
    const int p = f.pos[m];
    const float* cp = f.cos_t + (long)p * (f.head_dim >> 1) + ii;
    const float* sp = f.sin_t + (long)p * (f.head_dim >> 1) + ii;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      cs[j] = cp[j];
      sn[j] = sp[j];
    }
  }
  epi_qkv_rope4_core(e, m, n0, v, pr, cs, sn, f.slot_base + (f.slot_dev ? *f.slot_dev : 0));
}

__device__ __forceinline__ void epi_qkv_rope4(const EpiArgs& e, int m, int n0, f32x4 v) {
  if (e.bias && n0 < e.N) v += load4_guard(e.bias, n0, e.N);   // bias in packed (permuted) column order
  f32x4 pr;
#pragma unroll
  for (int j = 0; j < 4; ++j) pr[j] = xchg_xor32(v[j]);
  epi_qkv_rope4_pr(e, m, n0, v, pr);
}

// PG_EPI_F32_RES in two halves, so a row subtile's residual loads are all issued before its first store (the
// compiler cannot move a load of C above an earlier store to C: one load latency per store otherwise)
__device__ __forceinline__ f32x4 res_load4(const EpiArgs& e, int m, int n0) {
  f32x4 r = {0.f, 0.f, 0.f, 0.f};
  if (m >= e.M || n0 >= e.N) return r;
  const float* C = (const float*)e.C + (size_t)m * e.ldc;
  if (n0 + 3 < e.N) return *(const f32x4*)(C + n0);
#pragma unroll
  for (int j = 0; j < 4; ++j) if (n0 + j < e.N) r[j] = C[n0 + j];
  return r;
}
__device__ __forceinline__ void res_store4(const EpiArgs& e, int m, int n0, f32x4 v, f32x4 r) {
  if (m >= e.M || n0 >= e.N) return;
  if (e.bias) v += load4_guard(e.bias, n0, e.N);
  float* C = (float*)e.C + (size_t)m * e.ldc;
  const f32x4 o = r + v;                                 // (resid + (acc + bias): the norm kernel's one add)
  if (n0 + 3 < e.N) {
    *(f32x4*)(C + n0) = o;
  } else {
#pragma unroll
    for (int j = 0; j < 4; ++j) if (n0 + j < e.N) C[n0 + j] = o[j];
  }
}

// Store 4 consecutive columns n0..n0+3 of row m (values v).  z = split index.
template <int EPI>
__device__ __forceinline__ void epi_store4(const EpiArgs& e, int m, int n0, f32x4 v, int z) {
  if (m >= e.M || n0 >= e.N) return;
  if (e.bias && (EPI != PG_EPI_F32 || z == 0)) v += load4_guard(e.bias, n0, e.N);
  if constexpr (EPI == PG_EPI_F32) {
    const size_t srows = e.f.slab_rows > 0 ? (size_t)e.f.slab_rows : (size_t)e.M;
    float* C = (float*)e.C + ((size_t)z * srows + m) * e.ldc;
    if (n0 + 3 < e.N) {
      *(f32x4*)(C + n0) = v;
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) if (n0 + j < e.N) C[n0 + j] = v[j];
    }
  } else if constexpr (EPI == PG_EPI_F32_RES) {
    float* C = (float*)e.C + (size_t)m * e.ldc;
    if (n0 + 3 < e.N) {
      *(f32x4*)(C + n0) = *(const f32x4*)(C + n0) + v;      // (resid + (acc + bias): the norm kernel's one add)
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) if (n0 + j < e.N) C[n0 + j] = C[n0 + j] + v[j];
    }
  } else if constexpr (EPI == PG_EPI_F32_POS) {
    float* C = (float*)e.C + (size_t)m * e.ldc;
    v += load4_guard(e.aux + (size_t)(m % e.aux_rows) * e.ldc, n0, e.N);
    if (n0 + 3 < e.N) {
      *(f32x4*)(C + n0) = v;
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) if (n0 + j < e.N) C[n0 + j] = v[j];
    }
  } else {
    // bf16 outputs
    if constexpr (EPI == PG_EPI_BF16_GELU) {
#pragma unroll
      for (int j = 0; j < 4; ++j) v[j] = gelu_tanh(v[j]);
    }
    if constexpr (EPI == PG_EPI_BF16_VT) {
      if (n0 >= e.aux_n) {
#pragma unroll
        for (int j = 0; j < 4; ++j)
          if (n0 + j < e.N) e.aux_out[(size_t)(n0 + j - e.aux_n) * e.aux_ld + m] = f2bf(v[j]);
        return;
      }
    }
    bf16_t* C = (bf16_t*)e.C + (size_t)m * e.ldc;
    if (n0 + 3 < e.N) {
      u32x2 p;
      p[0] = pack_bf2(v[0], v[1]);
      p[1] = pack_bf2(v[2], v[3]);
      *(u32x2*)(C + n0) = p;
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) if (n0 + j < e.N) C[n0 + j] = f2bf(v[j]);
    }
  }
}

// C[m][n0..n0+3] += v (+ bias by split 0) with hardware float atomic adds (PG_EPI_F32_ADD; unordered over splits)
__device__ __forceinline__ void epi_add4(const EpiArgs& e, int m, int n0, f32x4 v, int z) {
  if (m >= e.M || n0 >= e.N) return;
  if (e.bias && z == 0) v += load4_guard(e.bias, n0, e.N);
  float* dst = (float*)e.C + (size_t)m * e.ldc + n0;
#pragma unroll
  for (int j = 0; j < 4; ++j)
    if (n0 + j < e.N) unsafeAtomicAdd(dst + j, v[j]);
}

// gelu(gate) * up for an interleaved pair: gate tile at global col base gb (multiple of 32),
// lane's 4 columns are gb + q..q+3 (gate) and gb + 16 + q.. (up); output col = gb/2 + q.
__device__ __forceinline__ void epi_gelu_mul4(const EpiArgs& e, int m, int gb, int q, f32x4 g, f32x4 u) {
  if (m >= e.M) return;
  const int oc = (gb >> 1) + q;
  if (oc + 3 >= (e.N >> 1)) return;
  u32x2 p;
  p[0] = pack_bf2(gelu_tanh(g[0]) * u[0], gelu_tanh(g[1]) * u[1]);
  p[1] = pack_bf2(gelu_tanh(g[2]) * u[2], gelu_tanh(g[3]) * u[3]);
  *(u32x2*)((bf16_t*)e.C + (size_t)m * e.ldc + oc) = p;
}

// epi_gelu_mul4 that also returns max |bf16 output| of the four (0 when not stored): the per-row amax the fp8 down
// projection's prologue quantises h with (PgFusedArgs.amax_out / amax_in, pg_quant_fp8's rule)
__device__ __forceinline__ float epi_gelu_mul4_amax(const EpiArgs& e, int m, int gb, int q, f32x4 g, f32x4 u) {
  if (m >= e.M) return 0.f;
  const int oc = (gb >> 1) + q;
  if (oc + 3 >= (e.N >> 1)) return 0.f;
  u32x2 p;
  p[0] = pack_bf2(gelu_tanh(g[0]) * u[0], gelu_tanh(g[1]) * u[1]);
  p[1] = pack_bf2(gelu_tanh(g[2]) * u[2], gelu_tanh(g[3]) * u[3]);
  *(u32x2*)((bf16_t*)e.C + (size_t)m * e.ldc + oc) = p;
  return fmaxf(fmaxf(fabsf(bf_lo(p[0])), fabsf(bf_hi(p[0]))), fmaxf(fabsf(bf_lo(p[1])), fabsf(bf_hi(p[1]))));
}

// PgFusedArgs.amax_zero: the first workgroup clears amax_zero[0 .. n) (a later launch's amax_out)
__device__ __forceinline__ void amax_clear(const EpiArgs& e) {
  if (e.f.amax_zero && blockIdx.x == 0 && blockIdx.y == 0)
    for (int i = threadIdx.x; i < e.f.amax_zero_n; i += blockDim.x) e.f.amax_zero[i] = 0u;
}

// --------------------------------------------------------------------------------------
// Launchers of each translation unit (epi = the PG_EPI_* value without flags; every call enqueues one kernel
// on st and returns 0, or hipErrorInvalidValue for an epilogue that unit does not implement)
// --------------------------------------------------------------------------------------
// gemm_tile.hip: M > 16.  f8: A / W are fp8 byte pairs (K, lda, ldw in 2-byte units).  m1: PG_TILE_M1, n64: PG_TILE_N64
int pg_dispatch_tile(int epi, bool frag, bool f8, const bf16_t* A, int lda, const bf16_t* W, int ldw, int K, int ksplit,
                     const EpiArgs& e, hipStream_t st, bool m1, bool n64);
// gemm_gemv.hip: M <= 16, bf16
int pg_dispatch_gemv(int epi, bool frag, const bf16_t* A, int lda, const bf16_t* W, int ldw, int K, int ksplit,
                     const EpiArgs& e, hipStream_t st);
// gemm_gemv8.hip: M <= 32, fp8 fragment-packed W
int pg_dispatch_gemv8(int epi, const uint8_t* X, int ldx, const uint8_t* W, int K, int ksplit, const EpiArgs& e,
                      hipStream_t st);

