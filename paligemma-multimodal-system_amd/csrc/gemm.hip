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
#include <cstdlib>
#include <type_traits>

#include "attn_common.h"

#ifndef PG_G256_STAGGER
#define PG_G256_STAGGER 1       // gemm256: wave groups one barrier apart (MFMA of one || LDS reads of the other); +4-14%
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
};

// the fixed-point residual accumulator (PG_EPI_FX_ADD, PgFusedArgs.fx): value = q * 2^-32, |value| < 2^31
#define PG_FX_SCALE 0x1p32f
#define PG_FX_INV 0x1p-32f
__device__ __forceinline__ long long fx_from_f32(float v) { return __float2ll_rn(v * PG_FX_SCALE); }
// (consumers convert every entry of a row in every workgroup, so this is 3 VALU ops instead of __ll2float_rn's 12:
// q = hi * 2^32 + lo with hi = q >> 32 (arithmetic), lo the unsigned low word; value = hi + lo * 2^-32, rounded twice --
// a fixed function of q's bits, so every reader gets the same float)
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
  // into.  pro_mode 1 normalises resid_in + fx (+ partials); PG_EPI_F32_FIN finalises fin_resid + fx + slabs and
  // clears the fx entries it finalised (the accumulator is zero again once the FIN launch ends)
  long long* fx;
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
  v *= e.f.a_scale[m] * load4_guard(e.f.w_scale, n0, e.N);
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
// Tiled GEMM (prefill)
// --------------------------------------------------------------------------------------
// BM x 128 output tile, BK = 64, 4 waves (BM=128: 2x2 waves of 64x64; BM=96: 2x2 of 48x64;
// BM=64: 1x4 waves of 64x32).
// A and W k-tiles are staged HBM->LDS with global_load_lds (16 B/lane, 1 KiB pieces of 8 rows x
// 128 B, XOR-swizzled through the SOURCE address) into an STAGES-deep ring; the wait for stage kt
// is a counted vmcnt (the younger stages stay in flight across the raw s_barrier), so each k-step's
// MFMAs overlap the next STAGES-1 stages' loads.  One __shared__ array only (a second one makes
// hipcc drain vmcnt before every ds_read).
#define TBN 128
#define TBK 64

// element offset of W[row][k0 + 8c .. +8) (k0 % 64 == 0, c < 8) in the fragment-packed layout (PG_W_FRAG)
__device__ __forceinline__ size_t frag_off(int row, int k0, int c, int K) {
  return (size_t)(row >> 4) * 16 * K + ((size_t)(k0 >> 6) * 2 + (c & 1)) * 512 + ((c >> 1) * 16 + (row & 15)) * 8;
}

// Stage a ROWS x 64-k bf16 tile: ROWS/8 pieces spread evenly over NW staging waves (wave < NW; others issue none).
// FRAG: src is fragment-packed (ld = K); each piece still reads 8 runs of 128 contiguous bytes.
// SKIP: pieces whose 8 rows all lie past rows_valid are not loaded (their LDS rows feed only outputs that are never
// stored); the caller counts the pieces a wave issues with stage_pieces.
template <int ROWS, bool FRAG = false, int NW = 4, int AUX = 0, bool SKIP = false>
__device__ __forceinline__ void stage_tile(const bf16_t* __restrict__ src, int ld, int row0, int rows_valid,
                                           int k0, char* lds_tile, int wave, int lane) {
  static_assert((ROWS / 8) % NW == 0, "pieces must split evenly over the staging waves");
  constexpr int PER_WAVE = ROWS / 8 / NW;
  if (wave >= NW) return;
#pragma unroll
  for (int it = 0; it < PER_WAVE; ++it) {
    const int blk = wave * PER_WAVE + it;          // 1 KiB piece = 8 rows x 128 B
    if (SKIP && blk * 8 >= rows_valid - row0) break;   // (wave-uniform)
    const int r = blk * 8 + (lane >> 3);
    const int c = (lane & 7) ^ ((r >> 1) & 7);     // logical 16-B chunk landing at physical chunk lane&7
    int gr = row0 + r;
    gr = gr < rows_valid ? gr : rows_valid - 1;
    const bf16_t* g = FRAG ? src + frag_off(gr, k0, c, ld) : src + (size_t)gr * ld + k0 + c * 8;
    __builtin_amdgcn_global_load_lds((const void*)g, (LDS_AS void*)(lds_tile + blk * 1024), 16, 0, AUX);
  }
}

// pieces stage_tile<ROWS, *, NW, *, SKIP> issues for this wave
template <int ROWS, int NW, bool SKIP>
__device__ __forceinline__ int stage_pieces(int row0, int rows_valid, int wave) {
  constexpr int PER_WAVE = ROWS / 8 / NW;
  if (wave >= NW) return 0;
  if (!SKIP) return PER_WAVE;
  const int valid = (rows_valid - row0 + 7) / 8;
  return min(PER_WAVE, max(0, valid - wave * PER_WAVE));
}

__device__ __forceinline__ bf16x8 lds_frag(const char* tile, int row, int chunk) {
  const int phys = chunk ^ ((row >> 1) & 7);
  return *(const bf16x8*)(tile + row * 128 + phys * 16);
}

__device__ __forceinline__ void wait_vm(int n) {   // s_waitcnt vmcnt(n), n in [0, 24]
  switch (n) {
    case 0: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
    case 2: asm volatile("s_waitcnt vmcnt(2)" ::: "memory"); break;
    case 3: asm volatile("s_waitcnt vmcnt(3)" ::: "memory"); break;
    case 4: asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); break;
    case 5: asm volatile("s_waitcnt vmcnt(5)" ::: "memory"); break;
    case 6: asm volatile("s_waitcnt vmcnt(6)" ::: "memory"); break;
    case 9: asm volatile("s_waitcnt vmcnt(9)" ::: "memory"); break;
    case 10: asm volatile("s_waitcnt vmcnt(10)" ::: "memory"); break;
    case 8: asm volatile("s_waitcnt vmcnt(8)" ::: "memory"); break;
    case 12: asm volatile("s_waitcnt vmcnt(12)" ::: "memory"); break;
    case 13: asm volatile("s_waitcnt vmcnt(13)" ::: "memory"); break;
    case 16: asm volatile("s_waitcnt vmcnt(16)" ::: "memory"); break;
    case 18: asm volatile("s_waitcnt vmcnt(18)" ::: "memory"); break;
    case 24: asm volatile("s_waitcnt vmcnt(24)" ::: "memory"); break;
    default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
  }
}

#ifndef PG_TILE_M1_WNT
#define PG_TILE_M1_WNT 0  // PG_TILE_M1 grids: stage W non-temporal (each W tile read by one workgroup)
#endif
#ifndef PG_TILE_PROBE
#define PG_TILE_PROBE 0   // tuning builds only: 1 = staging without MFMAs, 2 = MFMAs without staging (wrong results)
#endif
// WAVES (4, 8 or 12): waves per workgroup.  4: BM 64 as 1 x 4 waves of 64 x 32, BM 128 / 256 / 288 as 2 x 2.  More
// waves put 2-3 waves on every SIMD, so one wave's LDS fragment reads hide behind another's MFMAs (with 4 waves the
// single wave of a SIMD waits out every ds_read before its MFMAs): 8 = BM 64 as 2 x 4 waves of 32 x 32 and BM 256
// as 4 x 2 of 64 x 64; 12 = BM 288 as 6 x 2 waves of 48 x 64.  The A pieces of a stage spread over all waves, the
// W pieces over the first 8 (12 waves) so every wave's piece count -- its vmcnt step -- is a whole number.
// BN = 64 (PG_TILE_N64, BM 64 and 4 waves only: 2 x 2 waves of 32 x 32): twice the workgroups of the 64 x 128
// grid for the small-M prefill GEMMs whose 64 x 128 grid leaves most CUs idle, without a K split.
// KSUB = 2: a stage holds two 64-k sub-tiles (K % 128 == 0), one barrier / vmcnt wait per 128 k: half the
// per-k-step synchronisation of the latency-bound small-M tiles.
// WNT: the W pieces are staged non-temporal (aux 2): for grids where each W tile is read by ONE workgroup (PG_TILE_M1)
template <int EPI, int BM, int STAGES, bool FRAG, bool F8 = false, int WAVES = 4, int BN = TBN, int KSUB = 1,
          bool WNT = false>
__global__ __launch_bounds__(WAVES * 64) void gemm_tile_kernel(const bf16_t* __restrict__ A, int lda,
                                                               const bf16_t* __restrict__ W, int ldw, int K,
                                                               int kchunk, int tiles_m, int tiles_n, EpiArgs e) {
  constexpr int A_BYTES = BM * TBK * 2;
  static_assert(BN == TBN || (BN == 64 && BM == 64 && WAVES == 4), "BN 64: 64-row tiles of 4 waves only");
  constexpr int W_BYTES = BN * TBK * 2;
  constexpr int SUB_BYTES = A_BYTES + W_BYTES;
  constexpr int STAGE_BYTES = KSUB * SUB_BYTES;
  constexpr int WN = BN == 64 ? 2 : (WAVES == 4 ? (BM == 64 ? 4 : 2) : (WAVES == 8 ? (BM == 64 ? 4 : 2) : 2));
  constexpr int WM = WAVES / WN;                   // waves along M
  constexpr int NI = BM / WM / 16;                 // 16-row subtiles per wave
  constexpr int NJ = BN / WN / 16;                 // 16-col subtiles per wave
  static_assert(WM * NI * 16 == BM && WN * NJ * 16 == BN, "wave grid must tile the block");
  constexpr int NWA = WAVES;                       // waves staging A pieces
  constexpr int NWW = WAVES > 8 ? 8 : WAVES;       // waves staging W pieces
  __shared__ __attribute__((aligned(1024))) char smem[STAGES * STAGE_BYTES];
  const int lane = threadIdx.x & 63;
  // wave-uniform (SGPR): the per-wave piece counts and the vmcnt switch below then branch on scalars, not through
  // an exec-masked chain of every case
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wave / WN, wn = wave % WN;

  // XCD-aware bijective remap (blocks b and b+8 share an XCD), then grouped tile order.
  const int nwg = gridDim.x;
  int pid = blockIdx.x;
  {
    const int q = nwg >> 3, r = nwg & 7, xcd = pid & 7, idx = pid >> 3;
    pid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + idx;
  }
  const int GROUP = 8;
  const int group = pid / (GROUP * tiles_n);
  const int first_m = group * GROUP;
  const int gsize = min(tiles_m - first_m, GROUP);
  const int tm = first_m + (pid % gsize);
  const int tn = (pid % (GROUP * tiles_n)) / gsize;
  const int m0 = tm * BM, n0 = tn * BN;
  // glds pieces this wave issues per stage (wave-uniform): its vmcnt step per younger stage in flight; A pieces of
  // padding rows only (the last row tile: M = 264 in a 288-row tile) are not loaded
  const int P = KSUB * (stage_pieces<BM, NWA, true>(m0, e.M, wave) + stage_pieces<BN, NWW, false>(n0, e.N, wave));

  const int z = blockIdx.z;
  const int kbeg = z * kchunk;
  const int kend = min(K, kbeg + kchunk);
  const int nk = max(0, (kend - kbeg) / (TBK * KSUB));

  f32x4 acc[NI][NJ];
#pragma unroll
  for (int i = 0; i < NI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto issue = [&](int kt) {
    char* st = smem + (kt % STAGES) * STAGE_BYTES;
    if (PG_TILE_PROBE == 2) return;                // tuning probe: no loads (MFMA + barrier floor)
#pragma unroll
    for (int u = 0; u < KSUB; ++u) {
      const int k0 = kbeg + (kt * KSUB + u) * TBK;
      stage_tile<BM, false, NWA, 0, true>(A, lda, m0, e.M, k0, st + u * SUB_BYTES, wave, lane);
      stage_tile<BN, FRAG, NWW, WNT ? 2 : 0>(W, ldw, n0, e.N, k0, st + u * SUB_BYTES + A_BYTES, wave, lane);
    }
  };
#pragma unroll
  for (int s = 0; s < STAGES - 1; ++s)
    if (s < nk) issue(s);

  for (int kt = 0; kt < nk; ++kt) {
    // stage kt has landed once at most (issued stages after kt) * P pieces are outstanding
    const int younger = min(nk - 1, kt + STAGES - 2) - kt;
    wait_vm_n(younger * P);
    __builtin_amdgcn_s_barrier();                  // every wave's pieces of kt landed; kt-1 fully read
    if (kt + STAGES - 1 < nk) issue(kt + STAGES - 1);
#pragma unroll
    for (int u = 0; u < KSUB; ++u) {
    const char* tA = smem + (kt % STAGES) * STAGE_BYTES + u * SUB_BYTES;
    const char* tW = tA + A_BYTES;
    if constexpr (PG_TILE_PROBE == 1) {
      // tuning probe: no fragment reads or MFMAs (the staging pipeline's floor); one LDS word keeps the loads live
      if (lane == 0 && wave == 0) acc[0][0][0] += *(const float*)tA;
    } else if constexpr (F8) {
      // fp8: the 128-byte k-row holds 128 k; one 16x16x128 MFMA takes both chunk sets of the bf16 form
      bf16x8 fa[NI][2], fw[NJ][2];
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const int chunk = s * 4 + (lane >> 4);
#pragma unroll
        for (int i = 0; i < NI; ++i) fa[i][s] = lds_frag(tA, wm * (BM / WM) + i * 16 + (lane & 15), chunk);
#pragma unroll
        for (int j = 0; j < NJ; ++j) fw[j][s] = lds_frag(tW, wn * (BN / WN) + j * 16 + (lane & 15), chunk);
      }
#pragma unroll
      for (int i = 0; i < NI; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j) acc[i][j] = mfma8(fw[j][0], fw[j][1], fa[i][0], fa[i][1], acc[i][j]);
    } else {
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const int chunk = s * 4 + (lane >> 4);
        bf16x8 fa[NI], fw[NJ];
#pragma unroll
        for (int i = 0; i < NI; ++i) fa[i] = lds_frag(tA, wm * (BM / WM) + i * 16 + (lane & 15), chunk);
#pragma unroll
        for (int j = 0; j < NJ; ++j) fw[j] = lds_frag(tW, wn * (BN / WN) + j * 16 + (lane & 15), chunk);
#pragma unroll
        for (int i = 0; i < NI; ++i)
#pragma unroll
          for (int j = 0; j < NJ; ++j) acc[i][j] = mfma16(fw[j], fa[i], acc[i][j]);
      }
    }
    }
  }

  // epilogue: acc[i][j] lane holds C[m = m0+wm*(BM/WM)+i*16+(lane&15)][n = n0+wn*(BN/WN)+j*16+4*(lane>>4) + 0..3]
  const int q = 4 * (lane >> 4);
#pragma unroll
  for (int i = 0; i < NI; ++i) {
    const int m = m0 + wm * (BM / WM) + i * 16 + (lane & 15);
    const int nb = n0 + wn * (BN / WN);
    if constexpr (F8) {
#pragma unroll
      for (int j = 0; j < NJ; ++j) scale_acc(e, m, nb + j * 16 + q, acc[i][j]);
    }
    if constexpr (EPI == PG_EPI_BF16_GELU_MUL) {
#pragma unroll
      for (int j = 0; j < NJ; j += 2) epi_gelu_mul4(e, m, nb + j * 16, q, acc[i][j], acc[i][j + 1]);
    } else if constexpr (EPI == PG_EPI_QKV_ROPE) {
#pragma unroll
      for (int j = 0; j < NJ; ++j) epi_qkv_rope4(e, m, nb + j * 16 + q, acc[i][j]);
    } else {
#pragma unroll
      for (int j = 0; j < NJ; ++j) epi_store4<EPI>(e, m, nb + j * 16 + q, acc[i][j], z);
    }
  }
}

// --------------------------------------------------------------------------------------
// Large-M GEMM (prefill at batch x image tokens >= a few thousand rows): 256 x 256 x 64 tiles
// --------------------------------------------------------------------------------------
// 8 waves = 2 (M) x 4 (N), each owning 128 x 64 outputs (acc[8][4] 16x16 fragments), one workgroup per
// CU (128 KiB LDS).  A K-tile is staged as four 16 KiB half-images (128 rows x 128 B, XOR-swizzled through
// the source address, global_load_lds 16 B/lane, 2 per thread):
//   A0 = tile rows {0..63, 128..191}   A1 = rows {64..127, 192..255}      (wave rows wr*128 + [0,64) / [64,128))
//   B0 = W rows {64c + [0,32)}         B1 = W rows {64c + [32,64)}, c < 4 (wave columns wc*64 + [0,32) / [32,64))
// and consumed in four phases, one C quadrant each: (A0,B0) (A0 regs,B1) (A1,B1 regs) (A1,B0).  A half is
// restaged one phase after its last read (A0 of tile t+2 in phase 1 of t, B1 in phase 2, A1 in phase 3,
// B0 of t+1 in phase 0), so 3 half-tiles (6 loads per thread) stay in flight across the raw s_barrier that
// ends every phase; the single counted wait (vmcnt 6) sits in phase 3 and the tile it retires is read
// from phase 0 of the next tile on (MI355X guide: 256^2 8-phase template, counted vmcnt, T1/T2/T5).
template <int EPI, bool FRAG, bool F8 = false>
__global__ __launch_bounds__(512) void gemm256_kernel(const bf16_t* __restrict__ A, int lda,
                                                      const bf16_t* __restrict__ W, int ldw, int K,
                                                      int ktiles_per_split, int tiles_m, int tiles_n, EpiArgs e) {
  constexpr int HALF = 16384;
  __shared__ __attribute__((aligned(1024))) char smem[8 * HALF];
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int wr = wave >> 2, wc = wave & 3;

  const int nwg = gridDim.x;
  int pid = blockIdx.x;
  {
    const int q = nwg >> 3, r = nwg & 7, xcd = pid & 7, idx = pid >> 3;
    pid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + idx;
  }
  const int GROUP = 8;
  const int group = pid / (GROUP * tiles_n);
  const int first_m = group * GROUP;
  const int gsize = min(tiles_m - first_m, GROUP);
  const int tm = first_m + (pid % gsize);
  const int tn = (pid % (GROUP * tiles_n)) / gsize;
  const int m0 = tm * 256, n0 = tn * 256;
  // split-K (fp32 partial epilogue only): slice z covers k-tiles [kt0, kt0 + nk)
  const int z = blockIdx.z;
  const int kt0 = z * ktiles_per_split;
  const int nk = max(0, min(K / 64 - kt0, ktiles_per_split));

  auto stage = [&](int h, int kt) {
    char* dst = smem + ((kt & 1) * 4 + h) * HALF;
    const int k0 = (kt0 + kt) * 64;
#pragma unroll
    for (int it = 0; it < 2; ++it) {
      const int blk = wave * 2 + it;                 // 16 pieces of 8 rows x 128 B
      const int r = blk * 8 + (lane >> 3);           // half-image row
      const int c = (lane & 7) ^ ((r >> 1) & 7);
      // fp8: uniform base + 32-bit per-lane byte offset (the host checks both operands are < 4 GiB): the saddr
      // form, one VGPR per piece instead of a 64-bit pointer (the fp8 instance spilled its hoisted piece pointers)
      const char* src;
      if (h < 2) {
        const int gr = min(m0 + (r >> 6) * 128 + h * 64 + (r & 63), e.M - 1);
        if constexpr (F8)
          src = (const char*)A + (uint32_t)(((unsigned)gr * (unsigned)lda + (unsigned)(k0 + c * 8)) * 2u);
        else
          src = (const char*)(A + (size_t)gr * lda + k0 + c * 8);
      } else {
        const int gn = min(n0 + (r >> 5) * 64 + (h - 2) * 32 + (r & 31), e.N - 1);
        if constexpr (F8 && !FRAG)
          src = (const char*)W + (uint32_t)(((unsigned)gn * (unsigned)ldw + (unsigned)(k0 + c * 8)) * 2u);
        else
          src = (const char*)(FRAG ? W + frag_off(gn, k0, c, ldw) : W + (size_t)gn * ldw + k0 + c * 8);
      }
      __builtin_amdgcn_global_load_lds((const void*)src, (LDS_AS void*)(dst + blk * 1024), 16, 0, 0);
    }
  };

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  // fragment registers: A rows [0,64) / [64,128) of the wave (fa0 / fa1), B columns [0,32) / [32,64) (fb0 / fb1);
  // fp8: both 16-byte chunks of a row in one 8-register operand
  using FA = std::conditional_t<F8, i32x8[4], bf16x8[4][2]>;
  using FB = std::conditional_t<F8, i32x8[2], bf16x8[2][2]>;
  FA fa0, fa1;
  FB fb0, fb1;

  auto read_a = [&](const char* img, auto& fa) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = wr * 64 + i * 16 + (lane & 15);
      if constexpr (F8) {
        fa[i] = cat8(lds_frag(img, row, lane >> 4), lds_frag(img, row, 4 + (lane >> 4)));
      } else {
#pragma unroll
        for (int s = 0; s < 2; ++s) fa[i][s] = lds_frag(img, row, s * 4 + (lane >> 4));
      }
    }
  };
  auto read_b = [&](const char* img, auto& fb) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int row = wc * 32 + j * 16 + (lane & 15);
      if constexpr (F8) {
        fb[j] = cat8(lds_frag(img, row, lane >> 4), lds_frag(img, row, 4 + (lane >> 4)));
      } else {
#pragma unroll
        for (int s = 0; s < 2; ++s) fb[j][s] = lds_frag(img, row, s * 4 + (lane >> 4));
      }
    }
  };
  auto mma = [&](int rh, int ch, const auto& fa, const auto& fb) {
    __builtin_amdgcn_s_setprio(1);
    if constexpr (F8) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[rh * 4 + i][ch * 2 + j] = mfma8(fb[j], fa[i], acc[rh * 4 + i][ch * 2 + j]);
    } else {
#pragma unroll
      for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j)
            acc[rh * 4 + i][ch * 2 + j] = mfma16(fb[j][s], fa[i][s], acc[rh * 4 + i][ch * 2 + j]);
    }
    __builtin_amdgcn_s_setprio(0);
  };

  // prologue: all of tile 0, then the three halves of tile 1 that phases 1-3 of tile -1 would have issued
  // (a split past the end of K -- ksplit with ceil-sized slices -- stages nothing and stores a zero slab)
  if (nk > 0) {
#pragma unroll
    for (int h = 0; h < 4; ++h) stage(h, 0);
  }
  if (nk > 1) {
    stage(0, 1);
    stage(3, 1);
    stage(1, 1);
    wait_vm(6);
  } else {
    wait_vm(0);
  }
  __builtin_amdgcn_s_barrier();

  if constexpr (PG_G256_STAGGER && !F8) {
    // Wave groups wr = 0 / 1 (one wave of each per SIMD) run one barrier apart, two barriers per phase:
    // while one group issues its phase's LDS reads and DMA, the other runs its MFMAs.  With the offset, a
    // group's reads must be complete before its phase's first barrier (lgkmcnt(0) there: the other group
    // restages right after it) and the tile's vmcnt wait sits before phase 3's first barrier (the other
    // group reads the retired halves one barrier earlier than this one) -- guide: "one barrier MORE when
    // two wave groups run staggered".
    auto bar = [] { __builtin_amdgcn_s_barrier(); };
    auto lgkm0 = [] { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); };
    if (wr == 1) bar();
    for (int t = 0; t < nk; ++t) {
      const char* buf = smem + (t & 1) * 4 * HALF;
      read_a(buf, fa0);
      read_b(buf + 2 * HALF, fb0);
      if (t + 1 < nk) stage(2, t + 1);
      lgkm0();
      bar();
      mma(0, 0, fa0, fb0);
      bar();
      read_b(buf + 3 * HALF, fb0);
      if (t + 2 < nk) stage(0, t + 2);
      lgkm0();
      bar();
      mma(0, 1, fa0, fb0);
      bar();
      read_a(buf + 1 * HALF, fa0);
      if (t + 2 < nk) stage(3, t + 2);
      lgkm0();
      bar();
      mma(1, 1, fa0, fb0);
      bar();
      read_b(buf + 2 * HALF, fb0);
      if (t + 2 < nk) stage(1, t + 2);
      if (t + 2 < nk) wait_vm(6); else wait_vm(0);
      lgkm0();
      bar();
      mma(1, 0, fa0, fb0);
      bar();
    }
    if (wr == 0) bar();     // same barrier count for both groups
  } else
  for (int t = 0; t < nk; ++t) {
    const char* buf = smem + (t & 1) * 4 * HALF;
    if constexpr (PG_G256_PREFETCH && !F8) {   // (fp8: the early reads would spill)
    // the reads of phases 1-3 are issued one phase early, ahead of the current phase's MFMAs (tile t is
    // retired for every wave from phase 0 on; each half is still restaged only after its last read)
    read_a(buf, fa0);
    read_b(buf + 2 * HALF, fb0);
    if (t + 1 < nk) stage(2, t + 1);
    read_b(buf + 3 * HALF, fb1);
    mma(0, 0, fa0, fb0);
    __builtin_amdgcn_s_barrier();
    read_a(buf + 1 * HALF, fa1);
    if (t + 2 < nk) stage(0, t + 2);
    mma(0, 1, fa0, fb1);
    __builtin_amdgcn_s_barrier();
    read_b(buf + 2 * HALF, fb0);
    if (t + 2 < nk) stage(3, t + 2);
    mma(1, 1, fa1, fb1);
    __builtin_amdgcn_s_barrier();
    if (t + 2 < nk) stage(1, t + 2);
    mma(1, 0, fa1, fb0);
    } else {
    // phase 0: quadrant (rows 0-63, cols 0-31) from A0, B0; restage B0 of tile t+1
    read_a(buf, fa0);
    read_b(buf + 2 * HALF, fb0);
    if (t + 1 < nk) stage(2, t + 1);
    mma(0, 0, fa0, fb0);
    __builtin_amdgcn_s_barrier();
    // phase 1: (rows 0-63, cols 32-63) A regs kept, B1; restage A0 of tile t+2 (A0 was last read in phase 0)
    read_b(buf + 3 * HALF, fb0);
    if (t + 2 < nk) stage(0, t + 2);
    mma(0, 1, fa0, fb0);
    __builtin_amdgcn_s_barrier();
    // phase 2: (rows 64-127, cols 32-63) A1, B regs kept; restage B1 of tile t+2
    read_a(buf + 1 * HALF, fa0);
    if (t + 2 < nk) stage(3, t + 2);
    mma(1, 1, fa0, fb0);
    __builtin_amdgcn_s_barrier();
    // phase 3: (rows 64-127, cols 0-31) A regs kept, B0 again; restage A1 of tile t+2; retire tile t+1
    read_b(buf + 2 * HALF, fb0);
    if (t + 2 < nk) stage(1, t + 2);
    mma(1, 0, fa0, fb0);
    }
    if (t + 2 < nk) wait_vm(6); else wait_vm(0);
    __builtin_amdgcn_s_barrier();
  }

  // epilogue: acc[i][j] lane holds C[m][n..n+3], m = m0 + wr*128 + (i/4)*64 + (i%4)*16 + (lane&15),
  // n = n0 + wc*64 + (j/2)*32 + (j%2)*16 + 4*(lane>>4)
  const int q = 4 * (lane >> 4);
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int m = m0 + wr * 128 + (i >> 2) * 64 + (i & 3) * 16 + (lane & 15);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int nb = n0 + wc * 64 + (j >> 1) * 32 + (j & 1) * 16;
      if constexpr (F8) scale_acc(e, m, nb + q, acc[i][j]);
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int nb = n0 + wc * 64 + (j >> 1) * 32 + (j & 1) * 16;
      if constexpr (EPI == PG_EPI_BF16_GELU_MUL) {
        if ((j & 1) == 0) epi_gelu_mul4(e, m, nb, q, acc[i][j], acc[i][j + 1]);
      } else if constexpr (EPI == PG_EPI_QKV_ROPE) {
        epi_qkv_rope4(e, m, nb + q, acc[i][j]);
      } else {
        epi_store4<EPI>(e, m, nb + q, acc[i][j], z);
      }
    }
  }
}

// --------------------------------------------------------------------------------------
// Skinny GEMM / GEMV (M <= 16): weight streaming straight to VGPRs
// --------------------------------------------------------------------------------------
// One workgroup = 4 waves on NT adjacent 16-row tiles of W (NT = 2 for the interleaved gate/up
// pair); the 4 waves split the chunks of split blockIdx.y round-robin and reduce through LDS.
// Chunk = 32U k: lane (r = lane&15, g = lane>>4) loads 16U contiguous bytes of W row r at
// k = chunk + 8U*g; MFMA step s consumes k = chunk + 8U*g + 8s + [0,8) for BOTH operands, a
// permutation of k that leaves the dot product unchanged.  DEPTH chunks stay in flight in a
// statically indexed register ring.  Plain (temporal) loads: measured 1.2-1.6x faster than
// non-temporal ones on every decode shape (round-1 GEMV sweep).
//
// PRO (prologue, fuses the producer of x into the GEMV so a decode layer needs 5 launches):
//   0: x rows read from A (bf16)
//   1: x = RMSNorm(resid_in + sum_s partials[s]) * (1 + w)       (GemmaRMSNorm, modeling_gemma.py:172-181)
//      workgroup (0,0) also writes resid_out = resid_in + sum partials (ping-pong residual stream)
//   2: x = merge of the split-KV attention partials (2^(m_s - M) weighted, / sum l)
// For PRO != 0 the WG's K range of x is built in LDS (bf16, rows padded by 16 B against bank conflicts).
#define XPAD 8

// tuning knobs (scripts/tune/): issue the first weight chunks before the prologue; one-pass online
// merge of the split-KV partials in the attention-merge prologue
#ifndef PG_GEMV_PREW
#define PG_GEMV_PREW 1
#endif
#ifndef PG_GEMV_NT
#define PG_GEMV_NT 0
#endif
#ifndef PG_GEMV_CONTIG
#define PG_GEMV_CONTIG 0
#endif
#ifndef PG_T128_STAGES_F8
#define PG_T128_STAGES_F8 2  // stages of the 128 x 128 fp8 tile (2: two workgroups per CU; 3 / 4 = one per CU, pt-896 x32
                             // gate/up 10.1 -> 14.6 / 14.3 ms)
#endif
#ifndef PG_F8_G256
// fp8 GEMMs on the 256x256 kernel: 0 never, 1 the fp32-slab epilogue only (pt-896 x32 o + down 115.7 -> 102.5 ms per
// prefill), 2 every epilogue (gate/up 182 -> 211 ms and q|k|v 21 -> 48 ms: those instances still spill)
#define PG_F8_G256 1
#endif
#ifndef PG_G256_MIN_TILES
#define PG_G256_MIN_TILES 256   // large-M GEMM when its 256x256 grid fills every CU
#endif
#ifndef PG_GEMV_QKV_NT1
#define PG_GEMV_QKV_NT1 1   // batched (M > 4) q|k|v GEMV with one 16-row tile per workgroup
#endif
#ifndef PG_GEMV_D2
#define PG_GEMV_D2 4
#endif
#ifndef PG_GEMV_D1
#define PG_GEMV_D1 8      // chunks in flight of the one-tile GEMV (M <= 4: batch-1 decode o / down / q|k|v / lm_head)
#endif
#ifndef PG_GEMV_XLDS
#define PG_GEMV_XLDS 0
#endif
#ifndef PG_GEMV_HOT
#define PG_GEMV_HOT 1           // 1 = q|k|v, 2 = o_proj (merge prologue), 3 = both read their weights with
                                // default-policy loads (allocating in the Infinity Cache) while the others stay nt:
                                // the 18 layers' q|k|v (189 MB) then stay on-die across decode steps; pt-224 B=1
                                // A/B/A/B 1.1348/1.1363 -> 1.1325/1.1314 ms/token (2: neutral; 3: 1.142, they no
                                // longer fit; scripts/r02/gpu_s3f.sh)
#endif
#ifndef PG_GEMV_FRAG_NT
#define PG_GEMV_FRAG_NT 1
#endif
#ifndef PG_GEMV_CPW
#define PG_GEMV_CPW 1     // decode GEMV: straight-line chunk loop when every wave owns the same chunk count
#endif

// the GEMV's workgroup coordinates (blockIdx / gridDim of its launch)
struct GemvIdx {
  int bx, by, nx, ny;
};

template <int PRO>
__device__ __forceinline__ void gemv_prologue(const EpiArgs& e, int M, int K, int k0, int Kr, bf16_t* xs,
                                              float* scratch, const bf16_t* __restrict__ A, int lda,
                                              const GemvIdx& gi) {
  const PgFusedArgs& f = e.f;
  const int t = threadIdx.x;
  const int ldx = Kr + XPAD;
  if constexpr (PRO == 0 || PRO == 4) {
    // x rows [M][k0, k0 + Kr) copied from A into LDS (PG_GEMV_XLDS): one L2 read per workgroup
    const int K8 = Kr >> 3;
    for (int idx = t; idx < M * K8; idx += 256) {
      const int m = idx / K8, c = idx % K8;
      *(u32x4*)(xs + m * ldx + c * 8) = *(const u32x4*)(A + (size_t)m * lda + k0 + c * 8);
    }
  } else if constexpr (PRO == 1) {
    // RMSNorm over the FULL row (Kr == K): pass 1 sum of squares, pass 2 normalise into LDS
    const int K4 = K >> 2;
    const bool w0 = gi.bx == 0 && gi.by == 0 && f.resid_out != nullptr;
    float* red = scratch;   // [4 waves][16 rows]
    if (M == 1 && K4 <= 4 * 256) {
      // one row: keep it in registers between the two passes (one dependent round trip fewer)
      f32x4 v[4], wn[4];
      float ss = 0.f;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int c = t + i * 256;
        v[i] = f32x4{0.f, 0.f, 0.f, 0.f};
        if (c < K4) {
          wn[i] = ((const f32x4*)f.norm_w)[c];          // issued with the residual: one round trip
          f32x4 a = ((const f32x4*)f.resid_in)[c];
          if (f.fx) a += fx_load4(f.fx + 4 * c);
          for (int sp = 0; sp < f.nsplit; ++sp) a += ((const f32x4*)(f.partials + (size_t)sp * K))[c];
          v[i] = a;
          ss += a[0] * a[0] + a[1] * a[1] + a[2] * a[2] + a[3] * a[3];
          if (w0) ((f32x4*)f.resid_out)[c] = a;
        }
      }
      ss = wave_sum(ss);
      if ((t & 63) == 0) red[t >> 6] = ss;
      __syncthreads();
      const float rstd = rsqrtf((red[0] + red[1] + red[2] + red[3]) / (float)K + f.eps);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int c = t + i * 256;
        if (c < K4) {
          const f32x4 w = wn[i];
          u32x2 pk;
          pk[0] = pack_bf2((v[i][0] * rstd) * (1.0f + w[0]), (v[i][1] * rstd) * (1.0f + w[1]));
          pk[1] = pack_bf2((v[i][2] * rstd) * (1.0f + w[2]), (v[i][3] * rstd) * (1.0f + w[3]));
          *(u32x2*)(xs + c * 4) = pk;
        }
      }
      __syncthreads();
      return;
    }
    for (int m = 0; m < M; ++m) {
      float ss = 0.f;
      for (int c = t; c < K4; c += 256) {
        f32x4 v = ((const f32x4*)(f.resid_in + (size_t)m * K))[c];
        if (f.fx) v += fx_load4(f.fx + (size_t)m * K + 4 * c);
        for (int sp = 0; sp < f.nsplit; ++sp) v += ((const f32x4*)(f.partials + ((size_t)sp * M + m) * K))[c];
        ss += v[0] * v[0] + v[1] * v[1] + v[2] * v[2] + v[3] * v[3];
        if (w0) ((f32x4*)(f.resid_out + (size_t)m * K))[c] = v;
      }
      ss = wave_sum(ss);
      if ((t & 63) == 0) red[(t >> 6) * 16 + m] = ss;
    }
    __syncthreads();
    for (int m = 0; m < M; ++m) {
      const float rstd = rsqrtf((red[m] + red[16 + m] + red[32 + m] + red[48 + m]) / (float)K + f.eps);
      for (int c = t; c < K4; c += 256) {
        f32x4 v = ((const f32x4*)(f.resid_in + (size_t)m * K))[c];
        if (f.fx) v += fx_load4(f.fx + (size_t)m * K + 4 * c);
        for (int sp = 0; sp < f.nsplit; ++sp) v += ((const f32x4*)(f.partials + ((size_t)sp * M + m) * K))[c];
        const f32x4 w = ((const f32x4*)f.norm_w)[c];
        u32x2 pk;
        pk[0] = pack_bf2((v[0] * rstd) * (1.0f + w[0]), (v[1] * rstd) * (1.0f + w[1]));
        pk[1] = pack_bf2((v[2] * rstd) * (1.0f + w[2]), (v[3] * rstd) * (1.0f + w[3]));
        *(u32x2*)(xs + m * ldx + c * 4) = pk;
      }
    }
  } else if constexpr (PRO == 3) {
    // x = resid * (1 + w) over the full row (the residual was finalised by the producer's FIN epilogue);
    // per-row rstd from the producer's per-tile sums of squares, applied in the epilogue (scratch[64 + m])
    const int K4 = K >> 2;
    float* red = scratch;   // [4 waves][16 rows], then rstd [16] at +64
    for (int m = 0; m < M; ++m) {
      for (int c = t; c < K4; c += 256) {
        const f32x4 v = ((const f32x4*)(f.resid_in + (size_t)m * K))[c];
        const f32x4 w = ((const f32x4*)f.norm_w)[c];
        u32x2 pk;
        pk[0] = pack_bf2(v[0] * (1.0f + w[0]), v[1] * (1.0f + w[1]));
        pk[1] = pack_bf2(v[2] * (1.0f + w[2]), v[3] * (1.0f + w[3]));
        *(u32x2*)(xs + m * ldx + c * 4) = pk;
      }
      float ssum = 0.f;
      for (int i = t; i < f.ss_n; i += 256) ssum += f.ss_in[(size_t)m * f.ss_ld + i];
      ssum = wave_sum(ssum);
      if ((t & 63) == 0) red[(t >> 6) * 16 + m] = ssum;
    }
    __syncthreads();
    if (t < M) red[64 + t] = rsqrtf((red[t] + red[16 + t] + red[32 + t] + red[48 + t]) / (float)K + f.eps);
  } else if constexpr (PRO == 2) {
    // one pass per (row, head, 4 dims): merge over the splits, no LDS staging / barriers
    const int D = f.head_dim, G = f.q_per_kv, S = f.asplit;
    const int h0 = k0 / D, nh = Kr / D, D4 = D >> 2;
    const int items = M * nh * D4;
    if (S <= 16) {
      // every split's (m, l, o) loaded at once (one dependent L2 round trip, no read of the kv length:
      // splits past it hold m = -inf and weigh 0), then a two-pass max / weighted sum
      for (int idx = t; idx < M * nh * D4; idx += 256) {
        const int m = idx / (nh * D4), rem = idx % (nh * D4), hl = rem / D4, d4 = rem % D4;
        const int hq = h0 + hl;
        const long base0 = (((long)m * f.kv_heads + hq / G) * S) * 16 + (hq % G);
        float ms[16], ls[16];
        f32x4 o4[16];
        f32x2 mlv[16];
        // all 32 loads issued back to back before any is used (sched_barrier): the scheduler otherwise recycled
        // one register for six of the O loads, a load -> wait -> load chain of six round trips
#pragma unroll
        for (int sp = 0; sp < 16; ++sp) {
          const long bs = base0 + (long)min(sp, S - 1) * 16;
          mlv[sp] = *(const f32x2*)(f.part_ml + bs * 2);
          o4[sp] = *(const f32x4*)(f.part_o + bs * f.dtw + d4 * 4);
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int sp = 0; sp < 16; ++sp) {
          ms[sp] = sp < S ? mlv[sp][0] : -INFINITY;
          ls[sp] = mlv[sp][1];
        }
        float mx = ms[0];
#pragma unroll
        for (int sp = 1; sp < 16; ++sp) mx = fmaxf(mx, ms[sp]);
        float den = 0.f;
        f32x4 num = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int sp = 0; sp < 16; ++sp) {
          const float w = ms[sp] == -INFINITY ? 0.f : exp2f(ms[sp] - mx);
          den += w * ls[sp];
          num += w * o4[sp];
        }
        const float inv = 1.0f / den;
        u32x2 pk;
        pk[0] = pack_bf2(num[0] * inv, num[1] * inv);
        pk[1] = pack_bf2(num[2] * inv, num[3] * inv);
        *(u32x2*)(xs + m * ldx + hl * D + d4 * 4) = pk;
      }
      __syncthreads();
      return;
    }
    const int Seff = (f.slot_dev && f.akeys > 0) ? min(S, (*f.slot_dev + f.akeys) / f.akeys) : S;
    for (int idx = t; idx < items; idx += 256) {
      const int m = idx / (nh * D4), rem = idx % (nh * D4), hl = rem / D4, d4 = rem % D4;
      const int hq = h0 + hl;
      const long base0 = (((long)m * f.kv_heads + hq / G) * S) * 16 + (hq % G);
      float mx = -INFINITY, den = 0.f;
      f32x4 num = {0.f, 0.f, 0.f, 0.f};
#pragma unroll 8
      for (int sp = 0; sp < Seff; ++sp) {
        const long bs = base0 + (long)sp * 16;
        const float ms = f.part_ml[bs * 2], ls = f.part_ml[bs * 2 + 1];
        const f32x4 o4 = *(const f32x4*)(f.part_o + bs * f.dtw + d4 * 4);
        const float mn = fmaxf(mx, ms);
        const float ca = mx == -INFINITY ? 0.f : exp2f(mx - mn);
        const float cb = ms == -INFINITY ? 0.f : exp2f(ms - mn);
        den = den * ca + cb * ls;
        num = num * ca + cb * o4;
        mx = mn;
      }
      const float inv = 1.0f / den;
      u32x2 pk;
      pk[0] = pack_bf2(num[0] * inv, num[1] * inv);
      pk[1] = pack_bf2(num[2] * inv, num[3] * inv);
      *(u32x2*)(xs + m * ldx + hl * D + d4 * 4) = pk;
    }
  }
  __syncthreads();
}

// CPW > 0: every wave owns exactly CPW chunks (launch checks K / CH / ksplit == 4 * CPW).  The chunk loop is then
// straight-line code with unconditional loads, so hipcc's s_waitcnt bookkeeping stays exact: each chunk's MFMAs
// wait only for that chunk (vmcnt(N), N = younger loads), instead of the conservative vmcnt(0) that the runtime
// loop and its exec-masked loads produce at every ring turn (the ring drained before its first MFMA).
template <int EPI, int NT, int U, int DEPTH, int PRO, bool FRAG, int CPW = 0>
__device__ __forceinline__ void gemv_body(const bf16_t* __restrict__ A, int lda, const bf16_t* __restrict__ W,
                                          int ldw, int K, const EpiArgs& e, const GemvIdx gi) {
  constexpr int CH = U * 32;
  extern __shared__ __attribute__((aligned(16))) char dyn_smem[];
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int g = lane >> 4;
  const int r = lane & 15;
  const int tile0 = gi.bx * NT;
  const int M = e.M;
  const bool xvalid = r < M;

  const int z = gi.by;
  const int nch_all = K / CH;
  const int per_z = (nch_all + gi.ny - 1) / gi.ny;
  const int c0 = z * per_z;
  const int nch = min(nch_all - c0, per_z);
  const int mine = CPW > 0 ? CPW : (nch > wave ? (nch - wave + 3) / 4 : 0);   // chunks wave, wave+4, ...

  const bf16_t* wrow[NT];
  const bf16_t* wfrag[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    int n = (tile0 + t) * 16 + r;
    n = n < e.N ? n : e.N - 1;
    wrow[t] = W + (size_t)n * ldw;
    wfrag[t] = W + (size_t)min(tile0 + t, (e.N >> 4) - 1) * 16 * ldw;
  }
  f32x4 acc[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};

  bf16_t* xs = (bf16_t*)dyn_smem;
  const int Kr = per_z * CH;                    // K range of this split (LDS row length)
  // rows past M read row M-1 (their outputs are never stored): the x loads are unconditional, so the compiler
  // has no select or branch to resolve and no reason to wait for them before issuing the rest of the stream
  const bf16_t* xrow = (PRO == 0 || PRO == 4) ? A + (size_t)(xvalid ? r : M - 1) * lda : nullptr;
  // PRO 4 (M <= 2): wave 0 loads the producer's per-tile sums of squares before the weight stream (all
  // at once, clamped addresses; lanes [32*row, 32*row + 32) own a row) and sums them in the epilogue
  // M > 4 (two tiles per workgroup, <= 64 entries per row): lane (row r, group g) loads entries g + 4k of its
  // own row, so the row total is a reduction over the 4 lane groups
  // (one-tile workgroups at M > 4 -- the batched q|k|v, launch_gemv_pro -- use the same 16-entry layout as the
  // two-tile form)
  constexpr bool SS16 = PRO == 4 && (NT >= 2 || EPI == PG_EPI_QKV_ROPE);
  constexpr int SSL = SS16 ? 16 : 4;
  float ssv[SSL];
#pragma unroll
  for (int k = 0; k < SSL; ++k) ssv[k] = 0.f;
  if constexpr (PRO == 4) {
    if (wave == 0) {
      if (SS16 && M > 2) {
        const int rr = min(r, M - 1);
#pragma unroll
        for (int k = 0; k < SSL; ++k) ssv[k] = e.f.ss_in[(size_t)rr * e.f.ss_ld + min(g + 4 * k, e.f.ss_n - 1)];
      } else {
        const int lpr = M == 1 ? 64 : 32;
        const int rr = min(lane / lpr, M - 1);
#pragma unroll
        for (int k = 0; k < 4; ++k) ssv[k] = e.f.ss_in[(size_t)rr * e.f.ss_ld + min(lane % lpr + k * lpr, e.f.ss_n - 1)];
      }
    }
  }
  const bf16_t* xlds = xs + (xvalid ? r : M - 1) * (Kr + XPAD);
  // PG_EPI_QKV_ROPE: the epilogue's rotary positions and cache slot load before the weight stream, its cos/sin
  // right after the first chunks are issued, so the epilogue starts without a dependent round trip
  // (every wave loads them -- a few dwords -- so no divergent branch joins a loaded register, which would make
  // the compiler wait for it right there)
  int rope_p = 0, rope_slot_raw = 0;
  if constexpr (EPI == PG_EPI_QKV_ROPE) {
    rope_p = e.f.pos[r < M ? r : M - 1];
    // a vector load (counted in order with the stream, unlike a scalar load whose wait lands early); a null
    // slot_dev reads a zero word instead of a select on the loaded value
    rope_slot_raw = __hip_atomic_load(e.f.slot_dev ? e.f.slot_dev : &pg_zero_word, __ATOMIC_RELAXED,
                                      __HIP_MEMORY_SCOPE_AGENT);
  }

  // element offset of a lane's 16-B piece s inside a CH-element chunk: PG_GEMV_CONTIG lays piece s of the 4
  // lane groups side by side (one load instruction = 64 contiguous bytes per row); otherwise a lane owns 16U
  // contiguous elements.  x uses the same map, so the k order inside the MFMA is consistent either way.
  constexpr int S_STRIDE = PG_GEMV_CONTIG ? 32 : 8;
  const int LANE_OFF = PG_GEMV_CONTIG ? g * 8 : g * 8 * U;
  u32x4 wb[DEPTH][NT][U];
  u32x4 xb[DEPTH][U];
  auto loadw = [&](int j, u32x4 (&wv)[NT][U]) {
    if constexpr (FRAG) {
      // fragment-packed weights: tile t's chunk c is U wave-instructions of 1 KiB, lane-linear; read once,
      // so non-temporal (measured: gate/up 28.7 -> 23.0 us, down 17.0 -> 13.8 us vs row-major plain loads)
      const int cc = c0 + wave + j * 4;
#pragma unroll
      for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int s = 0; s < U; ++s) {
          const u32x4* src = (const u32x4*)(wfrag[t] + ((size_t)cc * U + s) * 512 + lane * 8);
          constexpr bool hot = ((PG_GEMV_HOT & 1) && EPI == PG_EPI_QKV_ROPE) || ((PG_GEMV_HOT & 2) && PRO == 2);
          if constexpr (PG_GEMV_FRAG_NT && !hot)
            wv[t][s] = __builtin_nontemporal_load(src);
          else
            wv[t][s] = *src;
        }
    } else {
      const int off = (c0 + wave + j * 4) * CH + LANE_OFF;
#pragma unroll
      for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int s = 0; s < U; ++s) {
#if PG_GEMV_NT
          wv[t][s] = __builtin_nontemporal_load((const u32x4*)(wrow[t] + off + S_STRIDE * s));
#else
          wv[t][s] = *(const u32x4*)(wrow[t] + off + S_STRIDE * s);
#endif
        }
    }
  };
  auto loadx = [&](int j, u32x4 (&xv)[U]) {
    const int koff = (wave + j * 4) * CH + LANE_OFF;      // offset inside this split
    if constexpr ((PRO == 0 || PRO == 4) && !PG_GEMV_XLDS) {
#pragma unroll
      for (int s = 0; s < U; ++s)
        xv[s] = *(const u32x4*)(xrow + c0 * CH + koff + S_STRIDE * s);
    } else {
#pragma unroll
      for (int s = 0; s < U; ++s) xv[s] = *(const u32x4*)(xlds + koff + S_STRIDE * s);
    }
  };
  constexpr bool STAGED = (PRO != 0 && PRO != 4) || PG_GEMV_XLDS;   // x built in LDS by a prologue
  // weights issued before the prologue (its loads are the critical path: the stream overlaps them)
  constexpr bool prew = STAGED && PG_GEMV_PREW;
  if (prew) {
#pragma unroll
    for (int d = 0; d < DEPTH; ++d)
      if (CPW > 0 ? d < CPW : d < mine) loadw(d, wb[d]);
  }
  if constexpr (STAGED) {
    float* scratch = (float*)(dyn_smem + (((size_t)M * (Kr + XPAD) * 2 + 15) & ~(size_t)15));
    gemv_prologue<PRO>(e, M, K, c0 * CH, nch * CH, xs, scratch, A, lda, gi);
  }
#pragma unroll
  for (int d = 0; d < DEPTH; ++d)
    if (CPW > 0 ? d < CPW : d < mine) {
      if (!prew) loadw(d, wb[d]);
      loadx(d, xb[d]);
    }
  // PG_EPI_F32_FIN: the residual rows and norm weights the tile's last-arriving split finalises are loaded now
  // (nothing else writes them in this launch), so the reducer's only round trip is the slab read
  f32x4 fin_r[NT], fin_w[NT];
  i64x2 fin_fa[NT], fin_fb[NT];     // the fixed-point accumulator's entries (PgFusedArgs.fx), converted when used
  if constexpr (EPI == PG_EPI_F32_FIN) {
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const int n0 = min((tile0 + t) * 16, e.N - 16) + 4 * g;
      fin_r[t] = *(const f32x4*)(e.f.fin_resid + (size_t)(r < M ? r : M - 1) * e.N + n0);
      if (e.f.fx) {
        const long long* p = e.f.fx + (size_t)(r < M ? r : M - 1) * e.N + n0;
        fin_fa[t] = *(const i64x2*)p;
        fin_fb[t] = *(const i64x2*)(p + 2);
      }
      // (no select on a loaded value -- it would make the compiler wait right here: a null norm_w reads the
      // residual row instead, unused)
      fin_w[t] = *(const f32x4*)((e.f.norm_w ? e.f.norm_w : e.f.fin_resid) + n0);
    }
  }
  f32x4 rope_cs[NT], rope_sn[NT];
  if constexpr (EPI == PG_EPI_QKV_ROPE) {
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      bool roped;   // (v columns load a valid, unused entry: no select on the loaded values)
      const int ii = rope_freq_index(e.f, min((tile0 + t) * 16, e.N - 16) + 4 * g, &roped);
      const long off = (long)rope_p * (e.f.head_dim >> 1) + ii;
      rope_cs[t] = *(const f32x4*)(e.f.cos_t + off);
      rope_sn[t] = *(const f32x4*)(e.f.sin_t + off);
    }
  }
  if constexpr (CPW > 0) {
    // sched_barrier: the scheduler may not sink the ring's loads below later MFMAs (it otherwise trades the
    // chunks in flight for registers: vmcnt(8) = two chunks in flight on the down projection)
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int j = 0; j < CPW; ++j) {
      const int d = j % DEPTH;
#pragma unroll
      for (int s = 0; s < U; ++s) {
        const bf16x8 xv = __builtin_bit_cast(bf16x8, xb[d][s]);
#pragma unroll
        for (int t = 0; t < NT; ++t) acc[t] = mfma16(__builtin_bit_cast(bf16x8, wb[d][t][s]), xv, acc[t]);
      }
      if (j + DEPTH < CPW) {
        loadw(j + DEPTH, wb[d]);
        loadx(j + DEPTH, xb[d]);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  } else {
    for (int base = 0; base < mine; base += DEPTH) {
#pragma unroll
      for (int d = 0; d < DEPTH; ++d) {
        const int j = base + d;
        if (j < mine) {
#pragma unroll
          for (int s = 0; s < U; ++s) {
            const bf16x8 xv = __builtin_bit_cast(bf16x8, xb[d][s]);
#pragma unroll
            for (int t = 0; t < NT; ++t) acc[t] = mfma16(__builtin_bit_cast(bf16x8, wb[d][t][s]), xv, acc[t]);
          }
          if (j + DEPTH < mine) {
            loadw(j + DEPTH, wb[d]);
            loadx(j + DEPTH, xb[d]);
          }
        }
      }
    }
  }

  __shared__ f32x4 red[4][NT][64];
#pragma unroll
  for (int t = 0; t < NT; ++t) red[wave][t][lane] = acc[t];
  __syncthreads();
  if (wave != 0) return;
#pragma unroll
  for (int t = 0; t < NT; ++t) acc[t] = red[0][t][lane] + red[1][t][lane] + red[2][t][lane] + red[3][t][lane];
  // lane holds C[m = lane&15][n = tile*16 + 4*(lane>>4) + 0..3]
  const int m = r;
  const int q = 4 * g;
  if constexpr (PRO == 3) {
    const float* scratch = (const float*)(dyn_smem + (((size_t)M * (Kr + XPAD) * 2 + 15) & ~(size_t)15));
    const float rs = scratch[64 + (m < M ? m : 0)];
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[t] *= rs;
  }
  if constexpr (PRO == 4) {
    // the raw per-tile entries were loaded with clamped indices (no select before the weight stream): mask here
    float ss = 0.f;
    if (SS16 && M > 2) {
#pragma unroll
      for (int k = 0; k < SSL; ++k) ss += g + 4 * k < e.f.ss_n ? ssv[k] : 0.f;
    } else {
      const int lpr = M == 1 ? 64 : 32;
#pragma unroll
      for (int k = 0; k < 4; ++k) ss += lane % lpr + k * lpr < e.f.ss_n ? ssv[k] : 0.f;
    }
    if (SS16 && M > 2) {
      ss = sum_xor16(ss);
      ss = sum_xor32(ss);
    } else {
      const int lpr = M == 1 ? 64 : 32;
      for (int o = 1; o < lpr; o <<= 1) ss += __shfl_xor(ss, o, 64);
      ss = __shfl(ss, (m < M ? m : 0) * lpr, 64);
    }
    const float rs = rsqrtf(ss / (float)K + e.f.eps);
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[t] *= rs;
  }
  if constexpr (EPI == PG_EPI_F32_FIN) {
    // 1. this split's slab; 2. release + ticket; 3. the last split of the tile reduces the slabs into the
    //    residual rows it owns and writes their sum of squares (MI355X guide: in-launch split-K reduction)
    // Slab stores are write-through (agent-scope relaxed 8-B atomic stores = global_store sc1), drained,
    // then one relaxed agent ticket: no release fence (an L2 write-back per workgroup cost 2x the kernel).
    // The reducer reads the slabs with sc1 loads (bypass its L1/L2), so no acquire fence either.
    const PgFusedArgs& f = e.f;
    typedef __attribute__((address_space(1))) unsigned long long gu64;
    // one sum-of-squares entry per tile pair (per tile at NT 1): a 4-tile workgroup writes two
    constexpr int SE = NT >= 2 ? NT / 2 : 1;
    auto finish = [&](int t, int n0, f32x4 v, float& ssl) {   // v = the finalised residual of (m, n0..n0+3)
      *(f32x4*)(f.fin_resid + (size_t)m * e.N + n0) = v;
      ssl += v[0] * v[0] + v[1] * v[1] + v[2] * v[2] + v[3] * v[3];
      if (f.fin_x) {
        const f32x4 w = fin_w[t];
        u32x2 pk;
        pk[0] = pack_bf2(v[0] * (1.0f + w[0]), v[1] * (1.0f + w[1]));
        pk[1] = pack_bf2(v[2] * (1.0f + w[2]), v[3] * (1.0f + w[3]));
        *(u32x2*)(f.fin_x + (size_t)m * e.N + n0) = pk;
      }
    };
    // the residual entering the finalisation: fin_resid (+ the fixed-point accumulator, whose entries this tile's
    // finalising workgroup then clears: every split of the tile loaded them before its ticket)
    auto fin_base = [&](int t) {
      f32x4 b = fin_r[t];
      if (f.fx) b += f32x4{fx_to_f32(fin_fa[t][0]), fx_to_f32(fin_fa[t][1]), fx_to_f32(fin_fb[t][0]),
                           fx_to_f32(fin_fb[t][1])};
      return b;
    };
    auto fx_clear = [&](int n0) {
      if (f.fx) {
        long long* p = f.fx + (size_t)m * e.N + n0;
        *(i64x2*)p = i64x2{0, 0};
        *(i64x2*)(p + 2) = i64x2{0, 0};
      }
    };
    auto put_ss = [&](float (&ssl)[SE]) {
#pragma unroll
      for (int p = 0; p < SE; ++p) {
        const float v = sum_xor32(sum_xor16(ssl[p]));
        if (g == 0 && m < M) f.ss_out[(size_t)m * f.ss_ld + gi.bx * SE + p] = v;
      }
    };
    if (gi.ny == 1) {
      // no split: this workgroup owns the tile -- no slab, no ticket (same sums: residual + (acc + bias))
      float ssl[SE];
#pragma unroll
      for (int p = 0; p < SE; ++p) ssl[p] = 0.f;
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        const int n0 = (tile0 + t) * 16 + q;
        if (m < M && n0 < e.N) {
          f32x4 v = acc[t];
          if (e.bias) v += load4_guard(e.bias, n0, e.N);
          finish(t, n0, fin_base(t) + v, ssl[t / 2 < SE ? t / 2 : 0]);
          fx_clear(n0);
        }
      }
      put_ss(ssl);
      return;
    }
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const int n0 = (tile0 + t) * 16 + q;
      if (m < M && n0 < e.N) {
        f32x4 v = acc[t];
        if (e.bias && z == 0) v += load4_guard(e.bias, n0, e.N);
        gu64* dst = (gu64*)((float*)e.C + ((size_t)z * M + m) * e.ldc + n0);
        __hip_atomic_store(dst, __builtin_bit_cast(unsigned long long, u32x2{__float_as_uint(v[0]),
                           __float_as_uint(v[1])}), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(dst + 1, __builtin_bit_cast(unsigned long long, u32x2{__float_as_uint(v[2]),
                           __float_as_uint(v[3])}), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    int old = 0;
    if (lane == 0) old = __hip_atomic_fetch_add(f.fin_cnt + gi.bx, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    old = __shfl(old, 0, 64);
    if (old != gi.ny - 1) return;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");   // compiler-only: keep the loads below the ticket
    float ssl[SE];
#pragma unroll
    for (int p = 0; p < SE; ++p) ssl[p] = 0.f;
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const int n0 = (tile0 + t) * 16 + q;
      if (m < M && n0 < e.N) {
        f32x4 v = fin_base(t);
        // all (<= 8) slabs in flight at once: clamped addresses + selects, no per-split branch / wait
        const int Z = gi.ny;
        u32x2 sa[8], sb[8];
#pragma unroll
        for (int zz = 0; zz < 8; ++zz) {
          gu64* src = (gu64*)((float*)e.C + ((size_t)(zz < Z ? zz : Z - 1) * M + m) * e.ldc + n0);
          sa[zz] = __builtin_bit_cast(u32x2, __hip_atomic_load(src, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
          sb[zz] = __builtin_bit_cast(u32x2, __hip_atomic_load(src + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
        }
#pragma unroll
        for (int zz = 0; zz < 8; ++zz) {
          const f32x4 sv = {__uint_as_float(sa[zz][0]), __uint_as_float(sa[zz][1]), __uint_as_float(sb[zz][0]),
                            __uint_as_float(sb[zz][1])};
          v += zz < Z ? sv : f32x4{0.f, 0.f, 0.f, 0.f};
        }
        finish(t, n0, v, ssl[t / 2 < SE ? t / 2 : 0]);
        fx_clear(n0);
      }
    }
    put_ss(ssl);
    if (lane == 0) __hip_atomic_store(f.fin_cnt + gi.bx, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return;
  }
  if constexpr (EPI == PG_EPI_F32_ADD) {
    // C[m][n] += acc (+ bias by split 0): hardware float atomic adds at the memory side, no slab, no ticket --
    // the launch ends one atomic round trip after its last MFMA (the F32_FIN tail is slab store -> ticket -> slab
    // load).  The split order of the adds is unordered (fp32 rounding of the sum may differ run to run).
    if (m < M) {
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        const int n0 = (tile0 + t) * 16 + q;
        if (n0 < e.N) {
          f32x4 v = acc[t];
          if (e.bias && z == 0) v += load4_guard(e.bias, n0, e.N);
          float* dst = (float*)e.C + (size_t)m * e.ldc + n0;
#pragma unroll
          for (int j = 0; j < 4; ++j) unsafeAtomicAdd(dst + j, v[j]);
        }
      }
    }
    return;
  }
  if constexpr (EPI == PG_EPI_FX_ADD) {
    // C[m][n] += rn(acc * 2^32) by 64-bit integer atomics (global_atomic_add_u64 at the memory side): the same one
    // round trip after the last MFMA as F32_ADD, but integer addition is associative, so the accumulated sum --
    // and every residual read from it -- is the same bits whatever order the splits arrive in
    if (m < M) {
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        const int n0 = (tile0 + t) * 16 + q;
        if (n0 < e.N) {
          f32x4 v = acc[t];
          if (e.bias && z == 0) v += load4_guard(e.bias, n0, e.N);
          unsigned long long* dst = (unsigned long long*)e.C + (size_t)m * e.ldc + n0;
#pragma unroll
          for (int j = 0; j < 4; ++j) atomicAdd(dst + j, (unsigned long long)fx_from_f32(v[j]));
        }
      }
    }
    return;
  }
  if constexpr (EPI == PG_EPI_BF16_GELU_MUL) {
#pragma unroll
    for (int t = 0; t < NT; t += 2) epi_gelu_mul4(e, m, (tile0 + t) * 16, q, acc[t], acc[t + 1]);
  } else if constexpr (EPI == PG_EPI_QKV_ROPE) {
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      f32x4 v = acc[t];
      const int n0 = (tile0 + t) * 16 + q;
      if (e.bias && n0 < e.N) v += load4_guard(e.bias, n0, e.N);
      f32x4 pr;
#pragma unroll
      for (int j = 0; j < 4; ++j) pr[j] = xchg_xor32(v[j]);
      epi_qkv_rope4_core(e, m, n0, v, pr, rope_cs[t], rope_sn[t], e.f.slot_base + rope_slot_raw);
    }
  } else {
#pragma unroll
    for (int t = 0; t < NT; ++t) epi_store4<EPI>(e, m, (tile0 + t) * 16 + q, acc[t], z);
  }
}

template <int EPI, int NT, int U, int DEPTH, int PRO, bool FRAG, int CPW = 0>
__global__ __launch_bounds__(256) void gemv_kernel(const bf16_t* __restrict__ A, int lda,
                                                   const bf16_t* __restrict__ W, int ldw, int K, EpiArgs e) {
  gemv_body<EPI, NT, U, DEPTH, PRO, FRAG, CPW>(A, lda, W, ldw, K, e,
                                               GemvIdx{(int)blockIdx.x, (int)blockIdx.y, (int)gridDim.x, (int)gridDim.y});
}

// --------------------------------------------------------------------------------------
// fp8 weight-streaming GEMV for 17..32 rows (batched decode on the fp8 path, BASELINE configs[4])
// --------------------------------------------------------------------------------------
// The batch-32 decode linears read each e4m3 weight once per step; as 64 x 128 / 128 x 128 tile GEMMs they staged
// W through LDS at 3.1-3.3 TB/s.  Here, as in gemv_body, W streams straight to VGPRs: the weights are stored
// fragment-packed (PG_W_FRAG with PG_FP8, weights.frag_pack8): W[16t + r][128c + 64s + 16g + e] (e < 16 bytes) at
// byte ((t * (K/128) + c) * 2 + s) * 1024 + (16g + r) * 16 + e, so piece s of a 16-row x 128-k chunk is one 1-KiB
// lane-linear non-temporal load.  Lane (r, g) loads x row r (and 16 + r) at the same k bytes, one
// v_mfma_scale_f32_16x16x128_f8f6f4 (unit block scales) per (W tile, 16-row x tile) and chunk; the 4 waves split
// the chunks of split blockIdx.y round-robin, DEPTH chunks in flight, and reduce through LDS.  The accumulator is
// scaled by a_scale[m] * w_scale[n] before the tile kernel's epilogues (bf16, gelu*up, fp32 slabs, RoPE + KV).
template <int EPI, int NT, int MT, int DEPTH, int CPW>
__global__ __launch_bounds__(256) void gemv8_kernel(const uint8_t* __restrict__ X, int ldx,
                                                    const uint8_t* __restrict__ W, int K, EpiArgs e) {
  amax_clear(e);
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int g = lane >> 4, r = lane & 15;
  const int tile0 = blockIdx.x * NT;
  const int M = e.M;
  const int z = blockIdx.y;
  const int nch_all = K >> 7;
  const int per_z = (nch_all + (int)gridDim.y - 1) / (int)gridDim.y;
  const int c0 = z * per_z;
  const int nch = min(nch_all - c0, per_z);
  const int mine = CPW > 0 ? CPW : (nch > wave ? (nch - wave + 3) / 4 : 0);   // chunks wave, wave + 4, ...
  const uint8_t* wt[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) wt[t] = W + (size_t)min(tile0 + t, (e.N >> 4) - 1) * 16 * K + lane * 16;
  const uint8_t* xr[MT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) xr[mt] = X + (size_t)min(mt * 16 + r, M - 1) * ldx + g * 16;
  f32x4 acc[NT][MT];
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) acc[t][mt] = f32x4{0.f, 0.f, 0.f, 0.f};
  u32x4 wb[DEPTH][NT][2], xb[DEPTH][MT][2];
  auto load = [&](int j, u32x4 (&wv)[NT][2], u32x4 (&xv)[MT][2]) {
    const size_t cc = (size_t)(c0 + wave + j * 4);
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int sp = 0; sp < 2; ++sp)
        wv[t][sp] = __builtin_nontemporal_load((const u32x4*)(wt[t] + (cc * 2 + sp) * 1024));
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int sp = 0; sp < 2; ++sp) xv[mt][sp] = *(const u32x4*)(xr[mt] + cc * 128 + sp * 64);
  };
  auto compute = [&](const u32x4 (&wv)[NT][2], const u32x4 (&xv)[MT][2]) {
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
        acc[t][mt] = mfma8(__builtin_bit_cast(bf16x8, wv[t][0]), __builtin_bit_cast(bf16x8, wv[t][1]),
                           __builtin_bit_cast(bf16x8, xv[mt][0]), __builtin_bit_cast(bf16x8, xv[mt][1]), acc[t][mt]);
  };
  // (QKV epilogue operands issued with the stream, as gemv_body does, are not needed: the tile epilogue loads them)
#pragma unroll
  for (int d = 0; d < DEPTH; ++d)
    if (CPW > 0 ? d < CPW : d < mine) load(d, wb[d], xb[d]);
  if constexpr (CPW > 0) {
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int j = 0; j < CPW; ++j) {
      const int d = j % DEPTH;
      compute(wb[d], xb[d]);
      if (j + DEPTH < CPW) load(j + DEPTH, wb[d], xb[d]);
      __builtin_amdgcn_sched_barrier(0);
    }
  } else {
    for (int base = 0; base < mine; base += DEPTH) {
#pragma unroll
      for (int d = 0; d < DEPTH; ++d) {
        const int j = base + d;
        if (j < mine) {
          compute(wb[d], xb[d]);
          if (j + DEPTH < mine) load(j + DEPTH, wb[d], xb[d]);
        }
      }
    }
  }
  __shared__ f32x4 red[4][NT][MT][64];
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) red[wave][t][mt][lane] = acc[t][mt];
  __syncthreads();
  if (wave != 0) return;
  const int q = 4 * g;
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) {
    const int m = mt * 16 + r;
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      acc[t][mt] = red[0][t][mt][lane] + red[1][t][mt][lane] + red[2][t][mt][lane] + red[3][t][mt][lane];
      scale_acc(e, m, (tile0 + t) * 16 + q, acc[t][mt]);
    }
    if constexpr (EPI == PG_EPI_BF16_GELU_MUL) {
#pragma unroll
      for (int t = 0; t < NT; t += 2) epi_gelu_mul4(e, m, (tile0 + t) * 16, q, acc[t][mt], acc[t + 1][mt]);
    } else if constexpr (EPI == PG_EPI_QKV_ROPE) {
#pragma unroll
      for (int t = 0; t < NT; ++t) epi_qkv_rope4(e, m, (tile0 + t) * 16 + q, acc[t][mt]);   // (all lanes: shuffle)
    } else if constexpr (EPI == PG_EPI_F32_ADD) {
#pragma unroll
      for (int t = 0; t < NT; ++t) epi_add4(e, m, (tile0 + t) * 16 + q, acc[t][mt], z);
    } else {
#pragma unroll
      for (int t = 0; t < NT; ++t) epi_store4<EPI>(e, m, (tile0 + t) * 16 + q, acc[t][mt], z);
    }
  }
}

// The wide form (large N: gate/up, down, the lm_head): x is staged ONCE per workgroup in LDS and the 4 waves split
// the W tiles instead of K (wave w owns tiles tile0 + w*NTW ...), so a workgroup reads x[32][Kr] once for 4 * NTW
// tiles -- at 32 rows x costs as many bytes per 16-row tile as the tile itself, and the per-CU load rate, not HBM,
// bounded the K-split form (gate/up 4.3 TB/s, down 2.9).  x [M <= 32][Kr] arrives by LDS-DMA (1 KiB pieces, the 16-B
// chunks of a row XOR-swizzled by row through the source address), issued before the W stream; each wave then
// streams its own W tiles DEPTH chunks deep and reads its x fragments from LDS.  No cross-wave reduction: every
// wave runs the epilogue of its own tiles (bf16, gelu*up on gate/up pairs, fp32 slabs, float-atomic residual add).
// XB (pro_mode 5): X is bf16 h [M][ldx elements] and row m's amax (amax_in, max-ed by the gate/up epilogue): each
// thread loads 16-element pieces, divides by s[m] = amax / 448 and packs e4m3 (pg_quant_fp8's bytes) into the same
// swizzled LDS layout -- the quantiser launch between gate/up and down is gone; x costs twice the bytes per
// workgroup (bf16), all issued before the W stream.
template <int EPI, int NTW, int MT, int DEPTH, int CPW, bool XB = false>
__global__ __launch_bounds__(256) void gemv8x_kernel(const uint8_t* __restrict__ X, int ldx,
                                                     const uint8_t* __restrict__ W, int K, EpiArgs e) {
  extern __shared__ __attribute__((aligned(16))) char xs8[];
  static_assert(!XB || CPW > 0, "the bf16-x form needs a compile-time chunk count");
  amax_clear(e);
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int g = lane >> 4, r = lane & 15;
  const int tile0 = (blockIdx.x * 4 + wave) * NTW;
  const int M = e.M;
  const int z = blockIdx.y;
  const int nch_all = K >> 7;
  const int per_z = (nch_all + (int)gridDim.y - 1) / (int)gridDim.y;
  const int c0 = z * per_z;
  const int nch = CPW > 0 ? CPW : max(0, min(nch_all - c0, per_z));
  const int Kr = nch * 128;                        // bytes of one x row in LDS
  // 1. x rows [0, 16 MT) x bytes [128 c0, +Kr) into LDS by DMA: LDS byte o = row * Kr + 16 pc holds logical chunk
  //    pc ^ (row & 7) of the row (rows past M repeat row M-1: their outputs are never stored)
  constexpr int XPT = XB ? MT * 16 * CPW * 8 / 256 : 1;   // XB: 16-element pieces per thread
  u32x4 xh[XPT][2];
  if constexpr (XB) {
    const bf16_t* Xb = (const bf16_t*)X;
#pragma unroll
    for (int i = 0; i < XPT; ++i) {
      const int ci = (int)threadIdx.x + i * 256;   // LDS chunk: row ci / (8 CPW), position pc
      const int row = ci / (8 * CPW), pc = ci % (8 * CPW);
      const bf16_t* src = Xb + (size_t)min(row, M - 1) * ldx + (size_t)c0 * 128 + (pc ^ (row & 7)) * 16;
      xh[i][0] = *(const u32x4*)src;
      xh[i][1] = *(const u32x4*)(src + 8);
    }
  } else {
    const int pieces = MT * 16 * Kr / 1024;        // 1 KiB each, dealt round-robin to the waves
    for (int pi = wave; pi < pieces; pi += 4) {
      const int o = pi * 1024 + lane * 16;
      const int row = o / Kr, pc = (o % Kr) >> 4;
      const int lc = pc ^ (row & 7);
      const uint8_t* src = X + (size_t)min(row, M - 1) * ldx + (size_t)c0 * 128 + lc * 16;
      __builtin_amdgcn_global_load_lds((const void*)src, (LDS_AS void*)(xs8 + pi * 1024), 16, 0, 0);
    }
  }
  // the x DMA pieces stay ahead of every W load in the vmcnt order (step 3 waits for "at most the W loads
  // outstanding"): the scheduler may not hoist a W load above them
  __builtin_amdgcn_sched_barrier(0);
  const uint8_t* wt[NTW];
#pragma unroll
  for (int t = 0; t < NTW; ++t) wt[t] = W + (size_t)min(tile0 + t, (e.N >> 4) - 1) * 16 * K + lane * 16;
  f32x4 acc[NTW][MT];
#pragma unroll
  for (int t = 0; t < NTW; ++t)
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) acc[t][mt] = f32x4{0.f, 0.f, 0.f, 0.f};
  u32x4 wb[DEPTH][NTW][2];
  auto loadw = [&](int j, u32x4 (&wv)[NTW][2]) {
    const size_t cc = (size_t)(c0 + j);
#pragma unroll
    for (int t = 0; t < NTW; ++t)
#pragma unroll
      for (int sp = 0; sp < 2; ++sp)
        wv[t][sp] = __builtin_nontemporal_load((const u32x4*)(wt[t] + (cc * 2 + sp) * 1024));
  };
  // 2. the W stream, DEPTH chunks deep, issued behind the x pieces
#pragma unroll
  for (int d = 0; d < DEPTH; ++d)
    if (CPW > 0 ? d < CPW : d < nch) loadw(d, wb[d]);
  // 3. this wave's x pieces have landed once at most its W loads are outstanding; the barrier covers the others'
  {
    const int wl = (CPW > 0 ? min(DEPTH, CPW) : min(DEPTH, nch)) * NTW * 2;
    wait_vm_n(wl);
    if constexpr (XB) {
#pragma unroll
      for (int i = 0; i < XPT; ++i) {
        const int ci = (int)threadIdx.x + i * 256;
        const int row = ci / (8 * CPW), pc = ci % (8 * CPW);
        const float am = __uint_as_float(e.f.amax_in[(size_t)min(row, M - 1) * e.f.amax_ld]);
        const float sc = am > 0.f ? am / 448.f : 1.f;
        u32x4 w8;
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
          for (int j = 0; j < 2; ++j)
            w8[2 * h + j] = pack_fp8x4(bf_lo(xh[i][h][2 * j]) / sc, bf_hi(xh[i][h][2 * j]) / sc,
                                       bf_lo(xh[i][h][2 * j + 1]) / sc, bf_hi(xh[i][h][2 * j + 1]) / sc);
        *(u32x4*)(xs8 + row * Kr + pc * 16) = w8;
      }
    }
    __syncthreads();
  }
  auto compute = [&](int j, const u32x4 (&wv)[NTW][2]) {
    bf16x8 xf[MT][2];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      const int row = mt * 16 + r;
#pragma unroll
      for (int sp = 0; sp < 2; ++sp) {
        const int lc = j * 8 + sp * 4 + g;
        xf[mt][sp] = *(const bf16x8*)(xs8 + row * Kr + ((lc ^ (row & 7)) << 4));
      }
    }
#pragma unroll
    for (int t = 0; t < NTW; ++t)
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
        acc[t][mt] = mfma8(__builtin_bit_cast(bf16x8, wv[t][0]), __builtin_bit_cast(bf16x8, wv[t][1]), xf[mt][0],
                           xf[mt][1], acc[t][mt]);
  };
  if constexpr (CPW > 0) {
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int j = 0; j < CPW; ++j) {
      const int d = j % DEPTH;
      compute(j, wb[d]);
      if (j + DEPTH < CPW) loadw(j + DEPTH, wb[d]);
      __builtin_amdgcn_sched_barrier(0);
    }
  } else {
    for (int base = 0; base < nch; base += DEPTH) {
#pragma unroll
      for (int d = 0; d < DEPTH; ++d) {
        const int j = base + d;
        if (j < nch) {
          compute(j, wb[d]);
          if (j + DEPTH < nch) loadw(j + DEPTH, wb[d]);
        }
      }
    }
  }
  const int q = 4 * g;
  float gam[MT];                                   // GELU_MUL with amax_out: this lane's max |h| per row tile
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) {
    const int m = mt * 16 + r;
    gam[mt] = 0.f;
    if constexpr (XB) {
      const float am = __uint_as_float(e.f.amax_in[(size_t)min(m, M - 1) * e.f.amax_ld]);
      const float sa = am > 0.f ? am / 448.f : 1.f;
#pragma unroll
      for (int t = 0; t < NTW; ++t) {
        const int n0 = (tile0 + t) * 16 + q;
        if (m < e.M && n0 < e.N) acc[t][mt] *= sa * load4_guard(e.f.w_scale, n0, e.N);
      }
    } else {
#pragma unroll
      for (int t = 0; t < NTW; ++t) scale_acc(e, m, (tile0 + t) * 16 + q, acc[t][mt]);
    }
    if constexpr (EPI == PG_EPI_BF16_GELU_MUL) {
      if (e.f.amax_out) {
#pragma unroll
        for (int t = 0; t < NTW; t += 2)
          gam[mt] = fmaxf(gam[mt], epi_gelu_mul4_amax(e, m, (tile0 + t) * 16, q, acc[t][mt], acc[t + 1][mt]));
      } else {
#pragma unroll
        for (int t = 0; t < NTW; t += 2) epi_gelu_mul4(e, m, (tile0 + t) * 16, q, acc[t][mt], acc[t + 1][mt]);
      }
    } else if constexpr (EPI == PG_EPI_F32_ADD) {
#pragma unroll
      for (int t = 0; t < NTW; ++t) epi_add4(e, m, (tile0 + t) * 16 + q, acc[t][mt], z);
    } else {
#pragma unroll
      for (int t = 0; t < NTW; ++t) epi_store4<EPI>(e, m, (tile0 + t) * 16 + q, acc[t][mt], z);
    }
  }
  if constexpr (EPI == PG_EPI_BF16_GELU_MUL) {
    if (e.f.amax_out) {                            // (uniform: every wave reaches the barrier)
      // row max over the 4 column groups of a lane's row, then over the 4 waves in LDS: one atomic per row per
      // workgroup (float bits of non-negative values order as unsigned)
      __shared__ float sam[4][16 * MT];
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        float v = gam[mt];
        v = fmaxf(v, __shfl_xor(v, 16, 64));
        v = fmaxf(v, __shfl_xor(v, 32, 64));
        if (g == 0) sam[wave][mt * 16 + r] = v;
      }
      __syncthreads();
      if ((int)threadIdx.x < 16 * MT && (int)threadIdx.x < M) {
        const float v = fmaxf(fmaxf(sam[0][threadIdx.x], sam[1][threadIdx.x]),
                              fmaxf(sam[2][threadIdx.x], sam[3][threadIdx.x]));
        if (v > 0.f)
          __hip_atomic_fetch_max(e.f.amax_out + (size_t)threadIdx.x * e.f.amax_ld, __float_as_uint(v),
                                 __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
  }
}

template <int EPI, int NTW, int MT, int DEPTH = 8>
static void launch_gemv8x_mt(const uint8_t* X, int ldx, const uint8_t* W, int K, int ksplit, const EpiArgs& e,
                             hipStream_t st) {
  const int tiles = e.N >> 4;
  const dim3 grid((tiles + 4 * NTW - 1) / (4 * NTW), ksplit);
  const int nch = K >> 7;
  const int per_z = (nch + ksplit - 1) / ksplit;
  const size_t lds = (size_t)MT * 16 * per_z * 128;
  const bool exact = nch % ksplit == 0;
  if constexpr (EPI == PG_EPI_F32) {
    if (e.f.pro_mode == 5) {                       // bf16 x quantised while staged (host: exact, 8 or 16 chunks)
      if (per_z == 16)
        hipLaunchKernelGGL((gemv8x_kernel<EPI, NTW, MT, 8, 16, true>), grid, dim3(256), lds, st, X, ldx, W, K, e);
      else
        hipLaunchKernelGGL((gemv8x_kernel<EPI, NTW, MT, 8, 8, true>), grid, dim3(256), lds, st, X, ldx, W, K, e);
      return;
    }
  }
  if (exact && per_z == 16)
    hipLaunchKernelGGL((gemv8x_kernel<EPI, NTW, MT, DEPTH, 16>), grid, dim3(256), lds, st, X, ldx, W, K, e);
  else if (exact && per_z == 8)
    hipLaunchKernelGGL((gemv8x_kernel<EPI, NTW, MT, DEPTH, 8>), grid, dim3(256), lds, st, X, ldx, W, K, e);
  else
    hipLaunchKernelGGL((gemv8x_kernel<EPI, NTW, MT, DEPTH, 0>), grid, dim3(256), lds, st, X, ldx, W, K, e);
}

#ifndef PG_GEMV8_DEPTH
#define PG_GEMV8_DEPTH 4
#endif
template <int EPI, int NT, int MT>
static void launch_gemv8_mt(const uint8_t* X, int ldx, const uint8_t* W, int K, int ksplit, const EpiArgs& e,
                            hipStream_t st) {
  const dim3 grid(((e.N >> 4) + NT - 1) / NT, ksplit);
  const int nch = K >> 7;
  const int cpw = (nch % ksplit == 0 && (nch / ksplit) % 4 == 0) ? nch / ksplit / 4 : 0;
  constexpr int D = PG_GEMV8_DEPTH;                // chunks in flight per wave
  switch (cpw) {
    case 2: hipLaunchKernelGGL((gemv8_kernel<EPI, NT, MT, 2, 2>), grid, dim3(256), 0, st, X, ldx, W, K, e); break;
    case 4: hipLaunchKernelGGL((gemv8_kernel<EPI, NT, MT, D, 4>), grid, dim3(256), 0, st, X, ldx, W, K, e); break;
    case 8: hipLaunchKernelGGL((gemv8_kernel<EPI, NT, MT, D, 8>), grid, dim3(256), 0, st, X, ldx, W, K, e); break;
    default: hipLaunchKernelGGL((gemv8_kernel<EPI, NT, MT, D, 0>), grid, dim3(256), 0, st, X, ldx, W, K, e); break;
  }
}

template <int EPI, int NT>
static void launch_gemv8_nt(const uint8_t* X, int ldx, const uint8_t* W, int K, int ksplit, const EpiArgs& e,
                            hipStream_t st) {
  if (e.M <= 16)
    launch_gemv8_mt<EPI, NT, 1>(X, ldx, W, K, ksplit, e, st);
  else
    launch_gemv8_mt<EPI, NT, 2>(X, ldx, W, K, ksplit, e, st);
}

#ifndef PG_GEMV8_NT_MAX
#define PG_GEMV8_NT_MAX 4
#endif
// NT W tiles per workgroup: every lane loads the x rows of its chunks once per workgroup, as many bytes per 16-row W
// tile as the tile itself at 32 rows, so wide tiles amortise x -- the most tiles per workgroup that still leave
// >= 256 workgroups (gelu*up: whole gate/up pairs); MT = 16-row x tiles
#ifndef PG_GEMV8_WIDE
#define PG_GEMV8_WIDE 1
#endif
template <int EPI>
static void launch_gemv8(const uint8_t* X, int ldx, const uint8_t* W, int K, int ksplit, const EpiArgs& e,
                         hipStream_t st) {
  const int tiles = e.N >> 4;
  // the wide form (x once per workgroup in LDS, waves split N) when its grid still has >= 256 workgroups and a
  // split's x rows fit the LDS; the K-split form otherwise (q|k|v: 160 tiles; o_proj)
  const int per_z = ((K >> 7) + ksplit - 1) / ksplit;
  if constexpr (EPI == PG_EPI_F32) {
    if (e.f.pro_mode == 5) {                       // bf16 x: the wide form only (host checked the chunk count)
      const int wgs2 = (tiles + 7) / 8 * ksplit;
      if (e.M <= 16) {
        if (wgs2 >= 256) launch_gemv8x_mt<EPI, 2, 1>(X, ldx, W, K, ksplit, e, st);
        else launch_gemv8x_mt<EPI, 1, 1>(X, ldx, W, K, ksplit, e, st);
      } else {
        if (wgs2 >= 256) launch_gemv8x_mt<EPI, 2, 2>(X, ldx, W, K, ksplit, e, st);
        else launch_gemv8x_mt<EPI, 1, 2>(X, ldx, W, K, ksplit, e, st);
      }
      return;
    }
  }
  if constexpr (EPI != PG_EPI_QKV_ROPE) {
    if (PG_GEMV8_WIDE && per_z * 128 <= 4096) {
      const int wgs2 = (tiles + 7) / 8 * ksplit, wgs1 = (tiles + 3) / 4 * ksplit;
      if (e.M <= 16) {
        if (wgs2 >= 256 || EPI == PG_EPI_BF16_GELU_MUL) { launch_gemv8x_mt<EPI, 2, 1>(X, ldx, W, K, ksplit, e, st); return; }
        if constexpr (EPI != PG_EPI_BF16_GELU_MUL)
          if (wgs1 >= 256) { launch_gemv8x_mt<EPI, 1, 1>(X, ldx, W, K, ksplit, e, st); return; }
      } else {
        if (wgs2 >= 256 || EPI == PG_EPI_BF16_GELU_MUL) { launch_gemv8x_mt<EPI, 2, 2>(X, ldx, W, K, ksplit, e, st); return; }
        if constexpr (EPI != PG_EPI_BF16_GELU_MUL)
          if (wgs1 >= 256) { launch_gemv8x_mt<EPI, 1, 2>(X, ldx, W, K, ksplit, e, st); return; }
      }
    }
  }
  if (PG_GEMV8_NT_MAX >= 4 && tiles % 4 == 0 && (tiles / 4) * ksplit >= 256)
    launch_gemv8_nt<EPI, 4>(X, ldx, W, K, ksplit, e, st);
  else if (EPI == PG_EPI_BF16_GELU_MUL || (PG_GEMV8_NT_MAX >= 2 && tiles % 2 == 0 && (tiles / 2) * ksplit >= 256))
    launch_gemv8_nt<EPI, 2>(X, ldx, W, K, ksplit, e, st);
  else if constexpr (EPI != PG_EPI_BF16_GELU_MUL)
    launch_gemv8_nt<EPI, 1>(X, ldx, W, K, ksplit, e, st);
}

// --------------------------------------------------------------------------------------
// Split-K finalisation for the bf16 epilogues (prefill at small M, where a full-K tile grid leaves CUs
// idle): the GEMM writes fp32 slabs [z][M][N] (bias in slab 0), this kernel sums them and applies the
// epilogue (bf16 / gelu / gelu*up / V^T side output / RoPE + KV-cache append).  One thread per 4 outputs.
template <int EPI>
__global__ __launch_bounds__(256) void gemm_finalize_kernel(const float* __restrict__ part, int nsplit, EpiArgs e) {
  const int NO = EPI == PG_EPI_BF16_GELU_MUL ? e.N / 2 : e.N;     // output columns
  const long idx = (long)blockIdx.x * 256 + threadIdx.x;
  const int q4 = NO / 4;
  if (idx >= (long)e.M * q4) return;
  const int m = (int)(idx / q4), c0 = (int)(idx % q4) * 4;
  const size_t slab = (size_t)e.M * e.N;
  auto sum4 = [&](int n) {
    f32x4 v = {0.f, 0.f, 0.f, 0.f};
    for (int z = 0; z < nsplit; ++z) v += *(const f32x4*)(part + z * slab + (size_t)m * e.N + n);
    return v;
  };
  if constexpr (EPI == PG_EPI_BF16_GELU_MUL) {
    // output column c0 <- gate column 32*(c0/16) + c0%16, up column +16
    const int gb = (c0 / 16) * 32, q = c0 % 16;
    epi_gelu_mul4(e, m, gb, q, sum4(gb + q), sum4(gb + 16 + q));
  } else if constexpr (EPI == PG_EPI_QKV_ROPE) {
    epi_qkv_rope4_pr(e, m, c0, sum4(c0), sum4(c0 ^ 8));
  } else {
    EpiArgs e2 = e;
    e2.bias = nullptr;                                            // already in slab 0
    epi_store4<EPI>(e2, m, c0, sum4(c0), 0);
  }
}

// --------------------------------------------------------------------------------------
// C ABI
// --------------------------------------------------------------------------------------
// Tile choice: 128-row tiles (2-stage ring, 64 KiB LDS -> 2 workgroups per CU) when that grid already
// has >= 256 workgroups; otherwise 64-row tiles with a 4-stage ring.  Split-K (fp32 partial epilogue
// only) is chosen by the caller.
// F8: A, W fp8 viewed as bf16-sized pairs (K, lda, ldw in 2-byte units: a 64-unit k-tile = 128 fp8 k)
// waves per workgroup of each gemm_tile_kernel shape (4, or 8 / 12 -- see the kernel).  8 / 8 / 8 / 12 measured
// 3-12 % faster than 4 on every batch-1 prefill GEMM and pt-224 prefill 5.29 -> 4.95 ms
// (profiles/r03_tile_waves_ab.txt)
#ifndef PG_TILE_KSUB
#define PG_TILE_KSUB 1    // 2: 64-row tiles stage 128 k per barrier (K % 128 == 0; 3 stages)
#endif
#ifndef PG_TILE_AUTO_N64
#define PG_TILE_AUTO_N64 1   // 64 x 64 tiles when the 64 x 128 grid has fewer workgroups than CUs (bf16)
#endif
#ifndef PG_TILE_W64
#define PG_TILE_W64 8
#endif
#ifndef PG_TILE_W128
#define PG_TILE_W128 8
#endif
#ifndef PG_TILE_W256
#define PG_TILE_W256 8
#endif
#ifndef PG_TILE_W288
#define PG_TILE_W288 12
#endif
// 64-row tiles, BN 128 (WV waves) or 64 (4 waves): 64-k stages (4 deep), or with PG_TILE_KSUB 2 and K % 128 == 0
// 128-k stages (3 deep)
template <int EPI, bool FRAG, bool F8, int BN, int WV>
static void launch_t64(const bf16_t* A, int lda, const bf16_t* W, int ldw, int K, int ksplit, const EpiArgs& e,
                       hipStream_t st) {
  const int m64 = (e.M + 63) / 64, tn = (e.N + BN - 1) / BN;
  if constexpr (PG_TILE_KSUB == 2) {
    if (K % 128 == 0) {
      const int kchunk = ((K / 128 + ksplit - 1) / ksplit) * 128;
      hipLaunchKernelGGL((gemm_tile_kernel<EPI, 64, 3, FRAG, F8, WV, BN, 2>), dim3(m64 * tn, 1, ksplit), dim3(64 * WV),
                         0, st, A, lda, W, ldw, K, kchunk, m64, tn, e);
      return;
    }
  }
  const int kchunk = ((K / TBK + ksplit - 1) / ksplit) * TBK;
  hipLaunchKernelGGL((gemm_tile_kernel<EPI, 64, 4, FRAG, F8, WV, BN>), dim3(m64 * tn, 1, ksplit), dim3(64 * WV), 0, st,
                     A, lda, W, ldw, K, kchunk, m64, tn, e);
}

template <int EPI, bool FRAG, bool F8 = false>
static void launch_tile(const bf16_t* A, int lda, const bf16_t* W, int ldw, int K, int ksplit, const EpiArgs& e,
                        hipStream_t st, bool m1 = false, bool n64 = false) {
  if (n64) {
    // (a 9-stage ring for one-round grids measured 3-10% slower on every batch-1 shape: r03_tile_sweep.txt)
    launch_t64<EPI, FRAG, F8, 64, 4>(A, lda, W, ldw, K, ksplit, e, st);
    return;
  }
  if constexpr (!F8) {
    if (m1) {
      // PG_TILE_M1 (batch-1 prefill: 256 image + a few text rows): ALL rows in one tile, so every weight tile
      // streams once and no 256-row tile is spent on an 8-row remainder (M = 264: 2 x 256 rows in gemm256)
      const int tiles_n = (e.N + TBN - 1) / TBN;
      const int kchunk = ((K / TBK + ksplit - 1) / ksplit) * TBK;
      constexpr bool WNT = PG_TILE_M1_WNT;
      if (e.M <= 256)
        hipLaunchKernelGGL((gemm_tile_kernel<EPI, 256, 3, FRAG, false, PG_TILE_W256, TBN, 1, WNT>),
                           dim3(tiles_n, 1, ksplit), dim3(64 * PG_TILE_W256), 0, st, A, lda,
                           W, ldw, K, kchunk, 1, tiles_n, e);
      else
        hipLaunchKernelGGL((gemm_tile_kernel<EPI, 288, 3, FRAG, false, PG_TILE_W288, TBN, 1, WNT>),
                           dim3(tiles_n, 1, ksplit), dim3(64 * PG_TILE_W288), 0, st, A, lda,
                           W, ldw, K, kchunk, 1, tiles_n, e);
      return;
    }
  }
  const int t256 = ((e.M + 255) / 256) * ((e.N + 255) / 256);
  // (fp8 on the 256 x 256 kernel addresses its operands by 32-bit byte offsets: both must be < 4 GiB)
  const bool off32 = (size_t)e.M * lda * 2 < (1ull << 32) && (size_t)e.N * ldw * 2 < (1ull << 32);
  constexpr bool g256 = !F8 || PG_F8_G256 == 2 || (PG_F8_G256 == 1 && EPI == PG_EPI_F32);
  if (g256 && (!F8 || off32) && t256 * ksplit >= PG_G256_MIN_TILES && (ksplit == 1 || EPI == PG_EPI_F32)) {
    const int kts = (K / 64 + ksplit - 1) / ksplit;
    hipLaunchKernelGGL((gemm256_kernel<EPI, FRAG, F8>), dim3(t256, 1, ksplit), dim3(512), 0, st, A, lda, W, ldw, K, kts,
                       (e.M + 255) / 256, (e.N + 255) / 256, e);
    return;
  }
  const int tiles_n = (e.N + TBN - 1) / TBN;
  int kchunk = ((K / TBK + ksplit - 1) / ksplit) * TBK;
  const int t128 = ((e.M + 127) / 128) * tiles_n;
  if (t128 >= 256) {
    const int tiles_m = (e.M + 127) / 128;
    hipLaunchKernelGGL((gemm_tile_kernel<EPI, 128, F8 ? PG_T128_STAGES_F8 : 2, FRAG, F8, PG_TILE_W128>),
                       dim3(tiles_m * tiles_n, 1, ksplit),
                       dim3(64 * PG_TILE_W128), 0, st,
                       A, lda, W, ldw, K, kchunk, tiles_m, tiles_n, e);
    return;
  }
  // (a 96-row tile wastes fewer padded rows at M = 264 but measured slower: fewer workgroups)
  const int m64 = (e.M + 63) / 64;
  if (!F8 && PG_TILE_AUTO_N64 && m64 * tiles_n * ksplit < 256) {
    // a 64 x 128 grid short of one workgroup per CU: 64 x 64 tiles, twice the workgroups (batch-1 prefill: SigLIP
    // q|k|v 13.7 -> 11.7 us, never slower on the other shapes; profiles/r03_tile_sweep.txt)
    launch_t64<EPI, FRAG, F8, 64, 4>(A, lda, W, ldw, K, ksplit, e, st);
    return;
  }
  launch_t64<EPI, FRAG, F8, TBN, PG_TILE_W64>(A, lda, W, ldw, K, ksplit, e, st);
}

// measured configs (round-1 GEMV sweep): M <= 4: one tile per WG, U=2, 8 chunks in flight;
// M > 4 and the gate/up pair: two tiles per WG, U=2, 4 chunks in flight.
// one gemv_kernel launch with the chunks-per-wave specialisation when the K split is exact (see gemv_kernel)
template <int EPI, int NT, int DEPTH, int PRO, bool FRAG>
static void launch_gemv_cpw(dim3 grid, size_t lds, hipStream_t st, const bf16_t* A, int lda, const bf16_t* W, int ldw,
                            int K, int ksplit, const EpiArgs& e) {
  const int nch = K / 64;                              // U = 2: 64-element chunks
  const int cpw = (nch % ksplit == 0 && (nch / ksplit) % 4 == 0) ? nch / ksplit / 4 : 0;
  switch (PG_GEMV_CPW ? cpw : 0) {
    case 4: hipLaunchKernelGGL((gemv_kernel<EPI, NT, 2, DEPTH, PRO, FRAG, 4>), grid, dim3(256), lds, st, A, lda, W, ldw, K, e); break;
    case 8: hipLaunchKernelGGL((gemv_kernel<EPI, NT, 2, DEPTH, PRO, FRAG, 8>), grid, dim3(256), lds, st, A, lda, W, ldw, K, e); break;
    case 16: hipLaunchKernelGGL((gemv_kernel<EPI, NT, 2, DEPTH, PRO, FRAG, 16>), grid, dim3(256), lds, st, A, lda, W, ldw, K, e); break;
    default: hipLaunchKernelGGL((gemv_kernel<EPI, NT, 2, DEPTH, PRO, FRAG, 0>), grid, dim3(256), lds, st, A, lda, W, ldw, K, e); break;
  }
}

// measured configs (round-1 GEMV sweep): M <= 4: one tile per WG, U=2, 8 chunks in flight;
// M > 4 and the gate/up pair: two tiles per WG, U=2, 4 chunks in flight.
template <int EPI, int PRO, bool FRAG>
static void launch_gemv_pro(const bf16_t* A, int lda, const bf16_t* W, int ldw, int K, int ksplit, const EpiArgs& e,
                            hipStream_t st) {
  const int ntiles = (e.N + 15) / 16;
  const int CH = 64;                                   // U = 2
  const int per_z = (K / CH + ksplit - 1) / ksplit;
  size_t lds = 0;
  if ((PRO != 0 && PRO != 4) || PG_GEMV_XLDS) {
    lds = (size_t)e.M * (per_z * CH + XPAD) * 2;
    lds = (lds + 15) & ~(size_t)15;
    if (PRO == 1) lds += 64 * sizeof(float);
    if (PRO == 3) lds += 80 * sizeof(float);
  }
  if constexpr (PG_GEMV_QKV_NT1 && EPI == PG_EPI_QKV_ROPE) {
    if (e.M > 4) {
      // batched q|k|v (2560 rows): one tile per workgroup doubles the grid to 160 workgroups
      launch_gemv_cpw<EPI, 1, PG_GEMV_D2, PRO, FRAG>(dim3(ntiles, ksplit), lds, st, A, lda, W, ldw, K, ksplit, e);
      return;
    }
  }
  // (four tiles per workgroup at 5..16 rows -- x's share of a workgroup's bytes 1/5 instead of 1/3 -- measured
  // slower on the pt-448 x16 gate/up and finalised down: 1.408 vs 1.380 ms/step; the epilogues take any even NT)
  // ring depths re-checked on the final round-2 code: two-tile kernels 4 chunks in flight, one-tile 8
  if (EPI == PG_EPI_BF16_GELU_MUL || e.M > 4) {
    launch_gemv_cpw<EPI, 2, PG_GEMV_D2, PRO, FRAG>(dim3((ntiles + 1) / 2, ksplit), lds, st, A, lda, W, ldw, K, ksplit, e);
  } else {
    launch_gemv_cpw<EPI, 1, PG_GEMV_D1, PRO, FRAG>(dim3(ntiles, ksplit), lds, st, A, lda, W, ldw, K, ksplit, e);
  }
}

template <int EPI, bool FRAG>
static void launch_gemv(const bf16_t* A, int lda, const bf16_t* W, int ldw, int K, int ksplit, const EpiArgs& e,
                        hipStream_t st) {
  if constexpr (EPI == PG_EPI_F32_ADD || EPI == PG_EPI_FX_ADD) {   // (plain x, or the attention merge: o / down)
    if (e.f.pro_mode == 2)
      launch_gemv_pro<EPI, 2, FRAG>(A, lda, W, ldw, K, ksplit, e, st);
    else
      launch_gemv_pro<EPI, 0, FRAG>(A, lda, W, ldw, K, ksplit, e, st);
    return;
  }
  switch (e.f.pro_mode) {
    case 1: launch_gemv_pro<EPI, 1, FRAG>(A, lda, W, ldw, K, ksplit, e, st); break;
    case 2: launch_gemv_pro<EPI, 2, FRAG>(A, lda, W, ldw, K, ksplit, e, st); break;
    case 3: launch_gemv_pro<EPI, 3, FRAG>(A, lda, W, ldw, K, ksplit, e, st); break;
    case 4: launch_gemv_pro<EPI, 4, FRAG>(A, lda, W, ldw, K, ksplit, e, st); break;
    default: launch_gemv_pro<EPI, 0, FRAG>(A, lda, W, ldw, K, ksplit, e, st); break;
  }
}

// M <= 16 -> weight-streaming GEMV, else the tile GEMM; FRAG (PG_W_FRAG) only for the Gemma epilogues
template <int EPI, bool FRAG>
static void launch_any(const bf16_t* A, int lda, const bf16_t* W, int ldw, int K, int ksplit, const EpiArgs& e,
                       hipStream_t st, bool m1 = false, bool n64 = false) {
  if (e.M <= 16)
    launch_gemv<EPI, FRAG>(A, lda, W, ldw, K, ksplit, e, st);
  else if constexpr (EPI != PG_EPI_F32_FIN && EPI != PG_EPI_F32_ADD && EPI != PG_EPI_FX_ADD)
    launch_tile<EPI, FRAG>(A, lda, W, ldw, K, ksplit, e, st, m1, n64);
}

static int gemm_impl(const void* A, int lda, const void* W, int ldw, const float* bias, void* C, int ldc,
                     int M, int N, int K, int epi_flags, int ksplit, const float* aux, int aux_rows, void* aux_out,
                     int aux_ld, int aux_n, const PgFusedArgs* fa, hipStream_t stream) {
  const bool frag = (epi_flags & PG_W_FRAG) != 0;
  const bool fp8 = (epi_flags & PG_FP8) != 0;
  const bool m1 = (epi_flags & PG_TILE_M1) != 0;
  const bool n64 = (epi_flags & PG_TILE_N64) != 0;
  const int epi = epi_flags & 0xFF;
  PG_REQUIRE((epi_flags & ~(0xFF | PG_W_FRAG | PG_FP8 | PG_TILE_M1 | PG_TILE_N64)) == 0);
  if (m1) PG_REQUIRE(!fp8 && !n64 && M >= 256 && M <= 288 && (fa == nullptr || fa->pro_mode == 0));
  if (n64) PG_REQUIRE(M > 16);
  PG_REQUIRE(M > 0 && N > 0 && K > 0 && ksplit >= 1);
  PG_REQUIRE(K % 32 == 0 && ldw >= K && (N % 4) == 0);
  if (frag && !fp8) PG_REQUIRE(N % 16 == 0 && K % 64 == 0 && ldw == K &&
                       (epi == PG_EPI_BF16 || epi == PG_EPI_BF16_GELU_MUL || epi == PG_EPI_F32 ||
                        epi == PG_EPI_QKV_ROPE || epi == PG_EPI_F32_FIN || epi == PG_EPI_F32_ADD ||
                        epi == PG_EPI_FX_ADD));
  PgFusedArgs f{};
  if (fa) f = *fa;
  EpiArgs e{bias, C, ldc, M, N, aux, aux_rows, (bf16_t*)aux_out, aux_ld, aux_n, f};
  PG_REQUIRE(f.pro_mode >= 0 && f.pro_mode <= 5);
  if (f.pro_mode == 5)
    PG_REQUIRE(fp8 && frag && epi == PG_EPI_F32 && M <= 32 && f.amax_in && f.amax_ld >= 1 && A != nullptr &&
               lda >= K && lda % 8 == 0 && ((uintptr_t)A & 15) == 0 && K % 128 == 0 && (K / 128) % ksplit == 0 &&
               (K / 128 / ksplit == 8 || K / 128 / ksplit == 16));
  if (f.amax_out) PG_REQUIRE(fp8 && frag && epi == PG_EPI_BF16_GELU_MUL && M <= 32 && f.amax_ld >= 1 &&
                             ((K >> 7) + ksplit - 1) / ksplit * 128 <= 4096 && PG_GEMV8_WIDE);
  if (f.amax_zero) PG_REQUIRE(fp8 && frag && f.amax_zero_n >= 0 && f.amax_zero_n <= 4096);
  if (f.pro_mode == 0 || f.pro_mode == 4) PG_REQUIRE(A != nullptr && lda >= K);
  // (M > 4 runs two 16-row tiles per workgroup: the per-row entries are loaded 16 per lane)
  if (f.pro_mode == 4) PG_REQUIRE(ksplit == 1 && f.ss_in && f.ss_n > 0 && f.ss_ld >= f.ss_n &&
                                  ((M <= 2 && f.ss_n <= 256 && (M == 1 || f.ss_n <= 128)) ||
                                   (M > 4 && M <= 16 && f.ss_n <= 64)));
  if (f.pro_mode != 0 && f.pro_mode != 5) PG_REQUIRE(M <= 16);
  if (f.pro_mode == 1) PG_REQUIRE(ksplit == 1 && f.resid_in && f.norm_w && (f.nsplit == 0 || f.partials) && K % 4 == 0);
  if (f.pro_mode == 2)
    PG_REQUIRE(f.part_o && f.part_ml && f.head_dim > 0 && (K / ksplit) % f.head_dim == 0 && f.asplit > 0 &&
               f.q_per_kv > 0 && f.kv_heads > 0);
  if (epi == PG_EPI_QKV_ROPE) PG_REQUIRE(f.head_dim % 16 == 0 && f.cos_t && f.sin_t && f.pos && f.kc && f.vtc &&
                                         f.rows_per_batch > 0 && f.smax > 0 && ksplit == 1 &&
                                         N == (f.q_heads + 2 * f.kv_heads) * f.head_dim);
  if (f.pro_mode == 3) PG_REQUIRE(ksplit == 1 && f.resid_in && f.norm_w && f.ss_in && f.ss_n > 0 &&
                                  f.ss_ld >= f.ss_n && K % 4 == 0);
  if (epi == PG_EPI_F32_FIN) PG_REQUIRE(M <= 16 && ksplit <= 8 && (f.fin_x == nullptr || f.norm_w != nullptr) && f.fin_cnt && f.fin_resid && f.ss_out && f.ss_ld >= (N + 15) / 16 &&
                                        ldc == N);
  if (epi == PG_EPI_F32_ADD) PG_REQUIRE((M <= 16 || (fp8 && frag && M <= 32)) && (f.pro_mode == 0 || f.pro_mode == 2) &&
                                        ldc >= N);
  if (epi == PG_EPI_FX_ADD) PG_REQUIRE(M <= 16 && !fp8 && (f.pro_mode == 0 || f.pro_mode == 2) && ldc >= N &&
                                       ((uintptr_t)C & 15) == 0 && ldc % 2 == 0);
  if (f.fx) PG_REQUIRE(((uintptr_t)f.fx & 15) == 0 && (f.pro_mode == 1) != (epi == PG_EPI_F32_FIN) && !fp8 &&
                       M <= 16);
  if (ksplit > 1) PG_REQUIRE(epi == PG_EPI_F32 || epi == PG_EPI_F32_FIN || epi == PG_EPI_F32_ADD || epi == PG_EPI_FX_ADD);
  if (epi == PG_EPI_BF16_GELU_MUL) PG_REQUIRE(N % 32 == 0);
  if (epi == PG_EPI_F32_POS) PG_REQUIRE(aux != nullptr && aux_rows > 0 && bias != nullptr);
  if (epi == PG_EPI_BF16_VT) PG_REQUIRE(aux_out != nullptr && aux_n % 4 == 0);
  if (M <= 16) PG_REQUIRE(K % 64 == 0);
  else PG_REQUIRE(K % TBK == 0 && (f.pro_mode == 0 || f.pro_mode == 5) && epi != PG_EPI_F32_FIN);
  const bf16_t* a = (const bf16_t*)A;
  const bf16_t* w = (const bf16_t*)W;
  if (fp8 && frag) {
    // fp8 weight-streaming GEMV (M <= 32): fp8 fragment-packed W (weights.frag_pack8), row-major e4m3 x
    PG_REQUIRE(M <= 32 && (f.pro_mode == 0 || f.pro_mode == 5) && (f.a_scale || f.pro_mode == 5) && f.w_scale &&
               K % 128 == 0 && N % 16 == 0 && ldw == K && lda >= K && (lda % 16 == 0 || f.pro_mode == 5) &&
               ((uintptr_t)A & 15) == 0 && ((uintptr_t)W & 15) == 0 && epi != PG_EPI_F32_FIN);
    const uint8_t* x8 = (const uint8_t*)A;
    const uint8_t* w8 = (const uint8_t*)W;
    switch (epi) {
      case PG_EPI_BF16: launch_gemv8<PG_EPI_BF16>(x8, lda, w8, K, ksplit, e, stream); break;
      case PG_EPI_BF16_GELU_MUL: launch_gemv8<PG_EPI_BF16_GELU_MUL>(x8, lda, w8, K, ksplit, e, stream); break;
      case PG_EPI_F32: launch_gemv8<PG_EPI_F32>(x8, lda, w8, K, ksplit, e, stream); break;
      case PG_EPI_QKV_ROPE: launch_gemv8<PG_EPI_QKV_ROPE>(x8, lda, w8, K, ksplit, e, stream); break;
      case PG_EPI_F32_ADD: launch_gemv8<PG_EPI_F32_ADD>(x8, lda, w8, K, ksplit, e, stream); break;
      default: return (int)hipErrorInvalidValue;
    }
    PG_LAUNCH_CHECK();
    return 0;
  }
  if (fp8) {
    // fp8 e4m3 operands, tile GEMMs only; the kernels see byte pairs, so K / lda / ldw are halved
    PG_REQUIRE(!frag && M > 16 && f.pro_mode == 0 && f.a_scale && f.w_scale && K % 128 == 0 && lda % 16 == 0 &&
               ldw % 16 == 0 && ((uintptr_t)A & 15) == 0 && ((uintptr_t)W & 15) == 0);
    switch (epi) {
      case PG_EPI_BF16: launch_tile<PG_EPI_BF16, false, true>(a, lda / 2, w, ldw / 2, K / 2, ksplit, e, stream, false, n64); break;
      case PG_EPI_BF16_GELU_MUL:
        launch_tile<PG_EPI_BF16_GELU_MUL, false, true>(a, lda / 2, w, ldw / 2, K / 2, ksplit, e, stream, false, n64);
        break;
      case PG_EPI_F32: launch_tile<PG_EPI_F32, false, true>(a, lda / 2, w, ldw / 2, K / 2, ksplit, e, stream, false, n64); break;
      case PG_EPI_QKV_ROPE:
        launch_tile<PG_EPI_QKV_ROPE, false, true>(a, lda / 2, w, ldw / 2, K / 2, ksplit, e, stream, false, n64);
        break;
      default: return (int)hipErrorInvalidValue;
    }
    PG_LAUNCH_CHECK();
    return 0;
  }
#define PG_CASE(E)                                                                             \
  case E:                                                                                      \
    if (frag) launch_any<E, true>(a, lda, w, ldw, K, ksplit, e, stream, m1, n64);              \
    else launch_any<E, false>(a, lda, w, ldw, K, ksplit, e, stream, m1, n64);                  \
    break;
#define PG_CASE_ROWMAJOR(E)                                                                    \
  case E: launch_any<E, false>(a, lda, w, ldw, K, ksplit, e, stream, m1, n64); break;
  switch (epi) {
    PG_CASE(PG_EPI_BF16)
    PG_CASE(PG_EPI_BF16_GELU_MUL)
    PG_CASE(PG_EPI_F32)
    PG_CASE(PG_EPI_QKV_ROPE)
    PG_CASE(PG_EPI_F32_FIN)
    PG_CASE(PG_EPI_F32_ADD)
    PG_CASE(PG_EPI_FX_ADD)
    PG_CASE_ROWMAJOR(PG_EPI_BF16_GELU)
    PG_CASE_ROWMAJOR(PG_EPI_F32_POS)
    PG_CASE_ROWMAJOR(PG_EPI_BF16_VT)
    default: return (int)hipErrorInvalidValue;
  }
#undef PG_CASE
#undef PG_CASE_ROWMAJOR
  PG_LAUNCH_CHECK();
  return 0;
}

extern "C" int pg_gemm(const void* A, int lda, const void* W, int ldw, const float* bias, void* C, int ldc,
                       int M, int N, int K, int epi, int ksplit, const float* aux, int aux_rows, void* aux_out,
                       int aux_ld, int aux_n, hipStream_t stream) {
  return gemm_impl(A, lda, W, ldw, bias, C, ldc, M, N, K, epi, ksplit, aux, aux_rows, aux_out, aux_ld, aux_n,
                   nullptr, stream);
}

// C = epilogue(sum_z part[z]) for a GEMM run as PG_EPI_F32 with ksplit slabs (bias was applied to slab 0)
extern "C" int pg_gemm_finalize(const float* part, int nsplit, void* C, int ldc, int M, int N, int epi,
                                void* aux_out, int aux_ld, int aux_n, const PgFusedArgs* fa, hipStream_t stream) {
  PG_REQUIRE(part != nullptr && nsplit >= 1 && M > 0 && N > 0 && N % 4 == 0);
  PgFusedArgs f{};
  if (fa) f = *fa;
  EpiArgs e{nullptr, C, ldc, M, N, nullptr, 0, (bf16_t*)aux_out, aux_ld, aux_n, f};
  const int NO = epi == PG_EPI_BF16_GELU_MUL ? N / 2 : N;
  const long items = (long)M * (NO / 4);
  const dim3 grid((unsigned)((items + 255) / 256));
  switch (epi) {
    case PG_EPI_F32: hipLaunchKernelGGL((gemm_finalize_kernel<PG_EPI_F32>), grid, dim3(256), 0, stream, part, nsplit, e); break;
    case PG_EPI_BF16: hipLaunchKernelGGL((gemm_finalize_kernel<PG_EPI_BF16>), grid, dim3(256), 0, stream, part, nsplit, e); break;
    case PG_EPI_BF16_GELU: hipLaunchKernelGGL((gemm_finalize_kernel<PG_EPI_BF16_GELU>), grid, dim3(256), 0, stream, part, nsplit, e); break;
    case PG_EPI_BF16_GELU_MUL:
      PG_REQUIRE(N % 32 == 0);
      hipLaunchKernelGGL((gemm_finalize_kernel<PG_EPI_BF16_GELU_MUL>), grid, dim3(256), 0, stream, part, nsplit, e); break;
    case PG_EPI_BF16_VT:
      PG_REQUIRE(aux_out != nullptr && aux_n % 4 == 0);
      hipLaunchKernelGGL((gemm_finalize_kernel<PG_EPI_BF16_VT>), grid, dim3(256), 0, stream, part, nsplit, e); break;
    case PG_EPI_QKV_ROPE:
      PG_REQUIRE(fa && f.head_dim % 16 == 0 && f.cos_t && f.sin_t && f.pos && f.kc && f.vtc && f.rows_per_batch > 0 &&
                 f.smax > 0 && N == (f.q_heads + 2 * f.kv_heads) * f.head_dim);
      hipLaunchKernelGGL((gemm_finalize_kernel<PG_EPI_QKV_ROPE>), grid, dim3(256), 0, stream, part, nsplit, e); break;
    default: return (int)hipErrorInvalidValue;
  }
  PG_LAUNCH_CHECK();
  return 0;
}

extern "C" int pg_gemm_fused(const void* A, int lda, const void* W, int ldw, const float* bias, void* C, int ldc,
                             int M, int N, int K, int epi, int ksplit, const PgFusedArgs* fused, hipStream_t stream) {
  return gemm_impl(A, lda, W, ldw, bias, C, ldc, M, N, K, epi, ksplit, nullptr, 0, nullptr, 0, 0, fused, stream);
}
