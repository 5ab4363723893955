// Attention pieces of attn.hip (the prefill / decode attention kernels): arguments, guarded loads, and the
// one-wave split-KV decode block.
#pragma once
#include "common.h"
#include <type_traits>


#ifndef PG_ATTN_STAMPS
#define PG_ATTN_STAMPS 0  // diagnostic variant only: per-wave s_memrealtime stamps of attn_decode_split (FULL)
#endif
#if PG_ATTN_STAMPS
__device__ unsigned long long pg_attn_stamp_buf[8192][4];
#define PG_STAMP(v) do { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); v = __builtin_amdgcn_s_memrealtime(); } while (0)
#else
#define PG_STAMP(v) do { } while (0)
#endif

struct AttnArgs {
  const bf16_t* q; long q_rs;
  bf16_t* o; long o_rs;
  const bf16_t* k; long k_bs, k_hs, k_rs;
  const bf16_t* vt; long vt_bs, vt_hs, vt_ds;
  const float* mask; long mask_bs, mask_rs;
  int Lq, Lkv, G, Hkv, D;
  const int* lkv_dev;      // if set: Lkv = *lkv_dev + Lkv
  float scale_log2;        // softmax scale * log2(e)
  int split_keys;          // split mode if > 0 (keys per wave)
  float* part_o;           // [B][Hkv][nsplit][16][DT*16]
  float* part_ml;          // [B][Hkv][nsplit][16][2]
  int kcap;                // decode: key rows readable per (b, kv head) in K and V^T (the static cache's Smax);
                           // > 0 lets a split issue its first block's loads before the kv length arrives
  int pf_splits;           // prefill key splits (> 1: attn_fa_kernel writes (O, m, l) partials to part_o / part_ml
                           // [B][Hkv][pf_splits][Lq*G][DT*16] / [..][2], merged by attn_pf_combine_kernel)
  const bf16_t* kd;        // decode-order cache copies [B][Hkv][kcap][D] (dec_koff / dec_voff): the kcap > 0 decode
  const bf16_t* vd;        // kernels read K and V only from these
};

// Decode-order copies of the static KV cache (ABI 6).  The QKV epilogue writes every appended k / v twice: to the
// canonical K [.][Smax][D] / V^T [.][D][Smax] (prefill attention, the reference KVCache views) and to these copies,
// laid out so that every load instruction of a decode split reads one contiguous KiB (scripts/tune/kv_pattern.hip:
// the cache read of pt-896 x32, 30.5 us per layer as 16 rows x 64 B per instruction, 22.8 us as 1 KB).  Per 32-key
// block, 16 KB each (D = 256):
//   K: [half h][D/8 chunks][16 MFMA rows][8 dims]; row r of half h is key 8(r/4) + 4h + r%4 (dec_krow's order), so
//      the (half, k-step s) fragment -- chunks 4s..4s+3 of 16 rows -- is 1 KB;
//   V: [D/16 d-tiles][4 key groups g][16 dims][8 keys 8g..8g+7], so the d-tile t fragment of V^T is 1 KB.
static __device__ __forceinline__ long dec_koff(int k, int d, int D) {
  const int blk = k >> 5, kk = k & 31, h = (kk >> 2) & 1, r = ((kk >> 3) << 2) | (kk & 3);
  return ((((long)blk * 2 + h) * (D >> 3) + (d >> 3)) * 16 + r) * 8 + (d & 7);
}
static __device__ __forceinline__ long dec_voff(int k, int d, int D) {
  const int blk = k >> 5, kk = k & 31;
  return ((((long)blk * (D >> 4) + (d >> 4)) * 4 + (kk >> 3)) * 16 + (d & 15)) * 8 + (kk & 7);
}
// a lane's 16-B fragment pieces: K half h, k-step s of block kl (lane (c, g): chunk 4s + g of MFMA row c), and the
// V^T d-tile t of block kl (lane (c, g): keys 8g..8g+7 of dim 16t + c)
static __device__ __forceinline__ long dec_kfrag(int kl, int h, int s, int c, int g, int D) {
  return ((((long)(kl >> 5) * 2 + h) * (D >> 3) + 4 * s + g) * 16 + c) * 8;
}
static __device__ __forceinline__ long dec_vfrag(int kl, int t, int c, int g, int D) {
  return ((((long)(kl >> 5) * (D >> 4) + t) * 4 + g) * 16 + c) * 8;
}

// Branch-free guarded loads: the address is always valid (callers clamp it), the value is
// zeroed by selects.  Conditional loads compiled to branches and, for partial blocks, to
// serialised per-element loads + vmcnt(0) waits (profiles/r01: decode attention 16 us -> fixed).
static __device__ __forceinline__ u32x4 ld16_sel(const bf16_t* p, bool ok) {
  const u32x4 v = *(const u32x4*)p;
  return u32x4{ok ? v[0] : 0u, ok ? v[1] : 0u, ok ? v[2] : 0u, ok ? v[3] : 0u};
}

// 4 consecutive keys of one Vt row (row padded so key+3 stays inside), zero beyond kend / invalid d
static __device__ __forceinline__ u32x2 ld_vt4(const bf16_t* row, int key, int kend, bool dok) {
  const u32x2 v = *(const u32x2*)(row + key);
  const int nv = dok ? kend - key : 0;   // number of valid keys among the 4
  const uint32_t lo = nv >= 2 ? v[0] : (nv == 1 ? (v[0] & 0xFFFFu) : 0u);
  const uint32_t hi = nv >= 4 ? v[1] : (nv == 3 ? (v[1] & 0xFFFFu) : 0u);
  return u32x2{lo, hi};
}

// Split-KV decode key order inside a 32-key block: MFMA row i of the first S^T half is key 8(i/4) + i%4, of the
// second 8(i/4) + 4 + i%4, so lane (c, g) ends up holding the scores of keys 8g..8g+7 -- P^T is 8 consecutive keys
// per lane and each V^T row is read as one 16-B chunk (keys 8g..8g+7) instead of two 8-B pieces: a load instruction
// covers 16 rows x 64 B of V^T, not 16 x 32 B (scripts/tune/kv_pattern.hip, pt-896 x32 decode shapes: the cache read
// alone 42.6 -> 30.5 us per layer).  The K rows are loaded in that order (any row order is free for K).
static __device__ __forceinline__ int dec_krow(int c) { return 8 * (c >> 2) + (c & 3); }

// a V^T chunk of 8 consecutive keys with the keys from the n-th on zeroed (n = valid keys in the chunk)
static __device__ __forceinline__ u32x4 vmask8(u32x4 v, int n) {
  return u32x4{n >= 2 ? v[0] : (n == 1 ? (v[0] & 0xFFFFu) : 0u), n >= 4 ? v[1] : (n == 3 ? (v[1] & 0xFFFFu) : 0u),
               n >= 6 ? v[2] : (n == 5 ? (v[2] & 0xFFFFu) : 0u), n >= 8 ? v[3] : (n == 7 ? (v[3] & 0xFFFFu) : 0u)};
}

typedef __attribute__((address_space(1))) unsigned long long pg_gu64;

// 16 bytes as two write-through (sc1) 8-B stores: visible to another CU's sc1 loads once the storing wave
// has drained vmcnt (MI355X guide, inter-workgroup hand-off without a release fence)
static __device__ __forceinline__ void st16_wt(float* p, f32x4 v) {
  pg_gu64* d = (pg_gu64*)p;
  __hip_atomic_store(d, __builtin_bit_cast(unsigned long long, f32x2{v[0], v[1]}), __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(d + 1, __builtin_bit_cast(unsigned long long, f32x2{v[2], v[3]}), __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
}
static __device__ __forceinline__ f32x4 ld16_wt(const float* p) {
  const pg_gu64* s = (const pg_gu64*)p;
  const f32x2 a = __builtin_bit_cast(f32x2, __hip_atomic_load(s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
  const f32x2 b = __builtin_bit_cast(f32x2, __hip_atomic_load(s + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
  return f32x4{a[0], a[1], b[0], b[1]};
}
static __device__ __forceinline__ f32x2 ld8_wt(const float* p) {
  return __builtin_bit_cast(f32x2, __hip_atomic_load((const pg_gu64*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}

// One decode split, one wave: keys [sp*split_keys, min(Lkv, (sp+1)*split_keys)) of kv head kvh, batch b, for
// the q rows r < Lq*G (Lq == 1: row r = q head kvh*G + r), written as (O, m, l) partials of split sp of nsplit.
// S^T = K.Q^T keeps each row's softmax statistics lane-local; O^T = V^T.P^T takes P from the S accumulators
// (key order permuted identically for V^T).  WT: write-through stores for a consumer inside the same launch.
// FULL (head_dim == DP): no lane-dependent selects on loaded values -- rows past Lq*G read row Lq*G-1 (never
// stored) -- so hipcc has no reason to wait for a load before the next one is issued, and the kv length is
// read with a vector load (in order with the stream; a scalar load's lgkmcnt wait lands before the first
// vector load, behind the kernel-argument loads).
template <int DP, int DT, bool WT, bool FULL = false>
__device__ __forceinline__ void attn_decode_split(const AttnArgs& a, int b, int kvh, int sp, int nsplit, int lane) {
  constexpr int KS = DP / 32;
  const int c = lane & 15, g = lane >> 4;
  const int R = a.Lq * a.G;
  const int D = FULL ? DP : a.D;
  const int kbeg = sp * a.split_keys;
  unsigned long long st0 = 0, st1 = 0, st2 = 0, st3 = 0;
  (void)st0; (void)st1; (void)st2; (void)st3;
#if PG_ATTN_STAMPS
  st0 = __builtin_amdgcn_s_memrealtime();
#endif
  const int r = c;
  const bool rvalid = r < R;
  const int rr = rvalid ? r : (FULL ? R - 1 : 0);
  const int pos = rr / a.G;
  const int hq = kvh * a.G + rr % a.G;
  int lkv_raw = 0;
  if constexpr (FULL)
    lkv_raw = __hip_atomic_load(a.lkv_dev ? a.lkv_dev : &pg_zero_word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);

  bf16x8 qf[KS];
  const bf16_t* qp = a.q + ((long)b * a.Lq + pos) * a.q_rs + (long)hq * D;
#pragma unroll
  for (int s = 0; s < KS; ++s) {
    const int d0 = 32 * s + 8 * g;
    if constexpr (FULL)
      qf[s] = __builtin_bit_cast(bf16x8, *(const u32x4*)(qp + d0));
    else
      qf[s] = __builtin_bit_cast(bf16x8, ld16_sel(qp + (d0 < D ? d0 : 0), rvalid && d0 < D));
  }
  const bf16_t* kbase = a.k + (long)b * a.k_bs + (long)kvh * a.k_hs;
  const bf16_t* vbase = a.vt + (long)b * a.vt_bs + (long)kvh * a.vt_hs;
  f32x4 o[DT];
#pragma unroll
  for (int t = 0; t < DT; ++t) o[t] = f32x4{0.f, 0.f, 0.f, 0.f};
  float m = -INFINITY, l = 0.f;
  // raw loads of one 32-key block: K rows for S^T (rows clamped below rowcap), 4-key runs of the V^T rows
  // (row padded to a multiple of 32 keys); masking by the kv length is applied after the loads land
  const bf16_t* kdb = FULL ? a.kd + ((long)b * a.Hkv + kvh) * a.kcap * DP : nullptr;
  const bf16_t* vdb = FULL ? a.vd + ((long)b * a.Hkv + kvh) * a.kcap * DP : nullptr;
  auto load_block = [&](int kb, int rowcap, u32x4 (&kfa)[KS], u32x4 (&kfb)[KS], u32x4 (&vr)[DT]) {
    if constexpr (FULL) {     // decode-order copies: one contiguous KiB per load instruction (block kb < kcap)
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        kfa[s] = *(const u32x4*)(kdb + dec_kfrag(kb, 0, s, c, g, DP));
        kfb[s] = *(const u32x4*)(kdb + dec_kfrag(kb, 1, s, c, g, DP));
      }
#pragma unroll
      for (int t = 0; t < DT; ++t) vr[t] = *(const u32x4*)(vdb + dec_vfrag(kb, t, c, g, DP));
      return;
    }
    const int ka = min(kb + dec_krow(c), rowcap - 1), kbk = min(kb + dec_krow(c) + 4, rowcap - 1);
    const bf16_t* pa = kbase + (long)ka * a.k_rs;
    const bf16_t* pb = kbase + (long)kbk * a.k_rs;
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      const int d0 = 32 * s + 8 * g;
      if constexpr (FULL) {
        kfa[s] = *(const u32x4*)(pa + d0);
        kfb[s] = *(const u32x4*)(pb + d0);
      } else {
        kfa[s] = ld16_sel(pa + (d0 < D ? d0 : 0), d0 < D);
        kfb[s] = ld16_sel(pb + (d0 < D ? d0 : 0), d0 < D);
      }
    }
#pragma unroll
    for (int t = 0; t < DT; ++t) {
      const int d = 16 * t + c;
      const bf16_t* vrow = vbase + (long)(d < D ? d : D - 1) * a.vt_ds;
      vr[t] = *(const u32x4*)(vrow + kb + 8 * g);
    }
  };
  // decode with a known cache capacity: the first block is in flight before the kv length is read.  FULL
  // (launched only with kcap > 0) loads it unconditionally -- a split past the cache reads the last block,
  // never used -- so no branch joins the loads (hipcc's wait bookkeeping stays exact)
  const bool pre = FULL || (a.kcap > 0 && kbeg < a.kcap);
  u32x4 kfa[KS], kfb[KS];
  u32x4 vr[DT];
  if (FULL) load_block(min(kbeg, a.kcap - 32), a.kcap, kfa, kfb, vr);
  else if (pre) load_block(kbeg, a.kcap, kfa, kfb, vr);
  const int Lkv = (FULL ? __builtin_amdgcn_readfirstlane(lkv_raw) : (a.lkv_dev ? *a.lkv_dev : 0)) + a.Lkv;
  const int kend = min(Lkv, kbeg + a.split_keys);
  // one 32-key block from the loaded registers: mask by the kv length, S^T, online softmax, P.V.  A block with
  // no valid key (a peeled first block past the kv length) leaves (o, m, l) = (0, -inf, 0) untouched.
  // first = the split's first block: (o, m, l) are still (0, -inf, 0), so O needs no rescale (64 multiplies of
  // accumulator registers skipped: a one-block split -- batch-1 decode -- never rescales)
  auto block = [&](int kb, auto first) {
    // every load of the block is issued before its first use (one memory round trip): the scheduler would
    // otherwise sink the V^T loads below the S^T MFMAs, behind the K loads' wait
    __builtin_amdgcn_sched_barrier(0);
    u32x4 vf[DT];
#pragma unroll
    for (int t = 0; t < DT; ++t) {
      const bool dok = 16 * t + c < D;
      vf[t] = vmask8(vr[t], dok ? kend - (kb + 8 * g) : 0);   // keys 8g..8g+7 of the block
    }
    f32x4 sA = {0.f, 0.f, 0.f, 0.f}, sB = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      sA = mfma16(__builtin_bit_cast(bf16x8, kfa[s]), qf[s], sA);
      sB = mfma16(__builtin_bit_cast(bf16x8, kfb[s]), qf[s], sB);
    }
    float x[8];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      x[j] = kb + 8 * g + j < kend ? sA[j] * a.scale_log2 : -INFINITY;
      x[4 + j] = kb + 8 * g + 4 + j < kend ? sB[j] * a.scale_log2 : -INFINITY;
    }
    float bm = x[0];
#pragma unroll
    for (int j = 1; j < 8; ++j) bm = fmaxf(bm, x[j]);
    bm = max_xor16(bm);
    bm = max_xor32(bm);
    const float mn = fmaxf(m, bm);
    const bool none = mn == -INFINITY;          // every key of the block masked and nothing before it
    const float alpha = none ? 1.f : exp2f(m - mn);
    float rs = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) { x[j] = none ? 0.f : exp2f(x[j] - mn); rs += x[j]; }
    rs = sum_xor16(rs);
    rs = sum_xor32(rs);
    m = mn;
    if constexpr (decltype(first)::value) {
      l = rs;
    } else {
      l = l * alpha + rs;
#pragma unroll
      for (int t = 0; t < DT; ++t) o[t] *= alpha;
    }
    u32x4 pw;
    pw[0] = pack_bf2(x[0], x[1]);
    pw[1] = pack_bf2(x[2], x[3]);
    pw[2] = pack_bf2(x[4], x[5]);
    pw[3] = pack_bf2(x[6], x[7]);
    const bf16x8 pf = __builtin_bit_cast(bf16x8, pw);
#pragma unroll
    for (int t = 0; t < DT; ++t) o[t] = mfma16(__builtin_bit_cast(bf16x8, vf[t]), pf, o[t]);
  };
  using first_t = std::integral_constant<bool, true>;
  using later_t = std::integral_constant<bool, false>;
  if constexpr (FULL) {
    // the prefetched first block runs unconditionally (straight-line from its loads: nothing for hipcc to sink
    // below a kv-length branch), later blocks of a multi-block split load as they go
    PG_STAMP(st1);
    block(kbeg, first_t{});
    for (int kb = kbeg + 32; kb < kend; kb += 32) {
      load_block(kb, kend, kfa, kfb, vr);
      block(kb, later_t{});
    }
  } else {
    for (int kb = kbeg; kb < kend; kb += 32) {
      if (!pre || kb != kbeg) load_block(kb, kend, kfa, kfb, vr);
      block(kb, later_t{});
    }
  }
  // lane holds O^T[d = 16t + 4g + j][q = c]
  const long base = (((long)b * a.Hkv + kvh) * nsplit + sp) * 16 + c;
#if PG_ATTN_STAMPS
  asm volatile("" :: "v"(o[0][0]), "v"(o[DT - 1][3]));
  st2 = __builtin_amdgcn_s_memrealtime();
#endif
  if (!rvalid) return;                       // rows past Lq*G are never merged
  float* po = a.part_o + base * (DT * 16);
#pragma unroll
  for (int t = 0; t < DT; ++t) {
    if (WT) st16_wt(po + 16 * t + 4 * g, o[t]);
    else *(f32x4*)(po + 16 * t + 4 * g) = o[t];
  }
  if (g == 0) {
    if (WT) {
      __hip_atomic_store((pg_gu64*)(a.part_ml + base * 2), __builtin_bit_cast(unsigned long long, f32x2{m, l}),
                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      a.part_ml[base * 2 + 0] = m;
      a.part_ml[base * 2 + 1] = l;
    }
  }
#if PG_ATTN_STAMPS
  PG_STAMP(st3);
  if (lane == 0) {
    const int id = (b * a.Hkv + kvh) * nsplit + sp;
    if (id < 8192) {
      pg_attn_stamp_buf[id][0] = st0; pg_attn_stamp_buf[id][1] = st1;
      pg_attn_stamp_buf[id][2] = st2; pg_attn_stamp_buf[id][3] = st3;
    }
  }
#endif
}

// One 32-key block [kb, kb + 32) of a decode split, one wave, head_dim == DP, known cache capacity (a.kcap >= 32):
// the block's K rows and V^T runs are issued before the kv length is read (rows past it masked after they land),
// exactly as attn_decode_split's FULL first block, and its (O^T, m, l) are returned in registers (lane holds
// O^T[d = 16t + 4g + j][q = c]; m, l of row c) for a caller that merges several blocks (attn_decode_wg_kernel).
template <int DP, int DT>
__device__ __forceinline__ void attn_decode_block32(const AttnArgs& a, int b, int kvh, int kb, int lane,
                                                    f32x4 (&o)[DT], float& m, float& l) {
  constexpr int KS = DP / 32;
  const int c = lane & 15, g = lane >> 4;
  const int R = a.Lq * a.G;
  const int rr = c < R ? c : R - 1;              // rows past Lq*G read row R - 1 (never stored): no select
  const int pos = rr / a.G;
  const int hq = kvh * a.G + rr % a.G;
  const int lkv_raw =
      __hip_atomic_load(a.lkv_dev ? a.lkv_dev : &pg_zero_word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  bf16x8 qf[KS];
  const bf16_t* qp = a.q + ((long)b * a.Lq + pos) * a.q_rs + (long)hq * DP;
#pragma unroll
  for (int s = 0; s < KS; ++s) qf[s] = __builtin_bit_cast(bf16x8, *(const u32x4*)(qp + 32 * s + 8 * g));
  const bf16_t* kbase = a.k + (long)b * a.k_bs + (long)kvh * a.k_hs;
  const bf16_t* vbase = a.vt + (long)b * a.vt_bs + (long)kvh * a.vt_hs;
  // a block past the cache reads the last block (never used: all its keys are masked)
  const int kl = min(kb, a.kcap - 32);
  u32x4 kfa[KS], kfb[KS];
  u32x4 vr[DT];
  {
    (void)kbase;
    (void)vbase;
    const bf16_t* kdb = a.kd + ((long)b * a.Hkv + kvh) * a.kcap * DP;
    const bf16_t* vdb = a.vd + ((long)b * a.Hkv + kvh) * a.kcap * DP;
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      kfa[s] = *(const u32x4*)(kdb + dec_kfrag(kl, 0, s, c, g, DP));
      kfb[s] = *(const u32x4*)(kdb + dec_kfrag(kl, 1, s, c, g, DP));
    }
#pragma unroll
    for (int t = 0; t < DT; ++t) vr[t] = *(const u32x4*)(vdb + dec_vfrag(kl, t, c, g, DP));
  }
  // every load of the block is issued before its first use (one memory round trip)
  __builtin_amdgcn_sched_barrier(0);
  const int Lkv = __builtin_amdgcn_readfirstlane(lkv_raw) + a.Lkv;
  const int kend = min(Lkv, kb + 32);
  u32x4 vf[DT];
#pragma unroll
  for (int t = 0; t < DT; ++t) vf[t] = vmask8(vr[t], kend - (kb + 8 * g));   // keys 8g..8g+7
  f32x4 sA = {0.f, 0.f, 0.f, 0.f}, sB = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int s = 0; s < KS; ++s) {
    sA = mfma16(__builtin_bit_cast(bf16x8, kfa[s]), qf[s], sA);
    sB = mfma16(__builtin_bit_cast(bf16x8, kfb[s]), qf[s], sB);
  }
  float x[8];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    x[j] = kb + 8 * g + j < kend ? sA[j] * a.scale_log2 : -INFINITY;
    x[4 + j] = kb + 8 * g + 4 + j < kend ? sB[j] * a.scale_log2 : -INFINITY;
  }
  float bm = x[0];
#pragma unroll
  for (int j = 1; j < 8; ++j) bm = fmaxf(bm, x[j]);
  bm = max_xor16(bm);
  bm = max_xor32(bm);
  const bool none = bm == -INFINITY;            // every key of the block masked
  float rs = 0.f;
#pragma unroll
  for (int j = 0; j < 8; ++j) { x[j] = none ? 0.f : exp2f(x[j] - bm); rs += x[j]; }
  rs = sum_xor16(rs);
  rs = sum_xor32(rs);
  m = bm;
  l = rs;
  u32x4 pw;
  pw[0] = pack_bf2(x[0], x[1]);
  pw[1] = pack_bf2(x[2], x[3]);
  pw[2] = pack_bf2(x[4], x[5]);
  pw[3] = pack_bf2(x[6], x[7]);
  const bf16x8 pf = __builtin_bit_cast(bf16x8, pw);
#pragma unroll
  for (int t = 0; t < DT; ++t) o[t] = mfma16(__builtin_bit_cast(bf16x8, vf[t]), pf, f32x4{0.f, 0.f, 0.f, 0.f});
}

// ---- batched decode (attn_decode_fused_kernel): one 32-key block's loads, and its online-softmax update ----

// K and V^T fragments of the 32-key block at kb from the decode-order copies of one (row, kv head) (kbase / vbase:
// a.kd / a.vd at that head), the block clamped below the cache capacity: a block past the kv length is read anyway
// (the last cache block at worst) and masked after its loads land, so the loads of a round are unconditional and
// hipcc's wait counting stays exact (head_dim == DP).
template <int DP, int DT>
__device__ __forceinline__ void dec_load_block(const AttnArgs& a, const bf16_t* kbase, const bf16_t* vbase, int kb,
                                               int c, int g, u32x4 (&kfa)[DP / 32], u32x4 (&kfb)[DP / 32],
                                               u32x4 (&vr)[DT]) {
  const int kl = min(kb, a.kcap - 32);
#pragma unroll
  for (int s = 0; s < DP / 32; ++s) {
    kfa[s] = *(const u32x4*)(kbase + dec_kfrag(kl, 0, s, c, g, DP));
    kfb[s] = *(const u32x4*)(kbase + dec_kfrag(kl, 1, s, c, g, DP));
  }
#pragma unroll
  for (int t = 0; t < DT; ++t) vr[t] = *(const u32x4*)(vbase + dec_vfrag(kl, t, c, g, DP));
}

// (o, m, l) <- the online-softmax update with the loaded block [kb, kb + 32), keys >= kend masked (the arithmetic of
// attn_decode_split's block).  S^T = K.Q^T keeps a row's statistics lane-local; P feeds O^T = V^T.P^T from the S
// accumulators, the key order inside the k-step permuted identically for V^T (lane holds keys 4g.., 16 + 4g..).
// MASK_V = false: V^T past kend is not zeroed (P is 0 there already): only for caches that hold finite values in every
// row (the engine's zero-initialised static cache, written only with model outputs) -- saves 64 registers.
// mid() runs once the scores are computed (the K registers are free: the staggered caller issues the next K there).
struct DecNoMid {
  __device__ void operator()() const {}
};
template <int DP, int DT, bool MASK_V = true, bool FIRST = false, typename Mid = DecNoMid>
__device__ __forceinline__ void dec_block_update(float scale_log2, int kb, int kend, int c, int g,
                                                 const bf16x8 (&qf)[DP / 32], const u32x4 (&kfa)[DP / 32],
                                                 const u32x4 (&kfb)[DP / 32], const u32x4 (&vr)[DT],
                                                 f32x4 (&o)[DT], float& m, float& l, Mid mid = Mid()) {
  (void)c;
  u32x4 vf[DT];
#pragma unroll
  for (int t = 0; t < DT; ++t) {
    if constexpr (MASK_V)
      vf[t] = vmask8(vr[t], kend - (kb + 8 * g));   // keys 8g..8g+7
    else
      vf[t] = vr[t];
  }
  f32x4 sA = {0.f, 0.f, 0.f, 0.f}, sB = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int s = 0; s < DP / 32; ++s) {
    sA = mfma16(__builtin_bit_cast(bf16x8, kfa[s]), qf[s], sA);
    sB = mfma16(__builtin_bit_cast(bf16x8, kfb[s]), qf[s], sB);
  }
  mid();
  float x[8];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    x[j] = kb + 8 * g + j < kend ? sA[j] * scale_log2 : -INFINITY;
    x[4 + j] = kb + 8 * g + 4 + j < kend ? sB[j] * scale_log2 : -INFINITY;
  }
  float bm = x[0];
#pragma unroll
  for (int j = 1; j < 8; ++j) bm = fmaxf(bm, x[j]);
  bm = max_xor16(bm);
  bm = max_xor32(bm);
  const float mn = fmaxf(m, bm);
  const bool none = mn == -INFINITY;          // every key so far masked
  const float alpha = none ? 1.f : exp2f(m - mn);
  float rs = 0.f;
#pragma unroll
  for (int j = 0; j < 8; ++j) { x[j] = none ? 0.f : exp2f(x[j] - mn); rs += x[j]; }
  rs = sum_xor16(rs);
  rs = sum_xor32(rs);
  m = mn;
  if constexpr (FIRST) {                        // (o, m, l) = (0, -inf, 0): nothing to rescale
    l = rs;
  } else {
    l = l * alpha + rs;
#pragma unroll
    for (int t = 0; t < DT; ++t) o[t] *= alpha;
  }
  u32x4 pw;
  pw[0] = pack_bf2(x[0], x[1]);
  pw[1] = pack_bf2(x[2], x[3]);
  pw[2] = pack_bf2(x[4], x[5]);
  pw[3] = pack_bf2(x[6], x[7]);
  const bf16x8 pf = __builtin_bit_cast(bf16x8, pw);
#pragma unroll
  for (int t = 0; t < DT; ++t) o[t] = mfma16(__builtin_bit_cast(bf16x8, vf[t]), pf, o[t]);
}

// 16-byte write-through (sc1) store / load through a buffer resource (MI355X guide: in-launch hand-off, R1 form)
static __device__ __forceinline__ __amdgpu_buffer_rsrc_t pg_rsrc(const void* base) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, 0x7fffffff, 0x00020000);
}
static __device__ __forceinline__ void st16_sc1(__amdgpu_buffer_rsrc_t r, int byte_off, f32x4 v) {
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), r, byte_off, 0, 16);
}
static __device__ __forceinline__ f32x4 ld16_sc1(__amdgpu_buffer_rsrc_t r, int byte_off) {
  return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, byte_off, 0, 16));
}
