// Attention pieces of attn.hip (the prefill / decode attention kernels): arguments, guarded loads, and the
// one-wave split-KV decode block.
#pragma once
#include "common.h"

#ifndef PG_VT_PROBE
#define PG_VT_PROBE 0     // tuning probe only: 1 = V^T blocks read as contiguous 16 KB regions (wrong values)
#endif

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
};

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
  auto load_block = [&](int kb, int rowcap, u32x4 (&kfa)[KS], u32x4 (&kfb)[KS], u32x2 (&vr)[DT][2]) {
    const int ka = min(kb + c, rowcap - 1), kbk = min(kb + 16 + c, rowcap - 1);
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
#if PG_VT_PROBE
      // timing probe (wrong values): the block's V^T bytes read from one contiguous 16 KB region
      const bf16_t* vrow = vbase + (long)(kb / 32) * (32 * DP) + (long)(d < D ? d : D - 1) * 32 - kb;
#else
      const bf16_t* vrow = vbase + (long)(d < D ? d : D - 1) * a.vt_ds;
#endif
      vr[t][0] = *(const u32x2*)(vrow + kb + 4 * g);
      vr[t][1] = *(const u32x2*)(vrow + kb + 16 + 4 * g);
    }
  };
  // decode with a known cache capacity: the first block is in flight before the kv length is read.  FULL
  // (launched only with kcap > 0) loads it unconditionally -- a split past the cache reads the last block,
  // never used -- so no branch joins the loads (hipcc's wait bookkeeping stays exact)
  const bool pre = FULL || (a.kcap > 0 && kbeg < a.kcap);
  u32x4 kfa[KS], kfb[KS];
  u32x2 vr[DT][2];
  if (FULL) load_block(min(kbeg, a.kcap - 32), a.kcap, kfa, kfb, vr);
  else if (pre) load_block(kbeg, a.kcap, kfa, kfb, vr);
  const int Lkv = (FULL ? __builtin_amdgcn_readfirstlane(lkv_raw) : (a.lkv_dev ? *a.lkv_dev : 0)) + a.Lkv;
  const int kend = min(Lkv, kbeg + a.split_keys);
  // one 32-key block from the loaded registers: mask by the kv length, S^T, online softmax, P.V.  A block with
  // no valid key (a peeled first block past the kv length) leaves (o, m, l) = (0, -inf, 0) untouched.
  auto block = [&](int kb) {
    // every load of the block is issued before its first use (one memory round trip): the scheduler would
    // otherwise sink the V^T loads below the S^T MFMAs, behind the K loads' wait
    __builtin_amdgcn_sched_barrier(0);
    u32x4 vf[DT];
#pragma unroll
    for (int t = 0; t < DT; ++t) {
      const bool dok = 16 * t + c < D;
      const int k0 = kb + 4 * g, k1 = kb + 16 + 4 * g;
      const int n0 = dok ? kend - k0 : 0, n1 = dok ? kend - k1 : 0;   // valid keys among each run of 4
      const u32x2 v0 = vr[t][0], v1 = vr[t][1];
      vf[t] = u32x4{n0 >= 2 ? v0[0] : (n0 == 1 ? (v0[0] & 0xFFFFu) : 0u),
                    n0 >= 4 ? v0[1] : (n0 == 3 ? (v0[1] & 0xFFFFu) : 0u),
                    n1 >= 2 ? v1[0] : (n1 == 1 ? (v1[0] & 0xFFFFu) : 0u),
                    n1 >= 4 ? v1[1] : (n1 == 3 ? (v1[1] & 0xFFFFu) : 0u)};
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
      const int k0 = kb + 4 * g + j, k1 = kb + 16 + 4 * g + j;
      x[j] = k0 < kend ? sA[j] * a.scale_log2 : -INFINITY;
      x[4 + j] = k1 < kend ? sB[j] * a.scale_log2 : -INFINITY;
    }
    float bm = x[0];
#pragma unroll
    for (int j = 1; j < 8; ++j) bm = fmaxf(bm, x[j]);
    bm = fmaxf(bm, __shfl_xor(bm, 16, 64));
    bm = fmaxf(bm, __shfl_xor(bm, 32, 64));
    const float mn = fmaxf(m, bm);
    const bool none = mn == -INFINITY;          // every key of the block masked and nothing before it
    const float alpha = none ? 1.f : exp2f(m - mn);
    float rs = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) { x[j] = none ? 0.f : exp2f(x[j] - mn); rs += x[j]; }
    rs += __shfl_xor(rs, 16, 64);
    rs += __shfl_xor(rs, 32, 64);
    l = l * alpha + rs;
    m = mn;
#pragma unroll
    for (int t = 0; t < DT; ++t) o[t] *= alpha;
    u32x4 pw;
    pw[0] = pack_bf2(x[0], x[1]);
    pw[1] = pack_bf2(x[2], x[3]);
    pw[2] = pack_bf2(x[4], x[5]);
    pw[3] = pack_bf2(x[6], x[7]);
    const bf16x8 pf = __builtin_bit_cast(bf16x8, pw);
#pragma unroll
    for (int t = 0; t < DT; ++t) o[t] = mfma16(__builtin_bit_cast(bf16x8, vf[t]), pf, o[t]);
  };
  if constexpr (FULL) {
    // the prefetched first block runs unconditionally (straight-line from its loads: nothing for hipcc to sink
    // below a kv-length branch), later blocks of a multi-block split load as they go
    PG_STAMP(st1);
    block(kbeg);
    for (int kb = kbeg + 32; kb < kend; kb += 32) {
      load_block(kb, kend, kfa, kfb, vr);
      block(kb);
    }
  } else {
    for (int kb = kbeg; kb < kend; kb += 32) {
      if (!pre || kb != kbeg) load_block(kb, kend, kfa, kfb, vr);
      block(kb);
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
  u32x2 vr[DT][2];
  {
    const bf16_t* pa = kbase + (long)(kl + c) * a.k_rs;
    const bf16_t* pb = kbase + (long)(kl + 16 + c) * a.k_rs;
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      kfa[s] = *(const u32x4*)(pa + 32 * s + 8 * g);
      kfb[s] = *(const u32x4*)(pb + 32 * s + 8 * g);
    }
#pragma unroll
    for (int t = 0; t < DT; ++t) {
#if PG_VT_PROBE
      const bf16_t* vrow = vbase + (long)(kl / 32) * (32 * DP) + (long)(16 * t + c) * 32 - kl;
#else
      const bf16_t* vrow = vbase + (long)(16 * t + c) * a.vt_ds;
#endif
      vr[t][0] = *(const u32x2*)(vrow + kl + 4 * g);
      vr[t][1] = *(const u32x2*)(vrow + kl + 16 + 4 * g);
    }
  }
  // every load of the block is issued before its first use (one memory round trip)
  __builtin_amdgcn_sched_barrier(0);
  const int Lkv = __builtin_amdgcn_readfirstlane(lkv_raw) + a.Lkv;
  const int kend = min(Lkv, kb + 32);
  u32x4 vf[DT];
#pragma unroll
  for (int t = 0; t < DT; ++t) {
    const int n0 = kend - (kb + 4 * g), n1 = kend - (kb + 16 + 4 * g);   // valid keys among each run of 4
    const u32x2 v0 = vr[t][0], v1 = vr[t][1];
    vf[t] = u32x4{n0 >= 2 ? v0[0] : (n0 == 1 ? (v0[0] & 0xFFFFu) : 0u),
                  n0 >= 4 ? v0[1] : (n0 == 3 ? (v0[1] & 0xFFFFu) : 0u),
                  n1 >= 2 ? v1[0] : (n1 == 1 ? (v1[0] & 0xFFFFu) : 0u),
                  n1 >= 4 ? v1[1] : (n1 == 3 ? (v1[1] & 0xFFFFu) : 0u)};
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
    x[j] = kb + 4 * g + j < kend ? sA[j] * a.scale_log2 : -INFINITY;
    x[4 + j] = kb + 16 + 4 * g + j < kend ? sB[j] * a.scale_log2 : -INFINITY;
  }
  float bm = x[0];
#pragma unroll
  for (int j = 1; j < 8; ++j) bm = fmaxf(bm, x[j]);
  bm = fmaxf(bm, __shfl_xor(bm, 16, 64));
  bm = fmaxf(bm, __shfl_xor(bm, 32, 64));
  const bool none = bm == -INFINITY;            // every key of the block masked
  float rs = 0.f;
#pragma unroll
  for (int j = 0; j < 8; ++j) { x[j] = none ? 0.f : exp2f(x[j] - bm); rs += x[j]; }
  rs += __shfl_xor(rs, 16, 64);
  rs += __shfl_xor(rs, 32, 64);
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
