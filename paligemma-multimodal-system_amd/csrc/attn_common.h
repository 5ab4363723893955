// Attention pieces shared by attn.hip (the attention kernels) and gemm.hip (the decode o_proj GEMV that
// computes the split-KV attention in-kernel, pg_attn_oproj).
#pragma once
#include "common.h"

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
template <int DP, int DT, bool WT>
__device__ __forceinline__ void attn_decode_split(const AttnArgs& a, int b, int kvh, int sp, int nsplit, int lane) {
  constexpr int KS = DP / 32;
  const int c = lane & 15, g = lane >> 4;
  const int Lkv = (a.lkv_dev ? *a.lkv_dev : 0) + a.Lkv;
  const int R = a.Lq * a.G;
  const int D = a.D;
  const int kbeg = sp * a.split_keys;
  const int kend = min(Lkv, kbeg + a.split_keys);
  const int r = c;
  const bool rvalid = r < R;
  const int pos = rvalid ? r / a.G : 0;
  const int hq = kvh * a.G + (rvalid ? r % a.G : 0);

  bf16x8 qf[KS];
  {
    const bf16_t* qp = a.q + ((long)b * a.Lq + pos) * a.q_rs + (long)hq * D;
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      const int d0 = 32 * s + 8 * g;
      qf[s] = __builtin_bit_cast(bf16x8, ld16_sel(qp + (d0 < D ? d0 : 0), rvalid && d0 < D));
    }
  }
  const bf16_t* kbase = a.k + (long)b * a.k_bs + (long)kvh * a.k_hs;
  const bf16_t* vbase = a.vt + (long)b * a.vt_bs + (long)kvh * a.vt_hs;
  f32x4 o[DT];
#pragma unroll
  for (int t = 0; t < DT; ++t) o[t] = f32x4{0.f, 0.f, 0.f, 0.f};
  float m = -INFINITY, l = 0.f;
  for (int kb = kbeg; kb < kend; kb += 32) {
    // every load of the block first (K rows for S^T, V^T rows for P.V): one memory round trip
    const int ka = min(kb + c, kend - 1), kbk = min(kb + 16 + c, kend - 1);
    u32x4 kfa[KS], kfb[KS];
    {
      const bf16_t* pa = kbase + (long)ka * a.k_rs;
      const bf16_t* pb = kbase + (long)kbk * a.k_rs;
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        const int d0 = 32 * s + 8 * g;
        kfa[s] = ld16_sel(pa + (d0 < D ? d0 : 0), d0 < D);
        kfb[s] = ld16_sel(pb + (d0 < D ? d0 : 0), d0 < D);
      }
    }
    u32x4 vf[DT];
#pragma unroll
    for (int t = 0; t < DT; ++t) {
      const int d = 16 * t + c;
      const bool dok = d < D;
      const bf16_t* vrow = vbase + (long)(dok ? d : D - 1) * a.vt_ds;
      const u32x2 v0 = ld_vt4(vrow, kb + 4 * g, kend, dok);
      const u32x2 v1 = ld_vt4(vrow, kb + 16 + 4 * g, kend, dok);
      vf[t] = u32x4{v0[0], v0[1], v1[0], v1[1]};
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
    const float alpha = exp2f(m - mn);
    float rs = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) { x[j] = exp2f(x[j] - mn); rs += x[j]; }
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
  }
  // lane holds O^T[d = 16t + 4g + j][q = c]
  const long base = (((long)b * a.Hkv + kvh) * nsplit + sp) * 16 + c;
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
}
