// bf16 decode GEMV (M <= 16): gemv_kernel and its launchers (see gemm_common.h).
#include "gemm_common.h"

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
#ifndef PG_GEMV_QKV_NT1
#define PG_GEMV_QKV_NT1 1   // batched (M > 4) q|k|v GEMV with one 16-row tile per workgroup
#endif
#ifndef PG_GEMV_D2
#define PG_GEMV_D2 4
#endif
// (round 5: the gate/up GEMV at batch 1 with two gate/up pairs per workgroup -- half the workgroups re-reading the row
// -- measured slower, 1.061 vs 1.059 ms/token at 3 chunks in flight, 1.073 at 2: profiles/r05_gateup_nt4_ab.jsonl)
#ifndef PG_GEMV_LM_NT
#define PG_GEMV_LM_NT 2   // the batch-1..4 lm_head GEMV with two 16-row tiles per workgroup (1: one; 2 with 6 chunks in
                          // flight: -5.5 us per token, 4 chunks: -3.5, profiles/r05_lm_head_nt2_ab.jsonl)
#endif
#ifndef PG_GEMV_LM_D
#define PG_GEMV_LM_D 6    // ... and that form's chunks in flight
#endif
#ifndef PG_GEMV_FIN_NT
#define PG_GEMV_FIN_NT 2  // (tuning) 16-column tiles per workgroup of the finalised batched (M > 4) GEMV: 2 or 4
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

#ifndef PG_GEMV_PRO_EARLY
#define PG_GEMV_PRO_EARLY 2     // 2: the q|k|v GEMV at M == 1; 1: gate/up too (152 VGPRs: 3 waves/SIMD, level); 0: off
                                // (measured and removed: the same loads as LDS DMA, slower; the o_proj merge prologue's
                                // partials loaded early, level -- profiles/r05_decode_early_prologue_ab.jsonl)
#endif
// A workgroup barrier that orders LDS only: the wave's LDS ops are waited for, its global loads (the weight ring) stay
// in flight (__syncthreads' fence would wait for them too: s_waitcnt vmcnt(0))
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
}
// The batch-1 RMSNorm prologue in two halves (PRO 1, M == 1, K <= 2048): the loads -- thread t owns the float4s
// c = t and t + 256 of the row, the residual's and the norm weight's, the fixed-point accumulator's raw words --
// and, after the weight ring is issued, the sum of squares, the normalisation and the LDS image.
struct Pro1Row {
  f32x4 a[2], w[2];
  i64x2 qa[2], qb[2];
};
__device__ __forceinline__ void pro1_row_load(const PgFusedArgs& f, int K, Pro1Row& p) {
  const int t = threadIdx.x, K4 = K >> 2;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int c = t + i * 256;
    p.a[i] = f32x4{0.f, 0.f, 0.f, 0.f};
    p.w[i] = p.a[i];
    p.qa[i] = i64x2{0, 0};
    p.qb[i] = p.qa[i];
    if (c < K4) {
      p.w[i] = ((const f32x4*)f.norm_w)[c];
      if (f.resid_in) p.a[i] = ((const f32x4*)f.resid_in)[c];
      if (f.fx) {
        p.qa[i] = *(const i64x2*)(f.fx + 4 * c);
        p.qb[i] = *(const i64x2*)(f.fx + 4 * c + 2);
      }
    }
  }
}
__device__ __forceinline__ void pro1_row_finish(const PgFusedArgs& f, int K, const Pro1Row& p, bf16_t* xs,
                                                float* red) {
  const int t = threadIdx.x, K4 = K >> 2;
  f32x4 v[2];
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    v[i] = p.a[i];
    if (f.fx) v[i] += f32x4{fx_to_f32(p.qa[i][0]), fx_to_f32(p.qa[i][1]), fx_to_f32(p.qb[i][0]), fx_to_f32(p.qb[i][1])};
    ss += v[i][0] * v[i][0] + v[i][1] * v[i][1] + v[i][2] * v[i][2] + v[i][3] * v[i][3];
  }
  ss = wave_sum(ss);
  if ((t & 63) == 0) red[t >> 6] = ss;
  lds_barrier();
  const float rstd = rsqrtf((red[0] + red[1] + red[2] + red[3]) / (float)K + f.eps);
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int c = t + i * 256;
    if (c < K4) {
      const f32x4 w = p.w[i];
      u32x2 pk;
      pk[0] = pack_bf2((v[i][0] * rstd) * (1.0f + w[0]), (v[i][1] * rstd) * (1.0f + w[1]));
      pk[1] = pack_bf2((v[i][2] * rstd) * (1.0f + w[2]), (v[i][3] * rstd) * (1.0f + w[3]));
      *(u32x2*)(xs + c * 4) = pk;
    }
  }
  lds_barrier();
}

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
          f32x4 a = f32x4{0.f, 0.f, 0.f, 0.f};
          if (f.resid_in) a = ((const f32x4*)f.resid_in)[c];
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
        f32x4 v = f32x4{0.f, 0.f, 0.f, 0.f};
        if (f.resid_in) v = ((const f32x4*)(f.resid_in + (size_t)m * K))[c];
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
        f32x4 v = f32x4{0.f, 0.f, 0.f, 0.f};
        if (f.resid_in) v = ((const f32x4*)(f.resid_in + (size_t)m * K))[c];
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
  // PRO 1 on one row of at most 2048 elements (batch-1 decode q|k|v and gate/up): the RMSNorm's loads go out BEFORE
  // the weight ring and are held in registers, so they return first and the normalisation runs while the weights
  // stream (issued after the ring, the prologue's loads made it wait for the whole ring: vmcnt counts in order)
  const bool early = PRO == 1 && (PG_GEMV_PRO_EARLY == 1 || (PG_GEMV_PRO_EARLY == 2 && EPI == PG_EPI_QKV_ROPE)) &&
                     M == 1 && (K >> 2) <= 512 && e.f.nsplit == 0 &&
                     e.f.resid_out == nullptr;
  Pro1Row p1;
  if constexpr (PRO == 1 && PG_GEMV_PRO_EARLY) {
    if (early) pro1_row_load(e.f, K, p1);
    __builtin_amdgcn_sched_barrier(0);         // (the prologue's loads stay ahead of the ring in the vmcnt order)
  }
  // weights issued before the prologue (its loads are the critical path: the stream overlaps them)
  constexpr bool prew = STAGED && PG_GEMV_PREW;
  if (prew) {
#pragma unroll
    for (int d = 0; d < DEPTH; ++d)
      if (CPW > 0 ? d < CPW : d < mine) loadw(d, wb[d]);
  }
  if constexpr (STAGED) {
    float* scratch = (float*)(dyn_smem + (((size_t)M * (Kr + XPAD) * 2 + 15) & ~(size_t)15));
    if (PRO == 1 && PG_GEMV_PRO_EARLY && early)
      pro1_row_finish(e.f, K, p1, xs, scratch);
    else
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
      const size_t ro = (size_t)(r < M ? r : M - 1) * e.N + n0;
      // both loads unconditional (a branch or select on them here would make the compiler wait for them before
      // the weight stream): without fx the fixed-point pair reads fin_resid's first 32 bytes, unused; fin_base picks
      fin_r[t] = *(const f32x4*)(e.f.fin_resid + ro);
      const long long* p = e.f.fx ? e.f.fx + ro : (const long long*)e.f.fin_resid;
      fin_fa[t] = *(const i64x2*)p;
      fin_fb[t] = *(const i64x2*)(p + 2);
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
  // PgFusedArgs.amax_zero (ABI 12 for this kernel): workgroup (0, 0) clears amax_zero[0 .. n) after its stream -- the
  // batch-1 decode step's first GEMV zeroes the fixed-point accumulator that the step's FX_ADD producers add into,
  // so no state carries over from an interrupted step (n % 4 == 0, 16-B aligned, host-checked)
  if (e.f.amax_zero && gi.bx == 0 && gi.by == 0)
    for (int i = 4 * (int)threadIdx.x; i < e.f.amax_zero_n; i += 1024) *(u32x4*)(e.f.amax_zero + i) = u32x4{0u, 0u, 0u, 0u};
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
    // the residual entering the finalisation: fin_resid, or with fx the fixed-point accumulator, which then holds the
    // whole residual (its entries are cleared by this tile's finalising workgroup: every split of the tile loaded
    // them before its ticket)
    auto fin_base = [&](int t) {
      return f.fx ? f32x4{fx_to_f32(fin_fa[t][0]), fx_to_f32(fin_fa[t][1]), fx_to_f32(fin_fb[t][0]),
                          fx_to_f32(fin_fb[t][1])}
                  : fin_r[t];
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
          // resid_in (optional): split 0 also adds the fp32 residual rows -- the accumulator then holds the whole
          // residual, and its consumers read it alone
          if (e.f.resid_in && z == 0) v += load4_guard(e.f.resid_in + (size_t)m * e.N, n0, e.N);
          unsigned long long* dst = (unsigned long long*)e.C + (size_t)m * e.ldc + n0;
#pragma unroll
          for (int j = 0; j < 4; ++j) atomicAdd(dst + j, (unsigned long long)fx_from_f32_checked(v[j], e.f.status));
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
  if constexpr (PG_GEMV_LM_NT == 2 && EPI == PG_EPI_F32) {
    if (e.M <= 4 && ntiles >= 8192 && ksplit == 1) {   // (tuning) the lm_head at batch 1-4 with two tiles per workgroup
      launch_gemv_cpw<EPI, 2, PG_GEMV_LM_D, PRO, FRAG>(dim3((ntiles + 1) / 2, 1), lds, st, A, lda, W, ldw, K, 1, e);
      return;
    }
  }
  if constexpr (PG_GEMV_FIN_NT == 4 && EPI == PG_EPI_F32_FIN) {
    if (e.M > 4 && ntiles % 4 == 0) {   // (tuning) the finalised batched down GEMV with four tiles per workgroup
      launch_gemv_cpw<EPI, 4, PG_GEMV_D2, PRO, FRAG>(dim3(ntiles / 4, ksplit), lds, st, A, lda, W, ldw, K, ksplit, e);
      return;
    }
  }
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

int pg_dispatch_gemv(int epi, bool frag, const bf16_t* A, int lda, const bf16_t* W, int ldw, int K, int ksplit,
                     const EpiArgs& e, hipStream_t st) {
#define PG_CASE(E)                                                                             \
  case E:                                                                                      \
    if (frag) launch_gemv<E, true>(A, lda, W, ldw, K, ksplit, e, st);                          \
    else launch_gemv<E, false>(A, lda, W, ldw, K, ksplit, e, st);                              \
    return 0;
#define PG_CASE_ROWMAJOR(E)                                                                    \
  case E: launch_gemv<E, false>(A, lda, W, ldw, K, ksplit, e, st); return 0;
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
}
