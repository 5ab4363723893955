// Flash-style attention on MFMA (bf16 in, fp32 softmax/accumulate), no N^2 scores in HBM.
//
// Restates the attention cores of SiglipAttention.forward (modeling_siglip.py:96-136,
// bidirectional, scale 1/sqrt(head_dim)) and GemmaAttention.forward
// (modeling_gemma.py:307-339: MQA via repeat_kv, scores/sqrt(head_dim) + additive
// mask, fp32 softmax, P.V) — but the MQA broadcast is free: the q heads that share a
// kv head are stacked as extra query ROWS of one problem (row r = pos * G + head%G),
// so one K/V tile feeds all of them.
//
// Per wave: 16 query rows.  S^T = K . Q^T (MFMA A = K tile, B = Q fragment) puts one
// query per lane column, so the online-softmax max/sum are lane-local plus two xor
// shuffles; O^T = V^T . P^T takes P straight from the S accumulators (the key order
// inside the k-step is permuted to match, SURVEY/guide 'accumulator as operand') and
// V^T from a transposed image (Vt[d][key], written transposed by the producer).
//
// Modes: normal (prefill): a wave walks all keys and writes normalised bf16 O;
// split (decode): each wave owns a key range and writes (O, m, l) partials that
// pg_attn_combine merges.
#include "attn_common.h"

// waves per workgroup in split (decode) mode: tuning knob (scripts/tune/), 1 = one split per workgroup
#ifndef PG_ATTN_FA
#define PG_ATTN_FA 1      // prefill: the LDS-DMA flash kernel (0: the register-staged kernels)
#endif
#ifndef PG_FA_W12
#define PG_FA_W12 1       // prefill, head_dim 256: 12-wave workgroups when they fill the one-per-CU rounds better
#endif
#ifndef PG_FA_W8R2
#define PG_FA_W8R2 1      // head_dim 256: 8 waves x 2 row groups (256 rows per workgroup) on 32-key blocks
#endif
#ifndef PG_FA_W8R2_NST
#define PG_FA_W8R2_NST 2  // (4 / 5 stages measured 4-5% slower at pt-896 x32)
#endif
#ifndef PG_FA_W8R2_HOIST
#define PG_FA_W8R2_HOIST 4
#endif
#ifndef PG_FA_UNROLL
#define PG_FA_UNROLL 1
#endif
#ifndef PG_FA_MASK_BRANCH
#define PG_FA_MASK_BRANCH 1
#endif
#ifndef PG_FA_STAGE32
#define PG_FA_STAGE32 1
#endif
#ifndef PG_FA_LAZY
#define PG_FA_LAZY 0      // lazy rescale threshold (log2); 8 measured faster but failed the pt-896 fp8 bound
#endif
#ifndef PG_FA_PRIO
#define PG_FA_PRIO 0
#endif
#ifndef PG_COMBINE_PF
#define PG_COMBINE_PF 12  // split-KV merge: O partials of the first 12 splits per thread loaded up front
#endif
#define PG_ATTN_PIPE 0x100 // pg_attn_decode: flag OR-ed into nw -- the double-buffered form (include/pghip.h)
#ifndef PG_ATTN_WG
#define PG_ATTN_WG 1      // decode splits of 2 / 4 / 8 blocks (head_dim 256): one wave per block, merged in LDS
#endif
#ifndef PG_ATTN_SPLIT_WAVES
#define PG_ATTN_SPLIT_WAVES 1
#endif
#ifndef PG_FA_DEEP
#define PG_FA_DEEP 0      // 4-wave prefill workgroups: a 5-8 stage ring; measured slower (pt-224 Gemma 25.2 vs 22.7 us,
                          // SigLIP 10.0 vs 10.0: not latency-bound; profiles/r03_prefill_breakdown_pt224.txt)
#endif
#ifndef PG_FA_SMALL
#define PG_FA_SMALL 0     // 1 = batch-1 prefill grids in 1- / 2-wave workgroups: measured slower (pt-224 prefill 5.69 vs
                          // 5.47 ms: a lone wave's staging latency is exposed; Gemma 33.0 vs 22.7 us, SigLIP 13.6 vs 10.0)
#endif

// Decode (split mode): one wave per (batch, kv head, split); grid (1, Hkv * nsplit, B).
template <int DP, int DT, bool FULL>
__global__ __launch_bounds__(64) void attn_decode_kernel(AttnArgs a) {
  const int nsplit = (int)gridDim.y / a.Hkv;
  attn_decode_split<DP, DT, false, FULL>(a, blockIdx.z, blockIdx.y / nsplit, blockIdx.y % nsplit, nsplit,
                                         threadIdx.x);
}

// Decode (split mode) with NW * NB-block splits (split_keys = 32 * NW * NB): one workgroup of NW waves per (batch,
// kv head, split); in round j < NB wave w takes the split's 32-key block j * NW + w (the NW waves' loads in flight
// at once, one memory round trip per round), folding its rounds into one running (O, m, l); then the waves'
// (O, m, l) are merged through LDS into ONE partial of the split (2^(m_w - M) weights, the merge of
// pg_attn_combine), so the combine still sees nsplit partials.  NB > 1 sizes the grid to one round of resident
// workgroups at long KV x batch (pt-896 x32: 12 splits of 384 keys, 384 workgroups, instead of 36 of 128 keys in
// 2.25 rounds).  Rounds past the kv length are skipped.  Needs a known cache capacity (kcap >= 32) and
// head_dim == DP.  grid (1, Hkv * nsplit, B).
template <int DP, int DT, int NW>
__global__ __launch_bounds__(NW * 64) void attn_decode_wg_kernel(AttnArgs a) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, c = lane & 15, g = lane >> 4;
  const int nsplit = (int)gridDim.y / a.Hkv;
  const int b = blockIdx.z, kvh = blockIdx.y / nsplit, sp = blockIdx.y % nsplit;
  const int NB = a.split_keys / (32 * NW);
  f32x4 o[DT];
  float m, l;
  attn_decode_block32<DP, DT>(a, b, kvh, sp * a.split_keys + 32 * wave, lane, o, m, l);
  // (the NB == 1 branch jumped straight to the LDS stores of o one instruction after the block's last MFMA, inside its
  // write latency -- found by tests/mfma_hazard.py: the accumulators are pinned past the MFMA latency first)
  mfma_fence(o);
  if (NB > 1) {
    const int lkv = __builtin_amdgcn_readfirstlane(
        __hip_atomic_load(a.lkv_dev ? a.lkv_dev : &pg_zero_word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) + a.Lkv;
    for (int j = 1; j < NB; ++j) {
      const int kb = sp * a.split_keys + (j * NW + wave) * 32;
      if (kb >= lkv) break;                        // wave-uniform: no key of this or a later round is valid
      f32x4 oj[DT];
      float mj, lj;
      attn_decode_block32<DP, DT>(a, b, kvh, kb, lane, oj, mj, lj);
      const float mn = fmaxf(m, mj);
      const float wa = m == -INFINITY ? 0.f : exp2f(m - mn), wb = mj == -INFINITY ? 0.f : exp2f(mj - mn);
      l = l * wa + lj * wb;
      m = mn;
#pragma unroll
      for (int t = 0; t < DT; ++t) o[t] = o[t] * wa + oj[t] * wb;
    }
  }
  __shared__ f32x4 so[NW - 1][DT][64];
  __shared__ float sml[NW - 1][2][16];
  if (wave > 0) {
#pragma unroll
    for (int t = 0; t < DT; ++t) so[wave - 1][t][lane] = o[t];
    if (g == 0) {
      sml[wave - 1][0][c] = m;
      sml[wave - 1][1][c] = l;
    }
  }
  __syncthreads();
  if (wave != 0) return;
  float M = m;
#pragma unroll
  for (int w = 0; w < NW - 1; ++w) M = fmaxf(M, sml[w][0][c]);
  const float w0 = m == -INFINITY ? 0.f : exp2f(m - M);
  float L = l * w0;
#pragma unroll
  for (int t = 0; t < DT; ++t) o[t] *= w0;
#pragma unroll
  for (int w = 0; w < NW - 1; ++w) {
    const float mw = sml[w][0][c];
    const float ww = mw == -INFINITY ? 0.f : exp2f(mw - M);
    L += ww * sml[w][1][c];
#pragma unroll
    for (int t = 0; t < DT; ++t) o[t] += ww * so[w][t][lane];
  }
  if (c >= a.Lq * a.G) return;                   // rows past Lq*G are never merged
  const long base = (((long)b * a.Hkv + kvh) * nsplit + sp) * 16 + c;
  float* po = a.part_o + base * (DT * 16);
#pragma unroll
  for (int t = 0; t < DT; ++t) *(f32x4*)(po + 16 * t + 4 * g) = o[t];
  if (g == 0) {
    a.part_ml[base * 2 + 0] = M;
    a.part_ml[base * 2 + 1] = L;
  }
}

// Batched decode (B > 2: the batch alone fills the chip) with the split merge in the same launch.
// One workgroup of NW waves per (split, kv head, batch).  Split sp owns the contiguous 32-key blocks
// [sp * nblk / S, (sp + 1) * nblk / S) -- floor or ceil of nblk / S each -- and its wave w takes every NW-th of them
// from the w-th, so the two 64-B halves of a 128-B V^T line (adjacent blocks) are read by one CU (dealing single
// blocks round-robin put them on two XCDs, each fetching the whole line).  The NW running (O, m, l)
// merge through LDS into the split's partial, stored write-through (sc1); one agent-scope ticket per (batch,
// kv head) then makes the workgroup of the last-arriving split merge the S partials (sc1 loads: the MI355X guide's
// in-launch hand-off with no release / acquire fence) and write the bf16 attention rows -- no combine launch.
// Stamps of the one-wave-per-split kernel it replaces for B > 2 (scripts/tune/attn_stamps.py): at 340 registers
// (one wave per SIMD) a split's compute (0.9 us) never overlapped another split's loads, and pt-896 x32 ran 4.25
// rounds of waves (54 us for 142 MB of K/V); this kernel holds 240 registers (two waves per SIMD).
// PIPE: each wave's blocks are staggered -- the next block's K / V loads are issued between the current block's
// phases, so its loads never drain during a compute phase (one wave per SIMD at pt-896 x32: each round's compute,
// 0.9 us, stalled the stream of the single-buffered form).
#ifndef PG_DEC_SHARE_MERGE
#define PG_DEC_SHARE_MERGE 1
#endif
// splits whose partials the merging workgroup loads per round trip (8: the engine's split cap, no clamped duplicates)
#ifndef PG_DEC_MERGE_MCH
#define PG_DEC_MERGE_MCH 8
#endif
template <int DP, int DT, int NW, bool PIPE>
__global__ __launch_bounds__(NW * 64, 2) void attn_decode_fused_kernel(AttnArgs a, int nb, int* __restrict__ cnt,
                                                                      uint8_t* __restrict__ q8, float* __restrict__ q8s,
                                                                      long q8_ld) {
  static_assert(NW == 2 || NW == 4, "2 or 4 waves per split");
  constexpr int KS = DP / 32;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, c = lane & 15, g = lane >> 4;
  const int S = gridDim.x, sp = blockIdx.x, kvh = blockIdx.y, b = blockIdx.z;
  const int G = a.G;
  const int rr = c < G ? c : G - 1;                // rows past G read row G - 1 (never stored): no select
#if PG_ATTN_STAMPS
  unsigned long long st0 = __builtin_amdgcn_s_memrealtime(), st1 = 0, st2 = 0, st3 = 0;
#endif
  const int lkv_raw =
      __hip_atomic_load(a.lkv_dev ? a.lkv_dev : &pg_zero_word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  // the G query rows of this (batch, kv head) in LDS, re-read per block (32 registers fewer: two waves per SIMD)
  // (loaded before the K/V stream, stored to LDS after it is issued: the store waits only for the q loads)
  __shared__ u32x4 sq[16][DP / 8];
  constexpr int QPT = (16 * (DP / 8) + NW * 64 - 1) / (NW * 64);
  const bf16_t* qrow0 = a.q + (long)b * a.q_rs + (long)(kvh * G) * DP;
  u32x4 qv[QPT];
#pragma unroll
  for (int k = 0; k < QPT; ++k) {
    const int i = min((int)threadIdx.x + k * NW * 64, 16 * (DP / 8) - 1);
    qv[k] = *(const u32x4*)(qrow0 + (long)min(i / (DP / 8), G - 1) * DP + 8 * (i % (DP / 8)));
  }
  __builtin_amdgcn_sched_barrier(0);               // (the q loads stay ahead of the K/V stream)
  const bf16_t* kbase = a.kd + ((long)b * a.Hkv + kvh) * a.kcap * DP;   // decode-order copies
  const bf16_t* vbase = a.vd + ((long)b * a.Hkv + kvh) * a.kcap * DP;
  // split sp owns the contiguous blocks [lo, hi) (at least NW: nsplit <= kcap / 128), wave w the blocks lo + w +
  // NW * j: every split reads ceil or floor of nblk / S blocks (dealing granules of NW blocks round-robin left the
  // first splits a whole extra round: pt-896 x32, 131 blocks, 20 vs 17 per CU)
  const int nblk = a.kcap >> 5;
  const int lo = (int)((long)sp * nblk / S), hi = (int)((long)(sp + 1) * nblk / S);
  auto qfrag = [&](bf16x8 (&qf)[KS]) {
#pragma unroll
    for (int s = 0; s < KS; ++s) qf[s] = __builtin_bit_cast(bf16x8, sq[rr][4 * s + g]);
  };
  u32x4 kfa[KS], kfb[KS];
  u32x4 vr[DT];
  f32x4 o[DT];
#pragma unroll
  for (int t = 0; t < DT; ++t) o[t] = f32x4{0.f, 0.f, 0.f, 0.f};
  float m = -INFINITY, l = 0.f;
  // round 0 (every split owns at least NW blocks: nsplit <= kcap / 128): its loads are issued before the kv length
  // arrives
  int blk = lo + wave;
  dec_load_block<DP, DT>(a, kbase, vbase, 32 * blk, c, g, kfa, kfb, vr);
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int k = 0; k < QPT; ++k) {
    const int i = (int)threadIdx.x + k * NW * 64;
    if ((16 * (DP / 8)) % (NW * 64) == 0 || i < 16 * (DP / 8)) sq[i / (DP / 8)][i % (DP / 8)] = qv[k];
  }
  __syncthreads();                                 // sq written (the block's loads stay in flight across it)
  __builtin_amdgcn_sched_barrier(0);
  const int Lkv = __builtin_amdgcn_readfirstlane(lkv_raw) + a.Lkv;
  if constexpr (!PIPE) {
    {
      bf16x8 qf[KS];
      qfrag(qf);
      dec_block_update<DP, DT, false, true>(a.scale_log2, 32 * blk, min(Lkv, 32 * blk + 32), c, g, qf, kfa, kfb, vr,
                                            o, m, l);
    }
    for (int j = 1; j < nb; ++j) {
      blk = lo + NW * j + wave;
      if (blk >= hi) break;
      dec_load_block<DP, DT>(a, kbase, vbase, 32 * blk, c, g, kfa, kfb, vr);
      __builtin_amdgcn_sched_barrier(0);
      bf16x8 qf[KS];
      qfrag(qf);
      dec_block_update<DP, DT, false>(a.scale_log2, 32 * blk, min(Lkv, 32 * blk + 32), c, g, qf, kfa, kfb, vr, o,
                                      m, l);
    }
  } else {
    // staggered: block j + 1's K is issued as soon as block j's scores are out of the K registers, its V as soon as
    // block j's P.V is out of the V registers -- one block of loads stays in flight through every compute phase with
    // no second register set.  The loads are unconditional inside the loop (wave-uniform trip count n - 1), so both
    // edges into the loop head carry the same [K, V] loads in flight and the compiler's vmcnt waits for the older half.
    const int n = (hi - lo - wave + NW - 1) / NW;  // this wave's blocks (>= 1)
    auto ldk = [&](int bk) {
#pragma unroll
      for (int s2 = 0; s2 < KS; ++s2) {
        const int kl = min(32 * bk, a.kcap - 32);
        kfa[s2] = *(const u32x4*)(kbase + dec_kfrag(kl, 0, s2, c, g, DP));
        kfb[s2] = *(const u32x4*)(kbase + dec_kfrag(kl, 1, s2, c, g, DP));
      }
      __builtin_amdgcn_sched_barrier(0);
    };
    auto ldv = [&](int bk) {
      const int kl = min(32 * bk, a.kcap - 32);
#pragma unroll
      for (int t = 0; t < DT; ++t) vr[t] = *(const u32x4*)(vbase + dec_vfrag(kl, t, c, g, DP));
      __builtin_amdgcn_sched_barrier(0);
    };
    auto none = [] {};
    bf16x8 qf[KS];
    qfrag(qf);
    if (n > 1) {
      dec_block_update<DP, DT, false, true>(a.scale_log2, 32 * blk, min(Lkv, 32 * blk + 32), c, g, qf, kfa, kfb, vr,
                                            o, m, l, [&] { ldk(blk + NW); });
      ldv(blk + NW);
      for (int j = 1; j < n - 1; ++j) {
        blk += NW;
        qfrag(qf);
        dec_block_update<DP, DT, false>(a.scale_log2, 32 * blk, min(Lkv, 32 * blk + 32), c, g, qf, kfa, kfb, vr, o,
                                        m, l, [&] { ldk(blk + NW); });
        ldv(blk + NW);
      }
      blk += NW;
      qfrag(qf);
      dec_block_update<DP, DT, false>(a.scale_log2, 32 * blk, min(Lkv, 32 * blk + 32), c, g, qf, kfa, kfb, vr, o, m,
                                      l, none);
    } else {
      dec_block_update<DP, DT, false, true>(a.scale_log2, 32 * blk, min(Lkv, 32 * blk + 32), c, g, qf, kfa, kfb, vr,
                                            o, m, l, none);
    }
  }
#if PG_ATTN_STAMPS
  PG_STAMP(st1);
#endif
  // the NW waves' (O, m, l) -> the split's partial, 2^(m_w - M) weights.  SHARE (4 waves, DT % 4 == 0): every wave
  // publishes its (O, m, l) and merges and stores a quarter of the columns (the same sum order as one wave merging
  // all of them, so the same bits), so the partial's stores drain from four waves before the ticket
  constexpr bool SHARE = PG_DEC_SHARE_MERGE && NW == 4 && DT % 4 == 0;
  constexpr int NSO = SHARE ? NW : (NW > 1 ? NW - 1 : 1);
  __shared__ f32x4 so[NSO][DT][64];
  __shared__ float sml[NSO][2][16];
  __shared__ int s_last;
  if (SHARE || (NW > 1 && wave > 0)) {
    const int ws = SHARE ? wave : wave - 1;
#pragma unroll
    for (int t = 0; t < DT; ++t) so[ws][t][lane] = o[t];
    if (g == 0) {
      sml[ws][0][c] = m;
      sml[ws][1][c] = l;
    }
  }
  __syncthreads();
  const long pbase = ((long)b * a.Hkv + kvh) * S * 16;          // partial rows of (b, kv head): [S][16]
  const __amdgpu_buffer_rsrc_t ro = pg_rsrc(a.part_o + pbase * (DT * 16));
  if constexpr (SHARE) {
    float M = sml[0][0][c];
#pragma unroll
    for (int w = 1; w < NW; ++w) M = fmaxf(M, sml[w][0][c]);
    float ww[NW];
#pragma unroll
    for (int w = 0; w < NW; ++w) ww[w] = sml[w][0][c] == -INFINITY ? 0.f : exp2f(sml[w][0][c] - M);
    float L = sml[0][1][c] * ww[0];
#pragma unroll
    for (int w = 1; w < NW; ++w) L += ww[w] * sml[w][1][c];
    if (c < G) {
      const int row = sp * 16 + c;
#pragma unroll
      for (int t0 = 0; t0 < DT / NW; ++t0) {
        const int t = wave * (DT / NW) + t0;
        f32x4 v = so[0][t][lane] * ww[0];
#pragma unroll
        for (int w = 1; w < NW; ++w) v += ww[w] * so[w][t][lane];
        st16_sc1(ro, (row * (DT * 16) + 16 * t + 4 * g) * 4, v);
      }
      if (wave == 0 && g == 0)
        __hip_atomic_store((pg_gu64*)(a.part_ml + (pbase + row) * 2), __builtin_bit_cast(unsigned long long,
                           f32x2{M, L}), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");             // every storing wave drained before the ticket
  } else if (wave == 0) {
    float M = m;
#pragma unroll
    for (int w = 0; w < NW - 1; ++w) M = fmaxf(M, sml[w][0][c]);
    const float w0 = m == -INFINITY ? 0.f : exp2f(m - M);
    float L = l * w0;
#pragma unroll
    for (int t = 0; t < DT; ++t) o[t] *= w0;
#pragma unroll
    for (int w = 0; w < NW - 1; ++w) {
      const float mw = sml[w][0][c];
      const float ww = mw == -INFINITY ? 0.f : exp2f(mw - M);
      L += ww * sml[w][1][c];
#pragma unroll
      for (int t = 0; t < DT; ++t) o[t] += ww * so[w][t][lane];
    }
    if (c < G) {
      const int row = sp * 16 + c;
#pragma unroll
      for (int t = 0; t < DT; ++t) st16_sc1(ro, (row * (DT * 16) + 16 * t + 4 * g) * 4, o[t]);
      if (g == 0)
        __hip_atomic_store((pg_gu64*)(a.part_ml + (pbase + row) * 2), __builtin_bit_cast(unsigned long long,
                           f32x2{M, L}), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");             // the storing wave drained before the ticket
  }
  __syncthreads();
  if (threadIdx.x == 0)
    s_last = __hip_atomic_fetch_add(cnt + b * a.Hkv + kvh, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == S - 1;
  __syncthreads();
#if PG_ATTN_STAMPS
  PG_STAMP(st2);
  st3 = st2;
  const int sid = (b * a.Hkv + kvh) * S + sp;
  if (threadIdx.x == 0 && sid < 8192 && !s_last) {
    pg_attn_stamp_buf[sid][0] = st0; pg_attn_stamp_buf[sid][1] = st1;
    pg_attn_stamp_buf[sid][2] = st2; pg_attn_stamp_buf[sid][3] = 0;
  }
#endif
  if (!s_last) return;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");        // compiler-only: the loads stay below the ticket
  // the last split's workgroup merges the S partials: one thread per (q row, 8 dims), MCH (8) splits per round trip
  constexpr int D8 = DP / 8, MCH = PG_DEC_MERGE_MCH;
  u32x4 pk = {0u, 0u, 0u, 0u};                      // this thread's last 8 outputs (the fp8 copy below)
  for (int it = threadIdx.x; it < G * D8; it += NW * 64) {
    const int r = it / D8, d8 = it % D8;
    float M = -INFINITY, den = 0.f;
    f32x4 n0 = {0.f, 0.f, 0.f, 0.f}, n1 = {0.f, 0.f, 0.f, 0.f};
    for (int s0 = 0; s0 < S; s0 += MCH) {
      f32x2 ml[MCH];
      f32x4 oa[MCH], ob[MCH];
#pragma unroll
      for (int k = 0; k < MCH; ++k) {
        const int row = min(s0 + k, S - 1) * 16 + r;
        ml[k] = ld8_wt(a.part_ml + (pbase + row) * 2);
        oa[k] = ld16_sc1(ro, (row * (DT * 16) + 8 * d8) * 4);
        ob[k] = ld16_sc1(ro, (row * (DT * 16) + 8 * d8 + 4) * 4);
      }
      __builtin_amdgcn_sched_barrier(0);
      float cm = -INFINITY;
#pragma unroll
      for (int k = 0; k < MCH; ++k) cm = s0 + k < S ? fmaxf(cm, ml[k][0]) : cm;
      const float Mn = fmaxf(M, cm);
      const float sc = M == -INFINITY ? 0.f : exp2f(M - Mn);
      den *= sc;
      n0 *= sc;
      n1 *= sc;
#pragma unroll
      for (int k = 0; k < MCH; ++k) {
        const float w = (s0 + k < S && ml[k][0] != -INFINITY) ? exp2f(ml[k][0] - Mn) : 0.f;
        den += w * ml[k][1];
        n0 += w * oa[k];
        n1 += w * ob[k];
      }
      M = Mn;
    }
    const float inv = 1.0f / den;
    pk[0] = pack_bf2(n0[0] * inv, n0[1] * inv);
    pk[1] = pack_bf2(n0[2] * inv, n0[3] * inv);
    pk[2] = pack_bf2(n1[0] * inv, n1[1] * inv);
    pk[3] = pack_bf2(n1[2] * inv, n1[3] * inv);
    *(u32x4*)(a.o + (long)b * a.o_rs + (long)(kvh * G + r) * DP + 8 * d8) = pk;
  }
  if (q8) {
    // e4m3 copy of the row for the fp8 o_proj (host: one kv head, so this workgroup wrote the whole row, and one
    // (q row, 8 dims) item per thread): pg_quant_fp8's bytes and scale from the same bf16 values
    __shared__ float red[NW];
    float amax = 0.f;
#pragma unroll
    for (int j = 0; j < 4; ++j) amax = fmaxf(amax, fmaxf(fabsf(bf_lo(pk[j])), fabsf(bf_hi(pk[j]))));
    amax = wave_max(amax);
    if (lane == 0) red[wave] = amax;
    __syncthreads();
#pragma unroll
    for (int w = 0; w < NW; ++w) amax = fmaxf(amax, red[w]);
    const float s = amax > 0.f ? amax / 448.f : 1.f;
    if (threadIdx.x == 0) q8s[b] = s;
    if ((int)threadIdx.x < G * D8) {
      const int r = threadIdx.x / D8, d8 = threadIdx.x % D8;
      u32x2 w8;
#pragma unroll
      for (int j = 0; j < 2; ++j)
        w8[j] = pack_fp8x4(bf_lo(pk[2 * j]) / s, bf_hi(pk[2 * j]) / s, bf_lo(pk[2 * j + 1]) / s,
                           bf_hi(pk[2 * j + 1]) / s);
      *(u32x2*)(q8 + b * q8_ld + (long)r * DP + 8 * d8) = w8;
    }
  }
  if (threadIdx.x == 0) __hip_atomic_store(cnt + b * a.Hkv + kvh, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#if PG_ATTN_STAMPS
  PG_STAMP(st3);
  if (threadIdx.x == 0 && sid < 8192) {
    pg_attn_stamp_buf[sid][0] = st0; pg_attn_stamp_buf[sid][1] = st1;
    pg_attn_stamp_buf[sid][2] = st2; pg_attn_stamp_buf[sid][3] = st3;
  }
#endif
}

template <int DP, int DT>
__global__ __launch_bounds__(256) void attn_kernel(AttnArgs a) {
  constexpr int KS = DP / 32;  // QK^T k-steps
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int c = lane & 15;
  const int g = lane >> 4;
  const int b = blockIdx.z;
  const bool split = a.split_keys > 0;
  const int wpg = (int)(blockDim.x >> 6);
  const int nsg = split ? (int)(gridDim.y / a.Hkv) : 1;
  const int kvh = blockIdx.y / nsg;
  const int sg = blockIdx.y % nsg;
  const int Lkv = (a.lkv_dev ? *a.lkv_dev : 0) + a.Lkv;
  const int R = a.Lq * a.G;
  const int D = a.D;

  if (split) {
    attn_decode_split<DP, DT, false>(a, b, kvh, sg * wpg + wave, nsg * wpg, lane);
    return;
  }
  const int r0 = split ? 0 : (blockIdx.x * (int)(blockDim.x >> 6) + wave) * 16;
  int kbeg = 0, kend = Lkv, sp = 0;
  if (split) {
    sp = sg * wpg + wave;
    kbeg = sp * a.split_keys;
    kend = min(Lkv, kbeg + a.split_keys);
  }
  if (!split && r0 >= R) return;

  const int r = r0 + c;
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
  const float* mrow = a.mask ? a.mask + (long)b * a.mask_bs + (long)pos * a.mask_rs : nullptr;

  f32x4 o[DT];
#pragma unroll
  for (int t = 0; t < DT; ++t) o[t] = f32x4{0.f, 0.f, 0.f, 0.f};
  float m = -INFINITY, l = 0.f;
  const float LOG2E = 1.4426950408889634f;

  for (int kb = kbeg; kb < kend; kb += 32) {
    // issue every load of the block first (K rows for S^T, V^T rows for P.V): one memory round trip
    // K rows past kend are clamped to a valid row: their scores are masked to -inf below
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
    // ---- S^T for keys kb..kb+15 (sA) and kb+16..kb+31 (sB)
    f32x4 sA = {0.f, 0.f, 0.f, 0.f}, sB = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      sA = mfma16(__builtin_bit_cast(bf16x8, kfa[s]), qf[s], sA);
      sB = mfma16(__builtin_bit_cast(bf16x8, kfb[s]), qf[s], sB);
    }
    // lane holds S[key = kb + 4g + j][q = c] (sA) and S[key = kb + 16 + 4g + j][q = c] (sB)
    float x[8];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int k0 = kb + 4 * g + j, k1 = kb + 16 + 4 * g + j;
      float v0 = sA[j] * a.scale_log2, v1 = sB[j] * a.scale_log2;
      if (mrow) {
        v0 += mrow[min(k0, kend - 1)] * LOG2E;
        v1 += mrow[min(k1, kend - 1)] * LOG2E;
      }
      x[j] = k0 < kend ? v0 : -INFINITY;
      x[4 + j] = k1 < kend ? v1 : -INFINITY;
    }
    float bm = x[0];
#pragma unroll
    for (int j = 1; j < 8; ++j) bm = fmaxf(bm, x[j]);
    bm = max_xor16(bm);
    bm = max_xor32(bm);
    const float mn = fmaxf(m, bm);
    const float alpha = exp2f(m - mn);
    float rs = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) { x[j] = exp2f(x[j] - mn); rs += x[j]; }
    rs = sum_xor16(rs);
    rs = sum_xor32(rs);
    l = l * alpha + rs;
    m = mn;
#pragma unroll
    for (int t = 0; t < DT; ++t) o[t] *= alpha;
    // P^T fragment: slot 8g+j <-> key kb+4g+j (j<4), kb+16+4g+(j-4) (j>=4)
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
  if (!split) {
    if (!rvalid) return;
    const float inv = 1.0f / l;
    bf16_t* op = a.o + ((long)b * a.Lq + pos) * a.o_rs + (long)hq * D;
#pragma unroll
    for (int t = 0; t < DT; ++t) {
      const int d = 16 * t + 4 * g;
      if (d < D) {
        u32x2 p;
        p[0] = pack_bf2(o[t][0] * inv, o[t][1] * inv);
        p[1] = pack_bf2(o[t][2] * inv, o[t][3] * inv);
        *(u32x2*)(op + d) = p;
      }
    }
  } else {
    const int nsplit = nsg * wpg;
    const long base = (((long)b * a.Hkv + kvh) * nsplit + sp) * 16 + c;
    if (!rvalid) return;                       // rows past Lq*G are never merged
    float* po = a.part_o + base * (DT * 16);
#pragma unroll
    for (int t = 0; t < DT; ++t) *(f32x4*)(po + 16 * t + 4 * g) = o[t];
    if (g == 0) {
      a.part_ml[base * 2 + 0] = m;
      a.part_ml[base * 2 + 1] = l;
    }
  }
}

// LDS-staged prefill attention for long sequences / large batches: a workgroup of 4 waves (64 query
// rows of one (b, kv head)) shares every 32-key block of K and V^T through a double-buffered LDS stage,
// so K/V leave L2 once per 64 rows instead of once per 16 (pt-448 x16: 1 MB of K/V per 16 rows).
// Rows are padded by 16 B so the MFMA fragment reads are bank-conflict free; K rows past Lkv are
// clamped (their scores are masked) and V^T keys past Lkv are zeroed at staging.
template <int DP, int DT>
__global__ __launch_bounds__(256) void attn_lds_kernel(AttnArgs a) {
  constexpr int KS = DP / 32;
  constexpr int KROW = DP * 2 + 16;          // bytes per staged K row
  constexpr int VROW = 64 + 16;              // bytes per staged V^T row (32 keys)
  constexpr int KBYTES = 32 * KROW;
  constexpr int STAGE = KBYTES + DT * 16 * VROW;
  constexpr int KCH = DP / 8;                // 16-B chunks per K row
  constexpr int KITEMS = 32 * KCH;
  constexpr int VITEMS = DT * 16 * 4;        // 4 chunks of 8 keys per V^T row
  constexpr int KPT = (KITEMS + 255) / 256, VPT = (VITEMS + 255) / 256;
  __shared__ __attribute__((aligned(16))) char smem[2 * STAGE];

  const int t = threadIdx.x;
  const int lane = t & 63, wave = t >> 6, c = lane & 15, g = lane >> 4;
  const int b = blockIdx.z, kvh = blockIdx.y;
  const int Lkv = (a.lkv_dev ? *a.lkv_dev : 0) + a.Lkv;
  const int R = a.Lq * a.G;
  const int D = a.D;
  const int r = (blockIdx.x * 4 + wave) * 16 + c;
  const bool rvalid = r < R;                 // invalid rows still stage and hit every barrier
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
  const float* mrow = a.mask ? a.mask + (long)b * a.mask_bs + (long)pos * a.mask_rs : nullptr;

  u32x4 kst[KPT], vst[VPT];
  auto gload = [&](int kb) {
#pragma unroll
    for (int i = 0; i < KPT; ++i) {
      const int idx = t + i * 256;
      if (idx < KITEMS) {
        const int key = idx / KCH, ch = idx % KCH;
        const int kk = min(kb + key, Lkv - 1);
        const bool ok = ch * 8 < D;
        kst[i] = ld16_sel(kbase + (long)kk * a.k_rs + (ok ? ch * 8 : 0), ok);
      }
    }
#pragma unroll
    for (int i = 0; i < VPT; ++i) {
      const int idx = t + i * 256;
      if (idx < VITEMS) {
        const int d = idx >> 2, key0 = kb + 8 * (idx & 3);
        const bool dok = d < D;
        const u32x4 v = *(const u32x4*)(vbase + (long)(dok ? d : D - 1) * a.vt_ds + key0);
        const int nv = dok ? Lkv - key0 : 0;  // valid keys among the 8
        u32x4 o;
#pragma unroll
        for (int j = 0; j < 4; ++j)
          o[j] = nv >= 2 * j + 2 ? v[j] : (nv == 2 * j + 1 ? (v[j] & 0xFFFFu) : 0u);
        vst[i] = o;
      }
    }
  };
  auto lstore = [&](int buf) {
    char* ks = smem + buf * STAGE;
    char* vs = ks + KBYTES;
#pragma unroll
    for (int i = 0; i < KPT; ++i) {
      const int idx = t + i * 256;
      if (idx < KITEMS) *(u32x4*)(ks + (idx / KCH) * KROW + (idx % KCH) * 16) = kst[i];
    }
#pragma unroll
    for (int i = 0; i < VPT; ++i) {
      const int idx = t + i * 256;
      if (idx < VITEMS) *(u32x4*)(vs + (idx >> 2) * VROW + (idx & 3) * 16) = vst[i];
    }
  };

  f32x4 o[DT];
#pragma unroll
  for (int tt = 0; tt < DT; ++tt) o[tt] = f32x4{0.f, 0.f, 0.f, 0.f};
  float m = -INFINITY, l = 0.f;
  const float LOG2E = 1.4426950408889634f;
  const int nblk = (Lkv + 31) / 32;

  gload(0);
  lstore(0);
  __syncthreads();
  for (int ib = 0; ib < nblk; ++ib) {
    const int kb = ib * 32;
    const int cur = ib & 1;
    if (ib + 1 < nblk) gload(kb + 32);        // next block in flight during this block's math
    const char* ks = smem + cur * STAGE;
    const char* vs = ks + KBYTES;
    f32x4 sA = {0.f, 0.f, 0.f, 0.f}, sB = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      const bf16x8 ka = *(const bf16x8*)(ks + c * KROW + (32 * s + 8 * g) * 2);
      const bf16x8 kb2 = *(const bf16x8*)(ks + (16 + c) * KROW + (32 * s + 8 * g) * 2);
      sA = mfma16(ka, qf[s], sA);
      sB = mfma16(kb2, qf[s], sB);
    }
    float x[8];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int k0 = kb + 4 * g + j, k1 = kb + 16 + 4 * g + j;
      float v0 = sA[j] * a.scale_log2, v1 = sB[j] * a.scale_log2;
      if (mrow) {
        v0 += mrow[min(k0, Lkv - 1)] * LOG2E;
        v1 += mrow[min(k1, Lkv - 1)] * LOG2E;
      }
      x[j] = k0 < Lkv ? v0 : -INFINITY;
      x[4 + j] = k1 < Lkv ? v1 : -INFINITY;
    }
    float bm = x[0];
#pragma unroll
    for (int j = 1; j < 8; ++j) bm = fmaxf(bm, x[j]);
    bm = max_xor16(bm);
    bm = max_xor32(bm);
    const float mn = fmaxf(m, bm);
    const float alpha = exp2f(m - mn);
    float rs = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) { x[j] = exp2f(x[j] - mn); rs += x[j]; }
    rs = sum_xor16(rs);
    rs = sum_xor32(rs);
    l = l * alpha + rs;
    m = mn;
    u32x4 pw;
    pw[0] = pack_bf2(x[0], x[1]);
    pw[1] = pack_bf2(x[2], x[3]);
    pw[2] = pack_bf2(x[4], x[5]);
    pw[3] = pack_bf2(x[6], x[7]);
    const bf16x8 pf = __builtin_bit_cast(bf16x8, pw);
#pragma unroll
    for (int tt = 0; tt < DT; ++tt) {
      const char* vr = vs + (16 * tt + c) * VROW;
      const u32x2 v0 = *(const u32x2*)(vr + 8 * g);
      const u32x2 v1 = *(const u32x2*)(vr + 32 + 8 * g);
      o[tt] = mfma16(__builtin_bit_cast(bf16x8, u32x4{v0[0], v0[1], v1[0], v1[1]}), pf, o[tt] * alpha);
    }
    if (ib + 1 < nblk) {
      lstore(cur ^ 1);                         // buffer cur^1 was last read before the previous barrier
      __syncthreads();
    }
  }
  if (!rvalid) return;
  const float inv = 1.0f / l;
  bf16_t* op = a.o + ((long)b * a.Lq + pos) * a.o_rs + (long)hq * D;
#pragma unroll
  for (int tt = 0; tt < DT; ++tt) {
    const int d = 16 * tt + 4 * g;
    if (d < D) {
      u32x2 p;
      p[0] = pack_bf2(o[tt][0] * inv, o[tt][1] * inv);
      p[1] = pack_bf2(o[tt][2] * inv, o[tt][3] * inv);
      *(u32x2*)(op + d) = p;
    }
  }
}

// Prefill flash attention, LDS-DMA staged (no mask, 16-B aligned strides).  A workgroup of WAVES waves
// (16 query rows each) walks KB-key blocks (KB 64 or 32); every block's K [KB keys][DP] and V^T [DT*16 d][KB keys]
// are pulled HBM->LDS by global_load_lds (16 B/lane, lane-linear destinations) into an NST-stage ring: NST - 1
// blocks in flight while one is computed, the wait for a block a counted vmcnt (its younger blocks stay in flight
// across the barrier).  NST 2 / KB 64 for grids that fill the chip; a deep ring (NST 5-8) for the batch-1 grids
// of a few dozen workgroups, whose time is otherwise one L2 round trip per block.  Images:
//   K   : 16-key groups of [DP/8 chunks][16 keys][16 B] -> a S^T fragment read (16 keys x 32 d) is one
//         contiguous KiB per wave-instruction (conflict-free ds_read_b128).  Image row i of group kt holds key
//         32 (kt / 2) + 8 (i / 4) + 4 (kt % 2) + i % 4 (the source address picks it), so the S^T lanes of a
//         32-key half hold 8 CONSECUTIVE keys 8g..8g+7 and a PV fragment of V^T is one 16-B chunk
//   V^T : rows of 2 KB bytes, 16-B chunk XOR-swizzled through the source address by (row >> 1) & 7 (KB 64) or
//         (row >> 2) & 2 (KB 32) -> the one ds_read_b128 of a PV fragment is conflict-free (16 distinct slots
//         in each of its 16-lane groups).  The earlier key order needed two 8-B reads per fragment, which the
//         compiler pairs into ds_read2st64_b64 (half the LDS rate, 2-way conflicts on the 32-bank modulus):
//         the LDS, not the MFMA, bounded the kernel
// Per block a wave does 4 x KS S^T MFMAs, an online softmax on 16 scores per lane (the rescale of O is
// skipped when no row's max moved), and 2 x DT PV MFMAs.  Keys past Lkv: K rows clamped, scores -inf,
// V^T chunks clamped to the last readable 8-key chunk (rup8(Lkv) keys must be readable per V^T row);
// K dims past D (D < DP) are never read from memory.
template <int DP, int DT, int WAVES, int RPW, int KB = 64, int NST = 2>
__global__ __launch_bounds__(WAVES * 64) void attn_fa_kernel(AttnArgs a) {
  static_assert(KB == 64 || KB == 32, "64- or 32-key blocks");
  constexpr int KS = DP / 32;
  constexpr int NCH = DP / 8;                      // 16-B chunks per K row
  constexpr int KIMG = KB * DP * 2;                // bytes
  constexpr int VROW = KB * 2;                     // bytes per V^T image row
  constexpr int VIMG = DT * 16 * VROW;
  constexpr int STAGE = KIMG + VIMG;
  constexpr int KINS = KIMG / 1024, VINS = VIMG / 1024;   // glds wave-instructions per block
  constexpr int FA_HOIST = (DP == 256 && WAVES == 8 && RPW == 2) ? PG_FA_W8R2_HOIST : 0;
  // lazy rescale (tuning knob, off): head_dim >= 128 only -- at head_dim 72 the rescale is cheap and the branch cost
  // more (pt-896 x32 SigLIP 3.79 -> 3.89 ms; Gemma 4.96 -> 4.75 ms)
  constexpr int LAZY = DP >= 128 ? PG_FA_LAZY : 0;
  static_assert(KIMG % 1024 == 0 && VIMG % 1024 == 0 && NST * STAGE <= 163840, "stage images");
  __shared__ __attribute__((aligned(1024))) char smem[NST * STAGE];

  const int t = threadIdx.x;
  const int lane = t & 63, c = lane & 15, g = lane >> 4;
  const int wave = __builtin_amdgcn_readfirstlane(t >> 6);   // wave-uniform: scalar branches on the piece counts
  const int b = blockIdx.z, kvh = blockIdx.y;
  const int Lkv = a.Lkv;
  const int R = a.Lq * a.G;
  const int D = a.D;
  // key split (a.pf_splits > 1): workgroup x = row tile * nks + split; split ks walks its share of the key blocks
  const int nks = a.pf_splits > 1 ? a.pf_splits : 1;
  const int rt = blockIdx.x / nks, ks = blockIdx.x % nks;
  // RPW groups of 16 query rows per wave: every K / V^T fragment read from LDS feeds RPW MFMAs
  int pos[RPW], hq[RPW], rrow[RPW];
  bool rvalid[RPW];
  bf16x8 qf[RPW][KS];
#pragma unroll
  for (int i = 0; i < RPW; ++i) {
    const int r = ((rt * WAVES + wave) * RPW + i) * 16 + c;
    rrow[i] = r;
    rvalid[i] = r < R;
    pos[i] = rvalid[i] ? r / a.G : 0;
    hq[i] = kvh * a.G + (rvalid[i] ? r % a.G : 0);
    const bf16_t* qp = a.q + ((long)b * a.Lq + pos[i]) * a.q_rs + (long)hq[i] * D;
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      const int d0 = 32 * s + 8 * g;
      qf[i][s] = __builtin_bit_cast(bf16x8, ld16_sel(qp + (d0 < D ? d0 : 0), rvalid[i] && d0 < D));
    }
  }
  const bf16_t* kbase = a.k + (long)b * a.k_bs + (long)kvh * a.k_hs;
  const bf16_t* vbase = a.vt + (long)b * a.vt_bs + (long)kvh * a.vt_hs;
  const int vkey_max = ((Lkv + 7) & ~7) - 8;       // last readable 8-key chunk of a V^T row

  auto stage = [&](int kb, int buf) {
    char* kimg = smem + buf * STAGE;
    char* vimg = kimg + KIMG;
    for (int i = wave; i < KINS; i += WAVES) {
      const int kg = i / (NCH / 4), cq = i % (NCH / 4);
      const int i16 = lane & 15;
      const int ch = 4 * cq + (lane >> 4), key = 32 * (kg >> 1) + 8 * (i16 >> 2) + 4 * (kg & 1) + (i16 & 3);
      // chunks past D (D < DP) re-read chunk 0: the matching q dims are zero, and 0 * (finite K) = 0, whereas
      // the bytes past a head's D may be another tensor's never-written memory (NaN * 0 = NaN)
      const int kr = min(kb + key, Lkv - 1), kc = ch * 8 < D ? ch * 8 : 0;
      // (PG_FA_STAGE32: uniform base + 32-bit lane offset -- the saddr form, no 64-bit address arithmetic per piece;
      // the host takes this kernel only where a head's K rows and V^T rows span < 4 GiB)
      const bf16_t* src = PG_FA_STAGE32 ? (const bf16_t*)((const char*)kbase + ((unsigned)kr * (unsigned)a.k_rs + (unsigned)kc) * 2u)
                                        : kbase + (long)kr * a.k_rs + kc;
      __builtin_amdgcn_global_load_lds((const void*)src, (LDS_AS void*)(kimg + i * 1024), 16, 0, 0);
    }
    for (int i = wave; i < VINS; i += WAVES) {
      const int row = KB == 64 ? 8 * i + (lane >> 3) : 16 * i + (lane >> 2);
      const int cl = KB == 64 ? (lane & 7) ^ ((row >> 1) & 7) : (lane & 3) ^ ((row >> 2) & 2);
      const int vr = min(row, D - 1), vc = min(kb + 8 * cl, vkey_max);
      const bf16_t* src = PG_FA_STAGE32 ? (const bf16_t*)((const char*)vbase + ((unsigned)vr * (unsigned)a.vt_ds + (unsigned)vc) * 2u)
                                        : vbase + (long)vr * a.vt_ds + vc;
      __builtin_amdgcn_global_load_lds((const void*)src, (LDS_AS void*)(vimg + i * 1024), 16, 0, 0);
    }
  };
  // glds pieces this wave issues per block (wave-uniform): its vmcnt step per younger block in flight
  const int P = (KINS > wave ? (KINS - 1 - wave) / WAVES + 1 : 0) + (VINS > wave ? (VINS - 1 - wave) / WAVES + 1 : 0);

  f32x4 o[RPW][DT];
  float m[RPW], l[RPW];
#pragma unroll
  for (int i = 0; i < RPW; ++i) {
    m[i] = -INFINITY;
    l[i] = 0.f;
#pragma unroll
    for (int tt = 0; tt < DT; ++tt) o[i][tt] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  const int nblk_all = (Lkv + KB - 1) / KB;
  const int per = (nblk_all + nks - 1) / nks;
  const int kb0 = ks * per * KB;                   // first key of this split
  const int nblk = max(0, min(nblk_all - ks * per, per));
  constexpr int NKT = KB / 16;                     // 16-key groups per block

#pragma unroll
  for (int sb = 0; sb < NST - 1; ++sb)
    if (sb < nblk) stage(kb0 + sb * KB, sb);
  // static priority for the second-dispatched half of a 2-wave-per-SIMD workgroup (tuning knob)
  if constexpr (PG_FA_PRIO) if (WAVES >= 8 && wave >= WAVES / 2) __builtin_amdgcn_s_setprio(1);
#if PG_FA_UNROLL == 2
#pragma unroll 2
#endif
  for (int ib = 0; ib < nblk; ++ib) {
    const int kb = kb0 + ib * KB;
    // block ib has landed once at most (blocks issued after it) * P of this wave's pieces are outstanding
    wait_vm_n((min(nblk - 1, ib + NST - 2) - ib) * P);
    __builtin_amdgcn_s_barrier();                  // every wave's pieces of ib landed; block ib - 1 fully read
    if (ib + NST - 1 < nblk) stage(kb + (NST - 1) * KB, (ib + NST - 1) % NST);   // the buffer block ib - 1 used
    const char* kimg = smem + (ib % NST) * STAGE;
    const char* vimg = kimg + KIMG;
    // ---- S^T for NKT groups of 16 keys
    f32x4 sc[RPW][NKT];
#pragma unroll
    for (int i = 0; i < RPW; ++i)
#pragma unroll
      for (int kt = 0; kt < NKT; ++kt) sc[i][kt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < KS; ++s) {
#pragma unroll
      for (int kt = 0; kt < NKT; ++kt) {
        const bf16x8 kf = *(const bf16x8*)(kimg + ((kt * NCH + 4 * s + g) * 16 + c) * 16);
#pragma unroll
        for (int i = 0; i < RPW; ++i) sc[i][kt] = mfma16(kf, qf[i][s], sc[i][kt]);
      }
      // (256 rows of head_dim 256 per 8-wave workgroup: at most FA_HOIST fragment reads ahead, or the
      // hoisted reads push the wave past its 256 registers)
      if constexpr (FA_HOIST > 0) if ((s + 1) % (FA_HOIST / NKT) == 0) __builtin_amdgcn_sched_barrier(0);
    }
    // lane holds S[key = kb + 32 (kt / 2) + 8g + 4 (kt % 2) + j][q = c] of each row group
    bf16x8 pf[RPW][KB / 32];
#pragma unroll
    for (int i = 0; i < RPW; ++i) {
      // raw scores (keys past Lkv -> -inf); the scale (> 0) goes onto the max and into one packed fma per pair of
      // scores before exp2 (v_pk_fma_f32 / v_pk_add_f32: the softmax, not the MFMA, bounds head_dim 72)
      float x[4 * NKT];
#pragma unroll
      for (int kt = 0; kt < NKT; ++kt)
#pragma unroll
        for (int j = 0; j < 4; ++j) x[4 * kt + j] = sc[i][kt][j];
      if (kb + KB > Lkv) {
        // (the empty volatile asm keeps this a branch: if-converted, the ~50 compares and selects of the key mask ran
        // on every block, a third of the softmax's VALU)
        if constexpr (PG_FA_MASK_BRANCH) asm volatile("");
#pragma unroll
        for (int kt = 0; kt < NKT; ++kt)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            if (kb + 32 * (kt >> 1) + 8 * g + 4 * (kt & 1) + j >= Lkv) x[4 * kt + j] = -INFINITY;
      }
      float bm = x[0];
#pragma unroll
      for (int j = 1; j < 4 * NKT; ++j) bm = fmaxf(bm, x[j]);
      bm = max_xor16(bm);
      bm = max_xor32(bm);
      float mn = fmaxf(m[i], bm * a.scale_log2);         // = the max of the scaled scores (scaling is monotonic)
      float alpha;
      if constexpr (LAZY > 0) {
        // lazy rescale: the running max moves (and O, l are rescaled) only when some row of the wave gained more than
        // 2^PG_FA_LAZY; otherwise the exponents are taken against the stale max (P <= 2^PG_FA_LAZY: same bf16
        // relative precision, fp32 O and l).  The volatile asm keeps it a branch (if-converted, the rescale of O ran
        // on every block)
        alpha = 1.0f;
        if (__builtin_amdgcn_ballot_w64(mn > m[i] + (float)LAZY)) {
          asm volatile("");
          alpha = __builtin_amdgcn_exp2f(m[i] - mn);
#pragma unroll
          for (int tt = 0; tt < DT; ++tt) o[i][tt] *= alpha;
          m[i] = mn;
        }
        mn = m[i];
      } else {
        alpha = __builtin_amdgcn_exp2f(m[i] - mn);
      }
      const f32x2 s2 = {a.scale_log2, a.scale_log2}, n2 = {-mn, -mn};
      f32x2 rs2 = {0.f, 0.f};
#pragma unroll
      for (int j = 0; j < 4 * NKT; j += 2) {
        const f32x2 t = __builtin_elementwise_fma(f32x2{x[j], x[j + 1]}, s2, n2);
        x[j] = __builtin_amdgcn_exp2f(t[0]);
        x[j + 1] = __builtin_amdgcn_exp2f(t[1]);
        rs2 += f32x2{x[j], x[j + 1]};
      }
      float rs = rs2[0] + rs2[1];
      rs = sum_xor16(rs);
      rs = sum_xor32(rs);
      l[i] = l[i] * alpha + rs;
      if constexpr (LAZY == 0) {
        m[i] = mn;
        if (__builtin_amdgcn_ballot_w64(alpha != 1.0f)) {   // a row's max moved: rescale O
#pragma unroll
          for (int tt = 0; tt < DT; ++tt) o[i][tt] *= alpha;
        }
      }
      // P^T operand of the 32-key steps; slot 8g+j <-> key 32h + 8g + j
#pragma unroll
      for (int h = 0; h < KB / 32; ++h) {
        u32x4 pw;
        pw[0] = pack_bf2(x[8 * h + 0], x[8 * h + 1]);
        pw[1] = pack_bf2(x[8 * h + 2], x[8 * h + 3]);
        pw[2] = pack_bf2(x[8 * h + 4], x[8 * h + 5]);
        pw[3] = pack_bf2(x[8 * h + 6], x[8 * h + 7]);
        pf[i][h] = __builtin_bit_cast(bf16x8, pw);
      }
    }
    // ---- O^T += V^T . P^T: one V^T fragment read feeds the RPW row groups
#pragma unroll
    for (int h = 0; h < KB / 32; ++h) {
#pragma unroll
      for (int tt = 0; tt < DT; ++tt) {
        const int row = 16 * tt + c;
        const char* vr = vimg + row * VROW;
        const int sw = KB == 64 ? (row >> 1) & 7 : (row >> 2) & 2;
        const bf16x8 vf = *(const bf16x8*)(vr + ((4 * h + g) ^ sw) * 16);   // keys 32h + 8g .. + 7
#pragma unroll
        for (int i = 0; i < RPW; ++i) o[i][tt] = mfma16(vf, pf[i][h], o[i][tt]);
        if constexpr (FA_HOIST > 0) if ((tt + 1) % FA_HOIST == 0) __builtin_amdgcn_sched_barrier(0);
      }
    }
  }
  if (nks > 1) {
    // unnormalised O and the row's (m, l) of this key split
#pragma unroll
    for (int i = 0; i < RPW; ++i) {
      if (!rvalid[i]) continue;
      const long prow = (((long)b * a.Hkv + kvh) * nks + ks) * R + rrow[i];
      float* po = a.part_o + prow * (DT * 16);
#pragma unroll
      for (int tt = 0; tt < DT; ++tt) *(f32x4*)(po + 16 * tt + 4 * g) = o[i][tt];
      if (g == 0) *(f32x2*)(a.part_ml + prow * 2) = f32x2{m[i], l[i]};
    }
    return;
  }
#pragma unroll
  for (int i = 0; i < RPW; ++i) {
    if (!rvalid[i]) continue;
    const float inv = 1.0f / l[i];
    bf16_t* op = a.o + ((long)b * a.Lq + pos[i]) * a.o_rs + (long)hq[i] * D;
#pragma unroll
    for (int tt = 0; tt < DT; ++tt) {
      const int d = 16 * tt + 4 * g;
      if (d < D) {
        u32x2 p;
        p[0] = pack_bf2(o[i][tt][0] * inv, o[i][tt][1] * inv);
        p[1] = pack_bf2(o[i][tt][2] * inv, o[i][tt][3] * inv);
        *(u32x2*)(op + d) = p;
      }
    }
  }
}

// Merge the split partials: out[b][hq][d] = sum_s 2^(m_s - M) O_s / sum_s 2^(m_s - M) l_s.
// One workgroup per (b, kv head, q row of the group), one thread per d.
__global__ __launch_bounds__(256) void attn_combine_kernel(const float* __restrict__ part_o,
                                                           const float* __restrict__ part_ml, int nsplit, int G,
                                                           int Hkv, int D, int DTW, bf16_t* __restrict__ o, long o_rs) {
  const int row = blockIdx.x % G;
  const int bk = blockIdx.x / G;  // b * Hkv + kvh
  const int b = bk / Hkv, kvh = bk % Hkv;
  __shared__ float wsh[256];
  __shared__ float inv_den;
  // thread (sg, dq): dims 4dq..4dq+3, splits sg, sg+4, ...; the first PG_COMBINE_PF of its splits' O partials
  // are loaded before the (m, l) reduction (clamped addresses, discarded by a select later), so the usual
  // split count (<= 4 * PG_COMBINE_PF) costs one memory round trip instead of two
  const int dq = threadIdx.x & 63, sg = threadIdx.x >> 6;
  const bool dok = 4 * dq < D;
  const float* po = part_o + ((long)bk * nsplit * 16 + row) * DTW + 4 * (dok ? dq : 0);
  f32x4 pre[PG_COMBINE_PF > 0 ? PG_COMBINE_PF : 1];
#pragma unroll
  for (int i = 0; i < PG_COMBINE_PF; ++i) pre[i] = *(const f32x4*)(po + (long)min(sg + 4 * i, nsplit - 1) * 16 * DTW);
  // split weights 2^(m_s - M) (thread s), and the denominator
  float ms = -INFINITY, ls = 0.f;
  if ((int)threadIdx.x < nsplit) {
    const long base = ((long)bk * nsplit + threadIdx.x) * 16 + row;
    ms = part_ml[base * 2];
    ls = part_ml[base * 2 + 1];
  }
  float M = wave_max(ms);
  __shared__ float red[4];
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = M;
  __syncthreads();
  M = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  const float wgt = (ms == -INFINITY) ? 0.f : exp2f(ms - M);
  if ((int)threadIdx.x < nsplit) wsh[threadIdx.x] = wgt;
  float den = wave_sum(wgt * ls);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = den;
  __syncthreads();
  if (threadIdx.x == 0) inv_den = 1.0f / (red[0] + red[1] + red[2] + red[3]);
  __syncthreads();
  // (16-B loads, 4 independent streams per dim group, no branch around a load); the four split groups are
  // summed in LDS
  f32x4 num = {0.f, 0.f, 0.f, 0.f};
  if (dok) {
#pragma unroll
    for (int i = 0; i < PG_COMBINE_PF; ++i) {
      const int s2 = sg + 4 * i;
      const float wv = s2 < nsplit ? wsh[s2] : 0.f;
      num += wv != 0.f ? wv * pre[i] : f32x4{0.f, 0.f, 0.f, 0.f};   // empty splits hold no partials
    }
#pragma unroll 4
    for (int s2 = sg + 4 * PG_COMBINE_PF; s2 < nsplit; s2 += 4) {
      const float wv = wsh[s2];
      const f32x4 pv = *(const f32x4*)(po + (long)s2 * 16 * DTW);
      num += wv != 0.f ? wv * pv : f32x4{0.f, 0.f, 0.f, 0.f};   // empty splits hold no partials
    }
  }
  __shared__ f32x4 part_sum[3][64];
  if (sg > 0) part_sum[sg - 1][dq] = num;
  __syncthreads();
  if (sg == 0 && 4 * dq < D) {
    num += part_sum[0][dq] + part_sum[1][dq] + part_sum[2][dq];
    num *= inv_den;
    u32x2 pk;
    pk[0] = pack_bf2(num[0], num[1]);
    pk[1] = pack_bf2(num[2], num[3]);
    *(u32x2*)(o + (long)b * o_rs + (long)(kvh * G + row) * D + 4 * dq) = pk;
  }
}

// Merge the key-split prefill partials: o[b][pos][hq][d] = sum_s 2^(m_s - M) O_s / sum_s 2^(m_s - M) l_s, one thread
// per (row, 4 dims), every split's (m, l, O) loaded before the first is used.
#define PF_MAXS 8
__global__ __launch_bounds__(256) void attn_pf_combine_kernel(const float* __restrict__ part_o,
                                                              const float* __restrict__ part_ml, int nks, int R, int G,
                                                              int Hkv, int D, int DW, int Lq, bf16_t* __restrict__ o,
                                                              long o_rs, long total) {
  const long idx = (long)blockIdx.x * 256 + threadIdx.x;
  if (idx >= total) return;
  const int D4 = D >> 2;
  const int d4 = (int)(idx % D4);
  const long rowg = idx / D4;
  const int r = (int)(rowg % R);
  const long bk = rowg / R;                        // b * Hkv + kvh
  f32x2 ml[PF_MAXS];
  f32x4 ov[PF_MAXS];
#pragma unroll
  for (int s = 0; s < PF_MAXS; ++s) {
    const long prow = (bk * nks + min(s, nks - 1)) * R + r;
    ml[s] = *(const f32x2*)(part_ml + prow * 2);
    ov[s] = *(const f32x4*)(part_o + prow * DW + 4 * d4);
  }
  __builtin_amdgcn_sched_barrier(0);
  float M = -INFINITY;
#pragma unroll
  for (int s = 0; s < PF_MAXS; ++s)
    if (s < nks) M = fmaxf(M, ml[s][0]);
  float den = 0.f;
  f32x4 num = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int s = 0; s < PF_MAXS; ++s) {
    const float w = (s < nks && ml[s][0] != -INFINITY) ? exp2f(ml[s][0] - M) : 0.f;
    den += w * ml[s][1];
    num += w * ov[s];
  }
  const float inv = 1.0f / den;
  const int b = (int)(bk / Hkv), kvh = (int)(bk % Hkv);
  const int pos = r / G, hq = kvh * G + r % G;
  u32x2 p;
  p[0] = pack_bf2(num[0] * inv, num[1] * inv);
  p[1] = pack_bf2(num[2] * inv, num[3] * inv);
  *(u32x2*)(o + ((long)b * Lq + pos) * o_rs + (long)hq * D + 4 * d4) = p;
}

// Flash attention, 16-row query groups per wave.  2 (one K / V^T fragment read feeding two row groups,
// 4 waves at head_dim 256) measured 0.81x at pt-448 Gemma, 0.95x / 1.03x at SigLIP 448 / 896: default 1.
#ifndef PG_FA_RPW
#define PG_FA_RPW 1
#endif

// the deep ring of a 4-wave workgroup: 64-key blocks when >= 4 stages fit the 160 KiB of LDS, else 32-key blocks
template <int DP, int DT>
struct FaDeep {
  static constexpr int S64 = 64 * DP * 2 + DT * 16 * 128, S32 = 32 * DP * 2 + DT * 16 * 64;
  static constexpr int KB = 163840 / S64 >= 4 ? 64 : 32;
  static constexpr int N = 163840 / (KB == 64 ? S64 : S32);
  static constexpr int NST = N > 8 ? 8 : N;
};

// the ring of the 8- / 12-wave workgroups (one per CU): KB-key blocks, as many stages as fit (capped at NST8)
#ifndef PG_FA_KB8
#define PG_FA_KB8 64
#endif
#ifndef PG_FA_NST8
#define PG_FA_NST8 2
#endif
template <int DP, int DT>
struct FaWide {
  static constexpr int KB = PG_FA_KB8;
  static constexpr int S = KB * DP * 2 + DT * 16 * KB * 2;
  static constexpr int N = 163840 / S;
  static constexpr int NST = N > PG_FA_NST8 ? PG_FA_NST8 : N;
};

template <int DP, int DT>
static void launch_fa(int waves, int rpw, bool deep, dim3 grid, hipStream_t stream, const AttnArgs& a) {
  if (deep && waves == 4 && rpw == 1) {
    hipLaunchKernelGGL((attn_fa_kernel<DP, DT, 4, 1, FaDeep<DP, DT>::KB, FaDeep<DP, DT>::NST>), grid, dim3(256), 0,
                       stream, a);
    return;
  }
  if constexpr (PG_FA_RPW == 2) {
    if constexpr (DP <= 96) {       // (DP 128 at 8 x 32 rows needs > 256 registers: 1 wave / SIMD)
      if (waves == 8 && rpw == 2) {
        hipLaunchKernelGGL((attn_fa_kernel<DP, DT, 8, 2>), grid, dim3(512), 0, stream, a);
        return;
      }
    }
    if (waves == 4 && rpw == 2) {
      hipLaunchKernelGGL((attn_fa_kernel<DP, DT, 4, 2>), grid, dim3(256), 0, stream, a);
      return;
    }
  }
  if constexpr (DP == 256) {
    if (waves == 8 && rpw == 2) {
      hipLaunchKernelGGL((attn_fa_kernel<DP, DT, 8, 2, 32, PG_FA_W8R2_NST>), grid, dim3(512), 0, stream, a);
      return;
    }
    if (waves == 12) {
      hipLaunchKernelGGL((attn_fa_kernel<DP, DT, 12, 1, FaWide<DP, DT>::KB, FaWide<DP, DT>::NST>), grid, dim3(768), 0,
                         stream, a);
      return;
    }
  }
  if (waves == 8)
    hipLaunchKernelGGL((attn_fa_kernel<DP, DT, 8, 1, FaWide<DP, DT>::KB, FaWide<DP, DT>::NST>), grid, dim3(512), 0,
                       stream, a);
  else if (waves == 2)
    hipLaunchKernelGGL((attn_fa_kernel<DP, DT, 2, 1>), grid, dim3(128), 0, stream, a);
  else if (waves == 1)
    hipLaunchKernelGGL((attn_fa_kernel<DP, DT, 1, 1>), grid, dim3(64), 0, stream, a);
  else
    hipLaunchKernelGGL((attn_fa_kernel<DP, DT, 4, 1>), grid, dim3(256), 0, stream, a);
}


#define ATTN_DISPATCH(DP_, DT_)                                                             \
  if (DP == DP_ && DT == DT_) {                                                              \
    if (fa_waves)                                                                            \
      launch_fa<DP_, DT_>(fa_waves, fa_rpw, fa_deep, grid, stream, a);                       \
    else if (use_lds)                                                                        \
      hipLaunchKernelGGL((attn_lds_kernel<DP_, DT_>), grid, dim3(256), 0, stream, a);        \
    else if (split_keys > 0 && PG_ATTN_SPLIT_WAVES == 1 && D == DP_ && kcap >= 32 && PG_ATTN_WG && DP_ == 256 && \
             (split_keys == 64 || split_keys % 128 == 0)) {                                  \
      if (split_keys == 64)                                                                  \
        hipLaunchKernelGGL((attn_decode_wg_kernel<DP_, DT_, 2>), grid, dim3(128), 0, stream, a); \
      else                                                                                   \
        hipLaunchKernelGGL((attn_decode_wg_kernel<DP_, DT_, 4>), grid, dim3(256), 0, stream, a); \
    } else if (split_keys > 0 && PG_ATTN_SPLIT_WAVES == 1 && D == DP_ && kcap >= 32)         \
      hipLaunchKernelGGL((attn_decode_kernel<DP_, DT_, true>), grid, dim3(64), 0, stream, a); \
    else if (split_keys > 0 && PG_ATTN_SPLIT_WAVES == 1)                                     \
      hipLaunchKernelGGL((attn_decode_kernel<DP_, DT_, false>), grid, dim3(64), 0, stream, a); \
    else                                                                                     \
      hipLaunchKernelGGL((attn_kernel<DP_, DT_>), grid, dim3(split_keys > 0 ? 64 * PG_ATTN_SPLIT_WAVES : 64), 0, \
                         stream, a);                                                         \
    launched = true;                                                                         \
  }

// V^T rows must be readable up to key 32*ceil(Lkv/32) (pad the row by 32 elements).
// q/o row for (b, pos, head): q + (b*Lq + pos)*q_rs + head*D.  k for (b, key, kvh): k + b*k_bs + kvh*k_hs + key*k_rs.
// vt for (b, d, key, kvh): vt + b*vt_bs + kvh*vt_hs + d*vt_ds + key.  mask (optional, additive fp32): mask + b*mask_bs
// + pos*mask_rs + key.  Lkv = (lkv_dev ? *lkv_dev : 0) + Lkv.
// split_keys == 0: prefill mode (writes bf16 o).  split_keys > 0: decode mode, Lq*Hq/Hkv <= 16, nsplit partials
// (nsplit multiple of 4) to part_o / part_ml, then call pg_attn_combine.  kcap > 0 (decode): K rows and V^T
// columns [0, kcap) are readable (a static cache's Smax, a multiple of 32), so each split issues its first block's
// loads before the kv length arrives from lkv_dev; 0 = rows clamped to the kv length.  Decode with kcap > 0 and
// D a multiple of 32 reads K and V only from the decode-order copies kd / vd ([B][Hkv][kcap][D], ABI 6).
extern "C" int pg_attention(const void* q, long q_rs, void* o, long o_rs, const void* k, long k_bs, long k_hs,
                            long k_rs, const void* vt, long vt_bs, long vt_hs, long vt_ds, const float* mask,
                            long mask_bs, long mask_rs, int B, int Lq, int Lkv, const int* lkv_dev, int Hq, int Hkv,
                            int D, float scale, int split_keys, int nsplit, float* part_o, float* part_ml,
                            int kcap, const void* kd, const void* vd, hipStream_t stream) {
  PG_REQUIRE(B > 0 && Lq > 0 && Hq > 0 && Hkv > 0 && Hq % Hkv == 0 && D > 0 && D % 8 == 0 && D <= 256);
  // (split mode writes partials only: o is read by nobody, the merge is pg_attn_combine's or the o_proj prologue's)
  PG_REQUIRE(kcap >= 0 && kcap % 32 == 0 && q && (split_keys == 0 ? o != nullptr : (part_o && part_ml)));
  const int G = Hq / Hkv;
  const int DP = ((D + 31) / 32) * 32;
  const int DT = (D + 15) / 16;
  if (split_keys > 0 && kcap >= 32 && D == DP)
    PG_REQUIRE(kd && vd && ((uintptr_t)kd & 15) == 0 && ((uintptr_t)vd & 15) == 0);
  AttnArgs a{(const bf16_t*)q, q_rs, (bf16_t*)o, o_rs, (const bf16_t*)k, k_bs, k_hs, k_rs,
             (const bf16_t*)vt, vt_bs, vt_hs, vt_ds, mask, mask_bs, mask_rs,
             Lq, Lkv, G, Hkv, D, lkv_dev, scale * 1.4426950408889634f, split_keys, part_o, part_ml,
             split_keys > 0 ? kcap : 0, 0, (const bf16_t*)kd, (const bf16_t*)vd};
  dim3 grid;
  // prefill with >= 1024 one-wave workgroups: the LDS-staged kernel (64 rows per workgroup share K/V);
  // needs 16-B aligned V^T rows / batch offsets
  const long wgs16 = (long)((Lq * G + 15) / 16) * Hkv * B;
  const bool aligned = vt_ds % 8 == 0 && vt_bs % 8 == 0 && vt_hs % 8 == 0 && k_rs % 8 == 0 && k_bs % 8 == 0 &&
                       k_hs % 8 == 0 && q_rs % 8 == 0 && ((uintptr_t)q & 15) == 0 && ((uintptr_t)k & 15) == 0 &&
                       ((uintptr_t)vt & 15) == 0;
  // LDS-DMA flash kernel for every unmasked prefill; 8 waves (128 rows) per workgroup once that fills the chip
  int fa_waves = 0, fa_rpw = 1;
  bool fa_deep = false;
  // (the flash kernel stages by 32-bit offsets from a head's K / V^T base)
  const bool off32 = (unsigned long)(Lkv + 64) * (unsigned long)k_rs * 2ul < (1ul << 32) &&
                     (unsigned long)D * (unsigned long)vt_ds * 2ul < (1ul << 32);
  if (split_keys == 0 && mask == nullptr && aligned && off32 && lkv_dev == nullptr && PG_ATTN_FA) {
    auto wgs = [&](int rows) { return (long)((Lq * G + rows - 1) / rows) * Hkv * B; };
    // two 16-row groups per wave (half the LDS fragment reads per flop) when the grid still fills the chip:
    // 8 waves x 32 rows for head_dim <= 96, else 4 waves x 32 rows (their accumulators need 1 wave / SIMD)
    auto rounds = [&](int rows) { return (wgs(rows) + 255) / 256; };
    // head_dim 256, 8 waves x 32 rows on 32-key blocks (twice the flops per LDS fragment read of 16-row waves, two
    // waves per SIMD at 256 registers): one round costs ~1.55 of an 8 x 16-row round (pt-896 x32 Gemma 5.03 vs
    // 6.29 ms), so it is taken where its rounds cost less than those of the 8- and 12-wave forms (pt-448 x16 keeps
    // 12 waves: 3 rounds of 256 rows cost more than 3 of 192)
    if (PG_FA_W8R2 && DP == 256 && wgs(256) >= 256 &&
        rounds(256) * 25 < rounds(128) * 16 && (!PG_FA_W12 || rounds(256) * 25 < rounds(192) * 24)) {
      fa_waves = 8;
      fa_rpw = 2;
    } else if (PG_FA_RPW == 2 && DP <= 96 && wgs(256) >= 256) {
      fa_waves = 8;
      fa_rpw = 2;
    } else if (PG_FA_RPW == 2 && wgs(128) >= 256) {
      fa_waves = 4;
      fa_rpw = 2;
    } else {
      fa_waves = wgs(128) >= 256 ? 8 : 4;
      // head_dim 256 (166 VGPRs, fits 3 waves / SIMD): 12 waves when the one-workgroup-per-CU rounds cost
      // less in total (pt-448 x16 Gemma: 688 workgroups in 3 rounds of 192 rows vs 1040 in 5 rounds of 128)
      if (PG_FA_W12 && DP == 256 && fa_waves == 8 && ((wgs(192) + 255) / 256) * 12 < ((wgs(128) + 255) / 256) * 8) fa_waves = 12;
      // batch 1 (pt-224: Gemma 2112 stacked rows on one kv head = 33 four-wave workgroups, SigLIP 16 heads x 256
      // rows = 64): narrower workgroups spread the same rows over 2-4x the CUs; each stages its own K / V^T copy
      // from L2 (the whole prefix is a few hundred KB)
      if (PG_FA_SMALL && fa_waves == 4 && wgs(64) < 256) fa_waves = wgs(32) >= 256 ? 2 : 1;
    }
    const int rows = 16 * fa_waves * fa_rpw;
    grid = dim3((Lq * G + rows - 1) / rows, Hkv, B);
    fa_deep = PG_FA_DEEP && fa_waves == 4 && fa_rpw == 1;
    if (nsplit > 1) {
      // prefill key split (caller's workspace: part_o [B][Hkv][nsplit][Lq*G][DT*16] fp32, part_ml [..][2])
      PG_REQUIRE(nsplit <= PF_MAXS && part_o && part_ml && D % 4 == 0);
      a.pf_splits = nsplit;
      grid.x *= nsplit;
    }
  } else if (split_keys == 0) {
    PG_REQUIRE(nsplit <= 1);                       // key splits need the flash kernel's shape conditions
  }
  const bool use_lds = fa_waves == 0 && split_keys == 0 && wgs16 >= 1024 && aligned;
  if (fa_waves) {
  } else if (use_lds) {
    grid = dim3((Lq * G + 63) / 64, Hkv, B);
  } else if (split_keys > 0) {
    PG_REQUIRE(Lq * G <= 16 && nsplit % 4 == 0 && part_o && part_ml && split_keys % 32 == 0);
    // a lane reads 8 consecutive keys of a V^T row as one 16-B load (dec_krow)
    PG_REQUIRE(vt_ds % 8 == 0 && vt_bs % 8 == 0 && vt_hs % 8 == 0 && ((uintptr_t)vt & 15) == 0);
    grid = dim3(1, Hkv * (nsplit / PG_ATTN_SPLIT_WAVES), B);
  } else {
    grid = dim3((Lq * G + 15) / 16, Hkv, B);   // one wave (16 query rows) per workgroup: 4x the workgroups
  }
  bool launched = false;
  ATTN_DISPATCH(32, 1)
  ATTN_DISPATCH(32, 2)     // head_dim 24 / 32 (test configs)
  ATTN_DISPATCH(64, 3)
  ATTN_DISPATCH(64, 4)
  ATTN_DISPATCH(96, 5)     // SigLIP head_dim 72
  ATTN_DISPATCH(96, 6)
  ATTN_DISPATCH(128, 8)
  ATTN_DISPATCH(256, 16)   // Gemma head_dim 256
  if (!launched) return (int)hipErrorInvalidValue;
  PG_LAUNCH_CHECK();
  if (a.pf_splits > 1) {
    const long total = (long)B * Hkv * Lq * G * (D / 4);
    hipLaunchKernelGGL(attn_pf_combine_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, stream, part_o,
                       part_ml, nsplit, Lq * G, G, Hkv, D, DT * 16, Lq, (bf16_t*)o, o_rs, total);
    PG_LAUNCH_CHECK();
  }
  return 0;
}

extern "C" int pg_attn_combine(const float* part_o, const float* part_ml, int B, int Hq, int Hkv, int D, int nsplit,
                               void* o, long o_rs, hipStream_t stream) {
  PG_REQUIRE(part_o && part_ml && o && B > 0 && Hq > 0 && Hkv > 0 && Hq % Hkv == 0 && Hq / Hkv <= 16 && nsplit >= 1 &&
             nsplit <= 256 && D > 0);
  const int DT = (D + 15) / 16;
  PG_REQUIRE(D <= 256 && D % 4 == 0 && o_rs % 4 == 0 && ((uintptr_t)o & 7) == 0 && nsplit <= 256);
  hipLaunchKernelGGL(attn_combine_kernel, dim3(B * Hq), dim3(256), 0, stream, part_o, part_ml, nsplit, Hq / Hkv,
                     Hkv, D, DT * 16, (bf16_t*)o, o_rs);
  PG_LAUNCH_CHECK();
  return 0;
}

// Batched split-KV decode with the merge in the same launch (attn_decode_fused_kernel): o[b][hq][:] (bf16, row stride
// o_rs per batch row) from q (one position per batch row) over the decode-order cache copies kd / vd ([B][Hkv][kcap][D],
// dec_koff / dec_voff) and the device kv length Lkv + *lkv_dev.  The kcap / 32 blocks of 32 keys are dealt to nsplit
// splits per (batch, kv head) in granules of nw (2 or 4) blocks, nb rounds each (nw * nsplit <= kcap / 32 <=
// nw * nsplit * nb); workspace part_o [B][Hkv][nsplit][16][D], part_ml [B][Hkv][nsplit][16][2] fp32; counters int32
// [B * Hkv], zero before the first call (every call leaves them zero).  head_dim 32 or 256, D == head_dim.
extern "C" int pg_attn_decode(const void* q, long q_rs, void* o, long o_rs, const void* kd, const void* vd, int B,
                              int Lkv, const int* lkv_dev, int Hq, int Hkv, int D, float scale, int kcap, int nsplit,
                              int nw, int nb, float* part_o, float* part_ml, int* counters, void* q8,
                              float* q8_scale, long q8_ld, hipStream_t stream) {
  PG_REQUIRE(q && B > 0 && Hq > 0 && Hkv > 0 && Hq % Hkv == 0 && Hq / Hkv <= 16 && (D == 32 || D == 256));
  const bool pipe = (nw & PG_ATTN_PIPE) != 0 && nb >= 2;      // the double-buffered form (head_dim 256, 4 waves)
  nw &= ~PG_ATTN_PIPE;
  // the fp8 copy: the merging workgroup holds the whole row (one kv head, one item per thread)
  if (q8) PG_REQUIRE(Hkv == 1 && Hq * (D / 8) <= nw * 64 && q8_scale && q8_ld >= (long)Hq * D && q8_ld % 8 == 0 &&
                     ((uintptr_t)q8 & 7) == 0);
  PG_REQUIRE((nw == 2 || nw == 4) && kcap % 32 == 0 && nsplit >= 1 && nw * nsplit <= kcap / 32 && nb >= 1 &&
             nsplit * nw * nb >= kcap / 32 && part_o && part_ml && counters && o && lkv_dev && kd && vd);
  PG_REQUIRE((long)B * Hkv * nsplit * 16 * D * 4 < 0x7fffffffL);
  PG_REQUIRE(q_rs % 8 == 0 && o_rs % 8 == 0 && ((uintptr_t)q & 15) == 0 && ((uintptr_t)kd & 15) == 0 &&
             ((uintptr_t)vd & 15) == 0 && ((uintptr_t)o & 15) == 0);
  AttnArgs a{(const bf16_t*)q, q_rs, (bf16_t*)o, o_rs, nullptr, 0, 0, 0, nullptr, 0, 0, 0, nullptr, 0, 0,
             1, Lkv, Hq / Hkv, Hkv, D, lkv_dev, scale * 1.4426950408889634f, 32 * 4 * nb, part_o, part_ml, kcap, 0,
             (const bf16_t*)kd, (const bf16_t*)vd};
  const dim3 grid(nsplit, Hkv, B);
#define PG_DEC_LAUNCH(DP_, DT_, NW_, PIPE_)                                                                 \
  hipLaunchKernelGGL((attn_decode_fused_kernel<DP_, DT_, NW_, PIPE_>), grid, dim3(NW_ * 64), 0, stream, a, nb, \
                     counters, (uint8_t*)q8, q8_scale, q8_ld)
  if (D == 256 && nw == 4 && pipe)
    PG_DEC_LAUNCH(256, 16, 4, true);
  else if (D == 256 && nw == 4)
    PG_DEC_LAUNCH(256, 16, 4, false);
  else if (D == 256)
    PG_DEC_LAUNCH(256, 16, 2, false);
  else if (nw == 4)
    PG_DEC_LAUNCH(32, 2, 4, false);
  else
    PG_DEC_LAUNCH(32, 2, 2, false);
#undef PG_DEC_LAUNCH
  PG_LAUNCH_CHECK();
  return 0;
}

// The attention weights the reference's modules return, for callers of the module API that read them: probs = 1
// (modeling_gemma.py:358) the softmax(Q K^T * scale + mask) probabilities, probs = 0 (modeling_siglip.py:157, which
// returns its scores from before the softmax) the scaled scores (+ mask), fp32.  Not on the hot path -- the flash
// kernels never form this matrix.  One 256-thread workgroup per (b, q head, query row): the q row in LDS as fp32,
// each thread a key at a time (fp32 dot product of the bf16 q / k rows), then the row max, exp and sum as
// workgroup reductions; out[((b * Hq + hq) * Lq + pos) * Lkv + key].
__global__ __launch_bounds__(256) void attn_probs_kernel(const bf16_t* __restrict__ q, long q_rs,
                                                         const bf16_t* __restrict__ k, long k_bs, long k_hs, long k_rs,
                                                         const float* __restrict__ mask, long mask_bs, long mask_rs,
                                                         int Lq, int Lkv, int Hq, int Hkv, int D, float scale,
                                                         int probs, float* __restrict__ out) {
  __shared__ float qs[256];
  __shared__ float red[8];
  const int pos = blockIdx.x, hq = blockIdx.y, b = blockIdx.z, t = threadIdx.x;
  const int kvh = hq / (Hq / Hkv);
  const bf16_t* qr = q + ((long)b * Lq + pos) * q_rs + (long)hq * D;
  for (int d = t; d < D; d += 256) qs[d] = bf2f(qr[d]);
  __syncthreads();
  const bf16_t* kb = k + (long)b * k_bs + (long)kvh * k_hs;
  const float* mr = mask ? mask + (long)b * mask_bs + (long)pos * mask_rs : nullptr;
  float* orow = out + (((long)b * Hq + hq) * Lq + pos) * Lkv;
  auto block_reduce = [&](float v, bool is_max) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const float w = __shfl_xor(v, o, 64);
      v = is_max ? fmaxf(v, w) : v + w;
    }
    if ((t & 63) == 0) red[t >> 6] = v;
    __syncthreads();
    float r = red[0];
    for (int i = 1; i < 4; ++i) r = is_max ? fmaxf(r, red[i]) : r + red[i];
    __syncthreads();
    return r;
  };
  float mx = -INFINITY;
  for (int j = t; j < Lkv; j += 256) {
    const bf16_t* kr = kb + (long)j * k_rs;
    float acc = 0.f;
    for (int d = 0; d < D; ++d) acc += qs[d] * bf2f(kr[d]);
    const float sc = acc * scale + (mr ? mr[j] : 0.f);
    orow[j] = sc;
    mx = fmaxf(mx, sc);
  }
  if (!probs) return;
  mx = block_reduce(mx, true);
  float sum = 0.f;
  for (int j = t; j < Lkv; j += 256) {
    const float e = __expf(orow[j] - mx);
    orow[j] = e;
    sum += e;
  }
  const float inv = 1.0f / block_reduce(sum, false);
  for (int j = t; j < Lkv; j += 256) orow[j] *= inv;
}

extern "C" int pg_attn_probs(const void* q, long q_rs, const void* k, long k_bs, long k_hs, long k_rs, const float* mask,
                             long mask_bs, long mask_rs, int B, int Lq, int Lkv, int Hq, int Hkv, int D, float scale,
                             int probs, float* out, hipStream_t stream) {
  PG_REQUIRE(q && k && out && B > 0 && Lq > 0 && Lkv > 0 && Hq > 0 && Hkv > 0 && Hq % Hkv == 0 && D > 0 && D <= 256);
  PG_REQUIRE(Lq <= 65535 * 32 && Hq <= 65535 && B <= 65535);
  hipLaunchKernelGGL(attn_probs_kernel, dim3(Lq, Hq, B), dim3(256), 0, stream, (const bf16_t*)q, q_rs,
                     (const bf16_t*)k, k_bs, k_hs, k_rs, mask, mask_bs, mask_rs, Lq, Lkv, Hq, Hkv, D, scale, probs, out);
  PG_LAUNCH_CHECK();
  return 0;
}

#if PG_ATTN_STAMPS
// diagnostic variant only (not in the product library): copy the decode-split stamps to the host
extern "C" int pg_attn_stamps_read(void* host, int n) {
  return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(pg_attn_stamp_buf), (size_t)n * 32, 0, hipMemcpyDeviceToHost);
}
#endif
