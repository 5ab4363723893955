// Decode MLP engine: the gate/up and down GEMVs of one Gemma decoder layer (batch 1) as ONE persistent launch
// built the way the MI355X guide's weight-streaming engine is (§5.6; price list rows ldsdma-fill, prefetch-credit,
// handoff-1to1, allgather): per CU one workgroup of two waves --
//   wave 0, the LOADER: streams the CU's weight slices HBM -> LDS with LDS-DMA (global_load_lds, 16 B per lane,
//     non-temporal) into a ring of EN_NS 16 KiB slots, EN_INFL fills in flight, each published behind a counted
//     vmcnt through a FULL word in LDS; it never waits on data, only on ring space (a FREE word per slot), so
//     the down projection's weights stream while the h hand-off is in flight;
//   wave 1, the CONSUMER: MFMAs over the slots (fragment-packed weights land in LDS in exactly the register
//     image the decode GEMV uses), the epilogues, and the hand-offs.  It issues no weight loads, so its
//     hand-off loads never wait behind the stream in its own vmcnt order.
// Work per CU c (256 CUs, Gemma-2B: H 2048, I 16384):
//   gate/up: tile pairs 4c .. 4c+3 (gate tile + up tile, 16 rows x 2048 k each = 4 fills per tile) ->
//     h[64c .. 64c+64) = gelu(rstd * gate) * (rstd * up), published as 8-byte granules {2 x bf16, tag}
//     (write-through), the tag being this launch's epoch;
//   down: rows [16t, 16t+16) over k-half z (t = c / 2, z = c % 2): gathers the 4096 granules of h half z
//     (sweeps until every tag matches), 16 fills of 16 rows x 512 k, and the tile's second-arriving half adds
//     both halves into the residual in half order and writes x' = bf16(resid * (1 + norm_w)) and the tile's
//     sum of squares (the PG_EPI_F32_FIN contract the next GEMV reads).
// Replaces GemmaMLP.forward (modeling_gemma.py:210-218) + the residual add (:413-418) of a decode step, i.e.
// pg_gemm_fused(gate/up, pro 4) + pg_gemm_fused(down, PG_EPI_F32_FIN) at batch 1.  Every spin is bounded by the
// wall clock (sync[EN_ERR] = 1 on a timeout; the outputs are then meaningless); the launch is refused unless one
// workgroup per CU covers the grid.
#include "attn_common.h"

#ifndef PG_EN_TIMEOUT_TICKS
#define PG_EN_TIMEOUT_TICKS 20000000ull    // 0.2 s of the 100 MHz constant clock
#endif
#ifndef PG_EN_INFL
#define PG_EN_INFL 4                        // fills in flight per loader (64 KiB per CU)
#endif
#ifndef PG_EN_THIN
#define PG_EN_THIN 0                        // loader keeps one fill in flight while the consumer gathers h
#endif
#ifndef PG_EN_GSLEEP
#define PG_EN_GSLEEP 2                      // s_sleep between gather sweeps
#endif
#define EN_NS 8                             // ring slots
#define EN_SLOT 16384                       // bytes per slot: 16 rows x 512 k bf16 (8 fragment chunks)
#define EN_H 2048
#define EN_I 16384
#define EN_CUS 256
#define EN_NF_GU 32                         // 4 pairs x 2 tiles x 4 fills
#define EN_NF_D 16                          // 16 rows x 8192 k
#define EN_NF (EN_NF_GU + EN_NF_D)
#define EN_EPOCH 0                          // sync words, each on a 256-B line of its own
#define EN_DONE 64
#define EN_ERR 128
#define EN_SYNC_INTS 192

struct MlpEngineArgs {
  const bf16_t* xq;              // [1][H] x' of the post-attention RMSNorm (o_proj F32_FIN, previous launch)
  const float* ss_in;            // [ss_n] its per-tile sums of squares
  int ss_n;
  float eps;
  const bf16_t* wgu;             // [2I][H] fragment-packed, gate / up interleaved in 16-row blocks
  const bf16_t* wd;              // [H][I] fragment-packed
  unsigned long long* hgran;     // [I / 2] granules {lo: bf16 pair, hi: tag}
  float* slab;                   // [2][H] down k-half partials (write-through)
  int* fin_cnt;                  // [H / 16] tickets, zero between launches (the second arriver resets)
  float* resid;                  // [1][H]
  float* ss_out;                 // [H / 16]
  bf16_t* fin_x;                 // [1][H] (may be null)
  const float* norm_w;           // next RMSNorm weight (with fin_x)
  int* sync;                     // [EN_SYNC_INTS] zeroed once: epoch, done, err
  unsigned long long* stamps;    // diagnostics: [CU][8] wall-clock stamps, or null
};

typedef __attribute__((address_space(1))) unsigned long long en_gu64;

static unsigned long long* g_en_stamps = nullptr;
extern "C" int pg_decode_mlp_engine_stamps(void* buf) {
  g_en_stamps = (unsigned long long*)buf;
  return 0;
}

__device__ __forceinline__ bool en_timed_out(unsigned long long t0, int* sync) {
  if (wall_clock64() - t0 <= PG_EN_TIMEOUT_TICKS) return false;
  __hip_atomic_store(sync + EN_ERR, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return true;
}

// The loader's ring words go through inline-asm LDS accesses: with LDS-DMA in flight, hipcc puts a vmcnt(0) in
// front of every ordinary LDS access of that wave (it cannot tell the ring words from the DMA destinations), which
// would drain the whole ring at each fill.  An asm statement is opaque to the waitcnt pass.
__device__ __forceinline__ unsigned en_lds_addr(const int* p) { return (unsigned)(size_t)(LDS_AS const int*)p; }
__device__ __forceinline__ int en_lds_load(unsigned addr) {
  int v;
  asm volatile("ds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(addr) : "memory");
  return __builtin_amdgcn_readfirstlane(v);
}
__device__ __forceinline__ void en_lds_store(unsigned addr, int v) {
  asm volatile("ds_write_b32 %0, %1" ::"v"(addr), "v"(v) : "memory");
}

// source of fill f of CU c (elements of bf16)
__device__ __forceinline__ const bf16_t* en_fill_src(const MlpEngineArgs& a, int c, int f) {
  if (f < EN_NF_GU) {
    const int p = f >> 3, half = (f >> 2) & 1, q = f & 3;
    const size_t tile = (size_t)2 * (4 * c + p) + half;
    return a.wgu + tile * 16 * EN_H + (size_t)q * 8 * 1024;
  }
  const int d = f - EN_NF_GU, t = c >> 1, z = c & 1;
  return a.wd + (size_t)t * 16 * EN_I + (size_t)(128 * z + 8 * d) * 1024;
}

__global__ __launch_bounds__(128) void mlp_engine_kernel(MlpEngineArgs a) {
  __shared__ __attribute__((aligned(1024))) char ring[EN_NS * EN_SLOT];
  __shared__ __attribute__((aligned(16))) bf16_t xg[EN_H];
  __shared__ __attribute__((aligned(16))) unsigned xd[EN_I / 4];      // h half: 8192 bf16 as pairs
  __shared__ int fullw[EN_NS], freew[EN_NS], gathw[1];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int c = blockIdx.x;
  unsigned long long* stamp = a.stamps ? a.stamps + (size_t)c * 8 : nullptr;
  if (threadIdx.x < EN_NS) {
    fullw[threadIdx.x] = 0;
    freew[threadIdx.x] = 0;
  }
  if (threadIdx.x == 0) gathw[0] = 0;
  __syncthreads();
  const unsigned long long t0 = wall_clock64();
  if (stamp && threadIdx.x == 0) stamp[0] = t0;

  if (wave == 0) {
    // ------------------------------------------------------------------ loader
    int pub = 0;                                               // fills published so far
    auto publish = [&](int upto) {
      if (lane == 0)
        for (int k = pub; k < upto; ++k) en_lds_store(en_lds_addr(&fullw[k % EN_NS]), k + 1);
      pub = upto;
    };
    for (int f = 0; f < EN_NF; ++f) {
      const int slot = f % EN_NS;
      if (f >= EN_NS) {
        while (en_lds_load(en_lds_addr(&freew[slot])) < f - EN_NS + 1) {
          if (en_timed_out(t0, a.sync)) break;
          __builtin_amdgcn_s_sleep(1);
        }
      }
      const bf16_t* src = en_fill_src(a, c, f) + lane * 8;
      char* dst = ring + slot * EN_SLOT;
#pragma unroll
      for (int i = 0; i < 16; ++i)
        __builtin_amdgcn_global_load_lds((const void*)(src + i * 512), (LDS_AS void*)(dst + i * 1024), 16, 0, 2);
      if (PG_EN_THIN && en_lds_load(en_lds_addr(&gathw[0])) != 0) {
        // the consumer is gathering h: one fill in flight, so its hand-off loads do not queue behind the ring
        asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
        publish(f);
      } else if (f >= PG_EN_INFL - 1) {
        // fill f - (INFL - 1) has landed once at most (INFL - 1) fills' 16 loads each are outstanding
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(16 * (PG_EN_INFL - 1)) : "memory");
        publish(max(pub, f - PG_EN_INFL + 2));
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    publish(EN_NF);
    return;
  }

  // -------------------------------------------------------------------- consumer (wave 1)
  const int g = lane >> 4, r = lane & 15;
  const unsigned tag = (unsigned)a.sync[EN_EPOCH] + 1u;       // this launch's epoch (previous launch's value + 1)
  // gate/up input: x' into LDS, rstd from the producer's per-tile sums
  {
    const u32x4* xs = (const u32x4*)a.xq;
#pragma unroll
    for (int i = 0; i < 4; ++i) ((u32x4*)xg)[lane + 64 * i] = xs[lane + 64 * i];
  }
  float ss = 0.f;
  for (int i = lane; i < a.ss_n; i += 64) ss += a.ss_in[i];
  ss = wave_sum(ss);
  const float rs = rsqrtf(ss / (float)EN_H + a.eps);
  // the down tile's residual and next-norm weight (previous launch's data; the finaliser uses them)
  const int t = c >> 1, z = c & 1;
  const int n0 = t * 16 + 4 * g;
  const f32x4 fin_r = *(const f32x4*)(a.resid + n0);
  const f32x4 fin_w = *(const f32x4*)((a.norm_w ? a.norm_w : a.resid) + n0);
  __builtin_amdgcn_s_waitcnt(0);
  __builtin_amdgcn_wave_barrier();

  auto wait_full = [&](int f) {
    const int slot = f % EN_NS;
    while (__hip_atomic_load(&fullw[slot], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < f + 1) {
      if (en_timed_out(t0, a.sync)) break;
      __builtin_amdgcn_s_sleep(0);
    }
  };
  auto release = [&](int f) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");        // the slot's fragments are in registers
    if (lane == 0) __hip_atomic_store(&freew[f % EN_NS], f + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  };

  // ---- gate/up: 4 pairs, 8 fills each (4 gate, 4 up)
#pragma unroll 1
  for (int p = 0; p < 4; ++p) {
    f32x4 acc[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int f = 8 * p + q;
      wait_full(f);
      const char* sb = ring + (f % EN_NS) * EN_SLOT;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int cg = (q & 3) * 8 + j;                           // 64-k chunk along H
        const bf16x8 w0 = *(const bf16x8*)(sb + (2 * j) * 1024 + lane * 16);
        const bf16x8 w1 = *(const bf16x8*)(sb + (2 * j + 1) * 1024 + lane * 16);
        const bf16x8 x0 = *(const bf16x8*)(xg + 64 * cg + 16 * g);
        const bf16x8 x1 = *(const bf16x8*)(xg + 64 * cg + 16 * g + 8);
        acc[q >> 2] = mfma16(w0, x0, acc[q >> 2]);
        acc[q >> 2] = mfma16(w1, x1, acc[q >> 2]);
      }
      release(f);
    }
    // lane (r, g) holds rows 4g .. 4g+3 of the gate / up tiles (every r the same: x is one row)
    if (r == 0) {
      const f32x4 gt = acc[0] * rs, up = acc[1] * rs;
      const unsigned h01 = pack_bf2(gelu_tanh(gt[0]) * up[0], gelu_tanh(gt[1]) * up[1]);
      const unsigned h23 = pack_bf2(gelu_tanh(gt[2]) * up[2], gelu_tanh(gt[3]) * up[3]);
      const size_t gi = (size_t)(16 * (4 * c + p) + 4 * g) / 2;
      __hip_atomic_store((en_gu64*)(a.hgran + gi), ((unsigned long long)tag << 32) | h01, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store((en_gu64*)(a.hgran + gi + 1), ((unsigned long long)tag << 32) | h23, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  if (stamp && lane == 0) stamp[1] = wall_clock64();

  // ---- down: 16 fills of 16 rows x 512 k over h half z.  Fill d needs only the 512 h values [512 d, 512 d + 512) of
  // the half, i.e. 256 granules from 8 producer CUs: they are gathered per fill (4 per lane, the next fill's loads
  // in flight while this one computes), so a fill starts as soon as ITS producers have published (all 16 fills'
  // loads at once measured slower: 1.24 vs 1.17 ms/token -- every stale re-read then waits for all of them)
  const en_gu64* hsrc = (const en_gu64*)a.hgran + (size_t)4096 * z;
  const bf16_t* xdb = (const bf16_t*)xd;
  unsigned long long hv[2][4];
  auto gather_issue = [&](int d, unsigned long long (&v)[4]) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
      v[i] = __hip_atomic_load(hsrc + 256 * d + 64 * i + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  };
  gather_issue(0, hv[0]);
  f32x4 ad = {0.f, 0.f, 0.f, 0.f};
#pragma unroll 2
  for (int d = 0; d < EN_NF_D; ++d) {
    unsigned long long (&v)[4] = hv[d & 1];
    // complete fill d's granules: re-read the stale ones until every tag is this launch's
    while (true) {
      bool stale = false;
#pragma unroll
      for (int i = 0; i < 4; ++i) stale |= (unsigned)(v[i] >> 32) != tag;
      if (!__builtin_amdgcn_ballot_w64(stale)) break;
      if (en_timed_out(t0, a.sync)) break;
      __builtin_amdgcn_s_sleep(PG_EN_GSLEEP);
#pragma unroll
      for (int i = 0; i < 4; ++i)
        if ((unsigned)(v[i] >> 32) != tag)
          v[i] = __hip_atomic_load(hsrc + 256 * d + 64 * i + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (d + 1 < EN_NF_D) gather_issue(d + 1, hv[(d + 1) & 1]);
#pragma unroll
    for (int i = 0; i < 4; ++i) xd[256 * d + 64 * i + lane] = (unsigned)v[i];
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (d == 0 && stamp && lane == 0) stamp[2] = wall_clock64();
    const int f = EN_NF_GU + d;
    wait_full(f);
    const char* sb = ring + (f % EN_NS) * EN_SLOT;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int cl = 8 * d + j;                                   // 64-k chunk within the half
      const bf16x8 w0 = *(const bf16x8*)(sb + (2 * j) * 1024 + lane * 16);
      const bf16x8 w1 = *(const bf16x8*)(sb + (2 * j + 1) * 1024 + lane * 16);
      const bf16x8 x0 = *(const bf16x8*)(xdb + 64 * cl + 16 * g);
      const bf16x8 x1 = *(const bf16x8*)(xdb + 64 * cl + 16 * g + 8);
      ad = mfma16(w0, x0, ad);
      ad = mfma16(w1, x1, ad);
    }
    release(f);
  }
  if (stamp && lane == 0) stamp[3] = wall_clock64();

  // ---- this half's partial (write-through), ticket; the second half finalises the tile in half order
  if (r == 0) {
    en_gu64* dst = (en_gu64*)(a.slab + (size_t)z * EN_H + n0);
    __hip_atomic_store(dst, __builtin_bit_cast(unsigned long long, f32x2{ad[0], ad[1]}), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(dst + 1, __builtin_bit_cast(unsigned long long, f32x2{ad[2], ad[3]}), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  int old = 0;
  if (lane == 0) old = __hip_atomic_fetch_add(a.fin_cnt + t, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  old = __shfl(old, 0, 64);
  if (old == 1) {
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");      // compiler-only: keep the loads below the ticket
    float ssl = 0.f;
    if (r == 0) {
      f32x4 v = fin_r;
#pragma unroll
      for (int zz = 0; zz < 2; ++zz) {
        const en_gu64* s = (const en_gu64*)(a.slab + (size_t)zz * EN_H + n0);
        const f32x2 lo = __builtin_bit_cast(f32x2, __hip_atomic_load(s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
        const f32x2 hi = __builtin_bit_cast(f32x2, __hip_atomic_load(s + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
        v += f32x4{lo[0], lo[1], hi[0], hi[1]};
      }
      *(f32x4*)(a.resid + n0) = v;
      ssl = v[0] * v[0] + v[1] * v[1] + v[2] * v[2] + v[3] * v[3];
      if (a.fin_x) {
        u32x2 pk;
        pk[0] = pack_bf2(v[0] * (1.0f + fin_w[0]), v[1] * (1.0f + fin_w[1]));
        pk[1] = pack_bf2(v[2] * (1.0f + fin_w[2]), v[3] * (1.0f + fin_w[3]));
        *(u32x2*)(a.fin_x + n0) = pk;
      }
    }
    ssl += __shfl_xor(ssl, 16, 64);
    ssl += __shfl_xor(ssl, 32, 64);
    if (lane == 0) {
      a.ss_out[t] = ssl;
      __hip_atomic_store(a.fin_cnt + t, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  if (lane == 0) {
    // every wait of this CU is over: the last CU to get here advances the epoch for the next launch
    if (__hip_atomic_fetch_add(a.sync + EN_DONE, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == EN_CUS - 1) {
      __hip_atomic_store(a.sync + EN_EPOCH, (int)tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(a.sync + EN_DONE, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (stamp) stamp[4] = wall_clock64();
  }
}

// hgran: I/2 u64 (any content: stale tags are never this launch's); slab: 2*H fp32; fin_cnt: H/16 zeroed ints;
// sync: EN_SYNC_INTS zeroed ints.  Batch 1, Gemma-2B shapes only; hipErrorNotSupported (nothing launched) when
// this device cannot hold one workgroup on each of 256 CUs at once.
extern "C" int pg_decode_mlp_engine(const void* xq, const float* ss_in, int ss_n, float eps, const void* wgu,
                                    const void* wd, void* hgran, float* slab, int* fin_cnt, float* resid,
                                    float* ss_out, void* fin_x, const float* norm_w, int* sync, int M, int H, int I,
                                    hipStream_t stream) {
  PG_REQUIRE(xq && ss_in && wgu && wd && hgran && slab && fin_cnt && resid && ss_out && sync);
  PG_REQUIRE(ss_n > 0 && (fin_x == nullptr || norm_w != nullptr));
  if (M != 1 || H != EN_H || I != EN_I) return (int)hipErrorNotSupported;
  static int ok = -1;
  if (ok < 0) {
    int nb = 0, dev = 0, cus = 0;
    ok = hipGetDevice(&dev) == hipSuccess &&
         hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess &&
         hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, mlp_engine_kernel, 128, 0) == hipSuccess && nb >= 1 &&
         cus == EN_CUS;
  }
  if (!ok) return (int)hipErrorNotSupported;
  MlpEngineArgs a{(const bf16_t*)xq, ss_in, ss_n, eps, (const bf16_t*)wgu, (const bf16_t*)wd,
                  (unsigned long long*)hgran, slab, fin_cnt, resid, ss_out, (bf16_t*)fin_x, norm_w, sync, g_en_stamps};
  hipLaunchKernelGGL(mlp_engine_kernel, dim3(EN_CUS), dim3(128), 0, stream, a);
  PG_LAUNCH_CHECK();
  return 0;
}
