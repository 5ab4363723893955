// Decode MLP block: the gate/up GEMV (RMSNorm folded in, gelu(gate) * up) and the down GEMV (split-K, residual
// add + the next RMSNorm's statistics) of one Gemma decoder layer as ONE launch, batch <= 2.
// Replaces GemmaMLP.forward (modeling_gemma.py:210-218) and the decoder layer's second residual add
// (modeling_gemma.py:413-418) for a decode step; the arithmetic is that of the two launches
// gemv_kernel<GELU_MUL, PRO 4> + gemv_kernel<F32_FIN> (csrc/gemm.hip) with the down projection split 8 ways,
// and the outputs are bit-identical to them.
//
// Why one launch: the down projection's weights (64 KiB per workgroup, every chunk of its ring) are issued the
// moment a workgroup's gate/up rows are done, while the h hand-off is still in flight, instead of after a kernel
// boundary and its ramp (MI355X guide: prefetch-credit, boundary).
//
// Grid: one 256-thread workgroup per gate/up tile pair p (I / 16 of them; 1024 for Gemma-2B), all co-resident
// (4 per CU; the launch is refused otherwise).  Workgroup p:
//   1. gate/up rows [32p, 32p + 32) of the interleaved matrix -> h[m][16p .. 16p + 16), stored write-through,
//      drained, then one relaxed agent-scope add to the arrival counter of its K slice (sync[p / per_slice]);
//   2. down unit (tile t = p % (H / 16), K slice z = p / (H / 16)): issues its weights, waits until all
//      per_slice producers of slice z arrived (one lane polls, bounded by the wall clock), reads that h slice
//      write-through into LDS, multiplies, and hands its fp32 partial to the tile's last-arriving split, which
//      adds the KS slabs into the residual (PG_EPI_F32_FIN, in split order) and writes x' and the sums of squares.
// The last workgroup to finish resets the counters (every wait is then over).  Hand-off form: MI355X guide,
// inter-workgroup hand-off table row 1 (sc1 stores drained by the storing wave, one agent-scope add per
// workgroup, an sc1 poll, a workgroup barrier, sc1 loads).
#include "attn_common.h"

#ifndef PG_MLP_TIMEOUT_TICKS
#define PG_MLP_TIMEOUT_TICKS 20000000ull   // 0.2 s of the 100 MHz constant clock: a wait gives up, sync[ERR] = 1
#endif
#ifndef PG_MLP_GU_DEPTH
#define PG_MLP_GU_DEPTH 3                  // gate/up chunks in flight per wave (4 workgroups per CU: <= 128 VGPRs)
#endif
#ifndef PG_MLP_D_DEPTH
#define PG_MLP_D_DEPTH 8                   // down chunks in flight per wave (8 = the whole unit)
#endif
#ifndef PG_MLP_SLEEP
#define PG_MLP_SLEEP 32                    // s_sleep between polls (x 64 cycles)
#endif
#ifndef PG_MLP_CSTRIDE
#define PG_MLP_CSTRIDE 64                  // ints between the slice counters: one 256-B line each (polls that share
                                           // a line with the arrivals measured 2x slower: 98 vs 45 us per layer)
#endif
#define MLP_XPAD 8
#define MLP_SYNC_DONE (8 * PG_MLP_CSTRIDE)          // after the (<= 8) slice counters, each on a line of its own
#define MLP_SYNC_ERR (8 * PG_MLP_CSTRIDE + 64)
#define MLP_SYNC_INTS (8 * PG_MLP_CSTRIDE + 128)    // pg_decode_mlp_block's sync buffer size (ints)

struct MlpBlockArgs {
  const bf16_t* xq;      // [M][H] x' = bf16(resid * (1 + post_w)) (the o_proj F32_FIN epilogue, previous launch)
  const float* ss_in;    // [M][ss_ld] per-tile sums of squares of that residual
  int ss_ld, ss_n;
  float eps;
  const bf16_t* wgu;     // [2I][H] fragment-packed, gate / up interleaved in 16-row blocks
  bf16_t* h;             // [M][I] gelu(gate) * up (write-through)
  const bf16_t* wd;      // [H][I] fragment-packed
  float* slab;           // [KS][M][H] split-K partials (write-through)
  int* fin_cnt;          // [H / 16] arrival tickets, zero between launches (the last arriver resets)
  float* resid;          // [M][H] residual, finalised in place
  float* ss_out;         // [M][ss_ld_out] per-tile sums of squares of the new residual
  int ss_ld_out;
  bf16_t* fin_x;         // [M][H] x' = bf16(resid * (1 + norm_w)) for the next GEMV (may be null)
  const float* norm_w;   // the next RMSNorm's weight (with fin_x)
  int* sync;             // slice arrivals [z * CSTRIDE], workgroups done, err (MLP_SYNC_*); zero before the first launch
  int M, H, I, KS;
  unsigned long long* stamps;   // diagnostics (pg_decode_mlp_stamps): [workgroup][4] wall-clock stamps, or null
};

static unsigned long long* g_mlp_stamps = nullptr;
// Diagnostics: every later pg_decode_mlp_block launch records per workgroup [start, h published, h slice ready, end]
// (100 MHz wall clock, u64) into buf [grid][4]; null turns it off.
extern "C" int pg_decode_mlp_stamps(void* buf) {
  g_mlp_stamps = (unsigned long long*)buf;
  return 0;
}

typedef __attribute__((address_space(1))) unsigned long long mlp_gu64;

__device__ __forceinline__ u32x4 mlp_ldw(const bf16_t* p) {   // read-once weights: non-temporal
  return __builtin_nontemporal_load((const u32x4*)p);
}

// Gate/up rows of tile pair p (the arithmetic of gemv_body<PG_EPI_BF16_GELU_MUL, NT 2, U 2, PRO 4, FRAG, CPW>)
template <int DEPTH, int CPW>
__device__ __forceinline__ void mlp_gate_up(const MlpBlockArgs& a, int p, f32x4 (*red)[2][64]) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, g = lane >> 4, r = lane & 15;
  const int M = a.M, K = a.H;
  const bf16_t* wt0 = a.wgu + (size_t)(2 * p) * 16 * K;
  const bf16_t* wt1 = wt0 + (size_t)16 * K;
  const bf16_t* xrow = a.xq + (size_t)(r < M ? r : M - 1) * K;   // rows past M read row M - 1 (never stored)
  // the producer's per-tile sums of squares, loaded by wave 0 before the weight stream (clamped, masked later)
  float ssv[16];
#pragma unroll
  for (int k = 0; k < 16; ++k) ssv[k] = 0.f;
  if (wave == 0) {
    if (M > 2) {
      const int rr = min(r, M - 1);
#pragma unroll
      for (int k = 0; k < 16; ++k) ssv[k] = a.ss_in[(size_t)rr * a.ss_ld + min(g + 4 * k, a.ss_n - 1)];
    } else {
      const int lpr = M == 1 ? 64 : 32;
      const int rr = min(lane / lpr, M - 1);
#pragma unroll
      for (int k = 0; k < 4; ++k) ssv[k] = a.ss_in[(size_t)rr * a.ss_ld + min(lane % lpr + k * lpr, a.ss_n - 1)];
    }
  }
  u32x4 wb[DEPTH][2][2];
  u32x4 xb[DEPTH][2];
  auto loadw = [&](int j, u32x4 (&wv)[2][2]) {
    const size_t cc = (size_t)(wave + 4 * j);
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      wv[0][s] = mlp_ldw(wt0 + (cc * 2 + s) * 512 + lane * 8);
      wv[1][s] = mlp_ldw(wt1 + (cc * 2 + s) * 512 + lane * 8);
    }
  };
  auto loadx = [&](int j, u32x4 (&xv)[2]) {
    const int koff = (wave + 4 * j) * 64 + 16 * g;
#pragma unroll
    for (int s = 0; s < 2; ++s) xv[s] = *(const u32x4*)(xrow + koff + 8 * s);
  };
#pragma unroll
  for (int d = 0; d < DEPTH; ++d)
    if (d < CPW) {
      loadw(d, wb[d]);
      loadx(d, xb[d]);
    }
  f32x4 acc[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int j = 0; j < CPW; ++j) {
    const int d = j % DEPTH;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const bf16x8 xv = __builtin_bit_cast(bf16x8, xb[d][s]);
      acc[0] = mfma16(__builtin_bit_cast(bf16x8, wb[d][0][s]), xv, acc[0]);
      acc[1] = mfma16(__builtin_bit_cast(bf16x8, wb[d][1][s]), xv, acc[1]);
    }
    if (j + DEPTH < CPW) {
      loadw(j + DEPTH, wb[d]);
      loadx(j + DEPTH, xb[d]);
    }
    __builtin_amdgcn_sched_barrier(0);
  }
  red[wave][0][lane] = acc[0];
  red[wave][1][lane] = acc[1];
  __syncthreads();
  if (wave != 0) return;
#pragma unroll
  for (int t = 0; t < 2; ++t) acc[t] = red[0][t][lane] + red[1][t][lane] + red[2][t][lane] + red[3][t][lane];
  const int m = r;
  // RMSNorm: rstd of row m from the producer's per-tile sums (W.(x*rstd) = rstd * W.x)
  float ss = 0.f;
  if (M > 2) {
#pragma unroll
    for (int k = 0; k < 16; ++k) ss += g + 4 * k < a.ss_n ? ssv[k] : 0.f;
    ss += __shfl_xor(ss, 16, 64);
    ss += __shfl_xor(ss, 32, 64);
  } else {
    const int lpr = M == 1 ? 64 : 32;
#pragma unroll
    for (int k = 0; k < 4; ++k) ss += lane % lpr + k * lpr < a.ss_n ? ssv[k] : 0.f;
    for (int o = 1; o < lpr; o <<= 1) ss += __shfl_xor(ss, o, 64);
    ss = __shfl(ss, (m < M ? m : 0) * lpr, 64);
  }
  const float rs = rsqrtf(ss / (float)K + a.eps);
  acc[0] *= rs;
  acc[1] *= rs;
  // gelu(gate) * up -> h[m][16p + 4g .. +4), write-through for the down units of this launch
  if (m < M) {
    const f32x4 gt = acc[0], up = acc[1];
    u32x2 pk;
    pk[0] = pack_bf2(gelu_tanh(gt[0]) * up[0], gelu_tanh(gt[1]) * up[1]);
    pk[1] = pack_bf2(gelu_tanh(gt[2]) * up[2], gelu_tanh(gt[3]) * up[3]);
    __hip_atomic_store((mlp_gu64*)(a.h + (size_t)m * a.I + 16 * p + 4 * g), __builtin_bit_cast(unsigned long long, pk),
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  const int per_slice = (a.I / 16) / a.KS;
  if (lane == 0) __hip_atomic_fetch_add(a.sync + (p / per_slice) * PG_MLP_CSTRIDE, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (a.stamps && lane == 0) a.stamps[(size_t)p * 4 + 1] = wall_clock64();
}

// Down unit (tile t, K slice z) (the arithmetic of gemv_body<PG_EPI_F32_FIN, NT 1, U 2, PRO 0, FRAG, CPW> at ksplit
// KS), x = the h slice of this launch
template <int DEPTH, int CPW>
__device__ __forceinline__ void mlp_down(const MlpBlockArgs& a, int t, int z, bf16_t* xs, f32x4 (*red)[64]) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, g = lane >> 4, r = lane & 15;
  const int M = a.M, N = a.H;
  const int Kz = a.I / a.KS, nchz = Kz / 64;
  const bf16_t* wt = a.wd + (size_t)t * 16 * a.I;
  u32x4 wb[DEPTH][2];
  auto loadw = [&](int j, u32x4 (&wv)[2]) {
    const size_t cc = (size_t)(z * nchz + wave + 4 * j);
#pragma unroll
    for (int s = 0; s < 2; ++s) wv[s] = mlp_ldw(wt + (cc * 2 + s) * 512 + lane * 8);
  };
  // the weights go out before the wait (they do not depend on h)
#pragma unroll
  for (int d = 0; d < DEPTH; ++d)
    if (d < CPW) loadw(d, wb[d]);
  // the residual rows and norm weights the tile's finaliser uses (previous launch's data: plain loads)
  const int n0 = t * 16 + 4 * g;
  const f32x4 fin_r = *(const f32x4*)(a.resid + (size_t)(r < M ? r : M - 1) * N + n0);
  const f32x4 fin_w = *(const f32x4*)((a.norm_w ? a.norm_w : a.resid) + n0);
  const int per_slice = (a.I / 16) / a.KS;
  if (threadIdx.x == 0) {
    const unsigned long long t0 = wall_clock64();
    while (__hip_atomic_load(a.sync + z * PG_MLP_CSTRIDE, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < per_slice) {
      if (wall_clock64() - t0 > PG_MLP_TIMEOUT_TICKS) {
        __hip_atomic_store(a.sync + MLP_SYNC_ERR, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
      __builtin_amdgcn_s_sleep(PG_MLP_SLEEP);
    }
    if (a.stamps) a.stamps[(size_t)blockIdx.x * 4 + 2] = wall_clock64();
  }
  __syncthreads();
  // the h slice [M][z*Kz, (z+1)*Kz) into LDS, write-through-readable loads
  const int ldx = Kz + MLP_XPAD, K8 = Kz >> 3;
  for (int idx = threadIdx.x; idx < M * K8; idx += 256) {
    const int mm = idx / K8, c = idx % K8;
    *(u32x4*)(xs + mm * ldx + c * 8) = ld16_wt_u(a.h + (size_t)mm * a.I + (size_t)z * Kz + c * 8);
  }
  __syncthreads();
  const bf16_t* xl = xs + (r < M ? r : M - 1) * ldx;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int j = 0; j < CPW; ++j) {
    const int d = j % DEPTH;
    const int koff = (wave + 4 * j) * 64 + 16 * g;
#pragma unroll
    for (int s = 0; s < 2; ++s)
      acc = mfma16(__builtin_bit_cast(bf16x8, wb[d][s]), *(const bf16x8*)(xl + koff + 8 * s), acc);
    if (j + DEPTH < CPW) loadw(j + DEPTH, wb[d]);
    __builtin_amdgcn_sched_barrier(0);
  }
  red[wave][lane] = acc;
  __syncthreads();
  if (wave != 0) return;
  acc = red[0][lane] + red[1][lane] + red[2][lane] + red[3][lane];
  const int m = r;
  // this split's slab, write-through; drain; ticket; the tile's last split reduces (split order) and finalises
  if (m < M) {
    mlp_gu64* dst = (mlp_gu64*)(a.slab + ((size_t)z * M + m) * N + n0);
    __hip_atomic_store(dst, __builtin_bit_cast(unsigned long long, u32x2{__float_as_uint(acc[0]), __float_as_uint(acc[1])}),
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(dst + 1, __builtin_bit_cast(unsigned long long, u32x2{__float_as_uint(acc[2]), __float_as_uint(acc[3])}),
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  int old = 0;
  if (lane == 0) old = __hip_atomic_fetch_add(a.fin_cnt + t, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  old = __shfl(old, 0, 64);
  if (old == a.KS - 1) {
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");   // compiler-only: keep the loads below the ticket
    float ssl = 0.f;
    if (m < M) {
      f32x4 v = fin_r;
      u32x2 sa[8], sb[8];
#pragma unroll
      for (int zz = 0; zz < 8; ++zz) {
        const mlp_gu64* src = (const mlp_gu64*)(a.slab + ((size_t)(zz < a.KS ? zz : a.KS - 1) * M + m) * N + n0);
        sa[zz] = __builtin_bit_cast(u32x2, __hip_atomic_load(src, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
        sb[zz] = __builtin_bit_cast(u32x2, __hip_atomic_load(src + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
      }
#pragma unroll
      for (int zz = 0; zz < 8; ++zz) {
        const f32x4 sv = {__uint_as_float(sa[zz][0]), __uint_as_float(sa[zz][1]), __uint_as_float(sb[zz][0]),
                          __uint_as_float(sb[zz][1])};
        v += zz < a.KS ? sv : f32x4{0.f, 0.f, 0.f, 0.f};
      }
      *(f32x4*)(a.resid + (size_t)m * N + n0) = v;
      ssl = v[0] * v[0] + v[1] * v[1] + v[2] * v[2] + v[3] * v[3];
      if (a.fin_x) {
        u32x2 pk;
        pk[0] = pack_bf2(v[0] * (1.0f + fin_w[0]), v[1] * (1.0f + fin_w[1]));
        pk[1] = pack_bf2(v[2] * (1.0f + fin_w[2]), v[3] * (1.0f + fin_w[3]));
        *(u32x2*)(a.fin_x + (size_t)m * N + n0) = pk;
      }
    }
    ssl += __shfl_xor(ssl, 16, 64);
    ssl += __shfl_xor(ssl, 32, 64);
    if (g == 0 && m < M) a.ss_out[(size_t)m * a.ss_ld_out + t] = ssl;
    if (lane == 0) __hip_atomic_store(a.fin_cnt + t, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

template <int GU_CPW, int D_CPW>
__global__ __launch_bounds__(256) void decode_mlp_kernel(MlpBlockArgs a) {
  __shared__ f32x4 red_gu[4][2][64];
  __shared__ f32x4 red_d[4][64];
  extern __shared__ __attribute__((aligned(16))) char mlp_smem[];
  const int p = blockIdx.x;
  if (a.stamps && threadIdx.x == 0) a.stamps[(size_t)p * 4] = wall_clock64();
  mlp_gate_up<PG_MLP_GU_DEPTH, GU_CPW>(a, p, red_gu);
  const int TD = a.H / 16;
  mlp_down<PG_MLP_D_DEPTH, D_CPW>(a, p % TD, p / TD, (bf16_t*)mlp_smem, red_d);
  if (threadIdx.x == 0) {
    // every wait of this workgroup is over: the last one to get here resets the counters for the next launch
    if (__hip_atomic_fetch_add(a.sync + MLP_SYNC_DONE, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
        (int)gridDim.x - 1) {
      for (int i = 0; i < a.KS; ++i)
        __hip_atomic_store(a.sync + i * PG_MLP_CSTRIDE, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(a.sync + MLP_SYNC_DONE, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (a.stamps) a.stamps[(size_t)p * 4 + 3] = wall_clock64();
  }
}

template <int GU_CPW, int D_CPW>
static int launch_mlp(const MlpBlockArgs& a, size_t lds, hipStream_t stream) {
  // every workgroup waits on others: the whole grid must be resident at once (256-thread workgroups are admitted up
  // to min(occupancy API, 8, SGPR bound >= 6) per CU -- MI355X guide, residency -- and this grid needs 4)
  static int cap = -1;
  if (cap < 0) {
    int nb = 0, dev = 0, cus = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, decode_mlp_kernel<GU_CPW, D_CPW>, 256, 16384) != hipSuccess)
      return (int)hipErrorNotSupported;
    cap = (nb < 6 ? nb : 6) * cus;
  }
  const int grid = a.I / 16;
  if (grid > cap) return (int)hipErrorNotSupported;
  hipLaunchKernelGGL((decode_mlp_kernel<GU_CPW, D_CPW>), dim3(grid), dim3(256), lds, stream, a);
  PG_LAUNCH_CHECK();
  return 0;
}

extern "C" int pg_decode_mlp_block(const void* xq, const float* ss_in, int ss_ld, int ss_n, float eps, const void* wgu,
                                   void* h, const void* wd, float* slab, int ksplit, int* fin_cnt, float* resid,
                                   float* ss_out, int ss_ld_out, void* fin_x, const float* norm_w, int* sync, int M,
                                   int H, int I, hipStream_t stream) {
  PG_REQUIRE(xq && ss_in && wgu && h && wd && slab && fin_cnt && resid && ss_out && sync);
  static_assert(MLP_SYNC_INTS <= 640, "pg_decode_mlp_block documents a 640-int sync buffer");
  PG_REQUIRE(M >= 1 && M <= 2 && ss_n > 0 && ss_ld >= ss_n && ss_n <= 256 && (M == 1 || ss_n <= 128));
  PG_REQUIRE(H % 16 == 0 && I % 16 == 0 && ksplit >= 1 && ksplit <= 8 && (I / 16) == (H / 16) * ksplit);
  PG_REQUIRE(ss_ld_out >= H / 16 && (fin_x == nullptr || norm_w != nullptr));
  // compiled for the Gemma-2B shapes (8 chunks per wave in both GEMVs); anything else: the two-launch form
  if (H % 256 != 0 || (I / ksplit) % 256 != 0) return (int)hipErrorNotSupported;
  MlpBlockArgs a{(const bf16_t*)xq, ss_in, ss_ld, ss_n, eps, (const bf16_t*)wgu, (bf16_t*)h, (const bf16_t*)wd, slab,
                 fin_cnt, resid, ss_out, ss_ld_out, (bf16_t*)fin_x, norm_w, sync, M, H, I, ksplit, g_mlp_stamps};
  const int Kz = I / ksplit;
  const size_t lds = (size_t)M * (Kz + MLP_XPAD) * 2;
  const int gu_cpw = H / 256, d_cpw = Kz / 256;
  if (gu_cpw == 8 && d_cpw == 8) return launch_mlp<8, 8>(a, lds, stream);
  return (int)hipErrorNotSupported;
}
