// Decode gate/up GEMV that banks its weights on-chip while the attention chain runs (batch 1).
//
// Why: a batch-1 decode layer is qkv -> attention -> o_proj (19 MB, latency-bound, ~17 us with HBM mostly idle)
// then gate/up (134 MB) and down (67 MB) at the per-CU load rate (~25 GB/s per CU).  This kernel is launched on a
// SECOND stream as soon as the previous layer's down projection ends, i.e. beside the chain (a parallel branch of
// the captured decode graph), and pulls half of its weights into registers and LDS before its input exists:
//   workgroup c (one per CU -- the 128 KiB LDS bank admits one) owns tile pairs 4c .. 4c+3 (gate tile + up tile,
//   16 rows x 2048 k each, fragment-packed, 128 KiB per pair):
//     pair 0 -> VGPRs (each wave: its 8 chunks of both tiles, exactly the decode GEMV's register image),
//     pair 1 -> LDS by LDS-DMA (non-temporal), each wave its own 32 KiB;
//   then it waits (one polling lane, bounded) until the o_proj launch has finalised every residual tile
//   (*wait_cnt >= wait_target: the F32_FIN producer's done counter, x' and the sums of squares stored
//   write-through before each add), reads x' and ss with write-through-readable (agent-scope) loads and
//   computes pair 0, streams pair 2 into the registers pair 0 used and pair 3 into the LDS pair 1 used, so
//   after the hand-off only 256 KiB per CU remain to load instead of 512.
// Arithmetic is the decode GEMV's (gemv_kernel<PG_EPI_BF16_GELU_MUL, 2, 2, DEPTH, 4, FRAG, 8>): wave w sums chunks
// w, w+4, .., w+28 in that order (two 16x16x32 MFMAs per chunk), the four wave partials are added in wave order,
// scaled by rstd (same lane reduction of the producer's per-tile sums) and gelu(gate)*up is rounded to bf16 --
// so h is bit-identical to that launch's.
// Replaces GemmaMLP's gate_proj/up_proj + gelu*up (modeling_gemma.py:210-218) of a batch-1 decode step.
#include <cstdlib>

#include "common.h"

#ifndef PG_BANK_TIMEOUT_TICKS
#define PG_BANK_TIMEOUT_TICKS 20000000ull   // 0.2 s of the 100 MHz constant clock
#endif
#define BK_H 2048
#define BK_PAIRS 4                          // tile pairs per workgroup (4 x 256 = 1024 = 16384 / 16)
#define BK_WG 256
#define BK_LDS (131072 + 4096)                // weight bank + x' slots

struct GateUpBankArgs {
  const bf16_t* xq;        // [1][H] x' = bf16(resid * (1 + norm_w)) from the o_proj F32_FIN producer
  const float* ss_in;      // [ss_n] its per-tile sums of squares
  int ss_n;
  float eps;
  const bf16_t* wgu;       // [2I][H] fragment-packed, gate / up interleaved in 16-row blocks
  bf16_t* h;               // [1][I] gelu(gate) * up
  const int* wait_cnt;     // producer's done counter (tiles finalised)
  int wait_target;
  int* exit_cnt;           // workgroups past the wait; the last one resets *wait_cnt and itself
  int* err;                // 1 if a wait gave up (the outputs are then meaningless)
  unsigned long long* stamps;   // diagnostics: [WG][4] wall clock (start, wait over, pairs done, end) or null
};

typedef __attribute__((address_space(1))) unsigned long long bk_gu64;
typedef __attribute__((address_space(1))) unsigned bk_gu32;

// diagnostics: with a buffer set, launch k (counted from the pg_gateup_bank_stamps call) records its workgroups'
// stamps into slot k % 64 of buf [64][BK_WG][4] (captured launches keep the slot they were captured with)
static unsigned long long* g_bank_stamps = nullptr;
static unsigned g_bank_launch = 0;
extern "C" int pg_gateup_bank_stamps(void* buf) {
  g_bank_stamps = (unsigned long long*)buf;
  g_bank_launch = 0;
  return 0;
}

// LDS reads through inline asm: opaque to hipcc's waitcnt pass, which would otherwise drain every outstanding
// load -- the LDS-DMA and the next pair's stream -- in front of each LDS read.
// a chunk of a banked pair (4 pieces, 1 KiB apart) and its two x' pieces (16 B apart)
__device__ __forceinline__ void bk_lds_read6(unsigned waddr, unsigned xaddr, u32x4& a, u32x4& b, u32x4& c, u32x4& d,
                                             u32x4& x0, u32x4& x1) {
  asm volatile(
      "ds_read_b128 %0, %6\n\t"
      "ds_read_b128 %1, %6 offset:1024\n\t"
      "ds_read_b128 %2, %6 offset:2048\n\t"
      "ds_read_b128 %3, %6 offset:3072\n\t"
      "ds_read_b128 %4, %7\n\t"
      "ds_read_b128 %5, %7 offset:64\n\t"
      "s_waitcnt lgkmcnt(0)"
      : "=&v"(a), "=&v"(b), "=&v"(c), "=&v"(d), "=&v"(x0), "=&v"(x1)
      : "v"(waddr), "v"(xaddr)
      : "memory");
}
__device__ __forceinline__ void bk_lds_read2(unsigned xaddr, u32x4& x0, u32x4& x1) {
  asm volatile(
      "ds_read_b128 %0, %2\n\t"
      "ds_read_b128 %1, %2 offset:64\n\t"
      "s_waitcnt lgkmcnt(0)"
      : "=&v"(x0), "=&v"(x1)
      : "v"(xaddr)
      : "memory");
}

// INFL > 0: the banked loads are paced -- a wave keeps at most INFL of its 1 KiB load instructions in flight, so the
// chain's latency-bound loads on the same CU do not queue behind 256 KiB of bank traffic
template <int INFL>
__global__ __launch_bounds__(256, 1) void gateup_bank_kernel(GateUpBankArgs a) {
  // bank: [wave][chunk j][tile t][piece s] x 1 KiB (lane-linear 16 B) = 128 KiB, reused for the wave partials;
  // then x' per wave: [wave][chunk j][piece s][lane group g] x 16 B = 4 KiB
  extern __shared__ __attribute__((aligned(1024))) char bank[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int g = lane >> 4, r = lane & 15;
  const int c = blockIdx.x;
  unsigned long long* stamp = a.stamps ? a.stamps + (size_t)c * 4 : nullptr;
  if (stamp && threadIdx.x == 0) stamp[0] = wall_clock64();

  // fragment source of (pair p, tile t, this wave's chunk j, piece s): 64 KiB per tile, 2 KiB per chunk
  auto src = [&](int p, int t, int j, int s) -> const bf16_t* {
    const size_t tile = (size_t)2 * (BK_PAIRS * c + p) + t;
    return a.wgu + tile * 16 * BK_H + ((size_t)(wave + 4 * j) * 2 + s) * 512 + lane * 8;
  };
  char* mybank = bank + wave * 32768;
  const unsigned mybank_addr = (unsigned)(size_t)(LDS_AS char*)mybank;
  auto dma = [&](int p) {
#pragma unroll
    for (int j = 0; j < 8; ++j)
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int s = 0; s < 2; ++s)
        {
          __builtin_amdgcn_global_load_lds((const void*)src(p, t, j, s),
                                           (LDS_AS void*)(mybank + ((j * 2 + t) * 2 + s) * 1024), 16, 0, 2);
          if (INFL > 0 && p == 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(INFL) : "memory");
        }
  };

  // ---- before the hand-off: pair 0 into registers, pair 1 into LDS
  u32x4 wb[8][2][2];
#pragma unroll
  for (int j = 0; j < 8; ++j)
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        wb[j][t][s] = __builtin_nontemporal_load((const u32x4*)src(0, t, j, s));
        if (INFL > 0 && (j * 2 + t) * 2 + s >= INFL) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(INFL) : "memory");
      }
  dma(1);

  // ---- wait for the o_proj launch (one polling lane; the other waves hold at the barrier)
  if (threadIdx.x == 0) {
    const unsigned long long t0 = wall_clock64();
    while (__hip_atomic_load(a.wait_cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < a.wait_target) {
      if (wall_clock64() - t0 > PG_BANK_TIMEOUT_TICKS) {
        __hip_atomic_store(a.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
    if (__hip_atomic_fetch_add(a.exit_cnt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == (int)gridDim.x - 1) {
      // every workgroup is past its wait: re-arm for the next step's producer
      __hip_atomic_store((int*)a.wait_cnt, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(a.exit_cnt, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (stamp) stamp[1] = wall_clock64();
  }
  asm volatile("s_barrier" ::: "memory");        // (no fence: the banked loads stay in flight)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // banked data landed (issued a chain ago)

  // x': lane (j, s, gg) of each wave loads the one 16-B piece x'[64 (wave + 4j) + 16 gg + 8 s ..] with agent-scope
  // loads (the producer stored it write-through and added to the counter after draining) and parks it in the
  // wave's own LDS slots (its lanes of group gg read it back as their MFMA B operand)
  const unsigned xl_addr = (unsigned)(size_t)(LDS_AS char*)(bank + 131072 + wave * 1024);
  {
    const int js = lane >> 2, gg = lane & 3, j = js >> 1, sp = js & 1;
    const bk_gu64* px = (const bk_gu64*)(a.xq + (size_t)(wave + 4 * j) * 64 + 16 * gg + 8 * sp);
    const unsigned long long lo = __hip_atomic_load(px, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned long long hi = __hip_atomic_load(px + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const u32x4 v = {(unsigned)lo, (unsigned)(lo >> 32), (unsigned)hi, (unsigned)(hi >> 32)};
    asm volatile("s_waitcnt vmcnt(0)\n\tds_write_b128 %0, %1\n\ts_waitcnt lgkmcnt(0)" ::"v"(xl_addr + lane * 16),
                 "v"(v) : "memory");
  }
  // lane (g, r) reads piece (j, s) of its group at xl + ((2 j + s) * 4 + g) * 16
  const unsigned xg_addr = xl_addr + g * 16;
  float ssv[4];
#pragma unroll
  for (int k = 0; k < 4; ++k)
    ssv[k] = __uint_as_float(__hip_atomic_load((const bk_gu32*)(a.ss_in + min(lane + 64 * k, a.ss_n - 1)),
                                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));

  f32x4 acc[BK_PAIRS][2];
#pragma unroll
  for (int p = 0; p < BK_PAIRS; ++p) acc[p][0] = acc[p][1] = f32x4{0.f, 0.f, 0.f, 0.f};
  auto mma = [&](int p, const u32x4 (&w)[2][2], const u32x4 (&xv2)[2]) {
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const bf16x8 xv = __builtin_bit_cast(bf16x8, xv2[s]);
#pragma unroll
      for (int t = 0; t < 2; ++t) acc[p][t] = mfma16(__builtin_bit_cast(bf16x8, w[t][s]), xv, acc[p][t]);
    }
  };
  auto from_regs = [&](int p) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      u32x4 xv2[2];
      bk_lds_read2(xg_addr + j * 128, xv2[0], xv2[1]);
      mma(p, wb[j], xv2);
    }
  };
  auto from_lds = [&](int p) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      u32x4 w[2][2], xv2[2];
      bk_lds_read6(mybank_addr + j * 4096 + lane * 16, xg_addr + j * 128, w[0][0], w[0][1], w[1][0], w[1][1], xv2[0],
                   xv2[1]);
      mma(p, w, xv2);
    }
  };

  // pair 0 (registers), then pair 2's stream into the same registers
  from_regs(0);
#pragma unroll
  for (int j = 0; j < 8; ++j)
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int s = 0; s < 2; ++s) wb[j][t][s] = __builtin_nontemporal_load((const u32x4*)src(2, t, j, s));
  // pair 1 (LDS), then pair 3's DMA into the same slots (every read of them has returned: lgkmcnt(0) above)
  from_lds(1);
  dma(3);
  from_regs(2);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  from_lds(3);
  if (stamp && threadIdx.x == 0) stamp[2] = wall_clock64();

  // ---- rstd (the decode GEMV's pro-4 reduction for one row: 64 lanes x 4 entries, butterfly, lane 0's value)
  float ss = 0.f;
#pragma unroll
  for (int k = 0; k < 4; ++k) ss += lane + 64 * k < a.ss_n ? ssv[k] : 0.f;
  for (int o = 1; o < 64; o <<= 1) ss += __shfl_xor(ss, o, 64);
  ss = __shfl(ss, 0, 64);
  const float rs = rsqrtf(ss / (float)BK_H + a.eps);

  // ---- wave partials -> LDS (each wave into its own bank region: nothing of another wave is overwritten),
  // then wave p finishes pair p: red[0] + red[1] + red[2] + red[3], * rstd, gelu(gate) * up
  f32x4* red = (f32x4*)bank;                     // [wave][pair][tile][lane] at wave * 32 KiB
#pragma unroll
  for (int p = 0; p < BK_PAIRS; ++p)
#pragma unroll
    for (int t = 0; t < 2; ++t) red[(size_t)wave * 2048 + (p * 2 + t) * 64 + lane] = acc[p][t];
  __syncthreads();
  f32x4 v[2];
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const int o = (wave * 2 + t) * 64 + lane;
    v[t] = red[o] + red[2048 + o] + red[4096 + o] + red[6144 + o];
    v[t] *= rs;
  }
  if (r == 0) {
    const int oc = 16 * (BK_PAIRS * c + wave) + 4 * g;
    u32x2 pk;
    pk[0] = pack_bf2(gelu_tanh(v[0][0]) * v[1][0], gelu_tanh(v[0][1]) * v[1][1]);
    pk[1] = pack_bf2(gelu_tanh(v[0][2]) * v[1][2], gelu_tanh(v[0][3]) * v[1][3]);
    *(u32x2*)(a.h + oc) = pk;
  }
  if (stamp && threadIdx.x == 0) stamp[3] = wall_clock64();
}

// Batch 1, Gemma-2B MLP shapes (H 2048, I 16384) only.  wait_cnt / exit_cnt: ints zeroed once (self re-arming);
// err: an int the caller checks.  Returns hipErrorNotSupported (nothing launched) on another device shape.
extern "C" int pg_gateup_bank(const void* xq, const float* ss_in, int ss_n, float eps, const void* wgu, void* h,
                              const int* wait_cnt, int wait_target, int* exit_cnt, int* err, int M, int H, int I,
                              hipStream_t stream) {
  PG_REQUIRE(xq && ss_in && wgu && h && wait_cnt && exit_cnt && err && ss_n > 0 && ss_n <= 256 && wait_target > 0);
  if (M != 1 || H != BK_H || I != BK_PAIRS * BK_WG * 16) return (int)hipErrorNotSupported;
  // PG_BANK_INFL (environment, tuning A/B): 0 = every banked load issued at once; default 8
  static const int infl = getenv("PG_BANK_INFL") ? atoi(getenv("PG_BANK_INFL")) : 8;
  static int ok = -1;
  if (ok < 0) {
    ok = hipFuncSetAttribute((const void*)gateup_bank_kernel<0>, hipFuncAttributeMaxDynamicSharedMemorySize, BK_LDS) ==
             hipSuccess &&
         hipFuncSetAttribute((const void*)gateup_bank_kernel<4>, hipFuncAttributeMaxDynamicSharedMemorySize, BK_LDS) ==
             hipSuccess &&
         hipFuncSetAttribute((const void*)gateup_bank_kernel<8>, hipFuncAttributeMaxDynamicSharedMemorySize, BK_LDS) ==
             hipSuccess &&
         hipFuncSetAttribute((const void*)gateup_bank_kernel<16>, hipFuncAttributeMaxDynamicSharedMemorySize, BK_LDS) ==
             hipSuccess;
  }
  if (!ok) return (int)hipErrorNotSupported;
  GateUpBankArgs args{(const bf16_t*)xq, ss_in, ss_n, eps, (const bf16_t*)wgu, (bf16_t*)h, wait_cnt, wait_target,
                      exit_cnt, err,
                      g_bank_stamps ? g_bank_stamps + (size_t)(g_bank_launch++ % 64) * BK_WG * 4 : nullptr};
  switch (infl) {
    case 0: hipLaunchKernelGGL(gateup_bank_kernel<0>, dim3(BK_WG), dim3(256), BK_LDS, stream, args); break;
    case 4: hipLaunchKernelGGL(gateup_bank_kernel<4>, dim3(BK_WG), dim3(256), BK_LDS, stream, args); break;
    case 16: hipLaunchKernelGGL(gateup_bank_kernel<16>, dim3(BK_WG), dim3(256), BK_LDS, stream, args); break;
    default: hipLaunchKernelGGL(gateup_bank_kernel<8>, dim3(BK_WG), dim3(256), BK_LDS, stream, args); break;
  }
  PG_LAUNCH_CHECK();
  return 0;
}
