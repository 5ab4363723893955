// Persistent decode MLP (batch <= 2): GemmaMLP.forward (modeling_gemma.py:210-218) + the residual add
// of DecoderLayer.forward (:412-416) + the next RMSNorm's statistics, in ONE launch per layer:
//
//   phase A  h = gelu_tanh(x.Wg^T * rstd) * (x.Wu^T * rstd)      one wave per 32-row gate/up pair
//   ------   grid barrier (the down weights are already streaming into registers)
//   phase B  down split-K slabs -> in-kernel finalisation          one wave per (16-row tile, K slice)
//            (last-arriving slice: resid += slabs, x' = resid*(1+w_next), per-tile sum of squares)
//
// Two kernel boundaries per layer become one, and the down projection's ramp overlaps the barrier.
// x is the previous finalisation's x' = bf16(resid*(1+w)); rstd comes from its per-tile sums of
// squares (RMSNorm as an output scale: W.(x*rstd) = rstd*(W.x)).
//
// Inter-workgroup protocol (MI355X: per-CU L1 and per-XCD L2 are not coherent): h and the split-K
// slabs are stored write-through (agent-scope relaxed 8-B atomic stores = global_store ... sc1),
// drained with s_waitcnt vmcnt(0) before the arrival ticket, and read back with sc1 loads, so no
// release / acquire fences are needed.  The barrier counter is a 64-bit ticket that only grows
// (target = (ticket / G + 1) * G), so graph replays need no reset; every spin is bounded and sets
// *err instead of hanging.  grid = one workgroup per CU (all co-resident).
#include "common.h"

typedef __attribute__((address_space(1))) unsigned long long gu64;

struct PgMlpArgs {
  const bf16_t* x;          // [M][H] x' of the post-attention RMSNorm
  const float* ss_in;       // [M][ss_ld] per-tile sums of squares of the residual (ss_n tiles)
  int ss_ld, ss_n;
  float eps;
  const bf16_t* gu_w;       // [2I][H], gate/up interleaved in 16-row blocks
  bf16_t* h;                // [M][I] scratch
  const bf16_t* down_w;     // [H][I]
  float* part;              // [Z][M][H] split-K slabs
  int* fin_cnt;             // [H/16] arrival tickets (zero, self-resetting)
  float* resid;             // [M][H] residual, updated in place
  float* ss_out;            // [M][ss_ld] sums of squares of the new residual per 16-column tile
  bf16_t* x_out;            // [M][H] x' = bf16(resid * (1 + norm_w_next))
  const float* norm_w_next; // next RMSNorm weight
  unsigned long long* bar;  // grid barrier ticket (monotonic, zero-initialised once)
  int* err;                 // set to 1 if a barrier spin gave up
  int M, H, I, Z;
};

static __device__ __forceinline__ u32x4 ld16_sc1(const bf16_t* p) {
  gu64* q = (gu64*)p;
  const u32x2 a = __builtin_bit_cast(u32x2, __hip_atomic_load(q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
  const u32x2 b = __builtin_bit_cast(u32x2, __hip_atomic_load(q + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
  return u32x4{a[0], a[1], b[0], b[1]};
}

static __device__ __forceinline__ void st8_sc1(void* p, u32x2 v) {
  __hip_atomic_store((gu64*)p, __builtin_bit_cast(unsigned long long, v), __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
}

static __device__ __forceinline__ void raw_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

#ifndef PG_MLP_WG_PER_CU
#define PG_MLP_WG_PER_CU 2
#endif
constexpr int DA = 6;   // phase A chunks in flight per lane (2 tiles x 32 B each)
constexpr int DB = 8;   // phase B chunks in flight per lane (32 B each)

__global__ __launch_bounds__(256) void decode_mlp_kernel(PgMlpArgs a) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int g = lane >> 4, r = lane & 15;
  const int M = a.M, H = a.H, I = a.I, Z = a.Z;
  const bool xvalid = r < M;
  const int rrow = xvalid ? r : 0;
  const int gw = blockIdx.x * 4 + wave, nw = gridDim.x * 4;

  // rstd of every row from the producer's per-tile sums of squares (lanes [lpr*m, lpr*(m+1)) own row m)
  float rs;
  {
    const int lpr = M == 1 ? 64 : 32;
    const int rr = min(lane / lpr, M - 1);
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int i = lane % lpr + k * lpr;
      const float v = a.ss_in[(size_t)rr * a.ss_ld + min(i, a.ss_n - 1)];
      s += i < a.ss_n ? v : 0.f;
    }
    for (int o = 1; o < lpr; o <<= 1) s += __shfl_xor(s, o, 64);
    s = __shfl(s, rrow * lpr, 64);
    rs = rsqrtf(s / (float)H + a.eps);
  }

  // ---------------- phase A: gate/up pairs
  const int npairs = I / 16;
  const int nchA = H / 64;                  // 64-element chunks; lane piece = elements 16g..16g+15
  const bf16_t* xrow = a.x + (size_t)rrow * H;
  for (int p = gw; p < npairs; p += nw) {
    const bf16_t* w0 = a.gu_w + (size_t)(32 * p + r) * H + 16 * g;
    const bf16_t* w1 = w0 + (size_t)16 * H;
    const bf16_t* xp = xrow + 16 * g;
    f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
    u32x4 wb[DA][4], xb[DA][2];
    auto load = [&](int c, u32x4 (&w)[4], u32x4 (&xv)[2]) {
      w[0] = *(const u32x4*)(w0 + c * 64);
      w[1] = *(const u32x4*)(w0 + c * 64 + 8);
      w[2] = *(const u32x4*)(w1 + c * 64);
      w[3] = *(const u32x4*)(w1 + c * 64 + 8);
      xv[0] = xvalid ? *(const u32x4*)(xp + c * 64) : u32x4{0u, 0u, 0u, 0u};
      xv[1] = xvalid ? *(const u32x4*)(xp + c * 64 + 8) : u32x4{0u, 0u, 0u, 0u};
    };
#pragma unroll
    for (int d = 0; d < DA; ++d)
      if (d < nchA) load(d, wb[d], xb[d]);
    for (int base = 0; base < nchA; base += DA) {
#pragma unroll
      for (int d = 0; d < DA; ++d) {
        const int c = base + d;
        if (c < nchA) {
          const bf16x8 x0 = __builtin_bit_cast(bf16x8, xb[d][0]), x1 = __builtin_bit_cast(bf16x8, xb[d][1]);
          acc0 = mfma16(__builtin_bit_cast(bf16x8, wb[d][0]), x0, acc0);
          acc0 = mfma16(__builtin_bit_cast(bf16x8, wb[d][1]), x1, acc0);
          acc1 = mfma16(__builtin_bit_cast(bf16x8, wb[d][2]), x0, acc1);
          acc1 = mfma16(__builtin_bit_cast(bf16x8, wb[d][3]), x1, acc1);
          if (c + DA < nchA) load(c + DA, wb[d], xb[d]);
        }
      }
    }
    // lane holds gate/up of row r, features 16p + 4g + 0..3
    if (xvalid) {
      u32x2 pk;
      pk[0] = pack_bf2(gelu_tanh(acc0[0] * rs) * (acc1[0] * rs), gelu_tanh(acc0[1] * rs) * (acc1[1] * rs));
      pk[1] = pack_bf2(gelu_tanh(acc0[2] * rs) * (acc1[2] * rs), gelu_tanh(acc0[3] * rs) * (acc1[3] * rs));
      st8_sc1(a.h + (size_t)r * I + 16 * p + 4 * g, pk);
    }
  }

  // ---------------- grid barrier, with this wave's first down-projection weights already in flight
  const int KS = I / Z;                     // K slice per item
  const int nchB = KS / 32;                 // 32-element chunks; lane piece = elements 8g..8g+7 (16 B)
  const int nitems = (H / 16) * Z;
  int item = gw;
  u32x4 wbB[DB], xbB[DB];
  const bf16_t* wrow = nullptr;
  const bf16_t* hrow = nullptr;
  auto setup = [&](int it) {
    const int tile = it / Z, z = it % Z;
    wrow = a.down_w + (size_t)(16 * tile + r) * I + (size_t)z * KS + 8 * g;
    hrow = a.h + (size_t)rrow * I + (size_t)z * KS + 8 * g;
  };
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this wave's h stores drained
  raw_barrier();                                      // ... and every wave's of this workgroup
  unsigned long long target = 0;
  if (wave == 0 && lane == 0) {
    const unsigned long long G = gridDim.x;
    const unsigned long long t = __hip_atomic_fetch_add(a.bar, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    target = (t / G + 1) * G;
  }
  if (item < nitems) {                                // down weights in flight while the barrier completes
    setup(item);
#pragma unroll
    for (int d = 0; d < DB; ++d)
      if (d < nchB) wbB[d] = *(const u32x4*)(wrow + d * 32);
  }
  if (wave == 0 && lane == 0) {
    unsigned spins = 0;
    while (__hip_atomic_load(a.bar, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
      __builtin_amdgcn_s_sleep(1);
      if (++spins > (1u << 22)) {
        __hip_atomic_store(a.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
    }
  }
  raw_barrier();

  // ---------------- phase B: down split-K items + finalisation
  for (; item < nitems; item += nw) {
    const int tile = item / Z, z = item % Z;
    if (item != gw) {
      setup(item);
#pragma unroll
      for (int d = 0; d < DB; ++d)
        if (d < nchB) wbB[d] = *(const u32x4*)(wrow + d * 32);
    }
#pragma unroll
    for (int d = 0; d < DB; ++d)
      if (d < nchB) xbB[d] = xvalid ? ld16_sc1(hrow + d * 32) : u32x4{0u, 0u, 0u, 0u};
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    for (int base = 0; base < nchB; base += DB) {
#pragma unroll
      for (int d = 0; d < DB; ++d) {
        const int c = base + d;
        if (c < nchB) {
          acc = mfma16(__builtin_bit_cast(bf16x8, wbB[d]), __builtin_bit_cast(bf16x8, xbB[d]), acc);
          if (c + DB < nchB) {
            wbB[d] = *(const u32x4*)(wrow + (c + DB) * 32);
            xbB[d] = xvalid ? ld16_sc1(hrow + (c + DB) * 32) : u32x4{0u, 0u, 0u, 0u};
          }
        }
      }
    }
    // slab (write-through), ticket, last slice reduces: lane holds C[m = r][n = 16*tile + 4g + 0..3]
    const int n0 = 16 * tile + 4 * g;
    if (xvalid) {
      float* dst = a.part + ((size_t)z * M + r) * H + n0;
      st8_sc1(dst, u32x2{__float_as_uint(acc[0]), __float_as_uint(acc[1])});
      st8_sc1(dst + 2, u32x2{__float_as_uint(acc[2]), __float_as_uint(acc[3])});
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    int old = 0;
    if (lane == 0) old = __hip_atomic_fetch_add(a.fin_cnt + tile, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    old = __shfl(old, 0, 64);
    if (old != Z - 1) continue;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");   // compiler-only: keep the loads below the ticket
    float ssl = 0.f;
    if (xvalid) {
      float* rp = a.resid + (size_t)r * H + n0;
      f32x4 v = *(const f32x4*)rp;
      const f32x4 w = *(const f32x4*)(a.norm_w_next + n0);
      u32x4 sl[8];
#pragma unroll
      for (int zz = 0; zz < 8; ++zz) sl[zz] = ld16_sc1((const bf16_t*)(a.part + ((size_t)min(zz, Z - 1) * M + r) * H + n0));
#pragma unroll
      for (int zz = 0; zz < 8; ++zz) {
        const f32x4 sv = {__uint_as_float(sl[zz][0]), __uint_as_float(sl[zz][1]), __uint_as_float(sl[zz][2]),
                          __uint_as_float(sl[zz][3])};
        v += zz < Z ? sv : f32x4{0.f, 0.f, 0.f, 0.f};
      }
      *(f32x4*)rp = v;
      ssl = v[0] * v[0] + v[1] * v[1] + v[2] * v[2] + v[3] * v[3];
      u32x2 pk;
      pk[0] = pack_bf2(v[0] * (1.0f + w[0]), v[1] * (1.0f + w[1]));
      pk[1] = pack_bf2(v[2] * (1.0f + w[2]), v[3] * (1.0f + w[3]));
      *(u32x2*)(a.x_out + (size_t)r * H + n0) = pk;
    }
    ssl += __shfl_xor(ssl, 16, 64);
    ssl += __shfl_xor(ssl, 32, 64);
    if (g == 0 && xvalid) a.ss_out[(size_t)r * a.ss_ld + tile] = ssl;
    if (lane == 0) __hip_atomic_store(a.fin_cnt + tile, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

static int g_num_cus = 0;

extern "C" int pg_decode_mlp(const PgMlpArgs* args, hipStream_t stream) {
  PG_REQUIRE(args != nullptr);
  const PgMlpArgs& a = *args;
  PG_REQUIRE(a.M >= 1 && a.M <= 2 && a.H % 64 == 0 && a.I % 64 == 0 && a.Z >= 1 && a.Z <= 8 &&
             (a.I / a.Z) % 32 == 0 && a.ss_n > 0 && a.ss_n <= (a.M == 1 ? 256 : 128) && a.ss_ld >= a.H / 16 &&
             a.x && a.ss_in && a.gu_w && a.h && a.down_w && a.part && a.fin_cnt && a.resid && a.ss_out &&
             a.x_out && a.norm_w_next && a.bar && a.err);
  if (g_num_cus == 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&g_num_cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || g_num_cus <= 0)
      return (int)hipErrorInvalidValue;
  }
  // two workgroups per CU (8 waves: 2 per SIMD at <= 256 VGPRs) -- all co-resident
  hipLaunchKernelGGL(decode_mlp_kernel, dim3(PG_MLP_WG_PER_CU * g_num_cus), dim3(256), 0, stream, a);
  PG_LAUNCH_CHECK();
  return 0;
}
