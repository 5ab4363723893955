// Shared device helpers for libpghip (gfx950 / CDNA4 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef uint16_t bf16_t;                                       // bf16 storage
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;     // MFMA A/B fragment (4 VGPRs)
typedef __attribute__((ext_vector_type(4))) float f32x4;       // 16x16 accumulator fragment
typedef __attribute__((ext_vector_type(2))) float f32x2;
typedef __attribute__((ext_vector_type(4))) uint32_t u32x4;    // 16-byte raw load
typedef __attribute__((ext_vector_type(2))) uint32_t u32x2;    // 8-byte raw load

#define LDS_AS __attribute__((address_space(3)))

__device__ __forceinline__ float bf2f(bf16_t v) { return __uint_as_float(((uint32_t)v) << 16); }

// round-to-nearest-even f32 -> bf16 (v_cvt_pk_bf16_f32 at -O3; keeps NaN a NaN)
__device__ __forceinline__ bf16_t f2bf(float f) {
  __bf16 b = (__bf16)f;
  return __builtin_bit_cast(bf16_t, b);
}
// two floats -> packed bf16 pair (RNE): one v_cvt_pk_bf16_f32 (converting each half separately costs two
// converts plus a shift and an OR per pair)
typedef __bf16 pg_bf16x2_t __attribute__((ext_vector_type(2)));
typedef float pg_f32x2_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t pack_bf2(float lo, float hi) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(pg_f32x2_t{lo, hi}, pg_bf16x2_t));
}

// the two bf16 halves of a packed pair as floats
__device__ __forceinline__ float bf_lo(uint32_t v) { return __uint_as_float(v << 16); }
__device__ __forceinline__ float bf_hi(uint32_t v) { return __uint_as_float(v & 0xffff0000u); }
// e4m3 bytes of four floats already divided by their row scale (clamped to +-448, round to nearest even)
__device__ __forceinline__ uint32_t pack_fp8x4(float a, float b, float c, float d) {
  int w = __builtin_amdgcn_cvt_pk_fp8_f32(fminf(fmaxf(a, -448.f), 448.f), fminf(fmaxf(b, -448.f), 448.f), 0, false);
  w = __builtin_amdgcn_cvt_pk_fp8_f32(fminf(fmaxf(c, -448.f), 448.f), fminf(fmaxf(d, -448.f), 448.f), w, true);
  return (uint32_t)w;
}

// combine lane l with lane l ^ 16 / l ^ 32 in registers: gfx950's v_permlane16_swap / v_permlane32_swap hand
// back both lanes' values (a VALU op; __shfl_xor is a ds_bpermute round trip through the LDS).  max and + are
// commutative, so the result has the same bits as op(v, __shfl_xor(v, 16 / 32)) in every lane.
__device__ __forceinline__ float max_xor16(float v) {
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
__device__ __forceinline__ float max_xor32(float v) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
__device__ __forceinline__ float sum_xor16(float v) {
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
__device__ __forceinline__ float sum_xor32(float v) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

// the value of lane l ^ 32 (v_permlane32_swap moves the upper half of its first operand's lanes into the lower
// half of the second and back: lanes 0-31 find their partner in the second result, lanes 32-63 in the first)
__device__ __forceinline__ float xchg_xor32(float v) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float((threadIdx.x & 32) ? r[0] : r[1]);
}

__device__ __forceinline__ float gelu_tanh(float x) {
  // torch gelu(approximate="tanh"): 0.5 x (1 + tanh(u)), u = sqrt(2/pi) (x + 0.044715 x^3), evaluated as
  // x * sigmoid(2u) = x / (1 + 2^(-2u log2 e)): one v_exp_f32 + one v_rcp_f32 (~1 ulp each) instead of
  // libm tanhf, exact limits at both tails (x -> 0 for u -> -inf, x for u -> +inf)
  const float u = 0.7978845608028654f * (x + 0.044715f * x * x * x);
  return x * __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(-2.8853900817779268f * u));
}

__device__ __forceinline__ f32x4 mfma16(const bf16x8& a, const bf16x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

typedef __attribute__((ext_vector_type(8))) int i32x8;
typedef __attribute__((ext_vector_type(4))) int i32x4;

// fp8 e4m3 (OCP) 16x16x128 with unit block scales (E8M0 127 = 2^0): 2x the bf16 MFMA rate.  Each operand is
// 32 bytes per lane, given as the two 16-byte chunks (a0, a1) that the bf16 form would consume in two k-steps;
// A and B take the same byte->k assignment, so any consistent k order gives the same dot product.
__device__ __forceinline__ f32x4 mfma8(const bf16x8& a0, const bf16x8& a1, const bf16x8& b0, const bf16x8& b1,
                                       const f32x4& c) {
  const i32x4 x0 = __builtin_bit_cast(i32x4, a0), x1 = __builtin_bit_cast(i32x4, a1);
  const i32x4 y0 = __builtin_bit_cast(i32x4, b0), y1 = __builtin_bit_cast(i32x4, b1);
  const i32x8 a = __builtin_shufflevector(x0, x1, 0, 1, 2, 3, 4, 5, 6, 7);
  const i32x8 b = __builtin_shufflevector(y0, y1, 0, 1, 2, 3, 4, 5, 6, 7);
  return __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, c, 0, 0, 0, 127, 0, 127);
}
// the same with a per-lane E8M0 block scale for B (MX rows: lane (r, g)'s 32 bytes are block g of row r of B)
__device__ __forceinline__ f32x4 mfma8s(const bf16x8& a0, const bf16x8& a1, const bf16x8& b0, const bf16x8& b1,
                                        const f32x4& c, int sb) {
  const i32x4 x0 = __builtin_bit_cast(i32x4, a0), x1 = __builtin_bit_cast(i32x4, a1);
  const i32x4 y0 = __builtin_bit_cast(i32x4, b0), y1 = __builtin_bit_cast(i32x4, b1);
  const i32x8 a = __builtin_shufflevector(x0, x1, 0, 1, 2, 3, 4, 5, 6, 7);
  const i32x8 b = __builtin_shufflevector(y0, y1, 0, 1, 2, 3, 4, 5, 6, 7);
  return __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, c, 0, 0, 0, 127, 0, sb);
}
// Pin finished MFMA accumulators in VGPRs here (straight-line, before any epilogue branch).  Without it the compiler may
// sink a whole v_mfma_scale chain into the epilogue's first guarded block and read its first result register a few
// SALU instructions after the last MFMA on the branch-skipping path -- before the MFMA has written it (measured: the
// last chunk missing from element 0 of every lane of one row tile, profiles/r05_mfma_sink_hazard.txt)
// (16 extra wait states on top of the hazard recognizer's own, once per kernel)
template <int N>
__device__ __forceinline__ void mfma_fence(f32x4 (&a)[N]) {
#ifdef PG_NO_MFMA_FENCE   // (test builds only: tests/test_host.py checks the hazard scan finds the unfenced form)
  return;
#endif
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_nop 7\n\ts_nop 7");
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int i = 0; i < N; ++i) asm volatile("" : "+v"(a[i]));
  __builtin_amdgcn_sched_barrier(0);
}
// E8M0 exponent of an MX block whose max |x| is amax: the smallest e with amax <= 448 * 2^e (0 for a zero block),
// clamped to [-127, 127].  amax = f * 2^k, f in [0.5, 1): f * 512 in [256, 512), so e = k - 9, or k - 8 when f > 7/8.
__device__ __forceinline__ int mx_exp(float amax) {
  if (!(amax > 0.f)) return 0;
  int k;
  const float f = frexpf(amax, &k);
  const int e = k - 9 + (f * 512.f > 448.f ? 1 : 0);
  return min(max(e, -127), 127);
}
__device__ __forceinline__ f32x4 mfma8(const i32x8& a, const i32x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, c, 0, 0, 0, 127, 0, 127);
}
// ... with the lane's E8M0 block scale for B in byte SEL of sb (MX rows in the prefill tile GEMM: one register holds
// the scales of the wave's row subtiles)
template <int SEL>
__device__ __forceinline__ f32x4 mfma8s_sel(const bf16x8& a0, const bf16x8& a1, const bf16x8& b0, const bf16x8& b1,
                                            const f32x4& c, int sb) {
  const i32x4 x0 = __builtin_bit_cast(i32x4, a0), x1 = __builtin_bit_cast(i32x4, a1);
  const i32x4 y0 = __builtin_bit_cast(i32x4, b0), y1 = __builtin_bit_cast(i32x4, b1);
  const i32x8 a = __builtin_shufflevector(x0, x1, 0, 1, 2, 3, 4, 5, 6, 7);
  const i32x8 b = __builtin_shufflevector(y0, y1, 0, 1, 2, 3, 4, 5, 6, 7);
  return __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, c, 0, 0, 0, 127, SEL, sb);
}
__device__ __forceinline__ i32x8 cat8(const bf16x8& lo, const bf16x8& hi) {
  return __builtin_shufflevector(__builtin_bit_cast(i32x4, lo), __builtin_bit_cast(i32x4, hi), 0, 1, 2, 3, 4, 5, 6, 7);
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Whole-block sum of one float per thread (blockDim.x multiple of 64, <= 1024).
__device__ __forceinline__ float block_sum(float v, float* red /* >= 16 floats of LDS */) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  v = wave_sum(v);
  __syncthreads();
  if (lane == 0) red[w] = v;
  __syncthreads();
  float s = 0.f;
  for (int i = 0; i < nw; ++i) s += red[i];
  return s;
}

// a zero word in device memory: read in place of an absent optional device-side scalar, so the load is
// unconditional (no branch or select on a loaded value, which makes hipcc wait for it on the spot)
static __device__ int pg_zero_word = 0;

// error reporting: every C entry point returns a hipError_t as int (0 = ok)
// s_waitcnt vmcnt(n) for a wave-uniform runtime n (the counter field takes an immediate); n > 40 waits for all
#define PG_VMC(k) case k: asm volatile("s_waitcnt vmcnt(" #k ")" ::: "memory"); break;
__device__ __forceinline__ void wait_vm_n(int n) {
  switch (n) {
    PG_VMC(1) PG_VMC(2) PG_VMC(3) PG_VMC(4) PG_VMC(5) PG_VMC(6) PG_VMC(7) PG_VMC(8) PG_VMC(9) PG_VMC(10)
    PG_VMC(11) PG_VMC(12) PG_VMC(13) PG_VMC(14) PG_VMC(15) PG_VMC(16) PG_VMC(17) PG_VMC(18) PG_VMC(19) PG_VMC(20)
    PG_VMC(21) PG_VMC(22) PG_VMC(23) PG_VMC(24) PG_VMC(25) PG_VMC(26) PG_VMC(27) PG_VMC(28) PG_VMC(29) PG_VMC(30)
    PG_VMC(31) PG_VMC(32) PG_VMC(33) PG_VMC(34) PG_VMC(35) PG_VMC(36) PG_VMC(37) PG_VMC(38) PG_VMC(39) PG_VMC(40)
    default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
  }
}
#undef PG_VMC

#define PG_LAUNCH_CHECK() do { hipError_t _e = hipGetLastError(); if (_e != hipSuccess) return (int)_e; } while (0)
#define PG_REQUIRE(cond) do { if (!(cond)) return (int)hipErrorInvalidValue; } while (0)
