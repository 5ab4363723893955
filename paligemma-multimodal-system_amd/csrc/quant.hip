// fp8 e4m3 (OCP) row quantisation for the fp8 GEMM path (BASELINE configs[4]; SURVEY.md §8(a) "fp8 MFMA").
//
// q[m][k] = e4m3(x[m][k] / s[m]), s[m] = max_k |x[m][k]| / 448 (1 for an all-zero row): one scale per
// activation row (token) here, one per output channel for the weights (pghip/weights.py, done once at load).
// The GEMM multiplies its fp32 accumulator by s_a[m] * s_w[n] before the epilogue (csrc/gemm.hip PG_FP8).
//
// x / s is a correctly rounded division (the same value torch computes in pghip/weights.py quant_rows_fp8),
// and the conversion rounds to nearest even, so both quantisers produce identical bytes.
// One 256-thread workgroup per row for K > 32768 (the row read twice), else quant_fp8_row1k_kernel below.
// HBM-bound: 2 + 1 bytes per element.
#include "common.h"

__global__ __launch_bounds__(256) void quant_fp8_rows_kernel(const bf16_t* __restrict__ x, int ldx, int K,
                                                             uint8_t* __restrict__ q, int ldq,
                                                             float* __restrict__ scale) {
  __shared__ float red[4];
  const int m = blockIdx.x, tid = threadIdx.x;
  const bf16_t* xr = x + (size_t)m * ldx;
  float amax = 0.f;
  for (int k = tid * 8; k < K; k += 2048) {
    const u32x4 v = *(const u32x4*)(xr + k);
#pragma unroll
    for (int j = 0; j < 4; ++j) amax = fmaxf(amax, fmaxf(fabsf(bf_lo(v[j])), fabsf(bf_hi(v[j]))));
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) amax = fmaxf(amax, __shfl_xor(amax, o, 64));
  if ((tid & 63) == 0) red[tid >> 6] = amax;
  __syncthreads();
  amax = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  const float s = amax > 0.f ? amax / 448.f : 1.f;
  if (tid == 0) scale[m] = s;
  uint8_t* qr = q + (size_t)m * ldq;
  for (int k = tid * 8; k < K; k += 2048) {
    const u32x4 v = *(const u32x4*)(xr + k);
    u32x2 o;
#pragma unroll
    for (int j = 0; j < 2; ++j)
      o[j] = pack_fp8x4(bf_lo(v[2 * j]) / s, bf_hi(v[2 * j]) / s, bf_lo(v[2 * j + 1]) / s, bf_hi(v[2 * j + 1]) / s);
    *(u32x2*)(qr + k) = o;
  }
}

// One 1024-thread workgroup per row, the row held in registers (V 16-byte pieces per thread, K <= 8192 V): one pass
// over x.  The 256-thread two-pass kernel above took 7.3 us for the 32 rows x 16384 of the batch-32 fp8 decode's h
// (32 workgroups, 64 correctly rounded divisions and two loads per thread in series).
template <int V>
__global__ __launch_bounds__(1024) void quant_fp8_row1k_kernel(const bf16_t* __restrict__ x, int ldx, int K,
                                                               uint8_t* __restrict__ q, int ldq,
                                                               float* __restrict__ scale) {
  __shared__ float red[16];
  const int m = blockIdx.x, tid = threadIdx.x;
  const bf16_t* xr = x + (size_t)m * ldx;
  u32x4 v[V];
  float amax = 0.f;
#pragma unroll
  for (int i = 0; i < V; ++i) {
    const int k = (tid + i * 1024) * 8;
    v[i] = k < K ? *(const u32x4*)(xr + k) : u32x4{0u, 0u, 0u, 0u};
  }
#pragma unroll
  for (int i = 0; i < V; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) amax = fmaxf(amax, fmaxf(fabsf(bf_lo(v[i][j])), fabsf(bf_hi(v[i][j]))));
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) amax = fmaxf(amax, __shfl_xor(amax, o, 64));
  if ((tid & 63) == 0) red[tid >> 6] = amax;
  __syncthreads();
  amax = red[0];
#pragma unroll
  for (int w = 1; w < 16; ++w) amax = fmaxf(amax, red[w]);
  const float s = amax > 0.f ? amax / 448.f : 1.f;
  if (tid == 0) scale[m] = s;
  uint8_t* qr = q + (size_t)m * ldq;
#pragma unroll
  for (int i = 0; i < V; ++i) {
    const int k = (tid + i * 1024) * 8;
    if (k < K) {
      u32x2 o;
#pragma unroll
      for (int j = 0; j < 2; ++j)
        o[j] = pack_fp8x4(bf_lo(v[i][2 * j]) / s, bf_hi(v[i][2 * j]) / s, bf_lo(v[i][2 * j + 1]) / s,
                          bf_hi(v[i][2 * j + 1]) / s);
      *(u32x2*)(qr + k) = o;
    }
  }
}

// One wave per row (4 rows per 256-thread workgroup), V 16-byte pieces per lane (K <= 512 V): for the many-row
// inputs of the fp8 prefill (pt-896 x32: 131,328 rows x 2048, the o_proj's attention rows), where the 1024-thread
// form leaves three quarters of its threads idle at K = 2048 (0.45 ms = 1.8 TB/s for 0.8 GB).  Same arithmetic (row
// max, correctly rounded x / s, round-to-nearest-even e4m3): the same bytes.
template <int V>
__global__ __launch_bounds__(256) void quant_fp8_wave_kernel(const bf16_t* __restrict__ x, int ldx, int M, int K,
                                                             uint8_t* __restrict__ q, int ldq,
                                                             float* __restrict__ scale) {
  const int lane = threadIdx.x & 63;
  const int m = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (m >= M) return;                                    // (wave-uniform: the rows past M leave whole)
  const bf16_t* xr = x + (size_t)m * ldx;
  u32x4 v[V];
#pragma unroll
  for (int i = 0; i < V; ++i) {
    const int k = (lane + i * 64) * 8;
    v[i] = k < K ? *(const u32x4*)(xr + k) : u32x4{0u, 0u, 0u, 0u};
  }
  float amax = 0.f;
#pragma unroll
  for (int i = 0; i < V; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) amax = fmaxf(amax, fmaxf(fabsf(bf_lo(v[i][j])), fabsf(bf_hi(v[i][j]))));
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) amax = fmaxf(amax, __shfl_xor(amax, o, 64));
  const float s = amax > 0.f ? amax / 448.f : 1.f;
  if (lane == 0) scale[m] = s;
  uint8_t* qr = q + (size_t)m * ldq;
#pragma unroll
  for (int i = 0; i < V; ++i) {
    const int k = (lane + i * 64) * 8;
    if (k < K) {
      u32x2 o;
#pragma unroll
      for (int j = 0; j < 2; ++j)
        o[j] = pack_fp8x4(bf_lo(v[i][2 * j]) / s, bf_hi(v[i][2 * j]) / s, bf_lo(v[i][2 * j + 1]) / s,
                          bf_hi(v[i][2 * j + 1]) / s);
      *(u32x2*)(qr + k) = o;
    }
  }
}

#ifndef PG_QUANT_WAVE_MIN_M
#define PG_QUANT_WAVE_MIN_M 1024   // rows from which the wave-per-row form is used
#endif

// x bf16 [M][K] (row stride ldx) -> q fp8 e4m3 [M][K] (row stride ldq bytes), scale f32 [M].
// K % 8 == 0, ldx % 8 == 0, ldq % 8 == 0, 16-byte aligned x.
extern "C" int pg_quant_fp8(const void* x, int ldx, int M, int K, void* q, int ldq, float* scale, hipStream_t stream) {
  PG_REQUIRE(x != nullptr && q != nullptr && scale != nullptr && M > 0 && K > 0 && K % 8 == 0 && ldx >= K &&
             ldx % 8 == 0 && ldq >= K && ldq % 8 == 0 && ((uintptr_t)x & 15) == 0 && ((uintptr_t)q & 7) == 0);
  if (M >= PG_QUANT_WAVE_MIN_M && K <= 4096) {
    const dim3 g((M + 3) / 4);
    if (K <= 2048)
      hipLaunchKernelGGL(quant_fp8_wave_kernel<4>, g, dim3(256), 0, stream, (const bf16_t*)x, ldx, M, K, (uint8_t*)q,
                         ldq, scale);
    else
      hipLaunchKernelGGL(quant_fp8_wave_kernel<8>, g, dim3(256), 0, stream, (const bf16_t*)x, ldx, M, K, (uint8_t*)q,
                         ldq, scale);
  } else if (K <= 8192)
    hipLaunchKernelGGL(quant_fp8_row1k_kernel<1>, dim3(M), dim3(1024), 0, stream, (const bf16_t*)x, ldx, K,
                       (uint8_t*)q, ldq, scale);
  else if (K <= 16384)
    hipLaunchKernelGGL(quant_fp8_row1k_kernel<2>, dim3(M), dim3(1024), 0, stream, (const bf16_t*)x, ldx, K,
                       (uint8_t*)q, ldq, scale);
  else if (K <= 32768)
    hipLaunchKernelGGL(quant_fp8_row1k_kernel<4>, dim3(M), dim3(1024), 0, stream, (const bf16_t*)x, ldx, K,
                       (uint8_t*)q, ldq, scale);
  else
    hipLaunchKernelGGL(quant_fp8_rows_kernel, dim3(M), dim3(256), 0, stream, (const bf16_t*)x, ldx, K, (uint8_t*)q,
                       ldq, scale);
  PG_LAUNCH_CHECK();
  return 0;
}
