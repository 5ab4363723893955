// Residual-stream normalisation with the split-K reduction of the producing GEMM fused in.
//
//   x        = resid[row] + sum_s partials[s][row]          (fp32; written back to resid if asked)
//   LayerNorm: y = (x - mean) / sqrt(var + eps) * w + b     (nn.LayerNorm, modeling_siglip.py:199,203,310)
//   RMSNorm  : y = x * rsqrt(mean(x^2) + eps) * (1 + w)     (GemmaRMSNorm, modeling_gemma.py:165-182)
//
// The residual stream stays fp32 in HBM (the reference is fp32 end to end); y goes out
// as bf16 for the next MFMA GEMM and optionally as fp32 (module-level API outputs).
// One 256-thread workgroup per row, values held in registers (H <= 4096, H % 4 == 0).
#include "common.h"

#define NORM_MAXV 4   // float4 per thread -> H <= 4096

__global__ __launch_bounds__(256) void norm_residual_kernel(float* __restrict__ resid, const float* __restrict__ partials,
                                                            int nsplit, int M_part, const float* __restrict__ w,
                                                            const float* __restrict__ b, bf16_t* __restrict__ out,
                                                            int ldo, float* __restrict__ out_f32,
                                                            const int* __restrict__ row_map, int H, int mode,
                                                            float eps, int write_resid) {
  __shared__ float red[16];
  const int orow = blockIdx.x;
  const int row = row_map ? row_map[orow] : orow;
  const int H4 = H >> 2;
  float* x = resid + (size_t)row * H;
  f32x4 v[NORM_MAXV];
#pragma unroll
  for (int i = 0; i < NORM_MAXV; ++i) {
    const int c = threadIdx.x + i * 256;
    if (c < H4) {
      f32x4 a = ((const f32x4*)x)[c];
      for (int s = 0; s < nsplit; ++s) a += ((const f32x4*)(partials + ((size_t)s * M_part + row) * H))[c];
      v[i] = a;
      if (write_resid && nsplit > 0) ((f32x4*)x)[c] = a;
    } else {
      v[i] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
  }
  float mean = 0.f, rstd;
  if (mode == 0) {
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < NORM_MAXV; ++i) s += v[i][0] + v[i][1] + v[i][2] + v[i][3];
    mean = block_sum(s, red) / (float)H;
    float q = 0.f;
#pragma unroll
    for (int i = 0; i < NORM_MAXV; ++i) {
      const int c = threadIdx.x + i * 256;
      if (c < H4) {
#pragma unroll
        for (int j = 0; j < 4; ++j) { float d = v[i][j] - mean; q += d * d; }
      }
    }
    rstd = rsqrtf(block_sum(q, red) / (float)H + eps);
  } else {
    float q = 0.f;
#pragma unroll
    for (int i = 0; i < NORM_MAXV; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) q += v[i][j] * v[i][j];
    rstd = rsqrtf(block_sum(q, red) / (float)H + eps);
  }
#pragma unroll
  for (int i = 0; i < NORM_MAXV; ++i) {
    const int c = threadIdx.x + i * 256;
    if (c < H4) {
      const f32x4 wv = ((const f32x4*)w)[c];
      f32x4 y;
      if (mode == 0) {
        const f32x4 bv = ((const f32x4*)b)[c];
#pragma unroll
        for (int j = 0; j < 4; ++j) y[j] = (v[i][j] - mean) * rstd * wv[j] + bv[j];
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) y[j] = (v[i][j] * rstd) * (1.0f + wv[j]);
      }
      if (out) {
        u32x2 p;
        p[0] = pack_bf2(y[0], y[1]);
        p[1] = pack_bf2(y[2], y[3]);
        *(u32x2*)(out + (size_t)orow * ldo + c * 4) = p;
      }
      if (out_f32) ((f32x4*)(out_f32 + (size_t)orow * H))[c] = y;
    }
  }
}

// mode: 0 = LayerNorm (w, b), 1 = Gemma RMSNorm (1 + w).  partials: [nsplit][M_part][H] (may be null).
// row_map (optional, device int32 [M_out]): output row i normalises input row row_map[i].
extern "C" int pg_norm_residual(float* resid, const float* partials, int nsplit, int M_part, const float* w,
                                const float* b, void* out, int ldo, float* out_f32, const int* row_map, int M_out,
                                int H, int mode, float eps, int write_resid, hipStream_t stream) {
  PG_REQUIRE(M_out > 0 && H > 0 && H % 4 == 0 && H <= 256 * 4 * NORM_MAXV);
  PG_REQUIRE(mode == 1 || b != nullptr);
  PG_REQUIRE(nsplit == 0 || partials != nullptr);
  hipLaunchKernelGGL(norm_residual_kernel, dim3(M_out), dim3(256), 0, stream, resid, partials, nsplit, M_part, w, b,
                     (bf16_t*)out, ldo, out_f32, row_map, H, mode, eps, write_resid);
  PG_LAUNCH_CHECK();
  return 0;
}
