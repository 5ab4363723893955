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
#ifndef PG_NORM_W_EARLY
#define PG_NORM_W_EARLY 1   // norm weights / bias loaded with the residual (not after the reductions)
#endif
// Split-K slabs loaded per round (SG) and float4 slots per thread (MAXV) are template parameters: 8 slabs per round
// pays where few rows carry many slabs (batch-1 prefill: 16-slab down projection), but its 214 registers (two
// waves per SIMD) tripled the 16 k-row norms of pt-448 x16 (55 -> 151 us each, 85 -> 93 ms per prefill): large
// launches take 2 slabs per round and the H <= 2048 slot count (pg_norm_residual picks).

// Q8: y goes out as fp8 e4m3 bytes (out = uint8 [M][ldo]) with its row scale in out_f32[orow] (the
// pg_quant_fp8 rule applied to the bf16-rounded y, so the bytes equal quantising the bf16 output).
template <bool Q8, int NORM_SG, int MAXV>
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
  const int nv = (H4 + 255) >> 8;                  // float4 slots in use per thread (wave-uniform)
  float* x = resid + (size_t)row * H;
  f32x4 v[MAXV];
  // the norm weights (and LayerNorm bias) are loaded with the residual, not after the reductions: one dependent
  // round trip fewer at the end of every launch
  f32x4 wv[MAXV], bv[MAXV];
#pragma unroll
  for (int i = 0; i < MAXV; ++i)
    if (PG_NORM_W_EARLY && i < nv) {
      const int c = min((int)threadIdx.x + i * 256, H4 - 1);
      wv[i] = ((const f32x4*)w)[c];
      bv[i] = mode == 0 ? ((const f32x4*)b)[c] : f32x4{0.f, 0.f, 0.f, 0.f};
    }
  // the residual and the split-K slabs, NORM_SG slabs per round with every load of a round issued before the
  // first add (columns past H re-read the last column, dropped after the loads): one memory round trip per round
  // instead of one per slab (the runtime-bounded add loop waited for each slab's load before issuing the next --
  // SigLIP's 6-slab LayerNorm took 6.9 us).  Slabs past nsplit are not loaded (wave-uniform guard): re-reading the
  // last slab in their place multiplied a one-slab norm's L2 reads by NORM_SG at pt-448 x16 (135 MB slabs)
#pragma unroll
  for (int i = 0; i < MAXV; ++i)
    if (i < nv) v[i] = ((const f32x4*)x)[min((int)threadIdx.x + i * 256, H4 - 1)];
  for (int s0 = 0; s0 < nsplit; s0 += NORM_SG) {
    f32x4 p[MAXV][NORM_SG];
#pragma unroll
    for (int i = 0; i < MAXV; ++i)
      if (i < nv) {
        const int c = min((int)threadIdx.x + i * 256, H4 - 1);
#pragma unroll
        for (int k = 0; k < NORM_SG; ++k)
          p[i][k] = s0 + k < nsplit ? ((const f32x4*)(partials + ((size_t)(s0 + k) * M_part + row) * H))[c]
                                    : f32x4{0.f, 0.f, 0.f, 0.f};
      }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int i = 0; i < MAXV; ++i)
      if (i < nv) {
#pragma unroll
        for (int k = 0; k < NORM_SG; ++k)
          if (s0 + k < nsplit) v[i] += p[i][k];
      }
  }
#pragma unroll
  for (int i = 0; i < MAXV; ++i) {
    const int c = threadIdx.x + i * 256;
    if (c >= H4 || i >= nv) v[i] = f32x4{0.f, 0.f, 0.f, 0.f};
    else if (write_resid && nsplit > 0) ((f32x4*)x)[c] = v[i];
  }
  float mean = 0.f, rstd;
  if (mode == 0) {
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < MAXV; ++i) s += v[i][0] + v[i][1] + v[i][2] + v[i][3];
    mean = block_sum(s, red) / (float)H;
    float q = 0.f;
#pragma unroll
    for (int i = 0; i < MAXV; ++i) {
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
    for (int i = 0; i < MAXV; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) q += v[i][j] * v[i][j];
    rstd = rsqrtf(block_sum(q, red) / (float)H + eps);
  }
  float amax = 0.f;
#pragma unroll
  for (int i = 0; i < MAXV; ++i) {
    const int c = threadIdx.x + i * 256;
    if (c < H4) {
      f32x4 y;
      if (!PG_NORM_W_EARLY) {
        wv[i] = ((const f32x4*)w)[c];
        bv[i] = mode == 0 ? ((const f32x4*)b)[c] : f32x4{0.f, 0.f, 0.f, 0.f};
      }
      if (mode == 0) {
#pragma unroll
        for (int j = 0; j < 4; ++j) y[j] = (v[i][j] - mean) * rstd * wv[i][j] + bv[i][j];
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) y[j] = (v[i][j] * rstd) * (1.0f + wv[i][j]);
      }
      if constexpr (Q8) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          v[i][j] = __uint_as_float((uint32_t)f2bf(y[j]) << 16);     // the bf16 value the GEMM would have read
          amax = fmaxf(amax, fabsf(v[i][j]));
        }
        continue;
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
  if constexpr (Q8) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) amax = fmaxf(amax, __shfl_xor(amax, o, 64));
    __syncthreads();
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = amax;
    __syncthreads();
    amax = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
    const float sc = amax > 0.f ? amax / 448.f : 1.f;
    if (threadIdx.x == 0) out_f32[orow] = sc;
    uint8_t* q = (uint8_t*)out + (size_t)orow * ldo;
#pragma unroll
    for (int i = 0; i < MAXV; ++i) {
      const int c = threadIdx.x + i * 256;
      if (c < H4) {
        float t[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) t[j] = fminf(fmaxf(v[i][j] / sc, -448.f), 448.f);
        int wq = __builtin_amdgcn_cvt_pk_fp8_f32(t[0], t[1], 0, false);
        wq = __builtin_amdgcn_cvt_pk_fp8_f32(t[2], t[3], wq, true);
        *(uint32_t*)(q + c * 4) = (uint32_t)wq;
      }
    }
  }
}

template <bool Q8>
static void norm_launch(int M_out, int H, int nsplit, hipStream_t stream, float* resid, const float* partials,
                        int M_part, const float* w, const float* b, void* out, int ldo, float* out_f32,
                        const int* row_map, int mode, float eps, int write_resid) {
  const bool deep = nsplit > 2 && M_out <= 2048;      // few rows, many slabs: one round trip per 8 slabs
  const bool wide = H > 2048;
#define PG_NORM_GO(SG_, MV_)                                                                                    \
  hipLaunchKernelGGL((norm_residual_kernel<Q8, SG_, MV_>), dim3(M_out), dim3(256), 0, stream, resid, partials,   \
                     nsplit, M_part, w, b, (bf16_t*)out, ldo, out_f32, row_map, H, mode, eps, write_resid)
  if (deep && wide) PG_NORM_GO(8, 4);
  else if (deep) PG_NORM_GO(8, 2);
  else if (wide) PG_NORM_GO(2, 4);
  else PG_NORM_GO(2, 2);
#undef PG_NORM_GO
}

// mode: 0 = LayerNorm (w, b), 1 = Gemma RMSNorm (1 + w).  partials: [nsplit][M_part][H] (may be null).
// row_map (optional, device int32 [M_out]): output row i normalises input row row_map[i].
extern "C" int pg_norm_residual(float* resid, const float* partials, int nsplit, int M_part, const float* w,
                                const float* b, void* out, int ldo, float* out_f32, const int* row_map, int M_out,
                                int H, int mode, float eps, int write_resid, hipStream_t stream) {
  PG_REQUIRE(resid && w && M_out > 0 && H > 0 && H % 4 == 0 && H <= 256 * 4 * NORM_MAXV);
  PG_REQUIRE(mode == 1 || b != nullptr);
  PG_REQUIRE(nsplit == 0 || partials != nullptr);
  norm_launch<false>(M_out, H, nsplit, stream, resid, partials, M_part, w, b, out, ldo, out_f32, row_map, mode, eps,
                     write_resid);
  PG_LAUNCH_CHECK();
  return 0;
}

// The same normalisation with y quantised to fp8 e4m3 for a PG_FP8 GEMM: q uint8 [M_out][ldq], scale [M_out]
// (pg_quant_fp8 of the bf16 output, fused: one launch and no bf16 round trip).  H % 4 == 0, ldq % 4 == 0.
extern "C" int pg_norm_residual_fp8(float* resid, const float* partials, int nsplit, int M_part, const float* w,
                                    const float* b, void* q, int ldq, float* scale, const int* row_map, int M_out,
                                    int H, int mode, float eps, int write_resid, hipStream_t stream) {
  PG_REQUIRE(resid && w && M_out > 0 && H > 0 && H % 4 == 0 && H <= 256 * 4 * NORM_MAXV && q != nullptr && scale != nullptr &&
             ldq >= H && ldq % 4 == 0);
  PG_REQUIRE(mode == 1 || b != nullptr);
  PG_REQUIRE(nsplit == 0 || partials != nullptr);
  norm_launch<true>(M_out, H, nsplit, stream, resid, partials, M_part, w, b, q, ldq, scale, row_map, mode, eps,
                    write_resid);
  PG_LAUNCH_CHECK();
  return 0;
}

// Gemma RMSNorm for MX fp8 consumers (17..32-row fp8 decode, engine.MX_NORM): x = resid + sum_s partials[s] (slab
// order; written back when write_resid), y = x * (1 + w) as e4m3 bytes q [M][ldq] with one E8M0 scale per 32
// columns (qs [M][4][H/128], the PgFusedArgs.mx_out rule and layout), and ss [M][ss_ld] the sum of x^2 over each
// 1024 columns.  The row's rstd is left to the consumer (PgFusedArgs.mx_in + ss_in): no row-wide reduction here, so
// every (1024 columns, row) is its own workgroup -- H/1024 x M workgroups, one memory round trip.
__global__ __launch_bounds__(256) void norm_mx_kernel(float* __restrict__ resid, const float* __restrict__ partials,
                                                      int nsplit, int M_part, const float* __restrict__ w,
                                                      uint8_t* __restrict__ q, int ldq, uint8_t* __restrict__ qs,
                                                      float* __restrict__ ss, int ss_ld, int H, int write_resid) {
  const int t = threadIdx.x, m = blockIdx.y, c = blockIdx.x * 1024 + 4 * t;
  const size_t o = (size_t)m * H + c;
  f32x4 x = *(const f32x4*)(resid + o);
  const f32x4 wv = *(const f32x4*)(w + c);
  constexpr int SG = 8;                            // slabs per round trip
  for (int s0 = 0; s0 < nsplit; s0 += SG) {
    f32x4 p[SG];
#pragma unroll
    for (int j = 0; j < SG; ++j) p[j] = *(const f32x4*)(partials + (size_t)min(s0 + j, nsplit - 1) * M_part * H + o);
#pragma unroll
    for (int j = 0; j < SG; ++j)
      if (s0 + j < nsplit) x += p[j];
  }
  if (write_resid) *(f32x4*)(resid + o) = x;
  f32x4 y;
  float am = 0.f;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    y[j] = x[j] * (1.f + wv[j]);
    am = fmaxf(am, fabsf(y[j]));
  }
  am = fmaxf(am, __shfl_xor(am, 1, 64));           // the 8 lanes of a 32-column block
  am = fmaxf(am, __shfl_xor(am, 2, 64));
  am = fmaxf(am, __shfl_xor(am, 4, 64));
  const int ex = mx_exp(am);
  const float inv = __builtin_ldexpf(1.0f, -ex);
  *(uint32_t*)(q + (size_t)m * ldq + c) = pack_fp8x4(y[0] * inv, y[1] * inv, y[2] * inv, y[3] * inv);
  if ((t & 7) == 0) {
    const int kb = c >> 5;
    qs[(size_t)m * (H >> 5) + (size_t)(kb & 3) * (H >> 7) + (kb >> 2)] = (uint8_t)(ex + 127);
  }
  __shared__ float sw[4];
  const float s2 = wave_sum(x[0] * x[0] + x[1] * x[1] + x[2] * x[2] + x[3] * x[3]);
  if ((t & 63) == 0) sw[t >> 6] = s2;
  __syncthreads();
  if (t == 0) ss[(size_t)m * ss_ld + blockIdx.x] = (sw[0] + sw[1]) + (sw[2] + sw[3]);
}

extern "C" int pg_norm_residual_mx(float* resid, const float* partials, int nsplit, int M_part, const float* w,
                                   void* q, int ldq, void* qs, float* ss, int ss_ld, int M, int H, int write_resid,
                                   hipStream_t stream) {
  PG_REQUIRE(resid && w && M > 0 && M <= M_part && H > 0 && H % 1024 == 0 && q && qs && ss && ldq >= H && ldq % 4 == 0 &&
             ss_ld >= H / 1024 && nsplit >= 0 && (nsplit == 0 || partials));
  PG_REQUIRE(((uintptr_t)resid & 15) == 0 && ((uintptr_t)w & 15) == 0 && ((uintptr_t)q & 3) == 0 &&
             ((uintptr_t)partials & 15) == 0);
  hipLaunchKernelGGL(norm_mx_kernel, dim3(H / 1024, M), dim3(256), 0, stream, resid, partials, nsplit, M_part, w,
                     (uint8_t*)q, ldq, (uint8_t*)qs, ss, ss_ld, H, write_resid);
  PG_LAUNCH_CHECK();
  return 0;
}
