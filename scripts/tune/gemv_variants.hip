// Tuning harness (not part of libpghip): decode GEMV variants y[M][N] = x[M][K] . W[N][K]^T, M <= 16.
// Built by scripts/tune/tune_gemv.py into its own .so; the winner is folded into csrc/gemm.hip.
//
// Template knobs:
//   U     : 16-byte loads per lane per 16-row tile per chunk (chunk = 32U k, lane bytes contiguous)
//   DEPTH : chunks kept in flight (register ring)
//   WPT   : waves cooperating on one tile (K split inside the workgroup, LDS reduce)
//   NT    : 16-row tiles per wave (shared x fragments)
//   NTL   : use non-temporal loads for W
#include "../../paligemma-multimodal-system_amd/csrc/common.h"

template <int U, int DEPTH, int WPT, int NT, bool NTL>
__global__ __launch_bounds__(256) void gemv_v(const bf16_t* __restrict__ A, int lda, const bf16_t* __restrict__ W,
                                              int ldw, int K, float* __restrict__ out, int N, int M) {
  constexpr int CH = U * 32;
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int g = lane >> 4, r = lane & 15;
  const int tgrp = wave / WPT;            // tile group inside the WG
  const int wk = wave % WPT;              // K slice of this wave
  constexpr int TG = 4 / WPT;             // tile groups per WG
  const int tile0 = (blockIdx.x * TG + tgrp) * NT;
  const bool xvalid = r < M;
  const bf16_t* xrow = A + (size_t)(xvalid ? r : 0) * lda;
  const bf16_t* wrow[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    int n = (tile0 + t) * 16 + r;
    n = n < N ? n : N - 1;
    wrow[t] = W + (size_t)n * ldw;
  }
  f32x4 acc[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int nch_all = K / CH;
  const int zsplit = gridDim.y, z = blockIdx.y;
  const int per_z = (nch_all + zsplit - 1) / zsplit;
  const int c0 = z * per_z;
  const int nch = min(nch_all - c0, per_z);  // chunks of this split; wave wk takes wk, wk+WPT, ...
  const int mine = nch > wk ? (nch - wk + WPT - 1) / WPT : 0;
  u32x4 wb[DEPTH][NT][U];
  u32x4 xb[DEPTH][U];
  auto load = [&](int d_unused, int j, u32x4 (&wv)[NT][U], u32x4 (&xv)[U]) {
    const int off = (c0 + wk + j * WPT) * CH + g * 8 * U;
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int s = 0; s < U; ++s) {
        const u32x4* p = (const u32x4*)(wrow[t] + off + 8 * s);
        wv[t][s] = NTL ? __builtin_nontemporal_load(p) : *p;
      }
#pragma unroll
    for (int s = 0; s < U; ++s) xv[s] = xvalid ? *(const u32x4*)(xrow + off + 8 * s) : u32x4{0u, 0u, 0u, 0u};
  };
#pragma unroll
  for (int d = 0; d < DEPTH; ++d)
    if (d < mine) load(d, d, wb[d], xb[d]);
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
        if (j + DEPTH < mine) load(d, j + DEPTH, wb[d], xb[d]);
      }
    }
  }
  if constexpr (WPT > 1) {
    __shared__ f32x4 red[4][NT][64];
#pragma unroll
    for (int t = 0; t < NT; ++t) red[wave][t][lane] = acc[t];
    __syncthreads();
    if (wk != 0) return;
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      f32x4 s = red[wave][t][lane];
#pragma unroll
      for (int w = 1; w < WPT; ++w) s += red[wave + w][t][lane];
      acc[t] = s;
    }
  }
  if (r < M) {
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const int n0 = (tile0 + t) * 16 + 4 * g;
      if (n0 + 3 < N) *(f32x4*)(out + ((size_t)z * M + r) * N + n0) = acc[t];
    }
  }
}

#define V(U, D, WPT, NT, NTL) \
  {U, D, WPT, NT, NTL, (void*)gemv_v<U, D, WPT, NT, NTL>}

struct Variant { int U, D, WPT, NT, NTL; void* fn; };
static Variant variants[] = {
  V(4, 2, 4, 1, false), V(2, 8, 1, 1, false), V(2, 4, 4, 1, false), V(2, 8, 4, 1, false),
  V(2, 8, 2, 1, false), V(4, 4, 1, 1, false), V(4, 4, 2, 1, false), V(4, 4, 4, 1, false),
  V(2, 4, 2, 1, false), V(1, 8, 4, 1, false), V(1, 16, 1, 1, false), V(2, 6, 1, 1, false),
  V(4, 3, 4, 1, false), V(2, 8, 1, 1, true), V(4, 2, 2, 2, false), V(2, 4, 4, 2, false),
};

extern "C" int gemv_variant_count() { return sizeof(variants) / sizeof(variants[0]); }
extern "C" void gemv_variant_desc(int i, int* d) {
  d[0] = variants[i].U; d[1] = variants[i].D; d[2] = variants[i].WPT; d[3] = variants[i].NT; d[4] = variants[i].NTL;
}
extern "C" int gemv_variant_run(int i, const void* A, int lda, const void* W, int ldw, int K, float* out, int N, int M,
                                int zsplit, hipStream_t st) {
  const Variant& v = variants[i];
  const int CH = v.U * 32;
  if (K % (CH * v.WPT) != 0 && K % CH != 0) return 1;
  const int tiles = (N + 15) / 16;
  const int tpw = (4 / v.WPT) * v.NT;   // tiles per WG
  dim3 grid((tiles + tpw - 1) / tpw, zsplit);
  void* args[] = {(void*)&A, (void*)&lda, (void*)&W, (void*)&ldw, (void*)&K, (void*)&out, (void*)&N, (void*)&M};
  return (int)hipLaunchKernel(v.fn, grid, dim3(256), args, 0, st);
}
