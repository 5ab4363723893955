// bf16 MFMA GEMMs with fused epilogues:  C[m][n] = sum_k A[m][k] * W[n][k]  (+ epilogue)
//
// A: activations, bf16 row-major (lda).  W: nn.Linear weight layout [N][K] (ldw),
// bf16, K zero-padded to a multiple of 64 at pack time.  fp32 accumulation.
//
// Two kernels:
//  * gemm_tile_kernel : 128x128x64 tiles, 4 waves (2x2, 64x64 each), A and W tiles
//    staged HBM->LDS by global_load_lds (16 B/lane) into a double-buffered,
//    XOR-swizzled LDS image; mfma_f32_16x16x32_bf16 with the operands swapped
//    (MFMA-A = W, MFMA-B = A) so each lane ends with 4 consecutive n of one m —
//    8/16-byte epilogue stores.  Used for prefill (M = tokens).
//  * gemv_kernel      : M <= 16 (decode).  Weight streaming: each wave reads
//    16 rows of W with 16U-byte contiguous non-temporal loads per lane straight
//    into VGPRs (no LDS round trip), the k order inside an MFMA step is permuted
//    identically for both operands so a lane's bytes are contiguous; 4 waves per
//    workgroup split K and reduce through LDS; an optional second level of
//    split-K writes fp32 partial slabs that the next norm kernel reduces.
//
// Replaces the nn.Linear call sites of modeling_siglip.py:59-62,177-178,
// modeling_paligemma.py:57, modeling_gemma.py:205-207,255-259,484.
#include "common.h"

enum {
  PG_EPI_BF16 = 0,          // C bf16 = acc + bias
  PG_EPI_BF16_GELU = 1,     // C bf16 = gelu_tanh(acc + bias)
  PG_EPI_BF16_GELU_MUL = 2, // W rows interleaved in 16-row blocks (gate, up); C bf16 [M][N/2] = gelu(g)*u
  PG_EPI_F32 = 3,           // C f32 [z][M][ldc] = acc (+ bias on split 0)
  PG_EPI_F32_POS = 4,       // C f32 = acc + bias + aux[(m % aux_rows) * ldc + n]  (patch + position emb)
  PG_EPI_BF16_VT = 5,       // n < aux_n: C bf16 = acc + bias ; n >= aux_n: aux_out bf16 [(n-aux_n)][m] (ld aux_ld)
};

struct EpiArgs {
  const float* bias;
  void* C;
  int ldc;
  int M, N;
  const float* aux;
  int aux_rows;
  bf16_t* aux_out;
  int aux_ld;
  int aux_n;
};

// Store 4 consecutive columns n0..n0+3 of row m (values v).  z = split index.
template <int EPI>
__device__ __forceinline__ void epi_store4(const EpiArgs& e, int m, int n0, f32x4 v, int z) {
  if (m >= e.M) return;
  if constexpr (EPI == PG_EPI_F32) {
    float* C = (float*)e.C + (size_t)z * e.M * e.ldc + (size_t)m * e.ldc;
    if (e.bias && z == 0) {
#pragma unroll
      for (int j = 0; j < 4; ++j) if (n0 + j < e.N) v[j] += e.bias[n0 + j];
    }
    if (n0 + 3 < e.N) {
      *(f32x4*)(C + n0) = v;
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) if (n0 + j < e.N) C[n0 + j] = v[j];
    }
  } else if constexpr (EPI == PG_EPI_F32_POS) {
    float* C = (float*)e.C + (size_t)m * e.ldc;
    const float* P = e.aux + (size_t)(m % e.aux_rows) * e.ldc;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      int n = n0 + j;
      if (n < e.N) C[n] = v[j] + e.bias[n] + P[n];
    }
  } else {
    // bf16 outputs
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      int n = n0 + j;
      float x = v[j];
      if (e.bias && n < e.N) x += e.bias[n];
      if constexpr (EPI == PG_EPI_BF16_GELU) x = gelu_tanh(x);
      v[j] = x;
    }
    if constexpr (EPI == PG_EPI_BF16_VT) {
      if (n0 >= e.aux_n) {
#pragma unroll
        for (int j = 0; j < 4; ++j)
          if (n0 + j < e.N) e.aux_out[(size_t)(n0 + j - e.aux_n) * e.aux_ld + m] = f2bf(v[j]);
        return;
      }
    }
    bf16_t* C = (bf16_t*)e.C + (size_t)m * e.ldc;
    if (n0 + 3 < e.N) {
      u32x2 p;
      p[0] = pack_bf2(v[0], v[1]);
      p[1] = pack_bf2(v[2], v[3]);
      *(u32x2*)(C + n0) = p;
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) if (n0 + j < e.N) C[n0 + j] = f2bf(v[j]);
    }
  }
}

// gelu(gate) * up for an interleaved pair: gate tile at global col base gb (multiple of 32),
// lane's 4 columns are gb + q..q+3 (gate) and gb + 16 + q.. (up); output col = gb/2 + q.
__device__ __forceinline__ void epi_gelu_mul4(const EpiArgs& e, int m, int gb, int q, f32x4 g, f32x4 u) {
  if (m >= e.M) return;
  const int oc = (gb >> 1) + q;
  if (oc + 3 >= (e.N >> 1)) return;
  u32x2 p;
  p[0] = pack_bf2(gelu_tanh(g[0]) * u[0], gelu_tanh(g[1]) * u[1]);
  p[1] = pack_bf2(gelu_tanh(g[2]) * u[2], gelu_tanh(g[3]) * u[3]);
  *(u32x2*)((bf16_t*)e.C + (size_t)m * e.ldc + oc) = p;
}

// --------------------------------------------------------------------------------------
// Tiled GEMM (prefill)
// --------------------------------------------------------------------------------------
#define TBM 128
#define TBN 128
#define TBK 64
#define TILE_BYTES (TBM * TBK * 2)   // 16 KiB per operand tile

// Stage a 128-row x 64-k bf16 tile into LDS (lane-linear 1 KiB pieces, XOR swizzle on the source).
__device__ __forceinline__ void stage_tile(const bf16_t* __restrict__ src, int ld, int row0, int rows_valid,
                                           int k0, char* lds_tile, int wave, int lane) {
#pragma unroll
  for (int it = 0; it < 4; ++it) {
    const int blk = wave * 4 + it;                 // 1 KiB piece = 8 rows x 128 B
    const int r = blk * 8 + (lane >> 3);
    const int c = (lane & 7) ^ ((r >> 1) & 7);     // logical 16-B chunk landing at physical chunk lane&7
    int gr = row0 + r;
    gr = gr < rows_valid ? gr : rows_valid - 1;
    const bf16_t* g = src + (size_t)gr * ld + k0 + c * 8;
    __builtin_amdgcn_global_load_lds((const void*)g, (LDS_AS void*)(lds_tile + blk * 1024), 16, 0, 0);
  }
}

__device__ __forceinline__ bf16x8 lds_frag(const char* tile, int row, int chunk) {
  const int phys = chunk ^ ((row >> 1) & 7);
  return *(const bf16x8*)(tile + row * 128 + phys * 16);
}

template <int EPI>
__global__ __launch_bounds__(256) void gemm_tile_kernel(const bf16_t* __restrict__ A, int lda,
                                                        const bf16_t* __restrict__ W, int ldw, int K, int kchunk,
                                                        int tiles_m, int tiles_n, EpiArgs e) {
  __shared__ __attribute__((aligned(1024))) char smem[4 * TILE_BYTES];   // 2 buffers x (A, W)
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int wm = wave >> 1, wn = wave & 1;

  // XCD-aware bijective remap (blocks b and b+8 share an XCD), then grouped tile order.
  const int nwg = gridDim.x;
  int pid = blockIdx.x;
  {
    const int q = nwg >> 3, r = nwg & 7, xcd = pid & 7, idx = pid >> 3;
    pid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + idx;
  }
  const int GROUP = 8;
  const int group = pid / (GROUP * tiles_n);
  const int first_m = group * GROUP;
  const int gsize = min(tiles_m - first_m, GROUP);
  const int tm = first_m + (pid % gsize);
  const int tn = (pid % (GROUP * tiles_n)) / gsize;
  const int m0 = tm * TBM, n0 = tn * TBN;

  const int z = blockIdx.z;
  const int kbeg = z * kchunk;
  const int kend = min(K, kbeg + kchunk);
  const int nk = (kend - kbeg) / TBK;

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // buffer b: A tile at smem + 2b*TILE_BYTES, W tile right after it
  if (nk > 0) {
    stage_tile(A, lda, m0, e.M, kbeg, smem, wave, lane);
    stage_tile(W, ldw, n0, e.N, kbeg, smem + TILE_BYTES, wave, lane);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    char* nxt = smem + (cur ^ 1) * 2 * TILE_BYTES;
    if (kt + 1 < nk) {
      stage_tile(A, lda, m0, e.M, kbeg + (kt + 1) * TBK, nxt, wave, lane);
      stage_tile(W, ldw, n0, e.N, kbeg + (kt + 1) * TBK, nxt + TILE_BYTES, wave, lane);
    }
    const char* tA = smem + cur * 2 * TILE_BYTES;
    const char* tW = tA + TILE_BYTES;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int chunk = s * 4 + (lane >> 4);
      bf16x8 fa[4], fw[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) fa[i] = lds_frag(tA, wm * 64 + i * 16 + (lane & 15), chunk);
#pragma unroll
      for (int j = 0; j < 4; ++j) fw[j] = lds_frag(tW, wn * 64 + j * 16 + (lane & 15), chunk);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = mfma16(fw[j], fa[i], acc[i][j]);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }

  // epilogue: acc[i][j] lane holds C[m = m0+wm*64+i*16+(lane&15)][n = n0+wn*64+j*16+4*(lane>>4) + 0..3]
  const int q = 4 * (lane >> 4);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int m = m0 + wm * 64 + i * 16 + (lane & 15);
    if constexpr (EPI == PG_EPI_BF16_GELU_MUL) {
#pragma unroll
      for (int j = 0; j < 4; j += 2) epi_gelu_mul4(e, m, n0 + wn * 64 + j * 16, q, acc[i][j], acc[i][j + 1]);
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) epi_store4<EPI>(e, m, n0 + wn * 64 + j * 16 + q, acc[i][j], z);
    }
  }
}

// --------------------------------------------------------------------------------------
// Skinny GEMM / GEMV (M <= 16): weight streaming straight to VGPRs
// --------------------------------------------------------------------------------------
// One workgroup = 4 waves = NT adjacent 16-row tiles of W (NT = 2 for the interleaved
// gate/up pair) over the K range of split blockIdx.y; the 4 waves split that range.
// lane (r = lane&15, g = lane>>4) covers k = kc + 8U*g + [0, 8U): MFMA step s uses k = kc + 8U*g + 8s + [0,8)
// for both operands (same permutation of k on both sides leaves the dot product unchanged).
template <int U>
__device__ __forceinline__ void gemv_w_load(const bf16_t* __restrict__ wrow, int kc, int g, u32x4* wv) {
  const int off = kc + g * 8 * U;
#pragma unroll
  for (int s = 0; s < U; ++s) wv[s] = __builtin_nontemporal_load((const u32x4*)(wrow + off + 8 * s));
}
template <int U>
__device__ __forceinline__ void gemv_x_load(const bf16_t* __restrict__ xrow, bool xvalid, int kc, int g, u32x4* xv) {
  const int off = kc + g * 8 * U;
#pragma unroll
  for (int s = 0; s < U; ++s) xv[s] = xvalid ? *(const u32x4*)(xrow + off + 8 * s) : u32x4{0u, 0u, 0u, 0u};
}

template <int EPI, int NT>
__global__ __launch_bounds__(256) void gemv_kernel(const bf16_t* __restrict__ A, int lda,
                                                   const bf16_t* __restrict__ W, int ldw, int K, int kchunk, EpiArgs e) {
  constexpr int U = 4;                       // MFMA steps per contiguous chunk (U*32 k, 16U bytes per lane)
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int g = lane >> 4;
  const int r = lane & 15;
  const int tile0 = blockIdx.x * NT;         // first 16-row tile of W
  const int z = blockIdx.y;
  const int kbeg = z * kchunk;
  const int kend = min(K, kbeg + kchunk);
  const int M = e.M;

  const bool xvalid = r < M;
  const bf16_t* xrow = A + (size_t)(xvalid ? r : 0) * lda;
  const bf16_t* wrow[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    int n = (tile0 + t) * 16 + r;
    n = n < e.N ? n : e.N - 1;
    wrow[t] = W + (size_t)n * ldw;
  }

  f32x4 acc[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};

  // big chunks of U*32 k, round-robin over the 4 waves, software-pipelined by one chunk
  const int CH = U * 32;
  const int nbig = (kend - kbeg) / CH;
  int c = wave;
  if (c < nbig) {
    u32x4 wv[NT][U], xv[U];
#pragma unroll
    for (int t = 0; t < NT; ++t) gemv_w_load<U>(wrow[t], kbeg + c * CH, g, wv[t]);
    gemv_x_load<U>(xrow, xvalid, kbeg + c * CH, g, xv);
    while (true) {
      const int cn = c + 4;
      u32x4 wn[NT][U], xn[U];
      if (cn < nbig) {
#pragma unroll
        for (int t = 0; t < NT; ++t) gemv_w_load<U>(wrow[t], kbeg + cn * CH, g, wn[t]);
        gemv_x_load<U>(xrow, xvalid, kbeg + cn * CH, g, xn);
      }
#pragma unroll
      for (int s = 0; s < U; ++s) {
        bf16x8 xb = __builtin_bit_cast(bf16x8, xv[s]);
#pragma unroll
        for (int t = 0; t < NT; ++t) acc[t] = mfma16(__builtin_bit_cast(bf16x8, wv[t][s]), xb, acc[t]);
      }
      if (cn >= nbig) break;
#pragma unroll
      for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int s = 0; s < U; ++s) wv[t][s] = wn[t][s];
#pragma unroll
      for (int s = 0; s < U; ++s) xv[s] = xn[s];
      c = cn;
    }
  }
  // tail: single MFMA steps (32 k) round-robin
  const int tbeg = kbeg + nbig * CH;
  const int ntail = (kend - tbeg) / 32;
  for (int ct = wave; ct < ntail; ct += 4) {
    u32x4 wv[NT][1], xv[1];
#pragma unroll
    for (int t = 0; t < NT; ++t) gemv_w_load<1>(wrow[t], tbeg + ct * 32, g, wv[t]);
    gemv_x_load<1>(xrow, xvalid, tbeg + ct * 32, g, xv);
    bf16x8 xb = __builtin_bit_cast(bf16x8, xv[0]);
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[t] = mfma16(__builtin_bit_cast(bf16x8, wv[t][0]), xb, acc[t]);
  }

  // reduce the 4 waves through LDS
  __shared__ f32x4 red[4][NT][64];
#pragma unroll
  for (int t = 0; t < NT; ++t) red[wave][t][lane] = acc[t];
  __syncthreads();
  if (wave != 0) return;
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    f32x4 s = red[0][t][lane];
#pragma unroll
    for (int w = 1; w < 4; ++w) s += red[w][t][lane];
    acc[t] = s;
  }
  // lane holds C[m = lane&15][n = tile*16 + 4*(lane>>4) + 0..3]
  const int m = r;
  const int q = 4 * g;
  if constexpr (EPI == PG_EPI_BF16_GELU_MUL) {
    epi_gelu_mul4(e, m, tile0 * 16, q, acc[0], acc[1]);
  } else {
#pragma unroll
    for (int t = 0; t < NT; ++t) epi_store4<EPI>(e, m, (tile0 + t) * 16 + q, acc[t], z);
  }
}

// --------------------------------------------------------------------------------------
// C ABI
// --------------------------------------------------------------------------------------
template <int EPI>
static void launch_tile(const bf16_t* A, int lda, const bf16_t* W, int ldw, int K, int ksplit, const EpiArgs& e,
                        hipStream_t st) {
  const int tiles_m = (e.M + TBM - 1) / TBM, tiles_n = (e.N + TBN - 1) / TBN;
  int kchunk = ((K / TBK + ksplit - 1) / ksplit) * TBK;
  dim3 grid(tiles_m * tiles_n, 1, ksplit);
  hipLaunchKernelGGL(gemm_tile_kernel<EPI>, grid, dim3(256), 0, st, A, lda, W, ldw, K, kchunk, tiles_m, tiles_n, e);
}

template <int EPI, int NT>
static void launch_gemv(const bf16_t* A, int lda, const bf16_t* W, int ldw, int K, int ksplit, const EpiArgs& e,
                        hipStream_t st) {
  const int ntiles = (e.N + 15) / 16;
  int kchunk = ((K / 32 + ksplit - 1) / ksplit) * 32;
  dim3 grid(ntiles / NT, ksplit);
  hipLaunchKernelGGL((gemv_kernel<EPI, NT>), grid, dim3(256), 0, st, A, lda, W, ldw, K, kchunk, e);
}

extern "C" int pg_gemm(const void* A, int lda, const void* W, int ldw, const float* bias, void* C, int ldc,
                       int M, int N, int K, int epi, int ksplit, const float* aux, int aux_rows, void* aux_out,
                       int aux_ld, int aux_n, hipStream_t stream) {
  PG_REQUIRE(M > 0 && N > 0 && K > 0 && ksplit >= 1);
  PG_REQUIRE(K % 32 == 0 && lda >= K && ldw >= K && (N % 4) == 0);
  EpiArgs e{bias, C, ldc, M, N, aux, aux_rows, (bf16_t*)aux_out, aux_ld, aux_n};
  if (ksplit > 1) PG_REQUIRE(epi == PG_EPI_F32);
  if (epi == PG_EPI_BF16_GELU_MUL) PG_REQUIRE(N % 32 == 0);
  if (epi == PG_EPI_F32_POS) PG_REQUIRE(aux != nullptr && aux_rows > 0 && bias != nullptr);
  if (epi == PG_EPI_BF16_VT) PG_REQUIRE(aux_out != nullptr && aux_n % 4 == 0);
  const bf16_t* a = (const bf16_t*)A;
  const bf16_t* w = (const bf16_t*)W;
  if (M <= 16) {
    PG_REQUIRE(N % 16 == 0 || epi == PG_EPI_F32 || epi == PG_EPI_BF16);
    switch (epi) {
      case PG_EPI_BF16: launch_gemv<PG_EPI_BF16, 1>(a, lda, w, ldw, K, ksplit, e, stream); break;
      case PG_EPI_BF16_GELU: launch_gemv<PG_EPI_BF16_GELU, 1>(a, lda, w, ldw, K, ksplit, e, stream); break;
      case PG_EPI_BF16_GELU_MUL: launch_gemv<PG_EPI_BF16_GELU_MUL, 2>(a, lda, w, ldw, K, ksplit, e, stream); break;
      case PG_EPI_F32: launch_gemv<PG_EPI_F32, 1>(a, lda, w, ldw, K, ksplit, e, stream); break;
      case PG_EPI_F32_POS: launch_gemv<PG_EPI_F32_POS, 1>(a, lda, w, ldw, K, ksplit, e, stream); break;
      case PG_EPI_BF16_VT: launch_gemv<PG_EPI_BF16_VT, 1>(a, lda, w, ldw, K, ksplit, e, stream); break;
      default: return (int)hipErrorInvalidValue;
    }
  } else {
    PG_REQUIRE(K % TBK == 0);
    switch (epi) {
      case PG_EPI_BF16: launch_tile<PG_EPI_BF16>(a, lda, w, ldw, K, ksplit, e, stream); break;
      case PG_EPI_BF16_GELU: launch_tile<PG_EPI_BF16_GELU>(a, lda, w, ldw, K, ksplit, e, stream); break;
      case PG_EPI_BF16_GELU_MUL: launch_tile<PG_EPI_BF16_GELU_MUL>(a, lda, w, ldw, K, ksplit, e, stream); break;
      case PG_EPI_F32: launch_tile<PG_EPI_F32>(a, lda, w, ldw, K, ksplit, e, stream); break;
      case PG_EPI_F32_POS: launch_tile<PG_EPI_F32_POS>(a, lda, w, ldw, K, ksplit, e, stream); break;
      case PG_EPI_BF16_VT: launch_tile<PG_EPI_BF16_VT>(a, lda, w, ldw, K, ksplit, e, stream); break;
      default: return (int)hipErrorInvalidValue;
    }
  }
  PG_LAUNCH_CHECK();
  return 0;
}
