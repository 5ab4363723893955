// Prefill tile GEMMs (M > 16): gemm_tile_kernel, gemm256_kernel and the split-K finalisation (see gemm_common.h).
#include "gemm_common.h"

// --------------------------------------------------------------------------------------
// Tiled GEMM (prefill)
// --------------------------------------------------------------------------------------
// BM x 128 output tile, BK = 64, 4 waves (BM=128: 2x2 waves of 64x64; BM=96: 2x2 of 48x64;
// BM=64: 1x4 waves of 64x32).
// A and W k-tiles are staged HBM->LDS with global_load_lds (16 B/lane, 1 KiB pieces of 8 rows x
// 128 B, XOR-swizzled through the SOURCE address) into an STAGES-deep ring; the wait for stage kt
// is a counted vmcnt (the younger stages stay in flight across the raw s_barrier), so each k-step's
// MFMAs overlap the next STAGES-1 stages' loads.  One __shared__ array only (a second one makes
// hipcc drain vmcnt before every ds_read).

// element offset of W[row][k0 + 8c .. +8) (k0 % 64 == 0, c < 8) in the fragment-packed layout (PG_W_FRAG)
__device__ __forceinline__ size_t frag_off(int row, int k0, int c, int K) {
  return (size_t)(row >> 4) * 16 * K + ((size_t)(k0 >> 6) * 2 + (c & 1)) * 512 + ((c >> 1) * 16 + (row & 15)) * 8;
}

// Stage a ROWS x 64-k bf16 tile: ROWS/8 pieces spread evenly over NW staging waves (wave < NW; others issue none).
// FRAG: src is fragment-packed (ld = K); each piece still reads 8 runs of 128 contiguous bytes.
// SKIP: pieces whose 8 rows all lie past rows_valid are not loaded (their LDS rows feed only outputs that are never
// stored); the caller counts the pieces a wave issues with stage_pieces.
template <int ROWS, bool FRAG = false, int NW = 4, int AUX = 0, bool SKIP = false>
__device__ __forceinline__ void stage_tile(const bf16_t* __restrict__ src, int ld, int row0, int rows_valid,
                                           int k0, char* lds_tile, int wave, int lane) {
  static_assert((ROWS / 8) % NW == 0, "pieces must split evenly over the staging waves");
  constexpr int PER_WAVE = ROWS / 8 / NW;
  if (wave >= NW) return;
#pragma unroll
  for (int it = 0; it < PER_WAVE; ++it) {
    const int blk = wave * PER_WAVE + it;          // 1 KiB piece = 8 rows x 128 B
    if (SKIP && blk * 8 >= rows_valid - row0) break;   // (wave-uniform)
    const int r = blk * 8 + (lane >> 3);
    const int c = (lane & 7) ^ ((r >> 1) & 7);     // logical 16-B chunk landing at physical chunk lane&7
    int gr = row0 + r;
    gr = gr < rows_valid ? gr : rows_valid - 1;
    const bf16_t* g = FRAG ? src + frag_off(gr, k0, c, ld) : src + (size_t)gr * ld + k0 + c * 8;
    __builtin_amdgcn_global_load_lds((const void*)g, (LDS_AS void*)(lds_tile + blk * 1024), 16, 0, AUX);
  }
}

// pieces stage_tile<ROWS, *, NW, *, SKIP> issues for this wave
template <int ROWS, int NW, bool SKIP>
__device__ __forceinline__ int stage_pieces(int row0, int rows_valid, int wave) {
  constexpr int PER_WAVE = ROWS / 8 / NW;
  if (wave >= NW) return 0;
  if (!SKIP) return PER_WAVE;
  const int valid = (rows_valid - row0 + 7) / 8;
  return min(PER_WAVE, max(0, valid - wave * PER_WAVE));
}

__device__ __forceinline__ bf16x8 lds_frag(const char* tile, int row, int chunk) {
  const int phys = chunk ^ ((row >> 1) & 7);
  return *(const bf16x8*)(tile + row * 128 + phys * 16);
}

__device__ __forceinline__ void wait_vm(int n) {   // s_waitcnt vmcnt(n), n in [0, 24]
  switch (n) {
    case 0: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
    case 2: asm volatile("s_waitcnt vmcnt(2)" ::: "memory"); break;
    case 3: asm volatile("s_waitcnt vmcnt(3)" ::: "memory"); break;
    case 4: asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); break;
    case 5: asm volatile("s_waitcnt vmcnt(5)" ::: "memory"); break;
    case 6: asm volatile("s_waitcnt vmcnt(6)" ::: "memory"); break;
    case 9: asm volatile("s_waitcnt vmcnt(9)" ::: "memory"); break;
    case 10: asm volatile("s_waitcnt vmcnt(10)" ::: "memory"); break;
    case 8: asm volatile("s_waitcnt vmcnt(8)" ::: "memory"); break;
    case 12: asm volatile("s_waitcnt vmcnt(12)" ::: "memory"); break;
    case 13: asm volatile("s_waitcnt vmcnt(13)" ::: "memory"); break;
    case 16: asm volatile("s_waitcnt vmcnt(16)" ::: "memory"); break;
    case 18: asm volatile("s_waitcnt vmcnt(18)" ::: "memory"); break;
    case 24: asm volatile("s_waitcnt vmcnt(24)" ::: "memory"); break;
    default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
  }
}

#ifndef PG_TILE_M1_WNT
#define PG_TILE_M1_WNT 0  // PG_TILE_M1 grids: stage W non-temporal (each W tile read by one workgroup)
#endif
#ifndef PG_TILE_PROBE
#define PG_TILE_PROBE 0   // tuning builds only: 1 = staging without MFMAs, 2 = MFMAs without staging (wrong results)
#endif
// WAVES (4, 8 or 12): waves per workgroup.  4: BM 64 as 1 x 4 waves of 64 x 32, BM 128 / 256 / 288 as 2 x 2.  More
// waves put 2-3 waves on every SIMD, so one wave's LDS fragment reads hide behind another's MFMAs (with 4 waves the
// single wave of a SIMD waits out every ds_read before its MFMAs): 8 = BM 64 as 2 x 4 waves of 32 x 32 and BM 256
// as 4 x 2 of 64 x 64; 12 = BM 288 as 6 x 2 waves of 48 x 64.  The A pieces of a stage spread over all waves, the
// W pieces over the first 8 (12 waves) so every wave's piece count -- its vmcnt step -- is a whole number.
// BN = 64 (PG_TILE_N64, BM 64 and 4 waves only: 2 x 2 waves of 32 x 32): twice the workgroups of the 64 x 128
// grid for the small-M prefill GEMMs whose 64 x 128 grid leaves most CUs idle, without a K split.
// KSUB = 2: a stage holds two 64-k sub-tiles (K % 128 == 0), one barrier / vmcnt wait per 128 k: half the
// per-k-step synchronisation of the latency-bound small-M tiles.
// WNT: the W pieces are staged non-temporal (aux 2): for grids where each W tile is read by ONE workgroup (PG_TILE_M1)
// MXA (fp8, ABI 12): A rows are MX (OCP microscaling) e4m3 with one E8M0 scale per 32 k, PgFusedArgs.mx_in [M][K/32]
// (the prefill gate/up epilogue's h, into the down projection): each stage also brings its BM rows' 4 block scales
// of the k-step into LDS -- one byte per lane of every wave (zero-extended into the lane's dword slot), stored
// transposed so that lane (r, g) of wave row wm reads its NI row subtiles' block-g scales with one 8-byte read -- and
// the MFMA of subtile i takes byte i of the packed pair (op_sel).  The MFMA
// reads block b's scale from lane group b: with the (g, 4 + g) chunk pairs below, lane group b holds block b's k
// ranges in the hardware's k order (k = 64 half + 16 g + byte), so MX block b is hardware block b.
template <int EPI, int BM, int STAGES, bool FRAG, bool F8 = false, int WAVES = 4, int BN = TBN, int KSUB = 1,
          bool WNT = false, bool MXA = false>
__global__ __launch_bounds__(WAVES * 64) void gemm_tile_kernel(const bf16_t* __restrict__ A, int lda,
                                                               const bf16_t* __restrict__ W, int ldw, int K,
                                                               int kchunk, int tiles_m, int tiles_n, EpiArgs e) {
  constexpr int A_BYTES = BM * TBK * 2;
  static_assert(BN == TBN || (BN == 64 && BM == 64 && WAVES == 4), "BN 64: 64-row tiles of 4 waves only");
  static_assert(!MXA || (F8 && KSUB == 1 && BM * 4 == WAVES * 64), "MX rows: fp8, one byte per lane per stage");
  constexpr int W_BYTES = BN * TBK * 2;
  // the stage's block scales (4 per row per 128-k step), one per dword: LDS DMA of a byte zero-extends it into the
  // lane's dword slot
  constexpr int S_BYTES = MXA ? BM * 4 * 4 : 0;
  constexpr int SUB_BYTES = A_BYTES + W_BYTES + S_BYTES;
  constexpr int STAGE_BYTES = KSUB * SUB_BYTES;
  constexpr int WN = BN == 64 ? 2 : (WAVES == 4 ? (BM == 64 ? 4 : 2) : (WAVES == 8 ? (BM == 64 ? 4 : 2) : 2));
  constexpr int WM = WAVES / WN;                   // waves along M
  constexpr int NI = BM / WM / 16;                 // 16-row subtiles per wave
  constexpr int NJ = BN / WN / 16;                 // 16-col subtiles per wave
  static_assert(WM * NI * 16 == BM && WN * NJ * 16 == BN, "wave grid must tile the block");
  constexpr int NWA = WAVES;                       // waves staging A pieces
  constexpr int NWW = WAVES > 8 ? 8 : WAVES;       // waves staging W pieces
  __shared__ __attribute__((aligned(1024))) char smem[STAGES * STAGE_BYTES];
  const int lane = threadIdx.x & 63;
  // wave-uniform (SGPR): the per-wave piece counts and the vmcnt switch below then branch on scalars, not through
  // an exec-masked chain of every case
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wave / WN, wn = wave % WN;

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
  const int m0 = tm * BM, n0 = tn * BN;
  // glds pieces this wave issues per stage (wave-uniform): its vmcnt step per younger stage in flight; A pieces of
  // padding rows only (the last row tile: M = 264 in a 288-row tile) are not loaded
  const int P = KSUB * (stage_pieces<BM, NWA, true>(m0, e.M, wave) + stage_pieces<BN, NWW, false>(n0, e.N, wave)) +
                (MXA ? 1 : 0);

  const int z = blockIdx.z;
  const int kbeg = z * kchunk;
  const int kend = min(K, kbeg + kchunk);
  const int nk = max(0, (kend - kbeg) / (TBK * KSUB));

  f32x4 acc[NI][NJ];
#pragma unroll
  for (int i = 0; i < NI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto issue = [&](int kt) {
    char* st = smem + (kt % STAGES) * STAGE_BYTES;
    if (PG_TILE_PROBE == 2) return;                // tuning probe: no loads (MFMA + barrier floor)
#pragma unroll
    for (int u = 0; u < KSUB; ++u) {
      const int k0 = kbeg + (kt * KSUB + u) * TBK;
      stage_tile<BM, false, NWA, 0, true>(A, lda, m0, e.M, k0, st + u * SUB_BYTES, wave, lane);
      stage_tile<BN, FRAG, NWW, WNT ? 2 : 0>(W, ldw, n0, e.N, k0, st + u * SUB_BYTES + A_BYTES, wave, lane);
      if constexpr (MXA) {
        // slot ((wm * 16 + r) * 4 + g) * NI + i = block g of tile row wm * (BM / WM) + i * 16 + r (transposed)
        const int idx = wave * 64 + lane;
        const int i = idx % NI, g = (idx / NI) & 3, r = (idx / (NI * 4)) & 15, wmr = idx / (NI * 64);
        const int gr = min(m0 + wmr * (BM / WM) + i * 16 + r, e.M - 1);
        // (uniform base + 32-bit offset: the scales are M * K / 16 bytes, host-checked < 4 GiB; K counts byte pairs)
        const char* src = (const char*)e.f.mx_in + (uint32_t)((unsigned)gr * (unsigned)(K >> 4) +
                                                              (unsigned)(k0 >> 6) * 4u + (unsigned)g);
        __builtin_amdgcn_global_load_lds((const void*)src, (LDS_AS void*)(st + A_BYTES + W_BYTES + wave * 256), 1, 0,
                                         0);
      }
    }
  };
#pragma unroll
  for (int s = 0; s < STAGES - 1; ++s)
    if (s < nk) issue(s);

  for (int kt = 0; kt < nk; ++kt) {
    // stage kt has landed once at most (issued stages after kt) * P pieces are outstanding
    const int younger = min(nk - 1, kt + STAGES - 2) - kt;
    wait_vm_n(younger * P);
    __builtin_amdgcn_s_barrier();                  // every wave's pieces of kt landed; kt-1 fully read
    if (kt + STAGES - 1 < nk) issue(kt + STAGES - 1);
#pragma unroll
    for (int u = 0; u < KSUB; ++u) {
    const char* tA = smem + (kt % STAGES) * STAGE_BYTES + u * SUB_BYTES;
    const char* tW = tA + A_BYTES;
    if constexpr (PG_TILE_PROBE == 1) {
      // tuning probe: no fragment reads or MFMAs (the staging pipeline's floor); one LDS word keeps the loads live
      if (lane == 0 && wave == 0) acc[0][0][0] += *(const float*)tA;
    } else if constexpr (F8) {
      // fp8: the 128-byte k-row holds 128 k; one 16x16x128 MFMA takes both chunk sets of the bf16 form
      bf16x8 fa[NI][2], fw[NJ][2];
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const int chunk = s * 4 + (lane >> 4);
#pragma unroll
        for (int i = 0; i < NI; ++i) fa[i][s] = lds_frag(tA, wm * (BM / WM) + i * 16 + (lane & 15), chunk);
#pragma unroll
        for (int j = 0; j < NJ; ++j) fw[j][s] = lds_frag(tW, wn * (BN / WN) + j * 16 + (lane & 15), chunk);
      }
      if constexpr (MXA) {
        static_assert(NI == 2, "MX rows: two row subtiles per wave (one 16-bit scale word per lane)");
        const u32x2 sv = *(const u32x2*)(tW + W_BYTES + ((wm * 16 + (lane & 15)) * 4 + (lane >> 4)) * NI * 4);
        const int scp = (int)(sv[0] | (sv[1] << 8));    // subtile 0's scale in byte 0, subtile 1's in byte 1
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
          acc[0][j] = mfma8s_sel<0>(fw[j][0], fw[j][1], fa[0][0], fa[0][1], acc[0][j], scp);
          acc[1][j] = mfma8s_sel<1>(fw[j][0], fw[j][1], fa[1][0], fa[1][1], acc[1][j], scp);
        }
      } else {
#pragma unroll
      for (int i = 0; i < NI; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j) acc[i][j] = mfma8(fw[j][0], fw[j][1], fa[i][0], fa[i][1], acc[i][j]);
      }
    } else {
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const int chunk = s * 4 + (lane >> 4);
        bf16x8 fa[NI], fw[NJ];
#pragma unroll
        for (int i = 0; i < NI; ++i) fa[i] = lds_frag(tA, wm * (BM / WM) + i * 16 + (lane & 15), chunk);
#pragma unroll
        for (int j = 0; j < NJ; ++j) fw[j] = lds_frag(tW, wn * (BN / WN) + j * 16 + (lane & 15), chunk);
#pragma unroll
        for (int i = 0; i < NI; ++i)
#pragma unroll
          for (int j = 0; j < NJ; ++j) acc[i][j] = mfma16(fw[j], fa[i], acc[i][j]);
      }
    }
    }
  }

  // epilogue: acc[i][j] lane holds C[m = m0+wm*(BM/WM)+i*16+(lane&15)][n = n0+wn*(BN/WN)+j*16+4*(lane>>4) + 0..3]
  const int q = 4 * (lane >> 4);
  if constexpr (EPI == PG_EPI_F32_RES) {
    // all NI x NJ residual loads of the wave in flight before its stores
    f32x4 rr[NI][NJ];
#pragma unroll
    for (int i = 0; i < NI; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int m = m0 + wm * (BM / WM) + i * 16 + (lane & 15), n = n0 + wn * (BN / WN) + j * 16 + q;
        if constexpr (F8) scale_acc(e, m, n, acc[i][j]);
        rr[i][j] = res_load4(e, m, n);
      }
#pragma unroll
    for (int i = 0; i < NI; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j)
        res_store4(e, m0 + wm * (BM / WM) + i * 16 + (lane & 15), n0 + wn * (BN / WN) + j * 16 + q, acc[i][j],
                   rr[i][j]);
    return;
  }
#pragma unroll
  for (int i = 0; i < NI; ++i) {
    const int m = m0 + wm * (BM / WM) + i * 16 + (lane & 15);
    const int nb = n0 + wn * (BN / WN);
    if constexpr (F8) {
#pragma unroll
      for (int j = 0; j < NJ; ++j) scale_acc(e, m, nb + j * 16 + q, acc[i][j]);
    }
    if constexpr (EPI == PG_EPI_BF16_GELU_MUL) {
      if constexpr (F8 && BN / WN == 64) {
        if (e.f.mx_out) {
          // (ABI 12) MX h for the prefill down projection: the wave's 64 W rows are 2 interleaved gate/up pairs = 32 h
          // columns = ONE MX block per row.  h rounded to bf16 (as the bf16 path stores it), the block max over the
          // lane's 8 values and the 4 lane groups of its row, e = mx_exp(max), e4m3 of h / 2^e; scales [M][N/64]
          f32x4 hv[2];
          float am = 0.f;
#pragma unroll
          for (int p = 0; p < 2; ++p)
#pragma unroll
            for (int jj = 0; jj < 4; ++jj) {
              hv[p][jj] = __uint_as_float((uint32_t)f2bf(gelu_tanh(acc[i][2 * p][jj]) * acc[i][2 * p + 1][jj]) << 16);
              am = fmaxf(am, fabsf(hv[p][jj]));
            }
          am = max_xor16(am);
          am = max_xor32(am);
          const int ex = mx_exp(am);
          const float inv = __builtin_ldexpf(1.0f, -ex);
          const int Nh = e.N >> 1, c0 = nb >> 1;          // the block's first h column (a multiple of 32)
          if (m < e.M && c0 + 31 < Nh) {
#pragma unroll
            for (int p = 0; p < 2; ++p)
              *(uint32_t*)((uint8_t*)e.C + (size_t)m * e.ldc + c0 + 16 * p + q) =
                  pack_fp8x4(hv[p][0] * inv, hv[p][1] * inv, hv[p][2] * inv, hv[p][3] * inv);
            if (q == 0) e.f.mx_out[(size_t)m * (Nh >> 5) + (c0 >> 5)] = (uint8_t)(ex + 127);
          }
          continue;
        }
      }
#pragma unroll
      for (int j = 0; j < NJ; j += 2) epi_gelu_mul4(e, m, nb + j * 16, q, acc[i][j], acc[i][j + 1]);
    } else if constexpr (EPI == PG_EPI_QKV_ROPE) {
#pragma unroll
      for (int j = 0; j < NJ; ++j) epi_qkv_rope4(e, m, nb + j * 16 + q, acc[i][j]);
    } else {
#pragma unroll
      for (int j = 0; j < NJ; ++j) epi_store4<EPI>(e, m, nb + j * 16 + q, acc[i][j], z);
    }
  }
}

// --------------------------------------------------------------------------------------
// Large-M GEMM (prefill at batch x image tokens >= a few thousand rows): 256 x 256 x 64 tiles
// --------------------------------------------------------------------------------------
// 8 waves = 2 (M) x 4 (N), each owning 128 x 64 outputs (acc[8][4] 16x16 fragments), one workgroup per
// CU (128 KiB LDS).  A K-tile is staged as four 16 KiB half-images (128 rows x 128 B, XOR-swizzled through
// the source address, global_load_lds 16 B/lane, 2 per thread):
//   A0 = tile rows {0..63, 128..191}   A1 = rows {64..127, 192..255}      (wave rows wr*128 + [0,64) / [64,128))
//   B0 = W rows {64c + [0,32)}         B1 = W rows {64c + [32,64)}, c < 4 (wave columns wc*64 + [0,32) / [32,64))
// and consumed in four phases, one C quadrant each: (A0,B0) (A0 regs,B1) (A1,B1 regs) (A1,B0).  A half is
// restaged one phase after its last read (A0 of tile t+2 in phase 1 of t, B1 in phase 2, A1 in phase 3,
// B0 of t+1 in phase 0), so 3 half-tiles (6 loads per thread) stay in flight across the raw s_barrier that
// ends every phase; the single counted wait (vmcnt 6) sits in phase 3 and the tile it retires is read
// from phase 0 of the next tile on (MI355X guide: 256^2 8-phase template, counted vmcnt, T1/T2/T5).
template <int EPI, bool FRAG, bool F8 = false>
__global__ __launch_bounds__(512) void gemm256_kernel(const bf16_t* __restrict__ A, int lda,
                                                      const bf16_t* __restrict__ W, int ldw, int K,
                                                      int ktiles_per_split, int tiles_m, int tiles_n, EpiArgs e) {
  constexpr int HALF = 16384;
  __shared__ __attribute__((aligned(1024))) char smem[8 * HALF];
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int wr = wave >> 2, wc = wave & 3;

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
  const int m0 = tm * 256, n0 = tn * 256;
  // split-K (fp32 partial epilogue only): slice z covers k-tiles [kt0, kt0 + nk)
  const int z = blockIdx.z;
  const int kt0 = z * ktiles_per_split;
  const int nk = max(0, min(K / 64 - kt0, ktiles_per_split));

  // fp8 (PG_G256_F8_BUF): the pieces are loaded through buffer resources (buffer_load ... lds): a lane's two pieces
  // of a half are 64 image rows apart (same swizzle), so every piece of a lane is ONE per-operand lane offset plus a
  // uniform row / k offset, and rows past M / N read zeros (out of range of the resource) instead of being clamped.
  // Two lane offsets live across the k loop instead of eight: the eight pushed the instance past 256 registers, and
  // the spill reloads inside the loop waited vmcnt(0), draining the half-tiles in flight every k-step (pt-896 x32
  // shapes: down 4.67 -> 4.00 ms, o_proj 0.81 -> 0.73 ms, gate/up 11.8 -> 9.9 ms; profiles/r06_g256_f8_buf_ab.txt).
  constexpr bool BUF = F8 && !FRAG && PG_G256_F8_BUF;
  unsigned la = 0, lw = 0;                         // (byte offsets < 4 GiB: host-checked, off32)
  if constexpr (BUF) {
    const int r0 = wave * 8 + (lane >> 3);           // piece rows r0 (it 0) and r0 + 64 (it 1)
    const int c = (lane & 7) ^ ((r0 >> 1) & 7);
    la = ((unsigned)r0 * (unsigned)lda + (unsigned)c * 8u) * 2u;
    lw = ((unsigned)((r0 >> 5) * 64 + (r0 & 31)) * (unsigned)ldw + (unsigned)c * 8u) * 2u;
  }
  auto stage = [&](int h, int kt) {
    char* dst = smem + ((kt & 1) * 4 + h) * HALF;
    const int k0 = (kt0 + kt) * 64;
    if constexpr (BUF) {
#pragma unroll
      for (int it = 0; it < 2; ++it) {
        const int blk = wave + 8 * it;
        // uniform byte offset of this piece's rows at k0 (through readfirstlane: an SGPR computed here, so the sum
        // below is not re-associated into per-piece loop-invariant lane offsets)
        const unsigned so = (unsigned)__builtin_amdgcn_readfirstlane((int)(
            h < 2 ? ((unsigned)(m0 + it * 128 + h * 64) * (unsigned)lda + (unsigned)k0) * 2u
                  : ((unsigned)(n0 + it * 128 + (h - 2) * 32) * (unsigned)ldw + (unsigned)k0) * 2u));
        // (the resource's size is the operand's M / N rows: pieces past them read zeros)
        const auto rs = h < 2 ? __builtin_amdgcn_make_buffer_rsrc((void*)A, 0,
                                                                  (int)((unsigned)e.M * (unsigned)lda * 2u), 0x00020000)
                              : __builtin_amdgcn_make_buffer_rsrc((void*)W, 0,
                                                                  (int)((unsigned)e.N * (unsigned)ldw * 2u), 0x00020000);
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (LDS_AS void*)(dst + blk * 1024), 16,
                                                 (int)((h < 2 ? la : lw) + so), 0, 0, 0);
      }
      return;
    }
#pragma unroll
    for (int it = 0; it < 2; ++it) {
      const int blk = wave * 2 + it;                 // 16 pieces of 8 rows x 128 B
      const int r = blk * 8 + (lane >> 3);           // half-image row
      const int c = (lane & 7) ^ ((r >> 1) & 7);
      // fp8: uniform base + 32-bit per-lane byte offset (the host checks both operands are < 4 GiB): the saddr
      // form, one VGPR per piece instead of a 64-bit pointer (the fp8 instance spilled its hoisted piece pointers)
      const char* src;
      if (h < 2) {
        const int gr = min(m0 + (r >> 6) * 128 + h * 64 + (r & 63), e.M - 1);
        if constexpr (F8)
          src = (const char*)A + (uint32_t)(((unsigned)gr * (unsigned)lda + (unsigned)(k0 + c * 8)) * 2u);
        else
          src = (const char*)(A + (size_t)gr * lda + k0 + c * 8);
      } else {
        const int gn = min(n0 + (r >> 5) * 64 + (h - 2) * 32 + (r & 31), e.N - 1);
        if constexpr (F8 && !FRAG)
          src = (const char*)W + (uint32_t)(((unsigned)gn * (unsigned)ldw + (unsigned)(k0 + c * 8)) * 2u);
        else
          src = (const char*)(FRAG ? W + frag_off(gn, k0, c, ldw) : W + (size_t)gn * ldw + k0 + c * 8);
      }
      __builtin_amdgcn_global_load_lds((const void*)src, (LDS_AS void*)(dst + blk * 1024), 16, 0, 0);
    }
  };

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  // fragment registers: A rows [0,64) / [64,128) of the wave (fa0 / fa1), B columns [0,32) / [32,64) (fb0 / fb1);
  // fp8: both 16-byte chunks of a row in one 8-register operand
  using FA = std::conditional_t<F8, i32x8[4], bf16x8[4][2]>;
  using FB = std::conditional_t<F8, i32x8[2], bf16x8[2][2]>;
  FA fa0, fa1;
  FB fb0, fb1;

  auto read_a = [&](const char* img, auto& fa) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = wr * 64 + i * 16 + (lane & 15);
      if constexpr (F8) {
        fa[i] = cat8(lds_frag(img, row, lane >> 4), lds_frag(img, row, 4 + (lane >> 4)));
      } else {
#pragma unroll
        for (int s = 0; s < 2; ++s) fa[i][s] = lds_frag(img, row, s * 4 + (lane >> 4));
      }
    }
  };
  auto read_b = [&](const char* img, auto& fb) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int row = wc * 32 + j * 16 + (lane & 15);
      if constexpr (F8) {
        fb[j] = cat8(lds_frag(img, row, lane >> 4), lds_frag(img, row, 4 + (lane >> 4)));
      } else {
#pragma unroll
        for (int s = 0; s < 2; ++s) fb[j][s] = lds_frag(img, row, s * 4 + (lane >> 4));
      }
    }
  };
  auto mma = [&](int rh, int ch, const auto& fa, const auto& fb) {
    __builtin_amdgcn_s_setprio(1);
    if constexpr (F8) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[rh * 4 + i][ch * 2 + j] = mfma8(fb[j], fa[i], acc[rh * 4 + i][ch * 2 + j]);
    } else {
#pragma unroll
      for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j)
            acc[rh * 4 + i][ch * 2 + j] = mfma16(fb[j][s], fa[i][s], acc[rh * 4 + i][ch * 2 + j]);
    }
    __builtin_amdgcn_s_setprio(0);
  };

  // prologue: all of tile 0, then the three halves of tile 1 that phases 1-3 of tile -1 would have issued
  // (a split past the end of K -- ksplit with ceil-sized slices -- stages nothing and stores a zero slab)
  if (nk > 0) {
#pragma unroll
    for (int h = 0; h < 4; ++h) stage(h, 0);
  }
  if (nk > 1) {
    stage(0, 1);
    stage(3, 1);
    stage(1, 1);
    wait_vm(6);
  } else {
    wait_vm(0);
  }
  __builtin_amdgcn_s_barrier();

  if constexpr (PG_G256_STAGGER && !F8) {
    // Wave groups wr = 0 / 1 (one wave of each per SIMD) run one barrier apart, two barriers per phase:
    // while one group issues its phase's LDS reads and DMA, the other runs its MFMAs.  With the offset, a
    // group's reads must be complete before its phase's first barrier (lgkmcnt(0) there: the other group
    // restages right after it) and the tile's vmcnt wait sits before phase 3's first barrier (the other
    // group reads the retired halves one barrier earlier than this one) -- guide: "one barrier MORE when
    // two wave groups run staggered".
    auto bar = [] { __builtin_amdgcn_s_barrier(); };
    auto lgkm0 = [] { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); };
    if (wr == 1) bar();
    for (int t = 0; t < nk; ++t) {
      const char* buf = smem + (t & 1) * 4 * HALF;
      read_a(buf, fa0);
      read_b(buf + 2 * HALF, fb0);
      if (t + 1 < nk) stage(2, t + 1);
      lgkm0();
      bar();
      mma(0, 0, fa0, fb0);
      bar();
      read_b(buf + 3 * HALF, fb0);
      if (t + 2 < nk) stage(0, t + 2);
      lgkm0();
      bar();
      mma(0, 1, fa0, fb0);
      bar();
      read_a(buf + 1 * HALF, fa0);
      if (t + 2 < nk) stage(3, t + 2);
      lgkm0();
      bar();
      mma(1, 1, fa0, fb0);
      bar();
      read_b(buf + 2 * HALF, fb0);
      if (t + 2 < nk) stage(1, t + 2);
      if (t + 2 < nk) wait_vm(6); else wait_vm(0);
      lgkm0();
      bar();
      mma(1, 0, fa0, fb0);
      bar();
    }
    if (wr == 0) bar();     // same barrier count for both groups
  } else
  for (int t = 0; t < nk; ++t) {
    const char* buf = smem + (t & 1) * 4 * HALF;
    if constexpr (PG_G256_PREFETCH && !F8) {   // (fp8: the early reads would spill)
    // the reads of phases 1-3 are issued one phase early, ahead of the current phase's MFMAs (tile t is
    // retired for every wave from phase 0 on; each half is still restaged only after its last read)
    read_a(buf, fa0);
    read_b(buf + 2 * HALF, fb0);
    if (t + 1 < nk) stage(2, t + 1);
    read_b(buf + 3 * HALF, fb1);
    mma(0, 0, fa0, fb0);
    __builtin_amdgcn_s_barrier();
    read_a(buf + 1 * HALF, fa1);
    if (t + 2 < nk) stage(0, t + 2);
    mma(0, 1, fa0, fb1);
    __builtin_amdgcn_s_barrier();
    read_b(buf + 2 * HALF, fb0);
    if (t + 2 < nk) stage(3, t + 2);
    mma(1, 1, fa1, fb1);
    __builtin_amdgcn_s_barrier();
    if (t + 2 < nk) stage(1, t + 2);
    mma(1, 0, fa1, fb0);
    } else {
    // phase 0: quadrant (rows 0-63, cols 0-31) from A0, B0; restage B0 of tile t+1
    read_a(buf, fa0);
    read_b(buf + 2 * HALF, fb0);
    if (t + 1 < nk) stage(2, t + 1);
    mma(0, 0, fa0, fb0);
    __builtin_amdgcn_s_barrier();
    // phase 1: (rows 0-63, cols 32-63) A regs kept, B1; restage A0 of tile t+2 (A0 was last read in phase 0)
    read_b(buf + 3 * HALF, fb0);
    if (t + 2 < nk) stage(0, t + 2);
    mma(0, 1, fa0, fb0);
    __builtin_amdgcn_s_barrier();
    // phase 2: (rows 64-127, cols 32-63) A1, B regs kept; restage B1 of tile t+2
    read_a(buf + 1 * HALF, fa0);
    if (t + 2 < nk) stage(3, t + 2);
    mma(1, 1, fa0, fb0);
    __builtin_amdgcn_s_barrier();
    // phase 3: (rows 64-127, cols 0-31) A regs kept, B0 again; restage A1 of tile t+2; retire tile t+1
    read_b(buf + 2 * HALF, fb0);
    if (t + 2 < nk) stage(1, t + 2);
    mma(1, 0, fa0, fb0);
    }
    if (t + 2 < nk) wait_vm(6); else wait_vm(0);
    __builtin_amdgcn_s_barrier();
  }

  // epilogue: acc[i][j] lane holds C[m][n..n+3], m = m0 + wr*128 + (i/4)*64 + (i%4)*16 + (lane&15),
  // n = n0 + wc*64 + (j/2)*32 + (j%2)*16 + 4*(lane>>4)
  const int q = 4 * (lane >> 4);
  if constexpr (EPI == PG_EPI_F32_RES) {
    // two row subtiles (i, i + 1: rows m, m + 16) at a time: their 8 residual loads in flight before the stores
#pragma unroll
    for (int i = 0; i < 8; i += 2) {
      const int m = m0 + wr * 128 + (i >> 2) * 64 + (i & 3) * 16 + (lane & 15);
      f32x4 rr[2][4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int n = n0 + wc * 64 + (j >> 1) * 32 + (j & 1) * 16 + q;
        if constexpr (F8) {
          scale_acc(e, m, n, acc[i][j]);
          scale_acc(e, m + 16, n, acc[i + 1][j]);
        }
        rr[0][j] = res_load4(e, m, n);
        rr[1][j] = res_load4(e, m + 16, n);
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int n = n0 + wc * 64 + (j >> 1) * 32 + (j & 1) * 16 + q;
        res_store4(e, m, n, acc[i][j], rr[0][j]);
        res_store4(e, m + 16, n, acc[i + 1][j], rr[1][j]);
      }
    }
    return;
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int m = m0 + wr * 128 + (i >> 2) * 64 + (i & 3) * 16 + (lane & 15);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int nb = n0 + wc * 64 + (j >> 1) * 32 + (j & 1) * 16;
      if constexpr (F8) scale_acc(e, m, nb + q, acc[i][j]);
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int nb = n0 + wc * 64 + (j >> 1) * 32 + (j & 1) * 16;
      if constexpr (EPI == PG_EPI_BF16_GELU_MUL) {
        if ((j & 1) == 0) epi_gelu_mul4(e, m, nb, q, acc[i][j], acc[i][j + 1]);
      } else if constexpr (EPI == PG_EPI_QKV_ROPE) {
        epi_qkv_rope4(e, m, nb + q, acc[i][j]);
      } else {
        epi_store4<EPI>(e, m, nb + q, acc[i][j], z);
      }
    }
  }
}

// --------------------------------------------------------------------------------------
// Split-K finalisation for the bf16 epilogues (prefill at small M, where a full-K tile grid leaves CUs
// idle): the GEMM writes fp32 slabs [z][M][N] (bias in slab 0), this kernel sums them and applies the
// epilogue (bf16 / gelu / gelu*up / V^T side output / RoPE + KV-cache append).  One thread per 4 outputs.
#ifndef PG_FIN_ROPE_EARLY
#define PG_FIN_ROPE_EARLY 1
#endif
template <int EPI>
__global__ __launch_bounds__(256) void gemm_finalize_kernel(const float* __restrict__ part, int nsplit, EpiArgs e) {
  const int NO = EPI == PG_EPI_BF16_GELU_MUL ? e.N / 2 : e.N;     // output columns
  const long idx = (long)blockIdx.x * 256 + threadIdx.x;
  const int q4 = NO / 4;
  if (idx >= (long)e.M * q4) return;
  const int m = (int)(idx / q4), c0 = (int)(idx % q4) * 4;
  const size_t slab = (size_t)e.M * e.N;
  auto sum4 = [&](int n) {
    f32x4 v = {0.f, 0.f, 0.f, 0.f};
    for (int z = 0; z < nsplit; ++z) v += *(const f32x4*)(part + z * slab + (size_t)m * e.N + n);
    return v;
  };
  if constexpr (EPI == PG_EPI_BF16_GELU_MUL) {
    // output column c0 <- gate column 32*(c0/16) + c0%16, up column +16
    const int gb = (c0 / 16) * 32, q = c0 % 16;
    epi_gelu_mul4(e, m, gb, q, sum4(gb + q), sum4(gb + 16 + q));
  } else if constexpr (EPI == PG_EPI_QKV_ROPE && !PG_FIN_ROPE_EARLY) {
    epi_qkv_rope4_pr(e, m, c0, sum4(c0), sum4(c0 ^ 8));
  } else if constexpr (EPI == PG_EPI_QKV_ROPE) {
    // the rotary position and cache slot are loaded before the slabs and the cos / sin right after them: two memory
    // round trips instead of three (slabs, then the position, then the table)
    bool roped;
    const int ii = rope_freq_index(e.f, c0, &roped);
    const int p = e.f.pos[m];
    const int slot0 = e.f.slot_base + (e.f.slot_dev ? *e.f.slot_dev : 0);
    const f32x4 v = sum4(c0), pr = sum4(c0 ^ 8);
    f32x4 cs = {1.f, 1.f, 1.f, 1.f}, sn = {0.f, 0.f, 0.f, 0.f};
    if (roped) {
      const long off = (long)p * (e.f.head_dim >> 1) + ii;
      cs = *(const f32x4*)(e.f.cos_t + off);
      sn = *(const f32x4*)(e.f.sin_t + off);
    }
    epi_qkv_rope4_core(e, m, c0, v, pr, cs, sn, slot0);
  } else {
    EpiArgs e2 = e;
    e2.bias = nullptr;                                            // already in slab 0
    epi_store4<EPI>(e2, m, c0, sum4(c0), 0);
  }
}

#ifndef PG_T128_STAGES_F8
#define PG_T128_STAGES_F8 2  // stages of the 128 x 128 fp8 tile (2: two workgroups per CU; 3 / 4 = one per CU, pt-896 x32
                             // gate/up 10.1 -> 14.6 / 14.3 ms)
#endif
#ifndef PG_F8_G256
// fp8 GEMMs on the 256x256 kernel: 0 never, 1 the fp32-slab epilogue only (round 4: pt-896 x32 o + down 115.7 -> 102.5
// ms per prefill), 2 every epilogue (gate/up 182 -> 211 ms and q|k|v 21 -> 48 ms: those instances still spill).
// Round 6: with the down projection on MX rows (the 128 x 128 tile, 5.3 ms vs 6.3 on the 256 kernel), the o_proj
// alone is faster on the 128 x 128 tile too: pt-896 x32 prefill 698.9 / 699.7 -> 695.3 / 696.5 ms
// (profiles/r06_fp8_prefill_ab.jsonl), so 0 -- until the spill-free staging (PG_G256_F8_BUF): o_proj 765 -> 742 us
// on the 256 kernel, q|k|v (RoPE epilogue, still spilling) 1.22 -> 2.29 ms, so 1 again
#define PG_F8_G256 1
#endif
#ifndef PG_G256_MIN_TILES
#define PG_G256_MIN_TILES 256   // large-M GEMM when its 256x256 grid fills every CU
#endif

// Tile choice: 128-row tiles (2-stage ring, 64 KiB LDS -> 2 workgroups per CU) when that grid already
// has >= 256 workgroups; otherwise 64-row tiles with a 4-stage ring.  Split-K (fp32 partial epilogue
// only) is chosen by the caller.
// F8: A, W fp8 viewed as bf16-sized pairs (K, lda, ldw in 2-byte units: a 64-unit k-tile = 128 fp8 k)
// waves per workgroup of each gemm_tile_kernel shape (4, or 8 / 12 -- see the kernel).  8 / 8 / 8 / 12 measured
// 3-12 % faster than 4 on every batch-1 prefill GEMM and pt-224 prefill 5.29 -> 4.95 ms
// (profiles/r03_tile_waves_ab.txt)
#ifndef PG_TILE_KSUB
#define PG_TILE_KSUB 1    // 2: 64-row tiles stage 128 k per barrier (K % 128 == 0; 3 stages)
#endif
#ifndef PG_TILE_AUTO_N64
#define PG_TILE_AUTO_N64 1   // 64 x 64 tiles when the 64 x 128 grid has fewer workgroups than CUs (bf16)
#endif
#ifndef PG_TILE_W64
#define PG_TILE_W64 8
#endif
#ifndef PG_TILE_W128
#define PG_TILE_W128 8
#endif
#ifndef PG_TILE_W256
#define PG_TILE_W256 8
#endif
#ifndef PG_TILE_W288
#define PG_TILE_W288 12
#endif
// 64-row tiles, BN 128 (WV waves) or 64 (4 waves): 64-k stages (4 deep), or with PG_TILE_KSUB 2 and K % 128 == 0
// 128-k stages (3 deep)
template <int EPI, bool FRAG, bool F8, int BN, int WV>
static void launch_t64(const bf16_t* A, int lda, const bf16_t* W, int ldw, int K, int ksplit, const EpiArgs& e,
                       hipStream_t st) {
  const int m64 = (e.M + 63) / 64, tn = (e.N + BN - 1) / BN;
  if constexpr (PG_TILE_KSUB == 2) {
    if (K % 128 == 0) {
      const int kchunk = ((K / 128 + ksplit - 1) / ksplit) * 128;
      hipLaunchKernelGGL((gemm_tile_kernel<EPI, 64, 3, FRAG, F8, WV, BN, 2>), dim3(m64 * tn, 1, ksplit), dim3(64 * WV),
                         0, st, A, lda, W, ldw, K, kchunk, m64, tn, e);
      return;
    }
  }
  const int kchunk = ((K / TBK + ksplit - 1) / ksplit) * TBK;
  hipLaunchKernelGGL((gemm_tile_kernel<EPI, 64, 4, FRAG, F8, WV, BN>), dim3(m64 * tn, 1, ksplit), dim3(64 * WV), 0, st,
                     A, lda, W, ldw, K, kchunk, m64, tn, e);
}

template <int EPI, bool FRAG, bool F8 = false>
static void launch_tile(const bf16_t* A, int lda, const bf16_t* W, int ldw, int K, int ksplit, const EpiArgs& e,
                        hipStream_t st, bool m1 = false, bool n64 = false) {
  if (n64) {
    // (a 9-stage ring for one-round grids measured 3-10% slower on every batch-1 shape: r03_tile_sweep.txt)
    launch_t64<EPI, FRAG, F8, 64, 4>(A, lda, W, ldw, K, ksplit, e, st);
    return;
  }
  if constexpr (!F8) {
    if (m1) {
      // PG_TILE_M1 (batch-1 prefill: 256 image + a few text rows): ALL rows in one tile, so every weight tile
      // streams once and no 256-row tile is spent on an 8-row remainder (M = 264: 2 x 256 rows in gemm256)
      const int tiles_n = (e.N + TBN - 1) / TBN;
      const int kchunk = ((K / TBK + ksplit - 1) / ksplit) * TBK;
      constexpr bool WNT = PG_TILE_M1_WNT;
      if (e.M <= 256)
        hipLaunchKernelGGL((gemm_tile_kernel<EPI, 256, 3, FRAG, false, PG_TILE_W256, TBN, 1, WNT>),
                           dim3(tiles_n, 1, ksplit), dim3(64 * PG_TILE_W256), 0, st, A, lda,
                           W, ldw, K, kchunk, 1, tiles_n, e);
      else
        hipLaunchKernelGGL((gemm_tile_kernel<EPI, 288, 3, FRAG, false, PG_TILE_W288, TBN, 1, WNT>),
                           dim3(tiles_n, 1, ksplit), dim3(64 * PG_TILE_W288), 0, st, A, lda,
                           W, ldw, K, kchunk, 1, tiles_n, e);
      return;
    }
  }
  if constexpr (F8 && (EPI == PG_EPI_F32 || EPI == PG_EPI_F32_RES || EPI == PG_EPI_BF16_GELU_MUL)) {
    if (e.f.mx_in || e.f.mx_out) {
      // (ABI 12) MX rows in (the prefill down projection) / MX h out (the prefill gate/up): the 128 x 128 fp8 tile, whose
      // waves own 32 rows x 64 W rows -- one 32-column h block per row (out), two row subtiles of scales (in)
      const int tiles_n = (e.N + TBN - 1) / TBN, tiles_m = (e.M + 127) / 128;
      const int kchunk = ((K / TBK + ksplit - 1) / ksplit) * TBK;
      if (e.f.mx_in)
        hipLaunchKernelGGL((gemm_tile_kernel<EPI, 128, PG_T128_STAGES_F8, FRAG, true, PG_TILE_W128, TBN, 1, false, true>),
                           dim3(tiles_m * tiles_n, 1, ksplit), dim3(64 * PG_TILE_W128), 0, st, A, lda, W, ldw, K,
                           kchunk, tiles_m, tiles_n, e);
      else
        hipLaunchKernelGGL((gemm_tile_kernel<EPI, 128, PG_T128_STAGES_F8, FRAG, true, PG_TILE_W128>),
                           dim3(tiles_m * tiles_n, 1, ksplit), dim3(64 * PG_TILE_W128), 0, st, A, lda, W, ldw, K,
                           kchunk, tiles_m, tiles_n, e);
      return;
    }
  }
  const int t256 = ((e.M + 255) / 256) * ((e.N + 255) / 256);
  // (fp8 on the 256 x 256 kernel addresses its operands by 32-bit byte offsets: both must be < 4 GiB)
  const bool off32 = (size_t)e.M * lda * 2 < (1ull << 32) && (size_t)e.N * ldw * 2 < (1ull << 32);
  constexpr bool g256 = !F8 || PG_F8_G256 == 2 || (PG_F8_G256 == 1 && (EPI == PG_EPI_F32 || EPI == PG_EPI_F32_RES));
  if (g256 && (!F8 || off32) && t256 * ksplit >= PG_G256_MIN_TILES && (ksplit == 1 || EPI == PG_EPI_F32)) {
    const int kts = (K / 64 + ksplit - 1) / ksplit;
    hipLaunchKernelGGL((gemm256_kernel<EPI, FRAG, F8>), dim3(t256, 1, ksplit), dim3(512), 0, st, A, lda, W, ldw, K, kts,
                       (e.M + 255) / 256, (e.N + 255) / 256, e);
    return;
  }
  const int tiles_n = (e.N + TBN - 1) / TBN;
  int kchunk = ((K / TBK + ksplit - 1) / ksplit) * TBK;
  const int t128 = ((e.M + 127) / 128) * tiles_n;
  if (t128 >= 256) {
    const int tiles_m = (e.M + 127) / 128;
    hipLaunchKernelGGL((gemm_tile_kernel<EPI, 128, F8 ? PG_T128_STAGES_F8 : 2, FRAG, F8, PG_TILE_W128>),
                       dim3(tiles_m * tiles_n, 1, ksplit),
                       dim3(64 * PG_TILE_W128), 0, st,
                       A, lda, W, ldw, K, kchunk, tiles_m, tiles_n, e);
    return;
  }
  // (a 96-row tile wastes fewer padded rows at M = 264 but measured slower: fewer workgroups)
  const int m64 = (e.M + 63) / 64;
  if (!F8 && PG_TILE_AUTO_N64 && m64 * tiles_n * ksplit < 256) {
    // a 64 x 128 grid short of one workgroup per CU: 64 x 64 tiles, twice the workgroups (batch-1 prefill: SigLIP
    // q|k|v 13.7 -> 11.7 us, never slower on the other shapes; profiles/r03_tile_sweep.txt)
    launch_t64<EPI, FRAG, F8, 64, 4>(A, lda, W, ldw, K, ksplit, e, st);
    return;
  }
  launch_t64<EPI, FRAG, F8, TBN, PG_TILE_W64>(A, lda, W, ldw, K, ksplit, e, st);
}

int pg_dispatch_tile(int epi, bool frag, bool f8, const bf16_t* A, int lda, const bf16_t* W, int ldw, int K, int ksplit,
                     const EpiArgs& e, hipStream_t st, bool m1, bool n64) {
  if (f8) {
    switch (epi) {
      case PG_EPI_BF16: launch_tile<PG_EPI_BF16, false, true>(A, lda, W, ldw, K, ksplit, e, st, false, n64); return 0;
      case PG_EPI_BF16_GELU_MUL:
        launch_tile<PG_EPI_BF16_GELU_MUL, false, true>(A, lda, W, ldw, K, ksplit, e, st, false, n64);
        return 0;
      case PG_EPI_F32: launch_tile<PG_EPI_F32, false, true>(A, lda, W, ldw, K, ksplit, e, st, false, n64); return 0;
      case PG_EPI_F32_RES:
        launch_tile<PG_EPI_F32_RES, false, true>(A, lda, W, ldw, K, ksplit, e, st, false, n64);
        return 0;
      case PG_EPI_QKV_ROPE:
        launch_tile<PG_EPI_QKV_ROPE, false, true>(A, lda, W, ldw, K, ksplit, e, st, false, n64);
        return 0;
      default: return (int)hipErrorInvalidValue;
    }
  }
#define PG_CASE(E)                                                                             \
  case E:                                                                                      \
    if (frag) launch_tile<E, true>(A, lda, W, ldw, K, ksplit, e, st, m1, n64);                 \
    else launch_tile<E, false>(A, lda, W, ldw, K, ksplit, e, st, m1, n64);                     \
    return 0;
#define PG_CASE_ROWMAJOR(E)                                                                    \
  case E: launch_tile<E, false>(A, lda, W, ldw, K, ksplit, e, st, m1, n64); return 0;
  switch (epi) {
    PG_CASE(PG_EPI_BF16)
    PG_CASE(PG_EPI_BF16_GELU_MUL)
    PG_CASE(PG_EPI_F32)
    PG_CASE(PG_EPI_F32_RES)
    PG_CASE(PG_EPI_QKV_ROPE)
    PG_CASE_ROWMAJOR(PG_EPI_BF16_GELU)
    PG_CASE_ROWMAJOR(PG_EPI_F32_POS)
    PG_CASE_ROWMAJOR(PG_EPI_BF16_VT)
    default: return (int)hipErrorInvalidValue;     // (F32_FIN / F32_ADD / FX_ADD: GEMV only)
  }
#undef PG_CASE
#undef PG_CASE_ROWMAJOR
}

// C = epilogue(sum_z part[z]) for a GEMM run as PG_EPI_F32 with ksplit slabs (bias was applied to slab 0)
extern "C" int pg_gemm_finalize(const float* part, int nsplit, void* C, int ldc, int M, int N, int epi,
                                void* aux_out, int aux_ld, int aux_n, const PgFusedArgs* fa, hipStream_t stream) {
  PG_REQUIRE(part != nullptr && C != nullptr && nsplit >= 1 && M > 0 && N > 0 && N % 4 == 0);
  PgFusedArgs f{};
  if (fa) f = *fa;
  EpiArgs e{nullptr, C, ldc, M, N, nullptr, 0, (bf16_t*)aux_out, aux_ld, aux_n, f};
  const int NO = epi == PG_EPI_BF16_GELU_MUL ? N / 2 : N;
  const long items = (long)M * (NO / 4);
  const dim3 grid((unsigned)((items + 255) / 256));
  switch (epi) {
    case PG_EPI_F32: hipLaunchKernelGGL((gemm_finalize_kernel<PG_EPI_F32>), grid, dim3(256), 0, stream, part, nsplit, e); break;
    case PG_EPI_BF16: hipLaunchKernelGGL((gemm_finalize_kernel<PG_EPI_BF16>), grid, dim3(256), 0, stream, part, nsplit, e); break;
    case PG_EPI_BF16_GELU: hipLaunchKernelGGL((gemm_finalize_kernel<PG_EPI_BF16_GELU>), grid, dim3(256), 0, stream, part, nsplit, e); break;
    case PG_EPI_BF16_GELU_MUL:
      PG_REQUIRE(N % 32 == 0);
      hipLaunchKernelGGL((gemm_finalize_kernel<PG_EPI_BF16_GELU_MUL>), grid, dim3(256), 0, stream, part, nsplit, e); break;
    case PG_EPI_BF16_VT:
      PG_REQUIRE(aux_out != nullptr && aux_n % 4 == 0);
      hipLaunchKernelGGL((gemm_finalize_kernel<PG_EPI_BF16_VT>), grid, dim3(256), 0, stream, part, nsplit, e); break;
    case PG_EPI_QKV_ROPE:
      PG_REQUIRE(fa && f.head_dim % 16 == 0 && f.cos_t && f.sin_t && f.pos && f.kc && f.vtc && f.rows_per_batch > 0 &&
                 f.smax > 0 && N == (f.q_heads + 2 * f.kv_heads) * f.head_dim);
      hipLaunchKernelGGL((gemm_finalize_kernel<PG_EPI_QKV_ROPE>), grid, dim3(256), 0, stream, part, nsplit, e); break;
    default: return (int)hipErrorInvalidValue;
  }
  PG_LAUNCH_CHECK();
  return 0;
}
