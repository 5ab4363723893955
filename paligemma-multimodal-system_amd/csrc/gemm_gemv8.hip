// fp8 decode GEMV (17..32 rows, fragment-packed e4m3 weights): gemv8_kernel / gemv8x_kernel and their launchers
// (see gemm_common.h).
#include "gemm_common.h"

// --------------------------------------------------------------------------------------
// fp8 weight-streaming GEMV for 17..32 rows (batched decode on the fp8 path, BASELINE configs[4])
// --------------------------------------------------------------------------------------
// The batch-32 decode linears read each e4m3 weight once per step; as 64 x 128 / 128 x 128 tile GEMMs they staged
// W through LDS at 3.1-3.3 TB/s.  Here, as in gemv_body, W streams straight to VGPRs: the weights are stored
// fragment-packed (PG_W_FRAG with PG_FP8, weights.frag_pack8): W[16t + r][128c + 64s + 16g + e] (e < 16 bytes) at
// byte ((t * (K/128) + c) * 2 + s) * 1024 + (16g + r) * 16 + e, so piece s of a 16-row x 128-k chunk is one 1-KiB
// lane-linear non-temporal load -- the MFMA's own k order (lane group g holds k 16g + e and 64 + 16g + e; measured,
// scripts/tune/mx_probe.hip).  Lane (r, g) loads x row r (and 16 + r) at the same k bytes, one
// v_mfma_scale_f32_16x16x128_f8f6f4 (unit block scales) per (W tile, 16-row x tile) and chunk; the 4 waves split
// the chunks of split blockIdx.y round-robin, DEPTH chunks in flight, and reduce through LDS.  The accumulator is
// scaled by a_scale[m] * w_scale[n] before the tile kernel's epilogues (bf16, gelu*up, fp32 slabs, RoPE + KV).
// MX: x rows carry E8M0 block scales (PgFusedArgs.mx_in, [M][4][K/128]).  The MFMA takes the scale of column r's
// 32-k block b (k 32b .. 32b + 31 of the chunk, spread over lane groups 2(b % 2) and 2(b % 2) + 1) from lane (r, b), so
// lane (r, g) loads block g's scale byte with its x bytes (no a_scale in the epilogue)
// RS (row split, MT 1): blockIdx.z picks the 16-row tile -- twice the workgroups for the 17..32-row q|k|v GEMV, whose
// 160 tiles alone leave 96 CUs idle, and for the o_proj's 256 (each weight tile is read by two workgroups at once)
template <int EPI, int NT, int MT, int DEPTH, int CPW, bool MX = false, bool RS = false>
__global__ __launch_bounds__(256) void gemv8_kernel(const uint8_t* __restrict__ X, int ldx,
                                                    const uint8_t* __restrict__ W, int K, EpiArgs e) {
  static_assert(!RS || MT == 1, "row split: one 16-row tile per workgroup");
  amax_clear(e);
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int g = lane >> 4, r0 = lane & 15;
  const int r = (RS ? (int)blockIdx.z * 16 : 0) + r0;   // (the row of this lane's first row tile)
  const int tile0 = blockIdx.x * NT;
  const int M = e.M;
  const int z = blockIdx.y;
  const int nch_all = K >> 7;
  const int per_z = (nch_all + (int)gridDim.y - 1) / (int)gridDim.y;
  const int c0 = z * per_z;
  const int nch = min(nch_all - c0, per_z);
  const int mine = CPW > 0 ? CPW : (nch > wave ? (nch - wave + 3) / 4 : 0);   // chunks wave, wave + 4, ...
  const uint8_t* wt[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) wt[t] = W + (size_t)min(tile0 + t, (e.N >> 4) - 1) * 16 * K + lane * 16;
  const uint8_t* xr[MT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) xr[mt] = X + (size_t)min(mt * 16 + r, M - 1) * ldx + g * 16;
  f32x4 acc[NT][MT];
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) acc[t][mt] = f32x4{0.f, 0.f, 0.f, 0.f};
  u32x4 wb[DEPTH][NT][2], xb[DEPTH][MT][2];
  int sbr[DEPTH][MT];
  const uint8_t* mxr[MT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
    mxr[mt] = MX ? e.f.mx_in + (size_t)min(mt * 16 + r, M - 1) * (K >> 5) + (size_t)g * nch_all : nullptr;
  // the epilogue's row factors (a_scale, or the MX rows' sums of squares) issued ahead of the weight stream
  Fp8RowLoads rl[MT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) rl[mt] = fp8_row_load(e, mt * 16 + r);
  auto load = [&](int j, u32x4 (&wv)[NT][2], u32x4 (&xv)[MT][2], int (&sv)[MT]) {
    const size_t cc = (size_t)(c0 + wave + j * 4);
    if constexpr (MX) {
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) sv[mt] = mxr[mt][cc];
    }
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int sp = 0; sp < 2; ++sp)
        wv[t][sp] = __builtin_nontemporal_load((const u32x4*)(wt[t] + (cc * 2 + sp) * 1024));
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int sp = 0; sp < 2; ++sp) xv[mt][sp] = *(const u32x4*)(xr[mt] + cc * 128 + sp * 64);
  };
  auto compute = [&](const u32x4 (&wv)[NT][2], const u32x4 (&xv)[MT][2], const int (&sv)[MT]) {
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        const bf16x8 w0 = __builtin_bit_cast(bf16x8, wv[t][0]), w1 = __builtin_bit_cast(bf16x8, wv[t][1]);
        const bf16x8 x0 = __builtin_bit_cast(bf16x8, xv[mt][0]), x1 = __builtin_bit_cast(bf16x8, xv[mt][1]);
        if constexpr (MX) acc[t][mt] = mfma8s(w0, w1, x0, x1, acc[t][mt], sv[mt]);
        else acc[t][mt] = mfma8(w0, w1, x0, x1, acc[t][mt]);
      }
  };
  // (QKV epilogue operands issued with the stream, as gemv_body does, are not needed: the tile epilogue loads them)
#pragma unroll
  for (int d = 0; d < DEPTH; ++d)
    if (CPW > 0 ? d < CPW : d < mine) load(d, wb[d], xb[d], sbr[d]);
  if constexpr (CPW > 0) {
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int j = 0; j < CPW; ++j) {
      const int d = j % DEPTH;
      compute(wb[d], xb[d], sbr[d]);
      if (j + DEPTH < CPW) load(j + DEPTH, wb[d], xb[d], sbr[d]);
      __builtin_amdgcn_sched_barrier(0);
    }
  } else {
    for (int base = 0; base < mine; base += DEPTH) {
#pragma unroll
      for (int d = 0; d < DEPTH; ++d) {
        const int j = base + d;
        if (j < mine) {
          compute(wb[d], xb[d], sbr[d]);
          if (j + DEPTH < mine) load(j + DEPTH, wb[d], xb[d], sbr[d]);
        }
      }
    }
  }
#pragma unroll
  for (int t = 0; t < NT; ++t) mfma_fence(acc[t]);
  __shared__ f32x4 red[4][NT][MT][64];
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) red[wave][t][mt][lane] = acc[t][mt];
  __syncthreads();
  if (wave != 0) return;
  const int q = 4 * g;
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) {
    const int m = mt * 16 + r;
    const float rf = fp8_row_finish(e, rl[mt]);
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      acc[t][mt] = red[0][t][mt][lane] + red[1][t][mt][lane] + red[2][t][mt][lane] + red[3][t][mt][lane];
      scale_acc_rf(e, m, (tile0 + t) * 16 + q, acc[t][mt], rf);
    }
    if constexpr (EPI == PG_EPI_BF16_GELU_MUL) {
#pragma unroll
      for (int t = 0; t < NT; t += 2) epi_gelu_mul4(e, m, (tile0 + t) * 16, q, acc[t][mt], acc[t + 1][mt]);
    } else if constexpr (EPI == PG_EPI_QKV_ROPE) {
#pragma unroll
      for (int t = 0; t < NT; ++t) epi_qkv_rope4(e, m, (tile0 + t) * 16 + q, acc[t][mt]);   // (all lanes: shuffle)
    } else if constexpr (EPI == PG_EPI_F32_ADD) {
#pragma unroll
      for (int t = 0; t < NT; ++t) epi_add4(e, m, (tile0 + t) * 16 + q, acc[t][mt], z);
    } else {
#pragma unroll
      for (int t = 0; t < NT; ++t) epi_store4<EPI>(e, m, (tile0 + t) * 16 + q, acc[t][mt], z);
    }
  }
}

// The wide form (large N: gate/up, down, the lm_head): x is staged ONCE per workgroup in LDS and the 4 waves split
// the W tiles instead of K (wave w owns tiles tile0 + w*NTW ...), so a workgroup reads x[32][Kr] once for 4 * NTW
// tiles -- at 32 rows x costs as many bytes per 16-row tile as the tile itself, and the per-CU load rate, not HBM,
// bounded the K-split form (gate/up 4.3 TB/s, down 2.9).  x [M <= 32][Kr] arrives by LDS-DMA (1 KiB pieces, the 16-B
// chunks of a row XOR-swizzled by row through the source address), issued before the W stream; each wave then
// streams its own W tiles DEPTH chunks deep and reads its x fragments from LDS.  No cross-wave reduction: every
// wave runs the epilogue of its own tiles (bf16, gelu*up on gate/up pairs, fp32 slabs, float-atomic residual add).
// XB (pro_mode 5): X is bf16 h [M][ldx elements] and row m's amax (amax_in, max-ed by the gate/up epilogue): each
// thread loads 16-element pieces, divides by s[m] = amax / 448 and packs e4m3 (pg_quant_fp8's bytes) into the same
// swizzled LDS layout -- the quantiser launch between gate/up and down is gone; x costs twice the bytes per
// workgroup (bf16), all issued before the W stream.
// MX (CPW > 0): x rows carry E8M0 block scales (PgFusedArgs.mx_in): lane (r, g)'s scale bytes (block g of each of
// the CPW chunks of its split, as in gemv8_kernel) are loaded before the W stream and handed to the MFMA per chunk.
// GELU_MUL with PgFusedArgs.mx_out (NTW 2: a wave's gate/up pair is 16 h columns, waves w and w ^ 1 hold the two halves
// of a 32-column MX block): h is written as e4m3 bytes with one E8M0 scale per block -- the block max of the
// bf16-rounded h exchanged between the two waves through LDS, no cross-workgroup reduction and no quantiser launch.
template <int EPI, int NTW, int MT, int DEPTH, int CPW, bool XB = false, bool MX = false>
__global__ __launch_bounds__(256) void gemv8x_kernel(const uint8_t* __restrict__ X, int ldx,
                                                     const uint8_t* __restrict__ W, int K, EpiArgs e) {
  extern __shared__ __attribute__((aligned(16))) char xs8[];
  static_assert(!XB || CPW > 0, "the bf16-x form needs a compile-time chunk count");
  static_assert(!MX || (CPW > 0 && !XB), "MX rows need a compile-time chunk count");
  amax_clear(e);
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int g = lane >> 4, r = lane & 15;
  const int tile0 = (blockIdx.x * 4 + wave) * NTW;
  const int M = e.M;
  const int z = blockIdx.y;
  const int nch_all = K >> 7;
  const int per_z = (nch_all + (int)gridDim.y - 1) / (int)gridDim.y;
  const int c0 = z * per_z;
  const int nch = CPW > 0 ? CPW : max(0, min(nch_all - c0, per_z));
  const int Kr = nch * 128;                        // bytes of one x row in LDS
  // 1. x rows [0, 16 MT) x bytes [128 c0, +Kr) into LDS by DMA: LDS byte o = row * Kr + 16 pc holds logical chunk
  //    pc ^ (row & 7) of the row (rows past M repeat row M-1: their outputs are never stored)
  constexpr int XPT = XB ? MT * 16 * CPW * 8 / 256 : 1;   // XB: 16-element pieces per thread
  u32x4 xh[XPT][2];
  if constexpr (XB) {
    const bf16_t* Xb = (const bf16_t*)X;
#pragma unroll
    for (int i = 0; i < XPT; ++i) {
      const int ci = (int)threadIdx.x + i * 256;   // LDS chunk: row ci / (8 CPW), position pc
      const int row = ci / (8 * CPW), pc = ci % (8 * CPW);
      const bf16_t* src = Xb + (size_t)min(row, M - 1) * ldx + (size_t)c0 * 128 + (pc ^ (row & 7)) * 16;
      xh[i][0] = *(const u32x4*)src;
      xh[i][1] = *(const u32x4*)(src + 8);
    }
  } else {
    const int pieces = MT * 16 * Kr / 1024;        // 1 KiB each, dealt round-robin to the waves
    for (int pi = wave; pi < pieces; pi += 4) {
      const int o = pi * 1024 + lane * 16;
      const int row = o / Kr, pc = (o % Kr) >> 4;
      const int lc = pc ^ (row & 7);
      const uint8_t* src = X + (size_t)min(row, M - 1) * ldx + (size_t)c0 * 128 + lc * 16;
      __builtin_amdgcn_global_load_lds((const void*)src, (LDS_AS void*)(xs8 + pi * 1024), 16, 0, 0);
    }
  }
  // MX rows: this lane's E8M0 scale of block g of each of its CPW chunks, rows r and 16 + r (loaded with the x pieces,
  // before the W stream; the step-3 wait covers them)
  // (the CPW bytes are consecutive and CPW-aligned: one 8- or 16-byte load per row tile)
  u32x4 sbv[MX ? MT : 1];
  if constexpr (MX) {
    static_assert(CPW == 8 || CPW == 16, "MX scale bytes load as one 8- or 16-byte vector");
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      const uint8_t* sp = e.f.mx_in + (size_t)min(mt * 16 + r, M - 1) * (K >> 5) + (size_t)g * nch_all + c0;
      if constexpr (CPW == 16) {
        sbv[mt] = *(const u32x4*)sp;
      } else {
        const u32x2 h = *(const u32x2*)sp;
        sbv[mt] = u32x4{h[0], h[1], 0u, 0u};
      }
    }
  }
  auto sbx = [&](int mt, int j) -> int { return (int)((sbv[mt][j >> 2] >> (8 * (j & 3))) & 0xffu); };
  // the epilogue's row factors, issued with the x pieces (not with XB: its scale comes from amax_in)
  Fp8RowLoads rl[XB ? 1 : MT];
  if constexpr (!XB) {
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) rl[mt] = fp8_row_load(e, mt * 16 + r);
  }
  // the x DMA pieces stay ahead of every W load in the vmcnt order (step 3 waits for "at most the W loads
  // outstanding"): the scheduler may not hoist a W load above them
  __builtin_amdgcn_sched_barrier(0);
  const uint8_t* wt[NTW];
#pragma unroll
  for (int t = 0; t < NTW; ++t) wt[t] = W + (size_t)min(tile0 + t, (e.N >> 4) - 1) * 16 * K + lane * 16;
  f32x4 acc[NTW][MT];
#pragma unroll
  for (int t = 0; t < NTW; ++t)
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) acc[t][mt] = f32x4{0.f, 0.f, 0.f, 0.f};
  u32x4 wb[DEPTH][NTW][2];
  auto loadw = [&](int j, u32x4 (&wv)[NTW][2]) {
    const size_t cc = (size_t)(c0 + j);
#pragma unroll
    for (int t = 0; t < NTW; ++t)
#pragma unroll
      for (int sp = 0; sp < 2; ++sp)
        wv[t][sp] = __builtin_nontemporal_load((const u32x4*)(wt[t] + (cc * 2 + sp) * 1024));
  };
  // 2. the W stream, DEPTH chunks deep, issued behind the x pieces
#pragma unroll
  for (int d = 0; d < DEPTH; ++d)
    if (CPW > 0 ? d < CPW : d < nch) loadw(d, wb[d]);
  // 3. this wave's x pieces have landed once at most its W loads are outstanding; the barrier covers the others'
  {
    const int wl = (CPW > 0 ? min(DEPTH, CPW) : min(DEPTH, nch)) * NTW * 2;
    wait_vm_n(wl);
    if constexpr (XB) {
#pragma unroll
      for (int i = 0; i < XPT; ++i) {
        const int ci = (int)threadIdx.x + i * 256;
        const int row = ci / (8 * CPW), pc = ci % (8 * CPW);
        const float am = __uint_as_float(e.f.amax_in[(size_t)min(row, M - 1) * e.f.amax_ld]);
        const float sc = am > 0.f ? am / 448.f : 1.f;
        u32x4 w8;
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
          for (int j = 0; j < 2; ++j)
            w8[2 * h + j] = pack_fp8x4(bf_lo(xh[i][h][2 * j]) / sc, bf_hi(xh[i][h][2 * j]) / sc,
                                       bf_lo(xh[i][h][2 * j + 1]) / sc, bf_hi(xh[i][h][2 * j + 1]) / sc);
        *(u32x4*)(xs8 + row * Kr + pc * 16) = w8;
      }
    }
    __syncthreads();
  }
  auto compute = [&](int j, const u32x4 (&wv)[NTW][2]) {
    bf16x8 xf[MT][2];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      const int row = mt * 16 + r;
#pragma unroll
      for (int sp = 0; sp < 2; ++sp) {
        const int lc = j * 8 + sp * 4 + g;           // the lane's 16-B pieces: k 64sp + 16g of chunk j
        xf[mt][sp] = *(const bf16x8*)(xs8 + row * Kr + ((lc ^ (row & 7)) << 4));
      }
    }
#pragma unroll
    for (int t = 0; t < NTW; ++t)
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        if constexpr (MX)
          acc[t][mt] = mfma8s(__builtin_bit_cast(bf16x8, wv[t][0]), __builtin_bit_cast(bf16x8, wv[t][1]), xf[mt][0],
                              xf[mt][1], acc[t][mt], sbx(mt, j));
        else
          acc[t][mt] = mfma8(__builtin_bit_cast(bf16x8, wv[t][0]), __builtin_bit_cast(bf16x8, wv[t][1]), xf[mt][0],
                             xf[mt][1], acc[t][mt]);
      }
  };
  if constexpr (CPW > 0) {
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int j = 0; j < CPW; ++j) {
      const int d = j % DEPTH;
      compute(j, wb[d]);
      if (j + DEPTH < CPW) loadw(j + DEPTH, wb[d]);
      __builtin_amdgcn_sched_barrier(0);
    }
  } else {
    for (int base = 0; base < nch; base += DEPTH) {
#pragma unroll
      for (int d = 0; d < DEPTH; ++d) {
        const int j = base + d;
        if (j < nch) {
          compute(j, wb[d]);
          if (j + DEPTH < nch) loadw(j + DEPTH, wb[d]);
        }
      }
    }
  }
#pragma unroll
  for (int t = 0; t < NTW; ++t) mfma_fence(acc[t]);
  const int q = 4 * g;
  float gam[MT];                                   // GELU_MUL with amax_out / mx_out: this lane's max |h| per row tile
  f32x4 mxh[MT];                                   // ... mx_out: the lane's h values
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) {
    const int m = mt * 16 + r;
    gam[mt] = 0.f;
    if constexpr (XB) {
      const float am = __uint_as_float(e.f.amax_in[(size_t)min(m, M - 1) * e.f.amax_ld]);
      const float sa = am > 0.f ? am / 448.f : 1.f;
#pragma unroll
      for (int t = 0; t < NTW; ++t) {
        const int n0 = (tile0 + t) * 16 + q;
        if (m < e.M && n0 < e.N) acc[t][mt] *= sa * load4_guard(e.f.w_scale, n0, e.N);
      }
    } else {
      const float rf = fp8_row_finish(e, rl[mt]);
#pragma unroll
      for (int t = 0; t < NTW; ++t) scale_acc_rf(e, m, (tile0 + t) * 16 + q, acc[t][mt], rf);
    }
    if constexpr (EPI == PG_EPI_BF16_GELU_MUL) {
      if (NTW == 2 && e.f.mx_out) {
        // MX h: the lane's 4 bf16-rounded values kept for the block scale below (stored there)
        const f32x4 gv = acc[0][mt], uv = acc[1][mt];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float hv = __uint_as_float((uint32_t)f2bf(gelu_tanh(gv[j]) * uv[j]) << 16);
          mxh[mt][j] = hv;
          gam[mt] = fmaxf(gam[mt], fabsf(hv));
        }
      } else if (e.f.amax_out) {
#pragma unroll
        for (int t = 0; t < NTW; t += 2)
          gam[mt] = fmaxf(gam[mt], epi_gelu_mul4_amax(e, m, (tile0 + t) * 16, q, acc[t][mt], acc[t + 1][mt]));
      } else {
#pragma unroll
        for (int t = 0; t < NTW; t += 2) epi_gelu_mul4(e, m, (tile0 + t) * 16, q, acc[t][mt], acc[t + 1][mt]);
      }
    } else if constexpr (EPI == PG_EPI_F32_ADD) {
#pragma unroll
      for (int t = 0; t < NTW; ++t) epi_add4(e, m, (tile0 + t) * 16 + q, acc[t][mt], z);
    } else {
#pragma unroll
      for (int t = 0; t < NTW; ++t) epi_store4<EPI>(e, m, (tile0 + t) * 16 + q, acc[t][mt], z);
    }
  }
  if constexpr (EPI == PG_EPI_BF16_GELU_MUL && NTW == 2) {
    if (e.f.mx_out) {                              // (uniform: every wave reaches the barrier)
      // block max over the 4 lanes of a row (16 columns), then with the partner wave's 16 (the block's other half)
      __shared__ float smx[4][16 * MT];
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        float v = gam[mt];
        v = fmaxf(v, __shfl_xor(v, 16, 64));
        v = fmaxf(v, __shfl_xor(v, 32, 64));
        gam[mt] = v;
        if (g == 0) smx[wave][mt * 16 + r] = v;
      }
      __syncthreads();
      const int pair = tile0 >> 1, kb = pair >> 1;  // this wave's 16 h columns [16 pair, +16) lie in 32-block kb
      const int Nh = e.N >> 1;
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        const int m = mt * 16 + r;
        const int ex = mx_exp(fmaxf(gam[mt], smx[wave ^ 1][mt * 16 + r]));
        const float inv = __builtin_ldexpf(1.0f, -ex);
        const int col = pair * 16 + q;
        if (m < e.M && col + 3 < Nh) {
          *(uint32_t*)((uint8_t*)e.C + (size_t)m * e.ldc + col) =
              pack_fp8x4(mxh[mt][0] * inv, mxh[mt][1] * inv, mxh[mt][2] * inv, mxh[mt][3] * inv);
          if ((wave & 1) == 0 && g == 0)
            e.f.mx_out[(size_t)m * (Nh >> 5) + (size_t)(kb & 3) * (Nh >> 7) + (kb >> 2)] = (uint8_t)(ex + 127);
        }
      }
    }
  }
  if constexpr (EPI == PG_EPI_BF16_GELU_MUL) {
    if (e.f.amax_out) {                            // (uniform: every wave reaches the barrier)
      // row max over the 4 column groups of a lane's row, then over the 4 waves in LDS: one atomic per row per
      // workgroup (float bits of non-negative values order as unsigned)
      __shared__ float sam[4][16 * MT];
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        float v = gam[mt];
        v = fmaxf(v, __shfl_xor(v, 16, 64));
        v = fmaxf(v, __shfl_xor(v, 32, 64));
        if (g == 0) sam[wave][mt * 16 + r] = v;
      }
      __syncthreads();
      if ((int)threadIdx.x < 16 * MT && (int)threadIdx.x < M) {
        const float v = fmaxf(fmaxf(sam[0][threadIdx.x], sam[1][threadIdx.x]),
                              fmaxf(sam[2][threadIdx.x], sam[3][threadIdx.x]));
        if (v > 0.f)
          __hip_atomic_fetch_max(e.f.amax_out + (size_t)threadIdx.x * e.f.amax_ld, __float_as_uint(v),
                                 __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
  }
}

template <int EPI, int NTW, int MT, int DEPTH = 8>
static void launch_gemv8x_mt(const uint8_t* X, int ldx, const uint8_t* W, int K, int ksplit, const EpiArgs& e,
                             hipStream_t st) {
  const int tiles = e.N >> 4;
  const dim3 grid((tiles + 4 * NTW - 1) / (4 * NTW), ksplit);
  const int nch = K >> 7;
  const int per_z = (nch + ksplit - 1) / ksplit;
  const size_t lds = (size_t)MT * 16 * per_z * 128;
  const bool exact = nch % ksplit == 0;
  if constexpr (EPI == PG_EPI_F32) {
    if (e.f.pro_mode == 5) {                       // bf16 x quantised while staged (host: exact, 8 or 16 chunks)
      if (per_z == 16)
        hipLaunchKernelGGL((gemv8x_kernel<EPI, NTW, MT, 8, 16, true>), grid, dim3(256), lds, st, X, ldx, W, K, e);
      else
        hipLaunchKernelGGL((gemv8x_kernel<EPI, NTW, MT, 8, 8, true>), grid, dim3(256), lds, st, X, ldx, W, K, e);
      return;
    }
  }
  if (e.f.mx_in) {                                 // MX rows (launch_gemv8 checked: exact, 8 or 16 chunks)
    if (per_z == 16)
      hipLaunchKernelGGL((gemv8x_kernel<EPI, NTW, MT, DEPTH, 16, false, true>), grid, dim3(256), lds, st, X, ldx, W, K,
                         e);
    else
      hipLaunchKernelGGL((gemv8x_kernel<EPI, NTW, MT, DEPTH, 8, false, true>), grid, dim3(256), lds, st, X, ldx, W, K,
                         e);
    return;
  }
  if (exact && per_z == 16)
    hipLaunchKernelGGL((gemv8x_kernel<EPI, NTW, MT, DEPTH, 16>), grid, dim3(256), lds, st, X, ldx, W, K, e);
  else if (exact && per_z == 8)
    hipLaunchKernelGGL((gemv8x_kernel<EPI, NTW, MT, DEPTH, 8>), grid, dim3(256), lds, st, X, ldx, W, K, e);
  else
    hipLaunchKernelGGL((gemv8x_kernel<EPI, NTW, MT, DEPTH, 0>), grid, dim3(256), lds, st, X, ldx, W, K, e);
}

#ifndef PG_GEMV8_DEPTH
#define PG_GEMV8_DEPTH 4
#endif
template <int EPI, int NT, int MT, bool MX = false, bool RS = false>
static void launch_gemv8_mt(const uint8_t* X, int ldx, const uint8_t* W, int K, int ksplit, const EpiArgs& e,
                            hipStream_t st) {
  const dim3 grid(((e.N >> 4) + NT - 1) / NT, ksplit, RS ? (e.M + 15) / 16 : 1);
  const int nch = K >> 7;
  const int cpw = (nch % ksplit == 0 && (nch / ksplit) % 4 == 0) ? nch / ksplit / 4 : 0;
  constexpr int D = PG_GEMV8_DEPTH;                // chunks in flight per wave
  switch (cpw) {
    case 2: hipLaunchKernelGGL((gemv8_kernel<EPI, NT, MT, 2, 2, MX, RS>), grid, dim3(256), 0, st, X, ldx, W, K, e); break;
    case 4: hipLaunchKernelGGL((gemv8_kernel<EPI, NT, MT, D, 4, MX, RS>), grid, dim3(256), 0, st, X, ldx, W, K, e); break;
    case 8: hipLaunchKernelGGL((gemv8_kernel<EPI, NT, MT, D, 8, MX, RS>), grid, dim3(256), 0, st, X, ldx, W, K, e); break;
    default: hipLaunchKernelGGL((gemv8_kernel<EPI, NT, MT, D, 0, MX, RS>), grid, dim3(256), 0, st, X, ldx, W, K, e); break;
  }
}

#ifndef PG_GEMV8_ROWSPLIT
#define PG_GEMV8_ROWSPLIT 1
#endif
template <int EPI, int NT>
static void launch_gemv8_nt(const uint8_t* X, int ldx, const uint8_t* W, int K, int ksplit, const EpiArgs& e,
                            hipStream_t st) {
  if constexpr (EPI == PG_EPI_QKV_ROPE || EPI == PG_EPI_F32) {
    // (a grid short of two workgroups per CU: the row split doubles it)
    if (PG_GEMV8_ROWSPLIT && e.M > 16 && ((e.N >> 4) + NT - 1) / NT * ksplit < 512) {
      if (e.f.mx_in) launch_gemv8_mt<EPI, NT, 1, true, true>(X, ldx, W, K, ksplit, e, st);
      else launch_gemv8_mt<EPI, NT, 1, false, true>(X, ldx, W, K, ksplit, e, st);
      return;
    }
  }
  if (e.f.mx_in) {
    if (e.M <= 16) launch_gemv8_mt<EPI, NT, 1, true>(X, ldx, W, K, ksplit, e, st);
    else launch_gemv8_mt<EPI, NT, 2, true>(X, ldx, W, K, ksplit, e, st);
    return;
  }
  if (e.M <= 16)
    launch_gemv8_mt<EPI, NT, 1>(X, ldx, W, K, ksplit, e, st);
  else
    launch_gemv8_mt<EPI, NT, 2>(X, ldx, W, K, ksplit, e, st);
}

#ifndef PG_GEMV8_NT_MAX
#define PG_GEMV8_NT_MAX 4
#endif
// NT W tiles per workgroup: every lane loads the x rows of its chunks once per workgroup, as many bytes per 16-row W
// tile as the tile itself at 32 rows, so wide tiles amortise x -- the most tiles per workgroup that still leave
// >= 256 workgroups (gelu*up: whole gate/up pairs); MT = 16-row x tiles
template <int EPI>
static void launch_gemv8(const uint8_t* X, int ldx, const uint8_t* W, int K, int ksplit, const EpiArgs& e,
                         hipStream_t st) {
  const int tiles = e.N >> 4;
  // the wide form (x once per workgroup in LDS, waves split N) when its grid still has >= 256 workgroups and a
  // split's x rows fit the LDS; the K-split form otherwise (q|k|v: 160 tiles; o_proj)
  const int per_z = ((K >> 7) + ksplit - 1) / ksplit;
  if constexpr (EPI == PG_EPI_F32) {
    if (e.f.pro_mode == 5) {                       // bf16 x: the wide form only (host checked the chunk count)
      const int wgs2 = (tiles + 7) / 8 * ksplit;
      if (e.M <= 16) {
        if (wgs2 >= 256) launch_gemv8x_mt<EPI, 2, 1>(X, ldx, W, K, ksplit, e, st);
        else launch_gemv8x_mt<EPI, 1, 1>(X, ldx, W, K, ksplit, e, st);
      } else {
        if (wgs2 >= 256) launch_gemv8x_mt<EPI, 2, 2>(X, ldx, W, K, ksplit, e, st);
        else launch_gemv8x_mt<EPI, 1, 2>(X, ldx, W, K, ksplit, e, st);
      }
      return;
    }
  }
  // (MX rows take the wide form only when its chunk count is a compile-time 8 or 16)
  const bool mx_ok = !e.f.mx_in || ((K >> 7) % ksplit == 0 && (per_z == 8 || per_z == 16));
  if constexpr (EPI != PG_EPI_QKV_ROPE) {
    if (PG_GEMV8_WIDE && per_z * 128 <= 4096 && mx_ok) {
      const int wgs2 = (tiles + 7) / 8 * ksplit, wgs1 = (tiles + 3) / 4 * ksplit;
      if (e.M <= 16) {
        if (wgs2 >= 256 || EPI == PG_EPI_BF16_GELU_MUL) { launch_gemv8x_mt<EPI, 2, 1>(X, ldx, W, K, ksplit, e, st); return; }
        if constexpr (EPI != PG_EPI_BF16_GELU_MUL)
          if (wgs1 >= 256) { launch_gemv8x_mt<EPI, 1, 1>(X, ldx, W, K, ksplit, e, st); return; }
      } else {
        if (wgs2 >= 256 || EPI == PG_EPI_BF16_GELU_MUL) { launch_gemv8x_mt<EPI, 2, 2>(X, ldx, W, K, ksplit, e, st); return; }
        if constexpr (EPI != PG_EPI_BF16_GELU_MUL)
          if (wgs1 >= 256) { launch_gemv8x_mt<EPI, 1, 2>(X, ldx, W, K, ksplit, e, st); return; }
      }
    }
  }
  if (PG_GEMV8_NT_MAX >= 4 && tiles % 4 == 0 && (tiles / 4) * ksplit >= 256)
    launch_gemv8_nt<EPI, 4>(X, ldx, W, K, ksplit, e, st);
  else if (EPI == PG_EPI_BF16_GELU_MUL || (PG_GEMV8_NT_MAX >= 2 && tiles % 2 == 0 && (tiles / 2) * ksplit >= 256))
    launch_gemv8_nt<EPI, 2>(X, ldx, W, K, ksplit, e, st);
  else if constexpr (EPI != PG_EPI_BF16_GELU_MUL)
    launch_gemv8_nt<EPI, 1>(X, ldx, W, K, ksplit, e, st);
}

int pg_dispatch_gemv8(int epi, const uint8_t* X, int ldx, const uint8_t* W, int K, int ksplit, const EpiArgs& e,
                      hipStream_t st) {
  switch (epi) {
    case PG_EPI_BF16: launch_gemv8<PG_EPI_BF16>(X, ldx, W, K, ksplit, e, st); return 0;
    case PG_EPI_BF16_GELU_MUL: launch_gemv8<PG_EPI_BF16_GELU_MUL>(X, ldx, W, K, ksplit, e, st); return 0;
    case PG_EPI_F32: launch_gemv8<PG_EPI_F32>(X, ldx, W, K, ksplit, e, st); return 0;
    case PG_EPI_QKV_ROPE: launch_gemv8<PG_EPI_QKV_ROPE>(X, ldx, W, K, ksplit, e, st); return 0;
    case PG_EPI_F32_ADD: launch_gemv8<PG_EPI_F32_ADD>(X, ldx, W, K, ksplit, e, st); return 0;
    default: return (int)hipErrorInvalidValue;
  }
}
