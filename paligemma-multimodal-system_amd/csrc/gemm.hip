// Argument checks and the C-ABI entry points of the GEMMs (include/pghip.h pg_gemm / pg_gemm_fused); the kernels live
// in gemm_tile.hip, gemm_gemv.hip and gemm_gemv8.hip (gemm_common.h).
#include "gemm_common.h"

static int gemm_impl(const void* A, int lda, const void* W, int ldw, const float* bias, void* C, int ldc,
                     int M, int N, int K, int epi_flags, int ksplit, const float* aux, int aux_rows, void* aux_out,
                     int aux_ld, int aux_n, const PgFusedArgs* fa, hipStream_t stream) {
  const bool frag = (epi_flags & PG_W_FRAG) != 0;
  const bool fp8 = (epi_flags & PG_FP8) != 0;
  const bool m1 = (epi_flags & PG_TILE_M1) != 0;
  const bool n64 = (epi_flags & PG_TILE_N64) != 0;
  const int epi = epi_flags & 0xFF;
  PG_REQUIRE((epi_flags & ~(0xFF | PG_W_FRAG | PG_FP8 | PG_TILE_M1 | PG_TILE_N64)) == 0 && epi <= PG_EPI_F32_RES);
  if (m1) PG_REQUIRE(!fp8 && !n64 && M >= 256 && M <= 288 && (fa == nullptr || fa->pro_mode == 0));
  if (n64) PG_REQUIRE(M > 16);
  PG_REQUIRE(M > 0 && N > 0 && K > 0 && ksplit >= 1 && W != nullptr && C != nullptr);
  PG_REQUIRE(K % 32 == 0 && ldw >= K && (N % 4) == 0);
  if (frag && !fp8) PG_REQUIRE(N % 16 == 0 && K % 64 == 0 && ldw == K &&
                       (epi == PG_EPI_BF16 || epi == PG_EPI_BF16_GELU_MUL || epi == PG_EPI_F32 ||
                        epi == PG_EPI_QKV_ROPE || epi == PG_EPI_F32_FIN || epi == PG_EPI_F32_ADD ||
                        epi == PG_EPI_FX_ADD || epi == PG_EPI_F32_RES));
  PgFusedArgs f{};
  if (fa) f = *fa;
  EpiArgs e{bias, C, ldc, M, N, aux, aux_rows, (bf16_t*)aux_out, aux_ld, aux_n, f};
  PG_REQUIRE(f.pro_mode >= 0 && f.pro_mode <= 5);
  if (f.pro_mode == 5)
    PG_REQUIRE(fp8 && frag && epi == PG_EPI_F32 && M <= 32 && f.amax_in && f.amax_ld >= 1 && A != nullptr &&
               lda >= K && lda % 8 == 0 && ((uintptr_t)A & 15) == 0 && K % 128 == 0 && (K / 128) % ksplit == 0 &&
               (K / 128 / ksplit == 8 || K / 128 / ksplit == 16));
  if (f.amax_out) PG_REQUIRE(fp8 && frag && epi == PG_EPI_BF16_GELU_MUL && M <= 32 && f.amax_ld >= 1 &&
                             ((K >> 7) + ksplit - 1) / ksplit * 128 <= 4096 && PG_GEMV8_WIDE);
  // (ABI 12: also the bf16 fragment-packed GEMV, which clears the batch-1 decode's fixed-point accumulator with it)
  if (f.amax_zero) PG_REQUIRE(frag && f.amax_zero_n >= 0 &&
                              (fp8 ? f.amax_zero_n <= 4096
                                   : (M <= 16 && f.amax_zero_n <= 16384 && f.amax_zero_n % 4 == 0 &&
                                      ((uintptr_t)f.amax_zero & 15) == 0)));
  if (f.pro_mode == 0 || f.pro_mode == 4) PG_REQUIRE(A != nullptr && lda >= K);
  // (M > 4 runs two 16-row tiles per workgroup: the per-row entries are loaded 16 per lane)
  if (f.pro_mode == 4) PG_REQUIRE(ksplit == 1 && f.ss_in && f.ss_n > 0 && f.ss_ld >= f.ss_n &&
                                  ((M <= 2 && f.ss_n <= 256 && (M == 1 || f.ss_n <= 128)) ||
                                   (M > 4 && M <= 16 && f.ss_n <= 64)));
  if (f.pro_mode != 0 && f.pro_mode != 5) PG_REQUIRE(M <= 16);
  if (f.pro_mode == 1) PG_REQUIRE(ksplit == 1 && (f.resid_in || f.fx) && f.norm_w && (f.nsplit == 0 || f.partials) &&
                                  K % 4 == 0);
  if (f.pro_mode == 2)
    PG_REQUIRE(f.part_o && f.part_ml && f.head_dim > 0 && (K / ksplit) % f.head_dim == 0 && f.asplit > 0 &&
               f.q_per_kv > 0 && f.kv_heads > 0);
  if (epi == PG_EPI_QKV_ROPE) PG_REQUIRE(f.head_dim % 16 == 0 && f.cos_t && f.sin_t && f.pos && f.kc && f.vtc &&
                                         f.rows_per_batch > 0 && f.smax > 0 && ksplit == 1 &&
                                         N == (f.q_heads + 2 * f.kv_heads) * f.head_dim);
  if (f.pro_mode == 3) PG_REQUIRE(ksplit == 1 && f.resid_in && f.norm_w && f.ss_in && f.ss_n > 0 &&
                                  f.ss_ld >= f.ss_n && K % 4 == 0);
  if (epi == PG_EPI_F32_FIN) PG_REQUIRE(M <= 16 && ksplit <= 8 && (f.fin_x == nullptr || f.norm_w != nullptr) && f.fin_cnt && f.fin_resid && f.ss_out && f.ss_ld >= (N + 15) / 16 &&
                                        ldc == N);
  if (epi == PG_EPI_F32_ADD) PG_REQUIRE((M <= 16 || (fp8 && frag && M <= 32)) && (f.pro_mode == 0 || f.pro_mode == 2) &&
                                        ldc >= N);
  // (ABI 13) the residual add moved into the producing tile GEMM: one producer per output, C 16-B aligned rows
  if (epi == PG_EPI_F32_RES) PG_REQUIRE(M > 16 && ksplit == 1 && f.pro_mode == 0 && ldc >= N && ldc % 4 == 0 &&
                                        ((uintptr_t)C & 15) == 0 && !f.mx_out);
  if (epi == PG_EPI_FX_ADD) PG_REQUIRE(M <= 16 && !fp8 && (f.pro_mode == 0 || f.pro_mode == 2) && ldc >= N &&
                                       ((uintptr_t)C & 15) == 0 && ldc % 2 == 0);
  if (f.mx_in && frag) PG_REQUIRE(fp8 && epi != PG_EPI_F32_ADD && M <= 32 && f.pro_mode == 0 && K % 128 == 0 &&
                                   A != nullptr && ((uintptr_t)f.mx_in & 15) == 0 &&
                                   (!f.ss_in || (f.ss_n > 0 && f.ss_n <= 4 && f.ss_ld >= f.ss_n && K == 1024 * f.ss_n)));
  // (ABI 12) the prefill tile form: MX rows [M][K] with scales [M][K/32] into the 256 x 256 fp32-slab GEMM
  if (f.mx_in && !frag) PG_REQUIRE(fp8 && (epi == PG_EPI_F32 || epi == PG_EPI_F32_RES) && M > 32 && f.pro_mode == 0 && K % 128 == 0 &&
                                   A != nullptr && ((uintptr_t)f.mx_in & 3) == 0 && !f.ss_in &&
                                   (size_t)M * (size_t)(K / 32) < (1ull << 32) &&
                                   (size_t)M * (size_t)lda < (1ull << 32) && (size_t)N * (size_t)ldw < (1ull << 32));
  // mx_out is written by the wide form only (gemv8x_kernel, NTW 2): launch_gemv8 takes it for GELU_MUL whenever a
  // split's x fits the LDS -- and, with MX rows in, when the split's chunk count is a compile-time 8 or 16
  if (f.mx_out && frag) PG_REQUIRE(fp8 && epi == PG_EPI_BF16_GELU_MUL && M <= 32 && f.pro_mode == 0 && !f.amax_out &&
                                    ksplit == 1 && (N / 2) % 128 == 0 && PG_GEMV8_WIDE && (K >> 7) * 128 <= 4096 &&
                                    (!f.mx_in || (K >> 7) == 8 || (K >> 7) == 16));
  // (ABI 12) the prefill tile form: e4m3 h [M][ldc bytes] + scales [M][N/64] from the 128 x 128 fp8 tile
  if (f.mx_out && !frag) PG_REQUIRE(fp8 && epi == PG_EPI_BF16_GELU_MUL && M > 32 && f.pro_mode == 0 && !f.mx_in &&
                                    ksplit == 1 && N % 128 == 0 && ldc >= N / 2);
  if (f.fx) PG_REQUIRE(((uintptr_t)f.fx & 15) == 0 && (f.pro_mode == 1) != (epi == PG_EPI_F32_FIN) && !fp8 &&
                       M <= 16);
  if (ksplit > 1) PG_REQUIRE(epi == PG_EPI_F32 || epi == PG_EPI_F32_FIN || epi == PG_EPI_F32_ADD || epi == PG_EPI_FX_ADD);
  if (epi == PG_EPI_BF16_GELU_MUL) PG_REQUIRE(N % 32 == 0);
  if (epi == PG_EPI_F32_POS) PG_REQUIRE(aux != nullptr && aux_rows > 0 && bias != nullptr);
  if (epi == PG_EPI_BF16_VT) PG_REQUIRE(aux_out != nullptr && aux_n % 4 == 0);
  if (M <= 16) PG_REQUIRE(K % 64 == 0);
  else PG_REQUIRE(K % TBK == 0 && (f.pro_mode == 0 || f.pro_mode == 5) && epi != PG_EPI_F32_FIN);
  const bf16_t* a = (const bf16_t*)A;
  const bf16_t* w = (const bf16_t*)W;
  if (fp8 && frag) {
    // fp8 weight-streaming GEMV (M <= 32): fp8 fragment-packed W (weights.frag_pack8), row-major e4m3 x
    PG_REQUIRE(M <= 32 && (f.pro_mode == 0 || f.pro_mode == 5) && (f.a_scale || f.pro_mode == 5 || f.mx_in) && f.w_scale &&
               K % 128 == 0 && N % 16 == 0 && ldw == K && lda >= K && (lda % 16 == 0 || f.pro_mode == 5) &&
               ((uintptr_t)A & 15) == 0 && ((uintptr_t)W & 15) == 0 && epi != PG_EPI_F32_FIN);
    const int rc = pg_dispatch_gemv8(epi, (const uint8_t*)A, lda, (const uint8_t*)W, K, ksplit, e, stream);
    if (rc) return rc;
    PG_LAUNCH_CHECK();
    return 0;
  }
  if (fp8) {
    // fp8 e4m3 operands, tile GEMMs only; the kernels see byte pairs, so K / lda / ldw are halved
    PG_REQUIRE(!frag && M > 16 && f.pro_mode == 0 && (f.a_scale || f.mx_in) && f.w_scale && K % 128 == 0 && lda % 16 == 0 &&
               ldw % 16 == 0 && ((uintptr_t)A & 15) == 0 && ((uintptr_t)W & 15) == 0);
    const int rc = pg_dispatch_tile(epi, false, true, a, lda / 2, w, ldw / 2, K / 2, ksplit, e, stream, false, n64);
    if (rc) return rc;
    PG_LAUNCH_CHECK();
    return 0;
  }
  // M <= 16 -> the weight-streaming GEMV, else the tile GEMM; PG_W_FRAG only for the Gemma epilogues (the
  // launchers run the row-major form of the others)
  const int rc = M <= 16 ? pg_dispatch_gemv(epi, frag, a, lda, w, ldw, K, ksplit, e, stream)
                         : pg_dispatch_tile(epi, frag, false, a, lda, w, ldw, K, ksplit, e, stream, m1, n64);
  if (rc) return rc;
  PG_LAUNCH_CHECK();
  return 0;
}

extern "C" int pg_gemm(const void* A, int lda, const void* W, int ldw, const float* bias, void* C, int ldc,
                       int M, int N, int K, int epi, int ksplit, const float* aux, int aux_rows, void* aux_out,
                       int aux_ld, int aux_n, hipStream_t stream) {
  return gemm_impl(A, lda, W, ldw, bias, C, ldc, M, N, K, epi, ksplit, aux, aux_rows, aux_out, aux_ld, aux_n,
                   nullptr, stream);
}

extern "C" int pg_gemm_fused(const void* A, int lda, const void* W, int ldw, const float* bias, void* C, int ldc,
                             int M, int N, int K, int epi, int ksplit, const PgFusedArgs* fused, hipStream_t stream) {
  return gemm_impl(A, lda, W, ldw, bias, C, ldc, M, N, K, epi, ksplit, nullptr, 0, nullptr, 0, 0, fused, stream);
}

