/* Host-side check of the C-ABI boundary (include/pghip.h) under AddressSanitizer + UndefinedBehaviorSanitizer.
 *
 * Built by tests/asan/asan_build.py from the csrc/ sources with the sanitizers on the host side only (the code a binding
 * calls; the device code is never run here) and run by tests/test_asan_host.py on a GPU box.  Every call below is
 * one the library must reject at the boundary -- a null operand, an empty or inconsistent shape, a size whose byte
 * count would overflow -- returning hipErrorInvalidValue (1) before any HIP call, or a pure host function
 * (pg_abi_version, pg_source_hash, the exchange-buffer sizes).  A rejected call that reached the runtime instead
 * would return hipErrorNoDevice (or crash here); a host overflow, division by zero or out-of-bounds write is reported
 * by the sanitizers and fails the run.
 */
#include <stdio.h>
#include <string.h>

#include "pghip.h"

static int fails = 0;
#define EXPECT(call, want)                                                                   \
  do {                                                                                       \
    int got_ = (call);                                                                       \
    if (got_ != (want)) {                                                                    \
      fprintf(stderr, "FAIL line %d: %s returned %d, expected %d\n", __LINE__, #call, got_,  \
              (int)(want));                                                                  \
      ++fails;                                                                               \
    }                                                                                        \
  } while (0)
#define REJECT(call) EXPECT(call, 1)

int main(void) {
  /* any non-null "device" pointer: never dereferenced on a rejection path */
  static float dummy[64] __attribute__((aligned(16)));
  void* d = dummy;
  float* f = dummy;
  int* ip = (int*)dummy;
  int64_t* lp = (int64_t*)dummy;
  hipStream_t s = NULL;

  /* ---- pure host functions */
  EXPECT(pg_abi_version(), 13);
  {
    char buf[200];
    memset(buf, 'x', sizeof buf);
    REJECT(pg_source_hash(buf, 0)); /* nothing written */
    if (buf[0] != 'x') { fprintf(stderr, "FAIL: pg_source_hash wrote into a 0-byte buffer\n"); ++fails; }
    REJECT(pg_source_hash(buf, 1));
    if (buf[0] != 0) { fprintf(stderr, "FAIL: pg_source_hash(n=1) did not terminate\n"); ++fails; }
    REJECT(pg_source_hash(buf, 8));
    if (strlen(buf) != 7) { fprintf(stderr, "FAIL: pg_source_hash(n=8) length %zu\n", strlen(buf)); ++fails; }
    REJECT(pg_source_hash(NULL, 65));
    EXPECT(pg_source_hash(buf, (int)sizeof buf), 0);
    if (strlen(buf) != 64) { fprintf(stderr, "FAIL: source hash length %zu\n", strlen(buf)); ++fails; }
    printf("source hash %s\n", buf);
  }
  {
    long bytes = -1, bytes2 = -1;
    EXPECT(pg_xgmi_buffer_bytes(8, 1L << 20, &bytes), 0);
    if (bytes != 4096 + 2L * 8 * (1L << 20) * 4) { fprintf(stderr, "FAIL: xgmi bytes %ld\n", bytes); ++fails; }
    EXPECT(pg_xgmi_rs_buffer_bytes(8, 1L << 20, &bytes2), 0);
    if (bytes2 <= 0) { fprintf(stderr, "FAIL: rs bytes %ld\n", bytes2); ++fails; }
    REJECT(pg_xgmi_buffer_bytes(0, 1024, &bytes));
    REJECT(pg_xgmi_buffer_bytes(9, 1024, &bytes));
    REJECT(pg_xgmi_buffer_bytes(2, 1022, &bytes));
    REJECT(pg_xgmi_buffer_bytes(2, 1024, NULL));
    REJECT(pg_xgmi_buffer_bytes(8, 0x7ffffffffffffffcL, &bytes)); /* would overflow a long */
    REJECT(pg_xgmi_rs_buffer_bytes(8, 0x7ffffffffffffffcL, &bytes));
    REJECT(pg_xgmi_rs_buffer_bytes(-1, 1024, &bytes));
    REJECT(pg_xgmi_alloc(0, (void**)&d));
    REJECT(pg_xgmi_alloc(1024, NULL));
    REJECT(pg_xgmi_ipc_handle(NULL, d));
    REJECT(pg_xgmi_ipc_open(NULL, (void**)&d));
  }

  /* ---- GEMM */
  REJECT(pg_gemm(d, 64, d, 64, NULL, d, 64, 0, 64, 64, PG_EPI_BF16, 1, NULL, 0, NULL, 0, 0, s));     /* M = 0 */
  REJECT(pg_gemm(d, 64, d, 64, NULL, d, 64, 32, 64, 48, PG_EPI_BF16, 1, NULL, 0, NULL, 0, 0, s));    /* K % 32 */
  REJECT(pg_gemm(d, 64, d, 64, NULL, d, 64, 32, 62, 64, PG_EPI_BF16, 1, NULL, 0, NULL, 0, 0, s));    /* N % 4 */
  REJECT(pg_gemm(d, 64, NULL, 64, NULL, d, 64, 32, 64, 64, PG_EPI_BF16, 1, NULL, 0, NULL, 0, 0, s)); /* no W */
  REJECT(pg_gemm(d, 64, d, 64, NULL, NULL, 64, 32, 64, 64, PG_EPI_BF16, 1, NULL, 0, NULL, 0, 0, s)); /* no C */
  REJECT(pg_gemm(NULL, 64, d, 64, NULL, d, 64, 32, 64, 64, PG_EPI_BF16, 1, NULL, 0, NULL, 0, 0, s)); /* no A */
  REJECT(pg_gemm(d, 64, d, 64, NULL, d, 64, 32, 64, 64, PG_EPI_F32_POS, 1, NULL, 0, NULL, 0, 0, s)); /* no aux */
  REJECT(pg_gemm(d, 64, d, 64, NULL, d, 64, 32, 64, 64, PG_EPI_BF16, 2, NULL, 0, NULL, 0, 0, s));    /* split bf16 */
  REJECT(pg_gemm(d, 64, d, 64, NULL, d, 64, 32, 64, 64, 0x7F, 1, NULL, 0, NULL, 0, 0, s));           /* epilogue */
  REJECT(pg_gemm(d, 64, d, 64, NULL, d, 64, 32, 64, 64, PG_EPI_BF16 | 0x1000, 1, NULL, 0, NULL, 0, 0, s));
  REJECT(pg_gemm(d, 64, d, 64, NULL, d, 64, 8, 64, 64, PG_EPI_F32_RES, 1, NULL, 0, NULL, 0, 0, s));  /* RES at M<=16 */
  {
    PgFusedArgs fa;
    memset(&fa, 0, sizeof fa);
    fa.pro_mode = 7;
    REJECT(pg_gemm_fused(d, 64, d, 64, NULL, d, 64, 4, 64, 64, PG_EPI_F32, 1, &fa, s));              /* pro_mode */
    fa.pro_mode = 1;                                                                                     /* no norm_w */
    REJECT(pg_gemm_fused(d, 64, d, 64, NULL, d, 64, 4, 64, 64, PG_EPI_F32, 1, &fa, s));
    fa.pro_mode = 0;
    REJECT(pg_gemm_fused(d, 64, d, 64, NULL, d, 64, 4, 64, 64, PG_EPI_QKV_ROPE, 1, &fa, s));         /* no tables */
    REJECT(pg_gemm_fused(d, 64, d, 64, NULL, d, 64, 4, 64, 64, PG_EPI_F32_FIN, 1, &fa, s));          /* no tickets */
    REJECT(pg_gemm_fused(d, 64, d, 64, NULL, d, 64, 64, 64, 64, PG_EPI_BF16 | PG_FP8, 1, &fa, s));   /* no scales */
    REJECT(pg_gemm_finalize(NULL, 2, d, 64, 32, 64, PG_EPI_BF16, NULL, 0, 0, &fa, s));
    REJECT(pg_gemm_finalize(f, 2, NULL, 64, 32, 64, PG_EPI_BF16, NULL, 0, 0, &fa, s));
    REJECT(pg_gemm_finalize(f, 0, d, 64, 32, 64, PG_EPI_BF16, NULL, 0, 0, &fa, s));
  }

  /* ---- attention */
  REJECT(pg_attention(NULL, 256, d, 256, d, 0, 0, 256, d, 0, 0, 64, NULL, 0, 0, 1, 64, 64, NULL, 1, 1, 256, 0.0625f,
                      0, 0, NULL, NULL, 0, NULL, NULL, s));                                           /* no q */
  REJECT(pg_attention(d, 256, NULL, 256, d, 0, 0, 256, d, 0, 0, 64, NULL, 0, 0, 1, 64, 64, NULL, 1, 1, 256, 0.0625f,
                      0, 0, NULL, NULL, 0, NULL, NULL, s));                                           /* no o */
  REJECT(pg_attention(d, 256, d, 256, d, 0, 0, 256, d, 0, 0, 64, NULL, 0, 0, 1, 64, 64, NULL, 8, 0, 256, 0.0625f,
                      0, 0, NULL, NULL, 0, NULL, NULL, s));                                           /* Hkv = 0 */
  REJECT(pg_attention(d, 256, d, 256, d, 0, 0, 256, d, 0, 0, 64, NULL, 0, 0, 1, 64, 64, NULL, 8, 3, 256, 0.0625f,
                      0, 0, NULL, NULL, 0, NULL, NULL, s));                                           /* Hq % Hkv */
  REJECT(pg_attention(d, 256, d, 256, d, 0, 0, 256, d, 0, 0, 64, NULL, 0, 0, 1, 1, 64, NULL, 8, 1, 256, 0.0625f,
                      256, 4, NULL, NULL, 64, d, d, s));                                              /* no partials */
  REJECT(pg_attn_combine(f, f, 1, 8, 0, 256, 4, d, 2048, s));                                       /* Hkv = 0 */
  REJECT(pg_attn_combine(NULL, f, 1, 8, 1, 256, 4, d, 2048, s));
  REJECT(pg_attn_combine(f, f, 1, 8, 1, 256, 0, d, 2048, s));                                       /* nsplit = 0 */
  REJECT(pg_attn_decode(NULL, 2048, d, 2048, d, d, 4, 0, ip, 8, 1, 256, 0.0625f, 256, 2, 4, 1, f, f, ip, NULL, NULL,
                        0, s));                                                                        /* no q */
  REJECT(pg_attn_decode(d, 2048, d, 2048, d, d, 4, 0, ip, 8, 0, 256, 0.0625f, 256, 2, 4, 1, f, f, ip, NULL, NULL, 0,
                        s));                                                                           /* Hkv = 0 */
  REJECT(pg_attn_decode(d, 2048, d, 2048, d, d, 4, 0, ip, 8, 1, 64, 0.0625f, 256, 2, 4, 1, f, f, ip, NULL, NULL, 0,
                        s));                                                                           /* D = 64 */
  REJECT(pg_attn_probs(NULL, 256, d, 0, 0, 256, NULL, 0, 0, 1, 64, 64, 8, 1, 256, 0.0625f, 1, f, s));
  REJECT(pg_attn_probs(d, 256, d, 0, 0, 256, NULL, 0, 0, 1, 64, 64, 8, 0, 256, 0.0625f, 1, f, s));

  /* ---- small ops */
  REJECT(pg_rope_kv_write(d, 2560, ip, 16, 16, 8, 1, 256, f, f, NULL, d, 64, 0, NULL, s));          /* no K cache */
  REJECT(pg_rope_kv_write(d, 2560, NULL, 16, 16, 8, 1, 256, f, f, d, d, 64, 0, NULL, s));          /* no positions */
  REJECT(pg_rope_kv_write(d, 2560, ip, 16, 0, 8, 1, 256, f, f, d, d, 64, 0, NULL, s));             /* L = 0 */
  REJECT(pg_patch_im2col(f, 1, 3, 224, 224, 0, d, 588, s));                                         /* patch 0 */
  REJECT(pg_patch_im2col(NULL, 1, 3, 224, 224, 14, d, 588, s));
  REJECT(pg_patch_im2col(f, 1, 3, 224, 224, 14, d, 500, s));                                        /* ldk short */
  REJECT(pg_image_rank(NULL, 16, 257152, ip, s));
  REJECT(pg_image_rank(lp, 0, 257152, ip, s));
  REJECT(pg_embed_merge(lp, ip, 16, NULL, 1024, f, 256, 2048, 257152, 0, 1.f, 45.25f, f, s));     /* no table */
  REJECT(pg_embed_merge(lp, ip, 16, d, 1024, NULL, 256, 2048, 257152, 0, 1.f, 45.25f, f, s));     /* no features */
  REJECT(pg_embed_merge(lp, ip, 16, d, 1024, f, 256, 2046, 257152, 0, 1.f, 45.25f, f, s));        /* H % 4 */
  REJECT(pg_argmax(NULL, 1024, 1, 1024, d, lp, NULL, 0, NULL, NULL, NULL, s));
  REJECT(pg_argmax(f, 1024, 1, 1024, NULL, lp, NULL, 0, NULL, NULL, NULL, s));
  REJECT(pg_argmax(f, 1024, 1, 1024, d, NULL, NULL, 0, NULL, NULL, NULL, s));
  REJECT(pg_argmax(f, 1022, 1, 1024, d, lp, NULL, 0, NULL, NULL, NULL, s));                         /* ld % 4 */
  REJECT(pg_argmax(f, 1024, 1, 1024, d, lp, lp, 0, ip, ip, ip, s));                                 /* hist rows */
  REJECT(pg_argmax_embed(f, 1024, 1, 1024, d, lp, NULL, 0, NULL, NULL, NULL, NULL, 1024, NULL, 0, 2048, 257152, 0,
                         1.f, 45.25f, f, s));                                                          /* no table */
  REJECT(pg_argmax_embed(f, 1024, 100000, 1024, d, lp, NULL, 0, NULL, NULL, NULL, d, 1024, NULL, 0, 2048, 257152, 0,
                         1.f, 45.25f, f, s));                                                          /* B too big */
  REJECT(pg_argmax_pairs(f, 1024, 1, 1024, (1 << 24), d, f, s));                                    /* offset */
  REJECT(pg_argmax_pairs(f, 1024, 1, 1024, 0, d, NULL, s));
  REJECT(pg_argmax_merge(f, 0, 1, lp, NULL, 0, NULL, NULL, NULL, s));                               /* world 0 */
  REJECT(pg_argmax_merge(f, 2, 1, NULL, NULL, 0, NULL, NULL, NULL, s));
  REJECT(pg_topp_sample(f, 1024, 1, 1024, 0.f, 0.9f, f, lp, lp, 4, ip, ip, ip, NULL, s));         /* T = 0 */
  REJECT(pg_topp_sample(f, 1024, 1, 1024, 1.f, 0.9f, NULL, lp, lp, 4, ip, ip, ip, NULL, s));      /* no uniforms */
  REJECT(pg_synth_fill(NULL, 1024, 1u, 0.02f, 0.f, 0, s));
  REJECT(pg_synth_fill(d, 0x100000000L, 1u, 0.02f, 0.f, 0, s));                                    /* > 2^32 */
  REJECT(pg_synth_fill(d, 1024, 1u, 0.02f, 0.f, 2, s));                                            /* kind */
  REJECT(pg_quant_fp8(d, 2048, 16, 2044, d, 2048, f, s));                                          /* K % 8 */
  REJECT(pg_quant_fp8(NULL, 2048, 16, 2048, d, 2048, f, s));
  REJECT(pg_image_preprocess(NULL, 224, 224, 224, NULL, NULL, 0, NULL, NULL, 0, 0, 224, f, NULL, f, s));
  REJECT(pg_image_preprocess((const uint8_t*)d, 300, 200, 224, NULL, NULL, 0, NULL, NULL, 0, 0, 224, f, NULL, f,
                             s));                                                                      /* no tables */

  /* ---- norms */
  REJECT(pg_norm_residual(NULL, NULL, 0, 16, f, f, d, 1152, NULL, NULL, 16, 1152, 0, 1e-6f, 0, s));  /* no resid */
  REJECT(pg_norm_residual(f, NULL, 0, 16, NULL, f, d, 1152, NULL, NULL, 16, 1152, 0, 1e-6f, 0, s)); /* no w */
  REJECT(pg_norm_residual(f, NULL, 0, 16, f, NULL, d, 1152, NULL, NULL, 16, 1152, 0, 1e-6f, 0, s)); /* LN b */
  REJECT(pg_norm_residual(f, NULL, 2, 16, f, f, d, 1152, NULL, NULL, 16, 1152, 0, 1e-6f, 0, s));    /* partials */
  REJECT(pg_norm_residual(f, NULL, 0, 16, f, f, d, 1152, NULL, NULL, 16, 1150, 0, 1e-6f, 0, s));    /* H % 4 */
  REJECT(pg_norm_residual_fp8(f, NULL, 0, 16, f, NULL, d, 2048, NULL, NULL, 16, 2048, 1, 1e-6f, 0, s)); /* scale */
  REJECT(pg_norm_residual_mx(f, NULL, 0, 16, f, d, 2048, d, f, 2, 16, 2000, 0, s));                  /* H % 1024 */
  REJECT(pg_norm_residual_mx(NULL, NULL, 0, 16, f, d, 2048, d, f, 2, 16, 2048, 0, s));

  /* ---- xGMI exchange (argument checks only: no buffer is mapped) */
  {
    void* peers[8] = {d, d, NULL, NULL, NULL, NULL, NULL, NULL};
    unsigned* ep = (unsigned*)dummy;
    REJECT(pg_allreduce_xgmi(f, 1024, 0, 2, NULL, 4096, ep, ip, s));                                 /* no peers */
    REJECT(pg_allreduce_xgmi(f, 1024, 2, 2, peers, 4096, ep, ip, s));                                /* rank */
    REJECT(pg_allreduce_xgmi(f, 8192, 0, 2, peers, 4096, ep, ip, s));                                /* n > cap */
    REJECT(pg_allreduce_xgmi(f, 1024, 0, 3, peers, 4096, ep, ip, s));                                /* null peer */
    REJECT(pg_allreduce_xgmi_slabs(f, 1024, 65, 1024, 0, 2, peers, 4096, ep, ip, s));               /* nslab */
    REJECT(pg_allgather_xgmi(f, 1024, f, 0, 2, peers, 4096, ep, ip, s));                             /* in == out */
    REJECT(pg_allreduce_xgmi_rs(f, 1024, 1, 0, 0, 2, peers, 4096, 0, ep, ip, s));                   /* nwg 0 */
    REJECT(pg_allreduce_xgmi_rs(f, 1024, 1, 0, 0, 2, peers, 4096, 257, ep, ip, s));                 /* nwg 257 */
  }

  if (fails) {
    fprintf(stderr, "%d boundary checks failed\n", fails);
    return 1;
  }
  printf("all boundary checks passed\n");
  return 0;
}
