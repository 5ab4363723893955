// Byte-moving / small kernels around the GEMMs and attention:
//   pg_patch_im2col   : Conv2d(k=s=patch) input as rows (SiglipVisionEmbeddings, modeling_siglip.py:258-263,285)
//   pg_image_rank     : exclusive count of image tokens (masked_scatter order, modeling_paligemma.py:121-122)
//   pg_embed_merge    : token-embedding gather + image-row scatter + pad zeroing + *sqrt(H)
//                       (modeling_paligemma.py:99-128,288; modeling_gemma.py:510-511)
//   pg_rope_kv_write  : RoPE on q (in place) and k, append k / v^T to the static KV cache
//                       (modeling_gemma.py:112-151, KVCache.update :18-57)
//   pg_argmax         : greedy next token, first index on ties (inference.py:68)
//   pg_argmax_embed   : pg_argmax + the next step's input rows (the embed of the next decode step folded in)
//   pg_topp_sample    : temperature softmax + top-p filter + explicit-uniform draw (inference.py:65,90-106)
//   pg_synth_fill     : name-seeded synthetic weights (oracle/synth.py formula, bit-identical)
#include <cstdlib>

#include "common.h"

// ---------------------------------------------------------------- im2col
// pixels f32 [B][C][H][W] -> rows bf16 [B*nh*nw][ldk], column (c*p + kh)*p + kw, zero for col >= C*p*p
__global__ void im2col_kernel(const float* __restrict__ px, int B, int C, int H, int W, int p, int nh, int nw,
                              bf16_t* __restrict__ out, int ldk) {
  const long total = (long)B * nh * nw * ldk;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int col = (int)(i % ldk);
    const long row = i / ldk;
    const int pw = (int)(row % nw);
    const int ph = (int)((row / nw) % nh);
    const int b = (int)(row / ((long)nw * nh));
    float v = 0.f;
    if (col < C * p * p) {
      const int c = col / (p * p), kh = (col / p) % p, kw = col % p;
      v = px[(((long)b * C + c) * H + ph * p + kh) * W + pw * p + kw];
    }
    out[i] = f2bf(v);
  }
}

extern "C" int pg_patch_im2col(const float* px, int B, int C, int H, int W, int p, void* out, int ldk,
                               hipStream_t stream) {
  PG_REQUIRE(px && out && B > 0 && C > 0 && p > 0 && ldk >= C * p * p && H >= p && W >= p);
  const int nh = H / p, nw = W / p;
  const long total = (long)B * nh * nw * ldk;
  const int grid = (int)min((total + 255) / 256, (long)8192);
  hipLaunchKernelGGL(im2col_kernel, dim3(grid), dim3(256), 0, stream, px, B, C, H, W, p, nh, nw, (bf16_t*)out, ldk);
  PG_LAUNCH_CHECK();
  return 0;
}

// ---------------------------------------------------------------- image-token rank (one workgroup)
__global__ __launch_bounds__(1024) void image_rank_kernel(const int64_t* __restrict__ ids, int n, int64_t image_id,
                                                          int* __restrict__ rank) {
  __shared__ int part[1024];
  const int t = threadIdx.x;
  const int per = (n + 1023) / 1024;
  const int s = min(n, t * per), e = min(n, s + per);
  int cnt = 0;
  for (int i = s; i < e; ++i) cnt += ids[i] == image_id;
  part[t] = cnt;
  __syncthreads();
  for (int off = 1; off < 1024; off <<= 1) {   // inclusive Hillis-Steele scan
    int v = t >= off ? part[t - off] : 0;
    __syncthreads();
    part[t] += v;
    __syncthreads();
  }
  int run = part[t] - cnt;
  for (int i = s; i < e; ++i) {
    rank[i] = run;
    run += ids[i] == image_id;
  }
}

extern "C" int pg_image_rank(const int64_t* ids, int n, long image_id, int* rank, hipStream_t stream) {
  PG_REQUIRE(ids && rank && n > 0);
  hipLaunchKernelGGL(image_rank_kernel, dim3(1), dim3(1024), 0, stream, ids, n, (int64_t)image_id, rank);
  PG_LAUNCH_CHECK();
  return 0;
}

// ---------------------------------------------------------------- embedding merge
// out f32 [n][H]: text row -> embed[id] * normalizer; image row -> feat[rank] * img_scale * normalizer;
// pad row -> 0.  rank may be null (then computed by scanning ids[0..row), meant for n <= 64).
// one output row: pad -> zeros, image token -> feat[rank] (zeros past n_feat) * img_scale * normalizer,
// text -> embed[clamp(id)] * normalizer; threads t, t + nt, ... of the caller each write 4 columns at a time
__device__ __forceinline__ void embed_row(float* __restrict__ o, int64_t id, int rk, int t, int nt,
                                          const bf16_t* __restrict__ embed, int V, const float* __restrict__ feat,
                                          int n_feat, int H, int64_t image_id, int64_t pad_id, float img_scale,
                                          float normalizer) {
  if (id == pad_id) {
    for (int c = t * 4; c < H; c += 4 * nt) *(f32x4*)(o + c) = f32x4{0.f, 0.f, 0.f, 0.f};
    return;
  }
  if (id == image_id) {
    const bool ok = rk < n_feat;
    const float* f = feat + (long)(ok ? rk : 0) * H;
    for (int c = t * 4; c < H; c += 4 * nt) {
      f32x4 v = ok ? *(const f32x4*)(f + c) : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int j = 0; j < 4; ++j) v[j] = (v[j] * img_scale) * normalizer;
      *(f32x4*)(o + c) = v;
    }
    return;
  }
  const int64_t tid = id < 0 ? 0 : (id >= V ? V - 1 : id);
  const bf16_t* e = embed + tid * (long)H;
  for (int c = t * 4; c < H; c += 4 * nt) {
    const u32x2 w = *(const u32x2*)(e + c);
    f32x4 v;
    v[0] = bf2f((bf16_t)(w[0] & 0xFFFF)) * normalizer;
    v[1] = bf2f((bf16_t)(w[0] >> 16)) * normalizer;
    v[2] = bf2f((bf16_t)(w[1] & 0xFFFF)) * normalizer;
    v[3] = bf2f((bf16_t)(w[1] >> 16)) * normalizer;
    *(f32x4*)(o + c) = v;
  }
}

__global__ __launch_bounds__(256) void embed_merge_kernel(const int64_t* __restrict__ ids, const int* __restrict__ rank,
                                                          int n, const bf16_t* __restrict__ embed, int V,
                                                          const float* __restrict__ feat, int n_feat, int H,
                                                          int64_t image_id, int64_t pad_id, float img_scale,
                                                          float normalizer, float* __restrict__ out) {
  const int row = blockIdx.x;
  const int64_t id = ids[row];
  int rk = 0;
  if (id == image_id) {
    if (rank) {
      rk = rank[row];
    } else {
      for (int i = 0; i < row; ++i) rk += ids[i] == image_id;
    }
  }
  embed_row(out + (long)row * H, id, rk, threadIdx.x, blockDim.x, embed, V, feat, n_feat, H, image_id, pad_id,
            img_scale, normalizer);
}

extern "C" int pg_embed_merge(const int64_t* ids, const int* rank, int n, const void* embed, int V, const float* feat,
                              int n_feat, int H, long image_id, long pad_id, float img_scale, float normalizer,
                              float* out, hipStream_t stream) {
  PG_REQUIRE(ids && embed && out && n > 0 && V > 0 && H > 0 && H % 4 == 0 && (n_feat == 0 || feat));
  hipLaunchKernelGGL(embed_merge_kernel, dim3(n), dim3(256), 0, stream, ids, rank, n, (const bf16_t*)embed, V, feat,
                     n_feat, H, (int64_t)image_id, (int64_t)pad_id, img_scale, normalizer, out);
  PG_LAUNCH_CHECK();
  return 0;
}

// ---------------------------------------------------------------- RoPE + KV-cache append
// qkv bf16 [T][ldq]: q = cols [0, Hq*D), k = [Hq*D, (Hq+Hkv)*D), v = next Hkv*D.  Row t = b*L + i.
// pos int32 [T] (rotary position).  Cache slot of row t = slot_base (+ *slot_dev) + i.
// kc bf16 [B][Smax][Hkv*D] (roped k);  vtc bf16 [B][Hkv*D][Smax] (v transposed).
// cos/sin tables f32 [P][D/2]: cos(inv_freq[j] * pos).
__global__ __launch_bounds__(256) void rope_kv_kernel(bf16_t* __restrict__ qkv, int ldq, const int* __restrict__ pos,
                                                      int L, int Hq, int Hkv, int D, const float* __restrict__ cosT,
                                                      const float* __restrict__ sinT, bf16_t* __restrict__ kc,
                                                      bf16_t* __restrict__ vtc, int Smax, int slot_base,
                                                      const int* __restrict__ slot_dev) {
  const int t = blockIdx.x;
  const int b = t / L, i = t % L;
  const int slot = slot_base + (slot_dev ? *slot_dev : 0) + i;
  const int p = pos[t];
  const int half = D / 2;
  const float* cs = cosT + (long)p * half;
  const float* sn = sinT + (long)p * half;
  bf16_t* row = qkv + (long)t * ldq;
  const int KV = Hkv * D;
  // q heads (in place) and k heads (to the cache): pairs (j, j + D/2)
  for (int idx = threadIdx.x; idx < (Hq + Hkv) * half; idx += blockDim.x) {
    const int h = idx / half, j = idx % half;
    bf16_t* x = row + h * D;
    const float x1 = bf2f(x[j]), x2 = bf2f(x[j + half]);
    const float c = cs[j], s = sn[j];
    const float y1 = x1 * c - x2 * s;   // q*cos + rotate_half(q)*sin, rotate_half = cat(-x2, x1)
    const float y2 = x2 * c + x1 * s;
    if (h < Hq) {
      x[j] = f2bf(y1);
      x[j + half] = f2bf(y2);
    } else {
      const int hk = h - Hq;
      bf16_t* kr = kc + ((long)b * Smax + slot) * KV + hk * D;
      kr[j] = f2bf(y1);
      kr[j + half] = f2bf(y2);
    }
  }
  const bf16_t* v = row + (Hq + Hkv) * D;
  for (int cidx = threadIdx.x; cidx < KV; cidx += blockDim.x)
    vtc[((long)b * KV + cidx) * Smax + slot] = v[cidx];
}

extern "C" int pg_rope_kv_write(void* qkv, int ldq, const int* pos, int T, int L, int Hq, int Hkv, int D,
                                const float* cosT, const float* sinT, void* kc, void* vtc, int Smax, int slot_base,
                                const int* slot_dev, hipStream_t stream) {
  PG_REQUIRE(qkv && pos && cosT && sinT && kc && vtc && T > 0 && L > 0 && T % L == 0 && D % 2 == 0);
  hipLaunchKernelGGL(rope_kv_kernel, dim3(T), dim3(256), 0, stream, (bf16_t*)qkv, ldq, pos, L, Hq, Hkv, D, cosT, sinT,
                     (bf16_t*)kc, (bf16_t*)vtc, Smax, slot_base, slot_dev);
  PG_LAUNCH_CHECK();
  return 0;
}

// ---------------------------------------------------------------- argmax (two passes)
#define AM_CHUNKS 64
__device__ __forceinline__ void am_better(float& bv, int& bi, float v, int i) {
  if (v > bv || (v == bv && i < bi)) { bv = v; bi = i; }
}
__device__ __forceinline__ void am_block(float& bv, int& bi, float* sv, int* si) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    float ov = __shfl_xor(bv, o, 64);
    int oi = __shfl_xor(bi, o, 64);
    am_better(bv, bi, ov, oi);
  }
  if (lane == 0) { sv[w] = bv; si[w] = bi; }
  __syncthreads();
  bv = sv[0]; bi = si[0];
  for (int i = 1; i < (int)(blockDim.x >> 6); ++i) am_better(bv, bi, sv[i], si[i]);
}

__global__ __launch_bounds__(256) void argmax_partial_kernel(const float* __restrict__ x, long ld, int V,
                                                             float* __restrict__ pv, int* __restrict__ pi) {
  __shared__ float sv[4];
  __shared__ int si[4];
  const int b = blockIdx.y, ch = blockIdx.x;
  const int per = ((V + AM_CHUNKS - 1) / AM_CHUNKS + 3) & ~3;
  const int s = ch * per, e = min(V, s + per);
  const float* row = x + (long)b * ld;
  float bv = -INFINITY;
  int bi = 0x7FFFFFFF;
  for (int i = s + threadIdx.x * 4; i < e; i += 1024) {
    if (i + 3 < e) {
      const f32x4 v = *(const f32x4*)(row + i);
#pragma unroll
      for (int j = 0; j < 4; ++j) am_better(bv, bi, v[j], i + j);
    } else {
      for (int j = 0; j < 4 && i + j < e; ++j) am_better(bv, bi, row[i + j], i + j);
    }
  }
  am_block(bv, bi, sv, si);
  if (threadIdx.x == 0) { pv[b * AM_CHUNKS + ch] = bv; pi[b * AM_CHUNKS + ch] = bi; }
}

// final pass; also advances the decode state when asked:
//   out_ids[b] = argmax ; hist[(*step) * B + b] = argmax ; pos[b] += 1 ; (*kv_len) += 1 ; (*step) += 1
__global__ __launch_bounds__(1024) void argmax_final_kernel(const float* __restrict__ pv, const int* __restrict__ pi,
                                                            int B, int64_t* __restrict__ out_ids, int64_t* __restrict__ hist,
                                                            int hist_rows, int* __restrict__ step, int* __restrict__ pos,
                                                            int* __restrict__ kv_len) {
  // one wave per row (rows strided over the block's waves): the rows' chunk winners load in parallel
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
  const int st = step ? *step : 0;
  __syncthreads();                             // every wave has read *step before thread 0 advances it
  for (int b = wave; b < B; b += nw) {
    float bv = pv[b * AM_CHUNKS + lane];
    int bi = pi[b * AM_CHUNKS + lane];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      float ov = __shfl_xor(bv, o, 64);
      int oi = __shfl_xor(bi, o, 64);
      am_better(bv, bi, ov, oi);
    }
    if (lane == 0) {
      out_ids[b] = bi;
      if (hist && st < hist_rows) hist[(long)st * B + b] = bi;   // a step past the history is not recorded
      if (pos) pos[b] += 1;
    }
  }
  if (threadIdx.x == 0) {
    if (kv_len) *kv_len += 1;
    if (step) *step = st + 1;
  }
}

// argmax_final_kernel, then the next decode step's input rows: res[b] = embedding of the winner of row b,
// exactly as pg_embed_merge(out_ids, rank = nullptr, ...) would write them (image-token rank = count of
// earlier rows whose winner is the image token).  Saves the step's leading embed launch.
#define AM_EMB_MAX_B 1024
struct AmEmbArgs {
  const bf16_t* embed;
  int V, n_feat, H;
  const float* feat;
  int64_t image_id, pad_id;
  float img_scale, normalizer;
  float* res;
};
__global__ __launch_bounds__(1024) void argmax_final_embed_kernel(const float* __restrict__ pv, const int* __restrict__ pi,
                                                                  int B, int64_t* __restrict__ out_ids,
                                                                  int64_t* __restrict__ hist, int hist_rows,
                                                                  int* __restrict__ step, int* __restrict__ pos,
                                                                  int* __restrict__ kv_len, AmEmbArgs ea) {
  __shared__ int win[AM_EMB_MAX_B];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
  const int st = step ? *step : 0;
  for (int b = wave; b < B; b += nw) {
    float bv = pv[b * AM_CHUNKS + lane];
    int bi = pi[b * AM_CHUNKS + lane];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      float ov = __shfl_xor(bv, o, 64);
      int oi = __shfl_xor(bi, o, 64);
      am_better(bv, bi, ov, oi);
    }
    if (lane == 0) {
      win[b] = bi;
      out_ids[b] = bi;
      if (hist && st < hist_rows) hist[(long)st * B + b] = bi;
      if (pos) pos[b] += 1;
    }
  }
  __syncthreads();                             // every wave has read *step and every winner is in LDS
  if (threadIdx.x == 0) {
    if (kv_len) *kv_len += 1;
    if (step) *step = st + 1;
  }
  for (int b = wave; b < B; b += nw) {
    const int64_t id = win[b];
    int rk = 0;
    if (id == ea.image_id)
      for (int i = 0; i < b; ++i) rk += win[i] == ea.image_id;
    embed_row(ea.res + (long)b * ea.H, id, rk, lane, 64, ea.embed, ea.V, ea.feat, ea.n_feat, ea.H, ea.image_id,
              ea.pad_id, ea.img_scale, ea.normalizer);
  }
}

static inline int am_waves(int B) { return B < 1 ? 1 : (B > 16 ? 16 : B); }

// vocabulary-parallel greedy (tensor parallelism): the local (max, first index + vocab_offset) per row,
// as float pairs [B][2] to be all-gathered; then pg_argmax_merge picks the global winner.
__global__ __launch_bounds__(1024) void argmax_pairs_kernel(const float* __restrict__ pv, const int* __restrict__ pi,
                                                            int B, int vocab_offset, float* __restrict__ pairs) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
  for (int b = wave; b < B; b += nw) {
    float bv = pv[b * AM_CHUNKS + lane];
    int bi = pi[b * AM_CHUNKS + lane];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      float ov = __shfl_xor(bv, o, 64);
      int oi = __shfl_xor(bi, o, 64);
      am_better(bv, bi, ov, oi);
    }
    if (lane == 0) { pairs[2 * b] = bv; pairs[2 * b + 1] = (float)(bi + vocab_offset); }
  }
}

// pairs [world][B][2] (rank-major, ascending vocabulary ranges): max value, lowest global index on ties
__global__ void argmax_merge_kernel(const float* __restrict__ pairs, int world, int B, int64_t* __restrict__ out_ids,
                                    int64_t* __restrict__ hist, int hist_rows, int* __restrict__ step, int* __restrict__ pos,
                                    int* __restrict__ kv_len) {
  if (threadIdx.x != 0) return;
  const int st = step ? *step : 0;
  for (int b = 0; b < B; ++b) {
    float bv = -INFINITY;
    int bi = 0x7FFFFFFF;
    for (int r = 0; r < world; ++r) am_better(bv, bi, pairs[(r * B + b) * 2], (int)pairs[(r * B + b) * 2 + 1]);
    out_ids[b] = bi;
    if (hist && st < hist_rows) hist[(long)st * B + b] = bi;
    if (pos) pos[b] += 1;
  }
  if (kv_len) *kv_len += 1;
  if (step) *step = st + 1;
}

extern "C" int pg_argmax_pairs(const float* logits, long ld, int B, int V, int vocab_offset, void* workspace,
                               float* pairs, hipStream_t stream) {
  PG_REQUIRE(logits && workspace && pairs && B > 0 && V > 0 && ld % 4 == 0 && vocab_offset >= 0 &&
             vocab_offset + V < (1 << 24));
  float* pv = (float*)workspace;
  int* pi = (int*)(pv + B * AM_CHUNKS);
  hipLaunchKernelGGL(argmax_partial_kernel, dim3(AM_CHUNKS, B), dim3(256), 0, stream, logits, ld, V, pv, pi);
  hipLaunchKernelGGL(argmax_pairs_kernel, dim3(1), dim3(64 * am_waves(B)), 0, stream, pv, pi, B, vocab_offset, pairs);
  PG_LAUNCH_CHECK();
  return 0;
}

extern "C" int pg_argmax_merge(const float* pairs, int world, int B, int64_t* out_ids, int64_t* hist, int hist_rows,
                               int* step, int* pos, int* kv_len, hipStream_t stream) {
  PG_REQUIRE(pairs && out_ids && world > 0 && B > 0 && (hist == nullptr || hist_rows > 0));
  hipLaunchKernelGGL(argmax_merge_kernel, dim3(1), dim3(64), 0, stream, pairs, world, B, out_ids, hist, hist_rows,
                     step, pos, kv_len);
  PG_LAUNCH_CHECK();
  return 0;
}

// workspace: >= B * AM_CHUNKS * 8 bytes
extern "C" int pg_argmax(const float* logits, long ld, int B, int V, void* workspace, int64_t* out_ids,
                         int64_t* hist, int hist_rows, int* step, int* pos, int* kv_len, hipStream_t stream) {
  PG_REQUIRE(logits && workspace && out_ids && B > 0 && V > 0 && ld % 4 == 0 && (hist == nullptr || hist_rows > 0));
  float* pv = (float*)workspace;
  int* pi = (int*)(pv + B * AM_CHUNKS);
  hipLaunchKernelGGL(argmax_partial_kernel, dim3(AM_CHUNKS, B), dim3(256), 0, stream, logits, ld, V, pv, pi);
  hipLaunchKernelGGL(argmax_final_kernel, dim3(1), dim3(64 * am_waves(B)), 0, stream, pv, pi, B, out_ids, hist, hist_rows, step, pos,
                     kv_len);
  PG_LAUNCH_CHECK();
  return 0;
}

// pg_argmax + the next step's embedding rows (see argmax_final_embed_kernel); workspace as pg_argmax
extern "C" int pg_argmax_embed(const float* logits, long ld, int B, int V, void* workspace, int64_t* out_ids,
                               int64_t* hist, int hist_rows, int* step, int* pos, int* kv_len, const void* embed,
                               int V_embed, const float* feat, int n_feat, int H, long image_id, long pad_id,
                               float img_scale, float normalizer, float* res, hipStream_t stream) {
  PG_REQUIRE(logits && workspace && out_ids && B > 0 && B <= AM_EMB_MAX_B && V > 0 && ld % 4 == 0 &&
             (hist == nullptr || hist_rows > 0));
  PG_REQUIRE(embed != nullptr && res != nullptr && V_embed > 0 && H > 0 && H % 4 == 0 && (n_feat == 0 || feat));
  float* pv = (float*)workspace;
  int* pi = (int*)(pv + B * AM_CHUNKS);
  const AmEmbArgs ea{(const bf16_t*)embed, V_embed, n_feat, H, feat, (int64_t)image_id, (int64_t)pad_id,
                     img_scale, normalizer, res};
  hipLaunchKernelGGL(argmax_partial_kernel, dim3(AM_CHUNKS, B), dim3(256), 0, stream, logits, ld, V, pv, pi);
  hipLaunchKernelGGL(argmax_final_embed_kernel, dim3(1), dim3(64 * am_waves(B)), 0, stream, pv, pi, B, out_ids, hist,
                     hist_rows, step, pos, kv_len, ea);
  PG_LAUNCH_CHECK();
  return 0;
}

// ---------------------------------------------------------------- top-p sampling (one workgroup per row)
// p_i = softmax(logits / T).  Included set = tokens whose probability mass strictly ranked before them is
// <= top_p, i.e. {e_i >= t0} with t0 the smallest value whose strictly-greater mass F(t0) <= top_p * Z.
// t0 is found by a 4-digit (8-bit) radix select over the float bit patterns of e_i (all positive,
// so bit order == value order), each digit choosing the bucket by mass.  The draw is an inverse CDF
// in vocabulary order over the included, renormalised mass: first i with prefix > u * Z_kept.
__global__ __launch_bounds__(1024) void topp_kernel(const float* __restrict__ logits, long ld, int V, float inv_temp,
                                                    float top_p, const float* __restrict__ uniforms,
                                                    int64_t* __restrict__ out_ids, int64_t* __restrict__ hist, int hist_rows,
                                                    int* __restrict__ step, int* __restrict__ pos, int B,
                                                    int* __restrict__ kv_len, float* __restrict__ probs_out) {
  __shared__ float red[16];
  __shared__ float hist_mass[256];
  __shared__ float scan[1024];
  __shared__ int sel;
  __shared__ float sel_above;
  const int b = blockIdx.x;
  const float* x = logits + (long)b * ld;
  const int tid = threadIdx.x;
  // 1. max of logits/T and the normaliser
  float mx = -INFINITY;
  for (int i = tid; i < V; i += 1024) mx = fmaxf(mx, x[i] * inv_temp);
  mx = wave_max(mx);
  if ((tid & 63) == 0) red[tid >> 6] = mx;
  __syncthreads();
  mx = red[0];
  for (int i = 1; i < 16; ++i) mx = fmaxf(mx, red[i]);
  __syncthreads();
  float z = 0.f;
  for (int i = tid; i < V; i += 1024) z += __expf(x[i] * inv_temp - mx);
  z = block_sum(z, red);
  const float target = top_p * z;
  // 2. radix select of t0 on the bit pattern, most significant byte first
  uint32_t prefix = 0;        // fixed high bits of t0
  float above = 0.f;          // mass strictly above the current prefix range
  for (int digit = 3; digit >= 0; --digit) {
    const int shift = digit * 8;
    const uint32_t hi_mask = digit == 3 ? 0u : (0xFFFFFFFFu << (shift + 8));
    for (int i = tid; i < 256; i += 1024) hist_mass[i] = 0.f;
    __syncthreads();
    for (int i = tid; i < V; i += 1024) {
      const float e = __expf(x[i] * inv_temp - mx);
      const uint32_t u = __float_as_uint(e);
      if ((u & hi_mask) == (prefix & hi_mask)) atomicAdd(&hist_mass[(u >> shift) & 255], e);
    }
    __syncthreads();
    if (tid == 0) {
      // walk buckets from the top: pick the highest bucket whose "mass strictly above it" stays <= target
      // while adding it would not... t0 lies in the lowest bucket k with above + mass(>k) <= target.
      float acc = above;
      int k = 255;
      for (; k >= 0; --k) {
        if (acc + hist_mass[k] > target && hist_mass[k] > 0.f) break;   // t0 inside bucket k
        acc += hist_mass[k];
      }
      if (k < 0) {   // everything fits: t0 is the minimum; keep descending to the lowest non-empty bucket
        acc = above;
        for (k = 0; k < 256 && hist_mass[k] == 0.f; ++k) {}
        for (int j = 255; j > k; --j) acc += hist_mass[j];
      }
      sel = k;
      sel_above = acc;
    }
    __syncthreads();
    prefix |= ((uint32_t)sel) << shift;
    above = sel_above;
    __syncthreads();
  }
  const float t0 = __uint_as_float(prefix);
  // 3. kept mass and the inverse-CDF draw in vocabulary order (contiguous chunk per thread)
  const int per = (V + 1023) / 1024;
  const int s = min(V, tid * per), e = min(V, s + per);
  float mine = 0.f;
  for (int i = s; i < e; ++i) {
    const float v = __expf(x[i] * inv_temp - mx);
    if (v >= t0) mine += v;
  }
  scan[tid] = mine;
  __syncthreads();
  for (int off = 1; off < 1024; off <<= 1) {
    float v = tid >= off ? scan[tid - off] : 0.f;
    __syncthreads();
    scan[tid] += v;
    __syncthreads();
  }
  const float kept = scan[1023];
  if (probs_out) {
    for (int i = s; i < e; ++i) {
      const float v = __expf(x[i] * inv_temp - mx);
      probs_out[(long)b * V + i] = v >= t0 ? v / kept : 0.f;
    }
  }
  // uniforms and hist hold hist_rows steps: a step past them reuses the last row / is not recorded
  const long srow = step ? (long)min(*step, hist_rows - 1) : 0;
  const float u = uniforms[srow * B + b] * kept;
  const float lo = scan[tid] - mine;
  __shared__ int chosen;
  if (tid == 0) chosen = -1;
  __syncthreads();
  if (mine > 0.f && u >= lo && u < scan[tid]) {
    float run = lo;
    int pick = -1, last = -1;
    for (int i = s; i < e; ++i) {
      const float v = __expf(x[i] * inv_temp - mx);
      if (v >= t0) {
        last = i;
        run += v;
        if (run > u) { pick = i; break; }
      }
    }
    atomicMax(&chosen, pick >= 0 ? pick : last);
  }
  __syncthreads();
  if (tid == 0) {
    int c = chosen;
    if (c < 0) {   // u at/after the total (rounding): last kept token
      for (int i = V - 1; i >= 0; --i) if (__expf(x[i] * inv_temp - mx) >= t0) { c = i; break; }
    }
    out_ids[b] = c;
    if (hist && (!step || *step < hist_rows)) hist[srow * B + b] = c;
    if (pos) pos[b] += 1;
  }
}

__global__ void advance_kernel(int* step, int* kv_len) {
  if (kv_len) *kv_len += 1;
  if (step) *step += 1;
}

// uniforms: [steps][B] (indexed by *step when step != null).  probs_out (optional) f32 [B][V]: the filtered,
// renormalised distribution in vocabulary order (for tests).
extern "C" int pg_topp_sample(const float* logits, long ld, int B, int V, float temperature, float top_p,
                              const float* uniforms, int64_t* out_ids, int64_t* hist, int hist_rows, int* step, int* pos,
                              int* kv_len, float* probs_out, hipStream_t stream) {
  PG_REQUIRE(logits && uniforms && out_ids && B > 0 && V > 0 && temperature > 0.f && hist_rows > 0);
  hipLaunchKernelGGL(topp_kernel, dim3(B), dim3(1024), 0, stream, logits, ld, V, 1.0f / temperature, top_p, uniforms,
                     out_ids, hist, hist_rows, step, pos, B, kv_len, probs_out);
  hipLaunchKernelGGL(advance_kernel, dim3(1), dim3(1), 0, stream, step, kv_len);
  PG_LAUNCH_CHECK();
  return 0;
}

// ---------------------------------------------------------------- synthetic weights
__device__ __forceinline__ uint32_t fmix32(uint32_t h) {
  h ^= h >> 16; h *= 0x85EBCA6Bu; h ^= h >> 13; h *= 0xC2B2AE35u; h ^= h >> 16;
  return h;
}
__device__ __forceinline__ uint32_t bf16_rne_bits(float v) {
  const uint32_t u = __float_as_uint(v);
  return (u + 0x7FFFu + ((u >> 16) & 1u)) >> 16;
}
// out_kind 0: bf16, 1: f32 (holding the bf16-rounded value)
__global__ void synth_kernel(void* out, long n, uint32_t seedmix, float a, float mean, int out_kind) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const uint32_t h = fmix32((uint32_t)i * 0x9E3779B1u + seedmix);
    float v = __fmul_rn((float)(h >> 8), 5.9604644775390625e-08f);   // * 2^-24 (exact)
    v = __fsub_rn(__fmul_rn(v, 2.0f), 1.0f);
    v = __fmul_rn(v, a);
    if (mean != 0.0f) v = __fadd_rn(v, mean);
    const uint32_t bits = bf16_rne_bits(v);
    if (out_kind == 0) ((bf16_t*)out)[i] = (bf16_t)bits;
    else ((float*)out)[i] = __uint_as_float(bits << 16);
  }
}

extern "C" int pg_synth_fill(void* out, long n, unsigned int seedmix, float a, float mean, int out_kind,
                             hipStream_t stream) {
  PG_REQUIRE(out && n > 0 && n <= 0xFFFFFFFFl && (out_kind == 0 || out_kind == 1));
  const int grid = (int)min((n + 255) / 256, (long)16384);
  hipLaunchKernelGGL(synth_kernel, dim3(grid), dim3(256), 0, stream, out, n, (uint32_t)seedmix, a, mean, out_kind);
  PG_LAUNCH_CHECK();
  return 0;
}

// ABI 4: the measured-slower decode variants removed (pg_attn_oproj, pg_decode_attn_block, pg_decode_mlp_block,
// pg_decode_mlp_engine, pg_gateup_bank, pg_prefetch, the *_stamps diagnostics) and PgFusedArgs slimmed to the
// fields the default path uses; pg_source_hash added.
extern "C" int pg_abi_version(void) { return 13; }

// sha256 (hex) over the csrc/ sources, include/pghip.h and the compile flags this library was built from
// (pghip/build.py passes it as PG_SOURCE_HASH): the loader compares it with the tree it runs from, so a stale
// prebuilt library cannot pass for the sources next to it.  The marker prefix lets the build read it from the file.
#ifndef PG_SOURCE_HASH
#define PG_SOURCE_HASH "unknown"
#endif
__attribute__((used)) static const char pg_source_hash_str[] = "PGHIP_SOURCE_HASH=" PG_SOURCE_HASH;
extern "C" int pg_source_hash(char* out, int n) {
  const char* h = pg_source_hash_str + 18;
  PG_REQUIRE(n <= 0 || out != nullptr);
  int i = 0;
  for (; h[i] && i + 1 < n; ++i) out[i] = h[i];
  if (n > 0) out[i] = 0;
  return h[i] ? (int)hipErrorInvalidValue : 0;
}

// ---------------------------------------------------------------- image pre-processing (processing_paligemma.py:13-73)
// PIL BICUBIC resize of an RGB uint8 image (Pillow Resample.c, 22-bit fixed point, coefficient tables from
// pghip/image.py) + the reference's rescale/normalise as a float32 lookup table, output CHW float32.
__device__ __forceinline__ uint8_t clip8_22(int acc) {
  const int v = acc >> 22;
  return (uint8_t)(v < 0 ? 0 : (v > 255 ? 255 : v));
}

// pass 1: tmp[r][xx][c] = clip8(2^21 + sum_x src[y0 + r][xmin + x][c] * hk[xx][x])
__global__ __launch_bounds__(256) void resize_h_kernel(const uint8_t* __restrict__ src, int W, int y0, int rows,
                                                       int S, const int* __restrict__ hb, const int* __restrict__ hk,
                                                       int hks, uint8_t* __restrict__ tmp) {
  const long total = (long)rows * S * 3;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int c = (int)(i % 3), xx = (int)((i / 3) % S);
    const long r = i / (3L * S);
    const int xmin = hb[2 * xx], n = hb[2 * xx + 1];
    const int* k = hk + (long)xx * hks;
    const uint8_t* p = src + ((long)(y0 + r) * W + xmin) * 3 + c;
    int acc = 1 << 21;
    for (int x = 0; x < n; ++x) acc += (int)p[3 * x] * k[x];
    tmp[i] = clip8_22(acc);
  }
}

// pass 2: out[c][yy][xx] = lut[clip8(2^21 + sum_y in[ymin - yshift + y][xx][c] * vk[yy][y])]  (vb == null: no
// vertical resize, out = lut[in[yy][xx][c]])
__global__ __launch_bounds__(256) void resize_v_kernel(const uint8_t* __restrict__ in, int Win, int yshift, int S,
                                                       const int* __restrict__ vb, const int* __restrict__ vk,
                                                       int vks, const float* __restrict__ lut,
                                                       float* __restrict__ out) {
  const long total = 3L * S * S;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int xx = (int)(i % S), yy = (int)((i / S) % S), c = (int)(i / ((long)S * S));
    int v;
    if (vb) {
      const int ymin = vb[2 * yy] - yshift, n = vb[2 * yy + 1];
      const int* k = vk + (long)yy * vks;
      const uint8_t* p = in + ((long)ymin * Win + xx) * 3 + c;
      int acc = 1 << 21;
      for (int y = 0; y < n; ++y) acc += (int)p[(long)y * Win * 3] * k[y];
      v = clip8_22(acc);
    } else {
      v = in[((long)yy * Win + xx) * 3 + c];
    }
    out[i] = lut[v];
  }
}

extern "C" int pg_image_preprocess(const uint8_t* src, int H, int W, int S, const int* hb, const int* hk, int hks,
                                   const int* vb, const int* vk, int vks, int y0, int rows, const float* lut,
                                   uint8_t* tmp, float* out, hipStream_t stream) {
  PG_REQUIRE(H > 0 && W > 0 && S > 0 && lut && out && src);
  PG_REQUIRE(hb ? (hk && hks > 0 && tmp && rows > 0 && y0 >= 0 && y0 + rows <= H) : W == S);
  PG_REQUIRE(vb ? (vk && vks > 0) : (hb ? rows == S : H == S));
  const uint8_t* in = src;
  int win = W, yshift = 0;
  if (hb) {
    const long n = (long)rows * S * 3;
    hipLaunchKernelGGL(resize_h_kernel, dim3((int)min((n + 255) / 256, 4096L)), dim3(256), 0, stream, src, W, y0,
                       rows, S, hb, hk, hks, tmp);
    in = tmp;
    win = S;
    yshift = y0;
  }
  const long n = 3L * S * S;
  hipLaunchKernelGGL(resize_v_kernel, dim3((int)min((n + 255) / 256, 4096L)), dim3(256), 0, stream, in, win, yshift,
                     S, vb, vk, vks, lut, out);
  PG_LAUNCH_CHECK();
  return 0;
}
