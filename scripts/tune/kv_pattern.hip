// Read-pattern probe for the decode KV cache (pt-448 x16 / pt-896 x32 shapes): the same bytes per wave, read as
//  0: the register-fragment pattern of attn_decode_split (K: 16 rows x 64 B per instruction, V^T: 16 rows x 32 B)
//  1: K as above, V^T as 16 rows x 64 B (keys 8g.. per lane, one 16-B load per row pair)
//  2: contiguous 1 KB per instruction (64 lanes x 16 B) over the same K block and a [block][256 d][32 keys] V image
// One wave per 32-key block, all blocks of B sequences; time per launch over 20 launches (hipEvents).
//   hipcc -O3 --offload-arch=gfx950 scripts/tune/kv_pattern.hip -o scripts/tune/kv_pattern && ./scripts/tune/kv_pattern
#include <hip/hip_runtime.h>
#include <cstdio>
typedef __attribute__((ext_vector_type(4))) unsigned u32x4;
typedef __attribute__((ext_vector_type(2))) unsigned u32x2;

template <int MODE>
__global__ __launch_bounds__(64) void probe(const unsigned short* k, const unsigned short* vt, int smax, int nblk,
                                            u32x4* out) {
  const int lane = threadIdx.x, c = lane & 15, g = lane >> 4;
  const int blk = blockIdx.x, b = blockIdx.y;
  const unsigned short* kb = k + ((long)b * smax + blk * 32) * 256;
  const unsigned short* vb = vt + (long)b * 256 * smax;
  u32x4 acc = {0, 0, 0, 0};
  if (MODE == 2) {
    const u32x4* kp = (const u32x4*)kb;                  // 16 KB contiguous
    const u32x4* vp = (const u32x4*)(vb + (long)blk * 32 * 256);   // blocked image: 16 KB contiguous
    u32x4 r[32];
#pragma unroll
    for (int i = 0; i < 16; ++i) r[i] = kp[i * 64 + lane];
#pragma unroll
    for (int i = 0; i < 16; ++i) r[16 + i] = vp[i * 64 + lane];
#pragma unroll
    for (int i = 0; i < 32; ++i) acc += r[i];
  } else {
    u32x4 ka[8], kb2[8];
#pragma unroll
    for (int s = 0; s < 8; ++s) {
      ka[s] = *(const u32x4*)(kb + (long)c * 256 + 32 * s + 8 * g);
      kb2[s] = *(const u32x4*)(kb + (long)(16 + c) * 256 + 32 * s + 8 * g);
    }
    if (MODE == 0) {
      u32x2 v[16][2];
#pragma unroll
      for (int t = 0; t < 16; ++t) {
        const unsigned short* row = vb + (long)(16 * t + c) * smax + blk * 32;
        v[t][0] = *(const u32x2*)(row + 4 * g);
        v[t][1] = *(const u32x2*)(row + 16 + 4 * g);
      }
#pragma unroll
      for (int t = 0; t < 16; ++t) acc += u32x4{v[t][0][0], v[t][0][1], v[t][1][0], v[t][1][1]};
    } else {
      u32x4 v[16];
#pragma unroll
      for (int t = 0; t < 16; ++t) v[t] = *(const u32x4*)(vb + (long)(16 * t + c) * smax + blk * 32 + 8 * g);
#pragma unroll
      for (int t = 0; t < 16; ++t) acc += v[t];
    }
#pragma unroll
    for (int s = 0; s < 8; ++s) acc += ka[s] + kb2[s];
  }
  if (acc[0] == 0x12345678u) out[lane] = acc;           // keep the loads live
}

int main() {
  const int cfg[2][3] = {{16, 1216, 1040}, {32, 4224, 4168}};
  for (auto& cf : cfg) {
    const int B = cf[0], smax = cf[1], L = cf[2];
    const int layers = 18;
    const size_t per = (size_t)B * smax * 256;           // elements per layer (K or V)
    unsigned short *k, *v;
    u32x4* out;
    hipMalloc(&k, per * 2 * layers);
    hipMalloc(&v, per * 2 * layers);
    hipMalloc(&out, 1024);
    hipMemset(k, 0x11, per * 2 * layers);
    hipMemset(v, 0x22, per * 2 * layers);
    const int nblk = (L + 31) / 32;
    const double bytes = (double)B * nblk * 32 * 1024;
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (int mode = 0; mode < 3; ++mode) {
      for (int rep = 0; rep < 2; ++rep) {
        hipEventRecord(e0);
        for (int it = 0; it < 20; ++it)
          for (int l = 0; l < layers; ++l) {
            const unsigned short* kl = k + per * l;
            const unsigned short* vl = v + per * l;
            if (mode == 0) probe<0><<<dim3(nblk, B), 64>>>(kl, vl, smax, nblk, out);
            if (mode == 1) probe<1><<<dim3(nblk, B), 64>>>(kl, vl, smax, nblk, out);
            if (mode == 2) probe<2><<<dim3(nblk, B), 64>>>(kl, vl, smax, nblk, out);
          }
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        const double us = ms * 1000.0 / (20 * layers);
        if (rep) printf("B=%d L=%d mode %d: %7.2f us per layer, %7.1f GB/s\n", B, L, mode, us, bytes / us / 1e3);
      }
    }
    hipFree(k);
    hipFree(v);
    hipFree(out);
  }
  return 0;
}
