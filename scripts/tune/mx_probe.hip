// Probe of v_mfma_scale_f32_16x16x128_f8f6f4's B-scale lane mapping: B data only in lane Ld, byte half h (e4m3 1.0),
// A all 1.0, scale B = 2 (E8M0 128) in lane Ls only.  Prints, per (Ld, h), the scale lanes that double the result.
#include <hip/hip_runtime.h>
#include <cstdio>

typedef int i32x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

__global__ void probe(float* out) {
  const int lane = threadIdx.x;
  for (int ld = 0; ld < 64; ++ld)
    for (int h = 0; h < 2; ++h)
      for (int ls = 0; ls < 64; ++ls) {
        i32x8 a, b;
        for (int i = 0; i < 8; ++i) {
          a[i] = 0x38383838;
          b[i] = (lane == ld && (i >> 2) == h) ? 0x38383838 : 0;
        }
        f32x4 c = {0.f, 0.f, 0.f, 0.f};
        const int sb = lane == ls ? 128 : 127;
        c = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, c, 0, 0, 0, 127, 0, sb);
        float s = c[0] + c[1] + c[2] + c[3];
        for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
        if (lane == 0) out[(ld * 2 + h) * 64 + ls] = s;
      }
}

int main() {
  float* d;
  hipMalloc(&d, 64 * 2 * 64 * sizeof(float));
  hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, d);
  static float h[64 * 2 * 64];
  hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  for (int ld = 0; ld < 64; ++ld)
    for (int hh = 0; hh < 2; ++hh) {
      const float* r = h + (ld * 2 + hh) * 64;
      float base = r[0] < r[1] ? r[0] : r[1];
      printf("data lane %2d half %d base %6.1f doubled by scale lanes:", ld, hh, base);
      for (int ls = 0; ls < 64; ++ls)
        if (r[ls] > base * 1.5f) printf(" %d", ls);
      printf("\n");
    }
  hipFree(d);
  return 0;
}
