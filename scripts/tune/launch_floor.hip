// Launch-floor microbenchmark: back-to-back dependent launches of a trivial kernel.
#include <hip/hip_runtime.h>
__global__ void tiny(float* p, int n) { if (threadIdx.x == 0 && blockIdx.x == 0) p[0] += 1.0f; }
extern "C" int launch_tiny(float* p, int grid, int block, hipStream_t s) {
  hipLaunchKernelGGL(tiny, dim3(grid), dim3(block), 0, s, p, 0);
  return (int)hipGetLastError();
}
