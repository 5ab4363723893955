// Grid-barrier cost microbenchmark (tuning only): one persistent launch of nwg workgroups (all co-resident: one or
// two per CU) that runs `iters` rounds of [each workgroup stores `words` floats to its own slice, grid barrier,
// reads its neighbour's slice].  The barrier: a device-scope release add on one counter by each workgroup, then
// a spin on an acquire load until the round's target; every spin gives up after ~0.5 s (err = 1), so a
// workgroup that is not resident cannot hang the GPU.
#include <hip/hip_runtime.h>

__global__ __launch_bounds__(256) void gb_kernel(unsigned* counter, int iters, float* buf, int words, int* err) {
  const int nwg = gridDim.x, wg = blockIdx.x;
  float acc = 0.f;
  for (int it = 0; it < iters; ++it) {
    float* mine = buf + (size_t)wg * words;
    for (int i = threadIdx.x; i < words; i += 256) mine[i] = (float)(it + i);
    __syncthreads();
    if (threadIdx.x == 0) {
      const unsigned target = (unsigned)(it + 1) * (unsigned)nwg;
      __hip_atomic_fetch_add(counter, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
      const unsigned long long t0 = wall_clock64();
      while (__hip_atomic_load(counter, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) < target) {
        if (wall_clock64() - t0 > 50000000ull) {   // 0.5 s at the 100 MHz wall clock
          *err = 1;
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
    }
    __syncthreads();
    const float* other = buf + (size_t)((wg + 1) % nwg) * words;
    for (int i = threadIdx.x; i < words; i += 256) acc += other[i];
  }
  if (acc == -1.f) buf[0] = acc;                 // keep the reads live
}

extern "C" int gb_run(unsigned* counter, int nwg, int iters, float* buf, int words, int* err, hipStream_t s) {
  hipLaunchKernelGGL(gb_kernel, dim3(nwg), dim3(256), 0, s, counter, iters, buf, words, err);
  return (int)hipGetLastError();
}
