// Weight prefetch into the Infinity Cache (MI355X L3 / MALL, 256 MiB, memory-side).
//
// A decode step streams 5 GB of weights through dependent kernels; the short ones (q|k|v, attention,
// o_proj) are latency-bound and leave HBM mostly idle.  pg_prefetch reads a byte range and discards it,
// so that a later kernel finds those lines on-die.  It is launched on a second stream beside the
// latency-bound kernels (a parallel branch of the captured decode graph): HBM time that the chain
// would leave idle moves the NEXT weight stream on-die.
//
// Each lane keeps UNR 16-byte loads in flight; loaded values are consumed by an empty asm sink, so
// nothing is written.  policy 1 = non-temporal loads.
#include "common.h"

template <int UNR, bool NT>
__global__ __launch_bounds__(256) void prefetch_kernel(const u32x4* __restrict__ p, long n16) {
  const long stride = (long)gridDim.x * blockDim.x;
  long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i + (UNR - 1) * stride < n16; i += UNR * stride) {
    u32x4 v[UNR];
#pragma unroll
    for (int u = 0; u < UNR; ++u) v[u] = NT ? __builtin_nontemporal_load(p + i + u * stride) : p[i + u * stride];
#pragma unroll
    for (int u = 0; u < UNR; ++u) asm volatile("" ::"v"(v[u][0]));
  }
  for (; i < n16; i += stride) {
    const u32x4 v = p[i];
    asm volatile("" ::"v"(v[0]));
  }
}

// Read [p, p + bytes) (p 16-B aligned, bytes a multiple of 16) on `stream` with `wgs` 256-thread workgroups.
extern "C" int pg_prefetch(const void* p, long bytes, int wgs, int policy, hipStream_t stream) {
  PG_REQUIRE(p != nullptr && bytes > 0 && bytes % 16 == 0 && ((uintptr_t)p & 15) == 0 && wgs > 0 && wgs <= 4096);
  const long n16 = bytes / 16;
  if (policy == 1)
    hipLaunchKernelGGL((prefetch_kernel<8, true>), dim3(wgs), dim3(256), 0, stream, (const u32x4*)p, n16);
  else
    hipLaunchKernelGGL((prefetch_kernel<8, false>), dim3(wgs), dim3(256), 0, stream, (const u32x4*)p, n16);
  PG_LAUNCH_CHECK();
  return 0;
}
