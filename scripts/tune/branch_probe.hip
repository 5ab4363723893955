// Probe: do two HIP streams (eager) and two branches of a captured hipGraph run concurrently, so that a
// resident "bank-ahead" kernel on one stream can wait (bounded) for a flag raised by a kernel chain on the
// other?  Standalone:  hipcc -O3 --offload-arch=gfx950 branch_probe.hip -o branch_probe && ./branch_probe
//
// waiter: 256 workgroups x 256 threads, 96 KiB dynamic LDS (one per CU), each polls a counter until it reaches
//         the epoch's target (relaxed agent loads + s_sleep), bounded by 20 ms of wall clock -> err.
// chain : a 1-workgroup spin of ~10 us, then `setter` (160 workgroups, 32 KiB LDS each, one add per workgroup).
// If the waiter's workgroups block the chain (no concurrency, or no co-residency) every wait times out.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

__device__ __forceinline__ unsigned long long wall() { return __builtin_amdgcn_s_memrealtime(); }   // 100 MHz

__global__ void begin_kernel(unsigned* epoch) { if (threadIdx.x == 0) atomicAdd(epoch, 1u); }

__global__ void spin_kernel(int ticks) {
  const unsigned long long t0 = wall();
  while (wall() - t0 < (unsigned long long)ticks) __builtin_amdgcn_s_sleep(1);
}

__global__ __launch_bounds__(256) void setter_kernel(unsigned* cnt, unsigned long long* stamp) {
  extern __shared__ char lds[];
  lds[threadIdx.x] = 1;
  __syncthreads();
  if (threadIdx.x == 0) {
    if (blockIdx.x == 0) stamp[0] = wall();
    __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

__global__ __launch_bounds__(256) void waiter_kernel(const unsigned* cnt, const unsigned* epoch, unsigned per,
                                                     unsigned* err, unsigned long long* stamp) {
  extern __shared__ char lds[];
  lds[threadIdx.x] = 2;
  if (threadIdx.x == 0) {
    const unsigned target = per * __hip_atomic_load(epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned long long t0 = wall();
    if (blockIdx.x == 0) stamp[1] = t0;
    while (__hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
      if (wall() - t0 > 2000000ull) { atomicAdd(err, 1u); break; }   // 20 ms
      __builtin_amdgcn_s_sleep(2);
    }
    if (blockIdx.x == 0) stamp[2] = wall();
  }
  __syncthreads();
}

int main() {
  unsigned *cnt, *epoch, *err;
  unsigned long long* stamp;
  CK(hipMalloc(&cnt, 4)); CK(hipMalloc(&epoch, 4)); CK(hipMalloc(&err, 4)); CK(hipMalloc(&stamp, 64));
  CK(hipMemset(cnt, 0, 4)); CK(hipMemset(epoch, 0, 4)); CK(hipMemset(err, 0, 4));
  CK(hipFuncSetAttribute((const void*)waiter_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, 96 * 1024));
  hipStream_t s1, s2;
  CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking)); CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
  hipEvent_t fork, join;
  CK(hipEventCreateWithFlags(&fork, hipEventDisableTiming)); CK(hipEventCreateWithFlags(&join, hipEventDisableTiming));
  const unsigned PER = 160;
  auto enqueue = [&](bool waiter_first) {
    begin_kernel<<<1, 64, 0, s1>>>(epoch);
    hipEventRecord(fork, s1);
    hipStreamWaitEvent(s2, fork, 0);
    if (waiter_first) waiter_kernel<<<256, 256, 96 * 1024, s2>>>(cnt, epoch, PER, err, stamp);
    spin_kernel<<<1, 64, 0, s1>>>(1000);   // 10 us
    setter_kernel<<<PER, 256, 32 * 1024, s1>>>(cnt, stamp);
    if (!waiter_first) waiter_kernel<<<256, 256, 96 * 1024, s2>>>(cnt, epoch, PER, err, stamp);
    hipEventRecord(join, s2);
    hipStreamWaitEvent(s1, join, 0);
  };
  unsigned long long h[4];
  unsigned herr = 0;
  // 1. eager, waiter enqueued first
  for (int it = 0; it < 5; ++it) enqueue(true);
  CK(hipStreamSynchronize(s1));
  CK(hipMemcpy(&herr, err, 4, hipMemcpyDeviceToHost));
  CK(hipMemcpy(h, stamp, 32, hipMemcpyDeviceToHost));
  printf("{\"case\": \"eager\", \"timeouts\": %u, \"wait_us\": %.2f, \"set_minus_waitstart_us\": %.2f}\n", herr,
         (h[2] - h[1]) / 100.0, ((long long)h[0] - (long long)h[1]) / 100.0);
  // 2/3. captured graph, waiter captured first / last
  for (int wf = 1; wf >= 0; --wf) {
    CK(hipMemset(err, 0, 4));
    CK(hipDeviceSynchronize());
    hipGraph_t g;
    hipGraphExec_t ge;
    CK(hipStreamBeginCapture(s1, hipStreamCaptureModeGlobal));
    enqueue(wf == 1);
    CK(hipStreamEndCapture(s1, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    hipEvent_t t0, t1;
    CK(hipEventCreate(&t0)); CK(hipEventCreate(&t1));
    CK(hipGraphLaunch(ge, s1));
    CK(hipStreamSynchronize(s1));
    CK(hipEventRecord(t0, s1));
    for (int it = 0; it < 20; ++it) CK(hipGraphLaunch(ge, s1));
    CK(hipEventRecord(t1, s1));
    CK(hipStreamSynchronize(s1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, t0, t1));
    CK(hipMemcpy(&herr, err, 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(h, stamp, 32, hipMemcpyDeviceToHost));
    printf("{\"case\": \"graph\", \"waiter_first\": %d, \"timeouts\": %u, \"replay_us\": %.2f, \"wait_us\": %.2f, "
           "\"set_minus_waitstart_us\": %.2f}\n", wf, herr, ms * 1000.f / 20, (h[2] - h[1]) / 100.0,
           ((long long)h[0] - (long long)h[1]) / 100.0);
    CK(hipGraphExecDestroy(ge)); CK(hipGraphDestroy(g));
  }
  // 4. cost of a cross-stream edge inside a graph: 36 short kernels alternating s1 / s2 (each waits for the
  //    previous one through an event) vs the same 36 kernels on s1 alone
  for (int pp = 0; pp < 2; ++pp) {
    CK(hipDeviceSynchronize());
    hipGraph_t g;
    hipGraphExec_t ge;
    std::vector<hipEvent_t> evs(40);
    for (auto& e : evs) CK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    CK(hipStreamBeginCapture(s1, hipStreamCaptureModeGlobal));
    hipEventRecord(evs[0], s1);
    hipStreamWaitEvent(s2, evs[0], 0);
    for (int i = 0; i < 36; ++i) {
      hipStream_t s = (pp == 1 && (i & 1)) ? s2 : s1;
      hipStream_t o = s == s1 ? s2 : s1;
      if (pp == 1 && i > 0) hipStreamWaitEvent(s, evs[i], 0);
      spin_kernel<<<1, 64, 0, s>>>(200);   // 2 us
      if (pp == 1) hipEventRecord(evs[i + 1], s);
      (void)o;
    }
    hipEventRecord(evs[38], s2);
    hipStreamWaitEvent(s1, evs[38], 0);
    CK(hipStreamEndCapture(s1, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    hipEvent_t t0, t1;
    CK(hipEventCreate(&t0)); CK(hipEventCreate(&t1));
    CK(hipGraphLaunch(ge, s1));
    CK(hipStreamSynchronize(s1));
    CK(hipEventRecord(t0, s1));
    for (int it = 0; it < 20; ++it) CK(hipGraphLaunch(ge, s1));
    CK(hipEventRecord(t1, s1));
    CK(hipStreamSynchronize(s1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, t0, t1));
    printf("{\"case\": \"graph36\", \"pingpong\": %d, \"replay_us\": %.2f}\n", pp, ms * 1000.f / 20);
    // the same, eager
    CK(hipEventRecord(t0, s1));
    for (int it = 0; it < 20; ++it) {
      hipEventRecord(evs[0], s1);
      hipStreamWaitEvent(s2, evs[0], 0);
      for (int i = 0; i < 36; ++i) {
        hipStream_t s = (pp == 1 && (i & 1)) ? s2 : s1;
        if (pp == 1 && i > 0) hipStreamWaitEvent(s, evs[i], 0);
        spin_kernel<<<1, 64, 0, s>>>(200);
        if (pp == 1) hipEventRecord(evs[i + 1], s);
      }
      hipEventRecord(evs[38], s2);
      hipStreamWaitEvent(s1, evs[38], 0);
    }
    CK(hipEventRecord(t1, s1));
    CK(hipStreamSynchronize(s1));
    CK(hipEventElapsedTime(&ms, t0, t1));
    printf("{\"case\": \"eager36\", \"pingpong\": %d, \"us\": %.2f}\n", pp, ms * 1000.f / 20);
    CK(hipGraphExecDestroy(ge)); CK(hipGraphDestroy(g));
  }
  return 0;
}
