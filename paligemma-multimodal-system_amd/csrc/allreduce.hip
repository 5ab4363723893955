// pg_allreduce_xgmi: one-shot SUM all-reduce of fp32 partials between the tensor-parallel ranks of one
// node, over xGMI peer-to-peer stores (the reference has no parallelism at all).
//
// Why not only RCCL: a decode step all-reduces two [B][hidden] fp32 slabs per layer (8-256 KB).  At
// that size a ring collective is latency-bound (2(W-1) dependent hops); a one-shot exchange is one
// hop: every rank stores its slab straight into slot `rank` of every peer's exchange buffer (the W-1
// stores go out over W-1 different xGMI links at once), raises a flag there, waits for the W flags
// in its own buffer and sums the W slots in rank order 0..W-1 -- so every rank computes the
// bit-identical sum (the vocabulary-parallel greedy merge depends on ranks agreeing).
//
// Exchange buffer of one rank (uncached device memory, mapped into the peers with IPC handles):
//   [0, 4096)   flags   u32 [2 sets][PG_XG_MAXWG workgroups][PG_XG_MAXW ranks]
//   [4096, ..)  slots   f32 [2 sets][W][cap]
// Every call launches all PG_XG_MAXWG workgroups and workgroup w always owns the same elements: the
// fixed PG_XG_CHUNK-float chunks w, w + PG_XG_MAXWG, w + 2*PG_XG_MAXWG, ... (a grid-stride loop; a
// workgroup with no chunk below n still does the flag handshake).  So every workgroup's local epoch
// counter `epochs[wg]` advances on every call, all workgroups agree on the call count e, and call e uses
// buffer set e&1.  A rank starts call e+2 only after its call e+1 finished, which needed every peer's
// flags for e+1; a peer raises those only after its call e (which read set e&1) finished (stream order).
// So the two sets make slot reuse race-free for any sequence of sizes, without a host sync between
// calls.  Everything the kernel needs lives on the device (epoch counters included), so the call is
// capturable into the decode hipGraph.
//
// pg_allgather_xgmi is the same exchange with a different step 3: instead of summing, every rank copies the W
// slots out in rank order (out = [W][n]), so the vocabulary-parallel logits travel once per rank instead of
// W times in a zero-padded SUM.  Both share the exchange buffer and the per-workgroup epochs, so calls of the
// two may be interleaved freely.
//
// pg_allreduce_xgmi_rs (ABI 12) is the large-message form (the prefill's row-chunk all-reduces, up to 32 MB): a
// reduce-scatter then an all-gather over the same kind of peer stores, 2(W-1)/W of the message leaving each rank
// instead of the one-shot's (W-1).  Chunk c of W*P floats is cut into W sub-pieces of P floats;
// rank p owns sub-piece p: every rank stores its sub-piece p into rank p's receive slot (phase 1), rank p sums the W
// contributions in rank order 0..W-1 -- the one-shot kernel's order, so both forms give the same bits -- and stores
// the sum into every rank's gather slot (phase 2), and every rank copies the gathered chunk out (phase 3).  Its own
// buffer, per-workgroup epochs and two buffer sets, with the same stream-order argument as the one-shot kernel, per
// kind: RS call e+2 can only begin on a peer after this rank finished RS call e+1, hence RS call e.
//
// Co-residency: workgroup w of a rank waits only for workgroup w of each peer (the same chunks), never for another
// workgroup of its own launch, so no kernel needs its whole grid resident.  It does need each peer's workgroup w
// to be dispatched eventually while it spins: true on a node with one device per rank (the spinning kernel holds at
// most nwg <= 256 workgroups of one device).  Ranks that SHARE a device (the tests) also need every rank's queue to be
// serviced while the others spin, and the sum of their grids to fit the device: XgmiComm sizes the RS grid by the
// ranks per device, and the test launcher keeps the hardware queues per process low.
//
// Waiting is bounded by the 100 MHz wall clock: a peer that never arrives sets err[0] and the kernel
// finishes (its output is then meaningless) instead of hanging the device.  err is int[8]: the first timeout also
// records (err[1] kind: 1 one-shot, 2 reduce-scatter, 3 all-gather phase; err[2] workgroup; err[3] the peer rank waited
// for; err[4] the epoch expected; err[5] the flag value seen; err[6] this rank).  Once err[0] is set, later exchanges
// skip their waits (their results are invalid anyway) so a dead peer costs one timeout, not one per call.
#include <cstring>

#include "common.h"

#define PG_XG_MAXW 8
#define PG_XG_MAXWG 64
#define PG_XG_MAXCAP (1L << 40)             // floats per slot: keeps the buffer byte counts inside a long
#define PG_XG_CHUNK 8192                    // floats per chunk (32 KB)
#define PG_XG_FLAG_BYTES 4096
#define PG_XG_TIMEOUT_TICKS 2000000000ull   // 20 s of the 100 MHz constant clock
#define PG_XR_MAXWG 256                     // reduce-scatter grid (<= 256 workgroups)
#define PG_XR_P 1024                        // floats per sub-piece: one 256-thread pass of 16 B per thread
#define PG_XR_FLAG_BYTES (2 * 2 * PG_XR_MAXWG * PG_XG_MAXW * 4)   // [2 phases][2 sets][wg][rank] u32

struct XgPeers {
  void* p[PG_XG_MAXW];
};

// the first timeout of this rank records where it waited (see the header); later ones only keep err[0] set
__device__ __forceinline__ void xg_timeout(int* err, int kind, int wg, int peer, unsigned expect, unsigned seen,
                                           int rank) {
  if (atomicCAS(err, 0, 1) == 0) {
    err[1] = kind;
    err[2] = wg;
    err[3] = peer;
    err[4] = (int)expect;
    err[5] = (int)seen;
    err[6] = rank;
  }
}

// one lane waits for flag f == e (bounded; records the diagnostics on a timeout)
__device__ __forceinline__ void xg_wait(const unsigned* f, unsigned e, int* err, int kind, int wg, int peer, int rank) {
  const unsigned long long t0 = wall_clock64();
  unsigned v;
  while ((v = __hip_atomic_load(f, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM)) != e) {
    if (wall_clock64() - t0 > PG_XG_TIMEOUT_TICKS) {
      xg_timeout(err, kind, wg, peer, e, v, rank);
      return;
    }
    __builtin_amdgcn_s_sleep(2);
  }
}

// this workgroup's stores are complete and visible system-wide, then lanes < W raise flag_at(lane) + rank = e (the flag
// of this workgroup and rank in peer `lane`'s buffer)
template <typename FlagAt>
__device__ __forceinline__ void xg_publish(FlagAt flag_at, int W, int rank, unsigned e) {
  __threadfence_system();
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // (the release's write-back waited for: MI355X guide hazard)
  __syncthreads();
  if ((int)threadIdx.x < W)
    __hip_atomic_store(flag_at((int)threadIdx.x) + rank, e, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

__device__ __forceinline__ unsigned* xg_flag(const XgPeers& peers, int r, int off, int set, int wg) {
  return (unsigned*)((char*)peers.p[r] + off) + (set * PG_XG_MAXWG + wg) * PG_XG_MAXW;
}
__device__ __forceinline__ unsigned* xr_flag(const XgPeers& peers, int r, int phase, int set, int wg) {
  return (unsigned*)peers.p[r] + ((phase * 2 + set) * PG_XR_MAXWG + wg) * PG_XG_MAXW;
}

template <int W, bool GATHER>
__global__ __launch_bounds__(256) void allreduce_xgmi_kernel(const float* __restrict__ data, long n, int nslab,
                                                             long slab_stride, int rank, XgPeers peers, long cap,
                                                             unsigned* __restrict__ epochs, int* __restrict__ err,
                                                             float* __restrict__ out) {
  const int wg = blockIdx.x, tid = threadIdx.x;
  const unsigned e = epochs[wg] + 1u;
  const bool dead = __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;
  __syncthreads();
  if (tid == 0) epochs[wg] = e;
  const int set = (int)(e & 1u);
  constexpr long STRIDE = (long)PG_XG_MAXWG * PG_XG_CHUNK;

  // 1. push this rank's chunks into slot `rank` of every peer (and of itself); with nslab > 1 this rank's
  //    contribution is the sum of its split-K slabs data[s * slab_stride + i], s = 0..nslab-1, in slab order
  for (long c0 = (long)wg * PG_XG_CHUNK; c0 < n; c0 += STRIDE) {
    const long c1 = c0 + PG_XG_CHUNK < n ? c0 + PG_XG_CHUNK : n;
    for (long i = c0 + 4 * tid; i < c1; i += 1024) {
      f32x4 v = *(const f32x4*)(data + i);
      for (int s = 1; s < nslab; ++s) v += *(const f32x4*)(data + (long)s * slab_stride + i);
#pragma unroll
      for (int p = 0; p < W; ++p) {
        float* dst = (float*)((char*)peers.p[p] + PG_XG_FLAG_BYTES) + ((long)set * W + rank) * cap + i;
        __builtin_nontemporal_store(v, (f32x4*)dst);
      }
    }
  }
  xg_publish([&](int r) { return xg_flag(peers, r, 0, set, wg); }, W, rank, e);

  // 2. wait for the W flags of this workgroup's chunks in the local buffer
  if (tid < W && !dead) xg_wait(xg_flag(peers, rank, 0, set, wg) + tid, e, err, 1, wg, tid, rank);
  __syncthreads();
  __atomic_thread_fence(__ATOMIC_ACQUIRE);

  // 3. sum the W slots in rank order (identical on every rank), or copy them out in rank order
  const float* slots = (const float*)((const char*)peers.p[rank] + PG_XG_FLAG_BYTES) + (long)set * W * cap;
  for (long c0 = (long)wg * PG_XG_CHUNK; c0 < n; c0 += STRIDE) {
    const long c1 = c0 + PG_XG_CHUNK < n ? c0 + PG_XG_CHUNK : n;
    for (long i = c0 + 4 * tid; i < c1; i += 1024) {
      if constexpr (GATHER) {
#pragma unroll
        for (int p = 0; p < W; ++p)
          *(f32x4*)(out + (long)p * n + i) = __builtin_nontemporal_load((const f32x4*)(slots + (long)p * cap + i));
      } else {
        f32x4 s = __builtin_nontemporal_load((const f32x4*)(slots + i));
#pragma unroll
        for (int p = 1; p < W; ++p) s += __builtin_nontemporal_load((const f32x4*)(slots + (long)p * cap + i));
        *(f32x4*)(out + i) = s;
      }
    }
  }
}

// Reduce-scatter + all-gather (pg_allreduce_xgmi_rs).  Buffer of one rank: flags (PG_XR_FLAG_BYTES), then
// recv f32 [2 sets][nc][W][P] (slot src of chunk c: rank src's sub-piece `rank` of chunk c), then
// gather f32 [2 sets][nc][W][P] (chunk c in its original order: sub-piece p summed by rank p).
template <int W>
__global__ __launch_bounds__(256) void allreduce_rs_kernel(const float* __restrict__ data, long n, int nslab,
                                                           long slab_stride, int rank, XgPeers peers, long nc,
                                                           unsigned* __restrict__ epochs, int* __restrict__ err,
                                                           float* __restrict__ out) {
  const int wg = blockIdx.x, nwg = gridDim.x, tid = threadIdx.x;
  const unsigned e = epochs[wg] + 1u;
  const bool dead = __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;
  __syncthreads();
  if (tid == 0) epochs[wg] = e;
  const int set = (int)(e & 1u);
  constexpr long CW = (long)W * PG_XR_P;
  const long nch = (n + CW - 1) / CW;
  const long set_floats = nc * CW;
  auto recv = [&](int r) { return (float*)((char*)peers.p[r] + PG_XR_FLAG_BYTES) + (long)set * set_floats; };
  auto gath = [&](int r) { return (float*)((char*)peers.p[r] + PG_XR_FLAG_BYTES) + (long)(2 + set) * set_floats; };
  const long t4 = 4 * tid;

  // 1. reduce-scatter, send: sub-piece p of each of this workgroup's chunks -> rank p's receive slot `rank`
  for (long c = wg; c < nch; c += nwg) {
#pragma unroll
    for (int p = 0; p < W; ++p) {
      const long i = c * CW + p * PG_XR_P + t4;
      f32x4 v = {0.f, 0.f, 0.f, 0.f};
      if (i < n) {
        v = *(const f32x4*)(data + i);
        for (int s = 1; s < nslab; ++s) v += *(const f32x4*)(data + (long)s * slab_stride + i);
      }
      __builtin_nontemporal_store(v, (f32x4*)(recv(p) + (c * W + rank) * PG_XR_P + t4));
    }
  }
  xg_publish([&](int r) { return xr_flag(peers, r, 0, set, wg); }, W, rank, e);
  if (tid < W && !dead) xg_wait(xr_flag(peers, rank, 0, set, wg) + tid, e, err, 2, wg, tid, rank);
  __syncthreads();
  __atomic_thread_fence(__ATOMIC_ACQUIRE);

  // 2. reduce this rank's sub-piece in rank order and all-gather it: -> every rank's gather slot
  const float* rv = recv(rank);
  for (long c = wg; c < nch; c += nwg) {
    const float* src = rv + c * CW + t4;
    f32x4 s = __builtin_nontemporal_load((const f32x4*)src);
#pragma unroll
    for (int q = 1; q < W; ++q) s += __builtin_nontemporal_load((const f32x4*)(src + q * PG_XR_P));
#pragma unroll
    for (int p = 0; p < W; ++p)
      __builtin_nontemporal_store(s, (f32x4*)(gath(p) + (c * W + rank) * PG_XR_P + t4));
  }
  xg_publish([&](int r) { return xr_flag(peers, r, 1, set, wg); }, W, rank, e);
  if (tid < W && !dead) xg_wait(xr_flag(peers, rank, 1, set, wg) + tid, e, err, 3, wg, tid, rank);
  __syncthreads();
  __atomic_thread_fence(__ATOMIC_ACQUIRE);

  // 3. the gathered chunks out, in their original order
  const float* gv = gath(rank);
  for (long c = wg; c < nch; c += nwg) {
#pragma unroll
    for (int p = 0; p < W; ++p) {
      const long i = c * CW + p * PG_XR_P + t4;
      if (i < n) *(f32x4*)(out + i) = __builtin_nontemporal_load((const f32x4*)(gv + i));
    }
  }
}

extern "C" int pg_xgmi_buffer_bytes(int world, long cap, long* bytes) {
  PG_REQUIRE(world >= 1 && world <= PG_XG_MAXW && cap > 0 && cap <= PG_XG_MAXCAP && cap % 4 == 0 && bytes != nullptr);
  *bytes = PG_XG_FLAG_BYTES + 2L * world * cap * (long)sizeof(float);
  return 0;
}

static long rs_chunks(int world, long rs_cap) { return (rs_cap + (long)world * PG_XR_P - 1) / ((long)world * PG_XR_P); }

extern "C" int pg_xgmi_rs_buffer_bytes(int world, long rs_cap, long* bytes) {
  PG_REQUIRE(world >= 1 && world <= PG_XG_MAXW && rs_cap > 0 && rs_cap <= PG_XG_MAXCAP && rs_cap % 4 == 0 &&
             bytes != nullptr);
  *bytes = PG_XR_FLAG_BYTES + 4L * rs_chunks(world, rs_cap) * world * PG_XR_P * (long)sizeof(float);
  return 0;
}

// Uncached device memory (flags and slots are read by the owner while peers write them over xGMI).
extern "C" int pg_xgmi_alloc(long bytes, void** out) {
  PG_REQUIRE(out != nullptr && bytes > 0);
  void* p = nullptr;
  hipError_t e = hipExtMallocWithFlags(&p, (size_t)bytes, hipDeviceMallocUncached);
  if (e != hipSuccess) return (int)e;
  e = hipMemset(p, 0, (size_t)bytes);
  // the zeroing must be complete before the IPC handle is exported and a peer's first flag or slot
  // store can land (a late memset would wipe it and the exchange would time out)
  if (e == hipSuccess) e = hipDeviceSynchronize();
  if (e != hipSuccess) {
    (void)hipFree(p);
    return (int)e;
  }
  *out = p;
  return 0;
}

extern "C" int pg_xgmi_free(void* p) { return (int)hipFree(p); }

extern "C" int pg_xgmi_ipc_handle(void* p, void* handle64) {
  PG_REQUIRE(p != nullptr && handle64 != nullptr);
  hipIpcMemHandle_t h;
  const hipError_t e = hipIpcGetMemHandle(&h, p);
  if (e != hipSuccess) return (int)e;
  std::memcpy(handle64, &h, sizeof(h));
  return 0;
}

extern "C" int pg_xgmi_ipc_open(const void* handle64, void** out) {
  PG_REQUIRE(handle64 != nullptr && out != nullptr);
  hipIpcMemHandle_t h;
  std::memcpy(&h, handle64, sizeof(h));
  return (int)hipIpcOpenMemHandle(out, h, hipIpcMemLazyEnablePeerAccess);
}

extern "C" int pg_xgmi_ipc_close(void* p) { return (int)hipIpcCloseMemHandle(p); }

static int xgmi_launch(const float* data, long n, int nslab, long slab_stride, float* out, bool gather, int rank,
                       int world, void* const* peers, long cap, unsigned* epochs, int* err, hipStream_t stream) {
  PG_REQUIRE(data != nullptr && out != nullptr && peers != nullptr && epochs != nullptr && err != nullptr);
  PG_REQUIRE(nslab >= 1 && nslab <= 64 && (nslab == 1 || (slab_stride >= n && slab_stride % 4 == 0)));
  PG_REQUIRE(world >= 1 && world <= PG_XG_MAXW && rank >= 0 && rank < world);
  PG_REQUIRE(n > 0 && n % 4 == 0 && n <= cap && cap % 4 == 0 && ((uintptr_t)data & 15) == 0 &&
             ((uintptr_t)out & 15) == 0);
  XgPeers pp = {};
  for (int r = 0; r < world; ++r) {
    PG_REQUIRE(peers[r] != nullptr && ((uintptr_t)peers[r] & 15) == 0);
    pp.p[r] = peers[r];
  }
  // always the full grid: every workgroup's epoch advances on every call (see the header)
#define PG_XG_CASE(WW)                                                                                         \
  case WW:                                                                                                     \
    if (gather)                                                                                                \
      hipLaunchKernelGGL((allreduce_xgmi_kernel<WW, true>), dim3(PG_XG_MAXWG), dim3(256), 0, stream, data, n,  \
                         nslab, slab_stride, rank, pp, cap, epochs, err, out);                                                     \
    else                                                                                                       \
      hipLaunchKernelGGL((allreduce_xgmi_kernel<WW, false>), dim3(PG_XG_MAXWG), dim3(256), 0, stream, data, n, \
                         nslab, slab_stride, rank, pp, cap, epochs, err, out);                                                     \
    break;
  switch (world) {
    PG_XG_CASE(1)
    PG_XG_CASE(2)
    PG_XG_CASE(3)
    PG_XG_CASE(4)
    PG_XG_CASE(5)
    PG_XG_CASE(6)
    PG_XG_CASE(7)
    PG_XG_CASE(8)
  }
#undef PG_XG_CASE
  PG_LAUNCH_CHECK();
  return 0;
}

// In-place SUM of data[0, n) over `world` ranks.  peers[r] = rank r's exchange buffer as mapped in this
// process (peers[rank] = the local one), each pg_xgmi_buffer_bytes(world, cap) long; epochs = PG_XG_MAXWG
// zero-initialised local u32 words owned by this communicator; err = 8 local ints (err[0] set on a timeout).
// n % 4 == 0, n <= cap, data 16-B aligned.  Every rank must issue the same sequence of calls.
extern "C" int pg_allreduce_xgmi(float* data, long n, int rank, int world, void* const* peers, long cap,
                                 unsigned* epochs, int* err, hipStream_t stream) {
  return xgmi_launch(data, n, 1, 0, data, false, rank, world, peers, cap, epochs, err, stream);
}

// The same SUM of this rank's nslab split-K slabs data[s * slab_stride + i] (s in order) over the ranks, written to
// data[0, n) (slab 0): a row-parallel linear's partial slabs are summed locally on the way into the exchange, so
// each rank moves n floats instead of nslab * n and no slab-sum launch precedes the exchange.
extern "C" int pg_allreduce_xgmi_slabs(float* data, long n, int nslab, long slab_stride, int rank, int world,
                                       void* const* peers, long cap, unsigned* epochs, int* err, hipStream_t stream) {
  return xgmi_launch(data, n, nslab, slab_stride, data, false, rank, world, peers, cap, epochs, err, stream);
}

// out[r * n + i] = rank r's in[i] for every rank r (all-gather in rank order); in / out 16-B aligned, not
// overlapping; the rest as pg_allreduce_xgmi (same buffer, same epochs).
extern "C" int pg_allgather_xgmi(const float* in, long n, float* out, int rank, int world, void* const* peers,
                                 long cap, unsigned* epochs, int* err, hipStream_t stream) {
  PG_REQUIRE(in != out);
  return xgmi_launch(in, n, 1, 0, out, true, rank, world, peers, cap, epochs, err, stream);
}

// (ABI 12) The same SUM as pg_allreduce_xgmi_slabs (nslab = 1: pg_allreduce_xgmi) as a reduce-scatter + all-gather over
// the ranks' RS buffers (pg_xgmi_rs_buffer_bytes(world, rs_cap) each, mapped like the exchange buffer): for messages
// of megabytes, 2(W-1)/W * n floats leave each rank instead of (W-1) * n.  The result has the same bits as the
// one-shot form's (rank-order sum) on every rank.  nwg (1..256) workgroups, the same on every rank and call; epochs =
// 256 local zero-initialised u32 words of this RS buffer (not the one-shot's); err = 8 local ints (see the header).
// n % 4 == 0, n <= rs_cap, data 16-B aligned.  Every rank must issue the same sequence of calls.
extern "C" int pg_allreduce_xgmi_rs(float* data, long n, int nslab, long slab_stride, int rank, int world,
                                    void* const* peers, long rs_cap, int nwg, unsigned* epochs, int* err,
                                    hipStream_t stream) {
  PG_REQUIRE(data != nullptr && peers != nullptr && epochs != nullptr && err != nullptr);
  PG_REQUIRE(nslab >= 1 && nslab <= 64 && (nslab == 1 || (slab_stride >= n && slab_stride % 4 == 0)));
  PG_REQUIRE(world >= 1 && world <= PG_XG_MAXW && rank >= 0 && rank < world && nwg >= 1 && nwg <= PG_XR_MAXWG);
  PG_REQUIRE(n > 0 && n % 4 == 0 && rs_cap % 4 == 0 && n <= rs_cap && ((uintptr_t)data & 15) == 0);
  XgPeers pp = {};
  for (int r = 0; r < world; ++r) {
    PG_REQUIRE(peers[r] != nullptr && ((uintptr_t)peers[r] & 15) == 0);
    pp.p[r] = peers[r];
  }
  const long nc = rs_chunks(world, rs_cap);
#define PG_XR_CASE(WW)                                                                                        \
  case WW:                                                                                                    \
    hipLaunchKernelGGL((allreduce_rs_kernel<WW>), dim3(nwg), dim3(256), 0, stream, data, n, nslab, slab_stride, \
                       rank, pp, nc, epochs, err, data);                                                      \
    break;
  switch (world) {
    PG_XR_CASE(1)
    PG_XR_CASE(2)
    PG_XR_CASE(3)
    PG_XR_CASE(4)
    PG_XR_CASE(5)
    PG_XR_CASE(6)
    PG_XR_CASE(7)
    PG_XR_CASE(8)
  }
#undef PG_XR_CASE
  PG_LAUNCH_CHECK();
  return 0;
}
