// One-shot all-reduce over xGMI peer memory (survey §5.8-3; the reference's per-step gradient all-reduce is
// ddp_tutorial_multi_gpu.py:94 through DDP's NCCL bucket).  An 8-GPU MI355X node is fully connected: every GPU
// has its own xGMI link to each peer.  A ring all-reduce sends 2(W-1) dependent messages through ONE link per
// step; for the latency-bound 247 KB (LeNet-5) / 473 KB (MLP) gradient slab, this kernel instead does ONE hop:
//   1. every rank PUSHES its slice of the slab into slot [rank] of every peer's receive buffer (W-1 remote
//      writes, one per link, all links busy at once) and raises a per-(source rank, block) flag there;
//   2. every rank waits for the W flags of its blocks (bounded spin) and sums the W slots of its OWN receive
//      buffer in rank order 0..W-1 -- a fixed order, so every replica gets bitwise the same sum.
// Receive buffers and flags are uncached device memory (hipDeviceMallocUncached) mapped into the peers over
// IPC: remote stores land in HBM, and the local reads see them without any cache maintenance.  Two buffer
// parities alternate per call: a rank can be at most one call ahead of any peer (it cannot pass a call
// without every peer's flags of that call), so the parity it writes is never the one a peer still reads.
// Each block keeps its own call sequence number; flags are monotonic (no reset between calls).
#include "common.h"
#include "launch.h"

namespace {

struct OneShotArgs {
  float* buf;                 // in/out gradient range (count floats, 16-byte aligned)
  int count;                  // floats, <= max_count
  int rank, world;
  int max_count;              // floats per slot (receive buffer: [2][world][max_count])
  float* const* peer_data;    // [world] base of every rank's receive buffer (own included), device array
  uint32_t* const* peer_flags;  // [world] base of every rank's flags [world][nblk]
  uint32_t* seq;              // [nblk] this rank's call sequence per block (local memory)
  uint32_t* err;              // [1] set to 1 on a flag timeout (host checks)
  unsigned long long timeout_ticks;  // 100 MHz wall clock
};

constexpr int OS_THREADS = 256;

__global__ __launch_bounds__(OS_THREADS) void oneshot_allreduce_kernel(OneShotArgs a) {
  const int b = blockIdx.x, nblk = gridDim.x, tid = threadIdx.x;
  const int nv = a.count >> 2;                       // float4 elements
  const int per = (nv + nblk - 1) / nblk;            // float4 per block
  const int v0 = b * per, v1 = min(nv, v0 + per);
  __shared__ uint32_t s_seq;
  if (tid == 0) s_seq = a.seq[b] + 1u;
  __syncthreads();
  const uint32_t s = s_seq;
  const int par = s & 1;
  // 1. push this block's slice into slot [rank] of every rank's receive buffer
  for (int v = v0 + tid; v < v1; v += OS_THREADS) {
    const f32x4 x = reinterpret_cast<const f32x4*>(a.buf)[v];
    for (int q = 0; q < a.world; ++q) {
      f32x4* dst = reinterpret_cast<f32x4*>(a.peer_data[q] + ((size_t)par * a.world + a.rank) * a.max_count);
      dst[v] = x;
    }
  }
  // tail (count % 4) by block 0
  if (b == 0 && tid < (a.count & 3)) {
    const int e = (nv << 2) + tid;
    for (int q = 0; q < a.world; ++q) a.peer_data[q][((size_t)par * a.world + a.rank) * a.max_count + e] = a.buf[e];
  }
  // every storing wave's stores are complete (system scope) before the block's flags are raised
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid < a.world) {
    __hip_atomic_store(a.peer_flags[tid] + (size_t)a.rank * nblk + b, s, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  // 2. wait for every rank's flag of this block (lane r polls source rank r), bounded
  if (tid < a.world) {
    const uint32_t* f = a.peer_flags[a.rank] + (size_t)tid * nblk + b;
    const unsigned long long t0 = wall_clock64();
    while (__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) < s) {
      if (wall_clock64() - t0 > a.timeout_ticks) {
        __hip_atomic_store(a.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
  __syncthreads();
  // 3. sum the W slots of the own receive buffer in rank order
  const float* rb = a.peer_data[a.rank] + (size_t)par * a.world * a.max_count;
  for (int v = v0 + tid; v < v1; v += OS_THREADS) {
    f32x4 acc = reinterpret_cast<const f32x4*>(rb)[v];
    for (int r = 1; r < a.world; ++r) acc += reinterpret_cast<const f32x4*>(rb + (size_t)r * a.max_count)[v];
    reinterpret_cast<f32x4*>(a.buf)[v] = acc;
  }
  if (b == 0 && tid < (a.count & 3)) {
    const int e = (nv << 2) + tid;
    float acc = rb[e];
    for (int r = 1; r < a.world; ++r) acc += rb[(size_t)r * a.max_count + e];
    a.buf[e] = acc;
  }
  if (tid == 0) a.seq[b] = s;
}

}  // namespace

void launch_oneshot_allreduce(float* buf, int count, int rank, int world, int max_count, float* const* peer_data,
                              uint32_t* const* peer_flags, uint32_t* seq, uint32_t* err, int nblk,
                              unsigned long long timeout_ticks, hipStream_t s) {
  OneShotArgs a{buf, count, rank, world, max_count, peer_data, peer_flags, seq, err, timeout_ticks};
  hipLaunchKernelGGL(oneshot_allreduce_kernel, dim3(nblk), dim3(OS_THREADS), 0, s, a);
}
