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
//
// Failure is latched, never silent: a flag wait that runs past the bound sets the error word and its block
// leaves WITHOUT writing a sum (the buffer keeps the local gradient there), and every later call sees the word
// at entry and does nothing at all -- no push (the one-call-ahead rule no longer holds once a call timed out, so
// a late peer could read a slot that was overwritten), no flag, no sum.  The update kernels of the step read the
// same word and skip the parameter update (launch_sgd_pack*: `skip`), so no parameter ever takes a partial sum;
// the host raises at its next wait (NativeTrainer.synchronize -> OneShotAllReduce::check).
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
  uint32_t* err;              // [1] latched: 1 after a flag wait timed out (host: check(); update kernels: skip)
  unsigned long long timeout_ticks;  // 100 MHz wall clock
  unsigned long long* stamps;  // optional [nblk][4] wall-clock stamps: entry, pushed, flags seen, summed
};

constexpr int OS_THREADS = 256;

// Ordering without cache-maintenance fences (a system-scope release / acquire pair wrote back and invalidated
// the whole L2 in every block: ~14 us per call at world 1, whatever the size): every payload byte moves with
// system-coherent write-through / cache-bypassing 16-byte buffer accesses (sc0 sc1), so (a) a storing wave's
// s_waitcnt vmcnt(0) means its pushes are performed at the destination before its block raises a flag
// (relaxed system-scope atomic store, also sc0 sc1), and (b) the receive slots are read with sc0 sc1 loads after
// the flag poll, which no cache line can serve stale -- the LLVM AMDGPU memory model's release / acquire minus
// the L2 write-back / invalidate that only non-coherent accesses need (MI355X_MICROARCH.md, visibility: "sc1
// stores and loads in place of the release and the acquire").
constexpr int SYS = 17;  // buffer-instruction cache policy: sc0 | sc1 (system coherent)
typedef __attribute__((address_space(1))) uint32_t gu32;  // flags: global (not flat) accesses
constexpr int RSRC3 = 0x00020000;  // raw buffer descriptor word 3 (32-bit data, untyped)
DEV __amdgpu_buffer_rsrc_t rsrc(const void* base, int bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, bytes, RSRC3);
}

__global__ __launch_bounds__(OS_THREADS) void oneshot_allreduce_kernel(OneShotArgs a) {
  const int b = blockIdx.x, nblk = gridDim.x, tid = threadIdx.x;
  const int nv = a.count >> 2;                       // float4 elements
  const int per = (nv + nblk - 1) / nblk;            // float4 per block
  const int v0 = b * per, v1 = min(nv, v0 + per);
  unsigned long long* st = a.stamps ? a.stamps + (size_t)b * 4 : nullptr;
  __shared__ uint32_t s_seq;
  __shared__ int s_fail;
  if (tid == 0) {
    if (st) st[0] = wall_clock64();
    s_fail = __hip_atomic_load((gu32*)a.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u;
    s_seq = a.seq[b] + 1u;
  }
  __syncthreads();
  if (s_fail) return;  // a previous call timed out: latched, this call does nothing (see the header)
  const uint32_t s = s_seq;
  const int par = s & 1;
  const int slot_bytes = a.max_count * 4;
  // 1. push this block's slice into slot [rank] of every rank's receive buffer
  for (int q = 0; q < a.world; ++q) {
    const float* slot = a.peer_data[q] + ((size_t)par * a.world + a.rank) * a.max_count;
    const __amdgpu_buffer_rsrc_t r = rsrc(slot, slot_bytes);
    for (int v = v0 + tid; v < v1; v += OS_THREADS)
      __builtin_amdgcn_raw_buffer_store_b128(reinterpret_cast<const u32x4*>(a.buf)[v], r, v * 16, 0, SYS);
    if (b == 0 && tid < (a.count & 3)) {  // tail (count % 4) by block 0
      const int e = (nv << 2) + tid;
      __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, a.buf[e]), r, e * 4, 0, SYS);
    }
  }
  // every storing wave's pushes are performed before the block's flags are raised
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (st && tid == 0) st[1] = wall_clock64();
  if (tid < a.world) {
    __hip_atomic_store((gu32*)(a.peer_flags[tid] + (size_t)a.rank * nblk + b), s, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_SYSTEM);
  }
  // 2. wait for every rank's flag of this block (lane r polls source rank r), bounded
  if (tid < a.world) {
    gu32* f = (gu32*)(a.peer_flags[a.rank] + (size_t)tid * nblk + b);
    const unsigned long long t0 = wall_clock64();
    while (__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) < s) {
      if (wall_clock64() - t0 > a.timeout_ticks) {
        __hip_atomic_store((gu32*)a.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        s_fail = 1;
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
  }
  __syncthreads();
  if (st && tid == 0) st[2] = wall_clock64();
  if (s_fail) return;  // no sum from missing slots: the update kernels skip on the latched word
  // 3. sum the W slots of the own receive buffer in rank order
  const float* rb = a.peer_data[a.rank] + (size_t)par * a.world * a.max_count;
  const __amdgpu_buffer_rsrc_t rr = rsrc(rb, a.world * slot_bytes);
  for (int v = v0 + tid; v < v1; v += OS_THREADS) {
    f32x4 acc = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rr, v * 16, 0, SYS));
    for (int r = 1; r < a.world; ++r)
      acc += __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rr, r * slot_bytes + v * 16, 0, SYS));
    reinterpret_cast<f32x4*>(a.buf)[v] = acc;
  }
  if (b == 0 && tid < (a.count & 3)) {
    const int e = (nv << 2) + tid;
    float acc = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rr, e * 4, 0, SYS));
    for (int r = 1; r < a.world; ++r)
      acc += __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rr, r * slot_bytes + e * 4, 0, SYS));
    a.buf[e] = acc;
  }
  if (tid == 0) {
    a.seq[b] = s;
    if (st) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      st[3] = wall_clock64();
    }
  }
}

}  // namespace

void launch_oneshot_allreduce(float* buf, int count, int rank, int world, int max_count, float* const* peer_data,
                              uint32_t* const* peer_flags, uint32_t* seq, uint32_t* err, int nblk,
                              unsigned long long timeout_ticks, hipStream_t s, unsigned long long* stamps) {
  OneShotArgs a{buf, count, rank, world, max_count, peer_data, peer_flags, seq, err, timeout_ticks, stamps};
  hipLaunchKernelGGL(oneshot_allreduce_kernel, dim3(nblk), dim3(OS_THREADS), 0, s, a);
}
