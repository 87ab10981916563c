// Gradient reduction, optimizer and operand packing kernels.
//
//  reduce_slabs : grad[p] = scale * sum_s slab[s][p] in a FIXED order (bitwise reproducible,
//                 no float atomics).  Replaces the per-parameter .grad accumulation + the DDP
//                 Reducer's bucket copy (survey N6/N9); `scale` carries the 1/B of the mean loss.
//  sgd_pack     : p -= lr * (mu*buf + g/W) over the flat fp32 master slab (torch SGD semantics,
//                 dampening 0, ddp_tutorial_cpu.py:61), 1/W of DDP averaging folded in, then the
//                 updated value is re-packed into the compute-dtype MFMA operand images
//                 (models.h) and the device step counters are advanced.  Replaces the
//                 _foreach_add_ multi-tensor apply (survey K15) plus any weight cast kernels.
#include <algorithm>
#include <type_traits>

#include "common.h"
#include "launch.h"
#include "models.h"

namespace {

// Wave w's share of sum_s slab[s][p]: rows [w*per, (w+1)*per), eight independent loads in flight
// per lane.  Shared by both reduce kernels so the fused single-GPU step and the reduce -> all-reduce
// -> SGD path produce bitwise-identical gradients.
constexpr int RNW = 16;  // waves per reduce block, for every slab count (keeps the tree fixed)

__device__ __forceinline__ float slab_partial(const float* __restrict__ slab, int ld, int nslab, int p, int w) {
  const int per = (nslab + RNW - 1) / RNW;
  const int sb = w * per, se = min(nslab, sb + per);
  int k = sb;
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  // 32 rows per round, all loads issued before the first add (the 512-row conv slab is one round per
  // wave instead of four dependent ones); same per-accumulator addition order as the 8-row loop below
  for (; k + 32 <= se; k += 32) {
    float v[32];
#pragma unroll
    for (int i = 0; i < 32; ++i) v[i] = slab[(size_t)(k + i) * ld + p];
#pragma unroll
    for (int g = 0; g < 4; ++g)
#pragma unroll
      for (int i = 0; i < 8; ++i) acc[i] += v[g * 8 + i];
  }
  for (; k + 8 <= se; k += 8) {
    float v[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = slab[(size_t)(k + i) * ld + p];
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[i] += v[i];
  }
  for (; k < se; ++k) acc[0] += slab[(size_t)k * ld + p];
  return ((acc[0] + acc[1]) + (acc[2] + acc[3])) + ((acc[4] + acc[5]) + (acc[6] + acc[7]));
}

// Slab counts up to DIRECT_MAX (the FC head's split-K slabs: 16 at B = 8192) are summed by ONE lane
// per parameter: no LDS, no cross-wave step, so the kernel fits beside conv_bwd, whose two
// workgroups per CU leave < 5 KB of LDS free (the LDS version of the FC update waited for CUs and
// stretched from ~5 to ~48 us on the aux stream).  Every path (fused or not) uses the same tree for
// a given slab count, so schedules stay bitwise equal.
constexpr int DIRECT_MAX = 64;

__device__ __forceinline__ float slab_sum_direct(const float* __restrict__ slab, int ld, int nslab, int p) {
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  int k = 0;
  for (; k + 8 <= nslab; k += 8) {
    float v[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = slab[(size_t)(k + i) * ld + p];
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[i] += v[i];
  }
  for (; k < nslab; ++k) acc[0] += slab[(size_t)k * ld + p];
  return 0.f + (((acc[0] + acc[1]) + (acc[2] + acc[3])) + ((acc[4] + acc[5]) + (acc[6] + acc[7])));
}

// One block = 64 consecutive parameters (lane) x RNW waves splitting the slab rows; the per-wave
// partial sums are combined in a fixed tree, so the result is bitwise reproducible.
template <int NW>
__global__ __launch_bounds__(NW * 64) void reduce_slabs_kernel(const float* __restrict__ slab, int ld, int nslab,
                                                               int p0, int p1, float scale, float* __restrict__ grad) {
  __shared__ float part[NW][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int p = p0 + blockIdx.x * 64 + lane;
  float s = 0.f;
  if (p < p1) {
    s = slab_partial(slab, ld, nslab, p, w);
  }
  part[w][lane] = s;
  __syncthreads();
  if (w == 0 && p < p1) {
    float t = 0.f;
#pragma unroll
    for (int i = 0; i < NW; ++i) t += part[i][lane];
    grad[p] = t * scale;
  }
}

__global__ __launch_bounds__(256) void reduce_direct_kernel(const float* __restrict__ slab, int ld, int nslab, int p0,
                                                            int p1, float scale, float* __restrict__ grad) {
  const int p = p0 + blockIdx.x * 256 + threadIdx.x;
  if (p < p1) grad[p] = slab_sum_direct(slab, ld, nslab, p) * scale;
}

template <class Model, typename T>
__global__ __launch_bounds__(256) void sgd_pack_kernel(float* __restrict__ params, const float* __restrict__ grad,
                                                       float* __restrict__ mom, T* __restrict__ pack, int p0, int n,
                                                       float lr, float mu, float gscale, int32_t* step_ptr,
                                                       int update, const uint32_t* skip) {
  // a latched collective failure (skip != 0): keep the parameters, re-pack them unchanged
  const bool upd = update && !(skip && __hip_atomic_load(const_cast<uint32_t*>(skip), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
  for (int p = p0 + blockIdx.x * blockDim.x + threadIdx.x; p < n; p += gridDim.x * blockDim.x) {
    float v = params[p];
    if (upd) {
      float g = grad[p] * gscale;
      if (mom) {
        const float b = mu * mom[p] + g;
        mom[p] = b;
        g = b;
      }
      v = v - lr * g;
      params[p] = v;
    }
    Packer<Model, T>::pack(p, v, pack);
  }
  if (update && step_ptr && blockIdx.x == 0 && threadIdx.x == 0) {
    step_ptr[0] += 1;  // step within epoch (batch addressing)
    step_ptr[1] += 1;  // global step (dropout stream)
  }
}

// Fused  grad = scale * sum_s slab[s]  ->  SGD(+momentum)  ->  re-pack, for runs without a gradient
// all-reduce (one GPU): saves two kernel boundaries and the grad round trip per step.  Parameters
// [p0, n): below `split` from slab_a, the rest from slab_b (LeNet: conv slab / FC slab; the concurrent
// schedule updates the FC range right after the FC wgrad, the conv range after conv_bwd).  One block = 64
// parameters x NW waves over the slab rows (same fixed summation tree as reduce_slabs_kernel).
template <class Model, typename T, int NW>
__global__ __launch_bounds__(NW * 64) void reduce_sgd_kernel(const float* __restrict__ slab_a, int lda, int na,
                                                             const float* __restrict__ slab_b, int ldb, int nb,
                                                             int split, int p0, int n, float scale, float* __restrict__ params,
                                                             float* __restrict__ grad, float* __restrict__ mom,
                                                             T* __restrict__ pack, float lr, float mu,
                                                             int32_t* step_ptr) {
  __shared__ float part[NW][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int p = p0 + blockIdx.x * 64 + lane;
  // the update's operands first: their latency overlaps the slab loads instead of following the reduction
  float pv = 0.f, mv = 0.f;
  if (w == 0 && p < n) {
    pv = params[p];
    if (mom) mv = mom[p];
  }
  float s = 0.f;
  if (p < n) {
    const bool a = p < split;
    const float* sl = a ? slab_a : slab_b;
    const int ld = a ? lda : ldb, ns = a ? na : nb;
    if (ns <= DIRECT_MAX) s = w == 0 ? slab_sum_direct(sl, ld, ns, p) : 0.f;  // same tree as the direct kernels
    else s = slab_partial(sl, ld, ns, p, w);
  }
  part[w][lane] = s;
  __syncthreads();
  if (w == 0 && p < n) {
    float g = 0.f;
#pragma unroll
    for (int i = 0; i < NW; ++i) g += part[i][lane];
    g *= scale;
    grad[p] = g;
    if (mom) {
      const float b = mu * mv + g;
      mom[p] = b;
      g = b;
    }
    const float v = pv - lr * g;
    params[p] = v;
    Packer<Model, T>::pack(p, v, pack);
  }
  if (step_ptr && blockIdx.x == 0 && threadIdx.x == 0) {
    step_ptr[0] += 1;
    step_ptr[1] += 1;
  }
}

// Fused reduce + SGD + pack of a parameter range whose slab count is <= DIRECT_MAX: no LDS.  Block size rd_block:
// the MLP (its update alone on the chip, after the weight gradient) takes one-wave blocks -- bf16 B=8192
// 0.0312-0.0315 vs 0.0314-0.0317 ms with 256-thread blocks, bitwise equal; LeNet's FC update, which runs beside
// conv_bwd, keeps 256 (one-wave blocks: 0.0971-0.0972 vs 0.0969-0.0971 ms); profiles/r6_session1/ab_reduce_direct_block.txt
template <class Model>
constexpr int rd_block() { return std::is_same<Model, MlpModel>::value ? 64 : 256; }
template <class Model, typename T>
__global__ __launch_bounds__(rd_block<Model>()) void reduce_sgd_direct_kernel(const float* __restrict__ slab, int ld, int ns, int p0,
                                                                int n, float scale, float* __restrict__ params,
                                                                float* __restrict__ grad, float* __restrict__ mom,
                                                                T* __restrict__ pack, float lr, float mu,
                                                                int32_t* step_ptr) {
  const int p = p0 + blockIdx.x * rd_block<Model>() + threadIdx.x;
  if (p < n) {
    const float pv = params[p], mv = mom ? mom[p] : 0.f;  // issued with the slab loads
    float g = slab_sum_direct(slab, ld, ns, p) * scale;
    grad[p] = g;
    if (mom) {
      const float b = mu * mv + g;
      mom[p] = b;
      g = b;
    }
    const float v = pv - lr * g;
    params[p] = v;
    Packer<Model, T>::pack(p, v, pack);
  }
  if (step_ptr && blockIdx.x == 0 && threadIdx.x == 0) {
    step_ptr[0] += 1;
    step_ptr[1] += 1;
  }
}

template <class Model, typename T>
void reduce_sgd_t(const float* sa, int lda, int na, const float* sb, int ldb, int nb, int split, int p0, int n, float scale,
                  float* params, float* grad, float* mom, void* pack, float lr, float mu, int32_t* step_ptr,
                  hipStream_t s) {
  if (n <= p0) return;
  const bool only_b = p0 >= split, only_a = n <= split;
  if ((only_b && nb <= DIRECT_MAX) || (only_a && na <= DIRECT_MAX)) {
    constexpr int RB = rd_block<Model>();
    hipLaunchKernelGGL((reduce_sgd_direct_kernel<Model, T>), dim3((n - p0 + RB - 1) / RB), dim3(RB), 0, s,
                       only_b ? sb : sa, only_b ? ldb : lda, only_b ? nb : na, p0, n, scale, params, grad, mom,
                       reinterpret_cast<T*>(pack), lr, mu, step_ptr);
    return;
  }
  const int grid = (n - p0 + 63) / 64;
  hipLaunchKernelGGL((reduce_sgd_kernel<Model, T, RNW>), dim3(grid), dim3(RNW * 64), 0, s, sa, lda, na, sb, ldb, nb, split,
                     p0, n, scale, params, grad, mom, reinterpret_cast<T*>(pack), lr, mu, step_ptr);
}

template <class Model, typename T>
void sgd_launch(float* params, const float* grad, float* mom, void* pack, int p0, int n, float lr, float mu,
                float gscale, int32_t* step_ptr, int update, hipStream_t s, const uint32_t* skip = nullptr) {
  const int grid = std::max(1, std::min(1024, (n - p0 + 255) / 256));
  hipLaunchKernelGGL((sgd_pack_kernel<Model, T>), dim3(grid), dim3(256), 0, s, params, grad, mom,
                     reinterpret_cast<T*>(pack), p0, n, lr, mu, gscale, step_ptr, update, skip);
}

// Bounded busy wait of `ticks` periods of the 100 MHz wall clock (one lane; tests of the collective
// watchdog use it to hold a stream busy for a known time).  Every wave exits once the deadline passes.
__global__ void spin_kernel(unsigned long long ticks) {
  const unsigned long long t0 = wall_clock64();
  while (wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(127);
}

template <typename T>
__global__ __launch_bounds__(256) void gather_normalize_kernel(BatchRef br, T* out, int ld) {
  const int r = blockIdx.x;
  if (r >= br.B) return;
  const int32_t* idx = br.idx_epoch + (size_t)br.step_ptr[0] * br.batch_stride;
  const uint8_t* img = br.images + (size_t)idx[r] * 784;
  for (int k = threadIdx.x; k < 784; k += blockDim.x) out[(size_t)r * ld + k] = to_t<T>(mnist_norm(img[k]));
}

}  // namespace

void launch_reduce(const float* slab, int slab_ld, int nslab, int p0, int p1, float scale, float* grad,
                   hipStream_t s) {
  if (p1 <= p0) return;
  if (nslab <= DIRECT_MAX) {
    hipLaunchKernelGGL(reduce_direct_kernel, dim3((p1 - p0 + 255) / 256), dim3(256), 0, s, slab, slab_ld, nslab, p0, p1,
                       scale, grad);
    return;
  }
  const int grid = (p1 - p0 + 63) / 64;
  hipLaunchKernelGGL(reduce_slabs_kernel<RNW>, dim3(grid), dim3(RNW * 64), 0, s, slab, slab_ld, nslab, p0, p1, scale,
                     grad);
}

void launch_sgd_pack_range(ModelKind m, DType t, float* params, const float* grad, float* mom, void* pack, int p0,
                           int p1, float lr, float momentum, float gscale, int32_t* step_ptr, hipStream_t s,
                           const uint32_t* skip) {
  if (p1 <= p0) return;
  float* mb = momentum != 0.f ? mom : nullptr;
  if (m == ModelKind::MLP) {
    if (t == DType::F32) sgd_launch<MlpModel, float>(params, grad, mb, pack, p0, p1, lr, momentum, gscale, step_ptr, 1, s, skip);
    else sgd_launch<MlpModel, bf16>(params, grad, mb, pack, p0, p1, lr, momentum, gscale, step_ptr, 1, s, skip);
  } else {
    if (t == DType::F32) sgd_launch<LenetModel, float>(params, grad, mb, pack, p0, p1, lr, momentum, gscale, step_ptr, 1, s, skip);
    else sgd_launch<LenetModel, bf16>(params, grad, mb, pack, p0, p1, lr, momentum, gscale, step_ptr, 1, s, skip);
  }
}

void launch_sgd_pack(ModelKind m, DType t, float* params, const float* grad, float* mom, void* pack, int nparam,
                     float lr, float momentum, float gscale, int32_t* step_ptr, hipStream_t s, const uint32_t* skip) {
  launch_sgd_pack_range(m, t, params, grad, mom, pack, 0, nparam, lr, momentum, gscale, step_ptr, s, skip);
}

void launch_spin(double seconds, hipStream_t s) {
  const unsigned long long ticks = (unsigned long long)(seconds * 1e8);  // wall_clock64 runs at 100 MHz
  hipLaunchKernelGGL(spin_kernel, dim3(1), dim3(64), 0, s, ticks);
}

void launch_pack(ModelKind m, DType t, const float* params, void* pack, int nparam, hipStream_t s) {
  float* p = const_cast<float*>(params);
  if (m == ModelKind::MLP) {
    if (t == DType::F32) sgd_launch<MlpModel, float>(p, nullptr, nullptr, pack, 0, nparam, 0.f, 0.f, 0.f, nullptr, 0, s);
    else sgd_launch<MlpModel, bf16>(p, nullptr, nullptr, pack, 0, nparam, 0.f, 0.f, 0.f, nullptr, 0, s);
  } else {
    if (t == DType::F32) sgd_launch<LenetModel, float>(p, nullptr, nullptr, pack, 0, nparam, 0.f, 0.f, 0.f, nullptr, 0, s);
    else sgd_launch<LenetModel, bf16>(p, nullptr, nullptr, pack, 0, nparam, 0.f, 0.f, 0.f, nullptr, 0, s);
  }
}

void launch_gather_normalize(DType t, const BatchRef& br, void* out, int ld, hipStream_t s) {
  if (br.B <= 0) return;
  if (t == DType::F32)
    hipLaunchKernelGGL(gather_normalize_kernel<float>, dim3(br.B), dim3(256), 0, s, br, reinterpret_cast<float*>(out), ld);
  else
    hipLaunchKernelGGL(gather_normalize_kernel<bf16>, dim3(br.B), dim3(256), 0, s, br, reinterpret_cast<bf16*>(out), ld);
}

int model_nparam(ModelKind m) { return m == ModelKind::MLP ? MlpModel::NPARAM : LenetModel::NPARAM; }
int model_conv_params(ModelKind m) { return m == ModelKind::MLP ? 0 : LenetModel::CONV_PARAMS; }
int model_phase_split(ModelKind m) { return m == ModelKind::MLP ? MlpModel::Head::W2 : LenetModel::CONV_PARAMS; }
int model_pack_size(ModelKind m) { return m == ModelKind::MLP ? MlpModel::PACK_SIZE : LenetModel::PACK_SIZE; }
int model_job_begin(ModelKind m, int job) {
  if (m == ModelKind::MLP) {
    using H = MlpModel::Head;
    const int b[4] = {H::W1, H::W2, H::W3, MlpModel::NPARAM};
    return b[std::min(std::max(job, 0), 3)];
  }
  using H = LenetModel::Head;
  const int b[4] = {H::W1, H::W2, H::W3, LenetModel::NPARAM};
  return b[std::min(std::max(job, 0), 3)];
}

void launch_reduce_sgd(ModelKind m, DType t, const float* slab_a, int lda, int na, const float* slab_b, int ldb,
                       int nb, int split, int p0, int n, float scale, float* params, float* grad, float* mom,
                       void* pack, float lr, float momentum, int32_t* step_ptr, hipStream_t s) {
  float* mb = momentum != 0.f ? mom : nullptr;
  if (m == ModelKind::MLP) {
    if (t == DType::F32) reduce_sgd_t<MlpModel, float>(slab_a, lda, na, slab_b, ldb, nb, split, p0, n, scale, params, grad, mb, pack, lr, momentum, step_ptr, s);
    else reduce_sgd_t<MlpModel, bf16>(slab_a, lda, na, slab_b, ldb, nb, split, p0, n, scale, params, grad, mb, pack, lr, momentum, step_ptr, s);
  } else {
    if (t == DType::F32) reduce_sgd_t<LenetModel, float>(slab_a, lda, na, slab_b, ldb, nb, split, p0, n, scale, params, grad, mb, pack, lr, momentum, step_ptr, s);
    else reduce_sgd_t<LenetModel, bf16>(slab_a, lda, na, slab_b, ldb, nb, split, p0, n, scale, params, grad, mb, pack, lr, momentum, step_ptr, s);
  }
}
