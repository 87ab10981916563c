// Issue rate of the MFMA forms an fp32-as-bf16-parts GEMM could use, on ONE SIMD (one wave per workgroup, one
// workgroup): v_mfma_f32_16x16x4_f32 (exact fp32, K = 4), v_mfma_f32_16x16x16_bf16 (K = 16, the lane layout of the
// fp32 K-chunk), v_mfma_f32_16x16x32_bf16 (K = 32).  Four independent accumulators, 4096 instructions each form;
// cycles from s_memtime (the shader clock).  Decides whether pre-split bf16 operand images could beat exact fp32:
// a 16-k fp32 chunk is 4 x 16x16x4 f32 = 4 c(f32); its 6-term split is 6 x c(16x16x16) or, with 32-k chunks,
// 6 x c(16x16x32) per 2 chunks.
// Build: hipcc --offload-arch=gfx950 -O3 -o /tmp/mfma_rate scripts/diag/mfma_rate.hip
#include <hip/hip_runtime.h>
#include <cstdio>

typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(4))) short s16x4;
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;

constexpr int N = 1024;  // iterations x 4 accumulators

__global__ void k_f32(float a, float b, float* out, long long* cyc) {
  f32x4 c0{}, c1{}, c2{}, c3{};
  const long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < N; ++i) {
    c0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c0, 0, 0, 0);
    c1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c1, 0, 0, 0);
    c2 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c2, 0, 0, 0);
    c3 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c3, 0, 0, 0);
  }
  const long long t1 = __builtin_amdgcn_s_memtime();
  out[threadIdx.x] = (c0 + c1 + c2 + c3).x;
  if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

__global__ void k_bf16_16(s16x4 a, s16x4 b, float* out, long long* cyc) {
  f32x4 c0{}, c1{}, c2{}, c3{};
  const long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < N; ++i) {
    c0 = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a, b, c0, 0, 0, 0);
    c1 = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a, b, c1, 0, 0, 0);
    c2 = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a, b, c2, 0, 0, 0);
    c3 = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a, b, c3, 0, 0, 0);
  }
  const long long t1 = __builtin_amdgcn_s_memtime();
  out[threadIdx.x] = (c0 + c1 + c2 + c3).x;
  if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

__global__ void k_bf16_32(bf16x8 a, bf16x8 b, float* out, long long* cyc) {
  f32x4 c0{}, c1{}, c2{}, c3{};
  const long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < N; ++i) {
    c0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c0, 0, 0, 0);
    c1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c1, 0, 0, 0);
    c2 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c2, 0, 0, 0);
    c3 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c3, 0, 0, 0);
  }
  const long long t1 = __builtin_amdgcn_s_memtime();
  out[threadIdx.x] = (c0 + c1 + c2 + c3).x;
  if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

int main() {
  float* out;
  long long* cyc;
  if (hipMalloc(&out, 64 * sizeof(float)) != hipSuccess || hipMalloc(&cyc, sizeof(long long)) != hipSuccess) return 1;
  s16x4 a16{0x3f80, 0x3f80, 0x3f80, 0x3f80};
  bf16x8 a32;
  for (int j = 0; j < 8; ++j) a32[j] = (__bf16)1.0f;
  const char* names[3] = {"v_mfma_f32_16x16x4_f32", "v_mfma_f32_16x16x16_bf16", "v_mfma_f32_16x16x32_bf16"};
  for (int rep = 0; rep < 3; ++rep) {
    for (int k = 0; k < 3; ++k) {
      if (k == 0) hipLaunchKernelGGL(k_f32, dim3(1), dim3(64), 0, 0, 1.0f, 1.0f, out, cyc);
      if (k == 1) hipLaunchKernelGGL(k_bf16_16, dim3(1), dim3(64), 0, 0, a16, a16, out, cyc);
      if (k == 2) hipLaunchKernelGGL(k_bf16_32, dim3(1), dim3(64), 0, 0, a32, a32, out, cyc);
      long long c = 0;
      if (hipMemcpy(&c, cyc, sizeof(c), hipMemcpyDeviceToHost) != hipSuccess) return 2;
      // s_memtime counts the 100 MHz reference clock on gfx9.4+; also print per-instruction ns
      if (rep == 2) printf("%-28s %8lld ticks for %d instr  %.3f ticks/instr\n", names[k], c, 4 * N, (double)c / (4 * N));
    }
  }
  return 0;
}
