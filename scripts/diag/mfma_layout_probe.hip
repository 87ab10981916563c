// Empirical operand layout of v_mfma_f32_16x16x16_bf16 on gfx950: for two hypotheses of which k each lane's
// 4 values carry, run one MFMA on bf16-exact inputs and compare with the host product.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cmath>
#include <cstdlib>
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(4))) short s16x4;

__device__ short bf(float x) { unsigned u = __builtin_bit_cast(unsigned, x); return (short)(u >> 16); }

__global__ void probe(const float* A, const float* B, float* C, int hyp) {
  const int l = threadIdx.x, r = l & 15, g = l >> 4;
  s16x4 a, b;
  for (int j = 0; j < 4; ++j) {
    const int k = hyp == 0 ? 4 * g + j : g + 4 * j;
    a[j] = bf(A[r * 16 + k]);
    b[j] = bf(B[r * 16 + k]);
  }
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  acc = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a, b, acc, 0, 0, 0);
  for (int i = 0; i < 4; ++i) C[(4 * g + i) * 16 + r] = acc[i];
}

int main() {
  float hA[256], hB[256], hC[256];
  srand(2);
  for (int i = 0; i < 256; ++i) {  // bf16-exact values
    hA[i] = (float)((rand() % 17) - 8) / 8.f;
    hB[i] = (float)((rand() % 17) - 8) / 8.f;
  }
  float *dA, *dB, *dC;
  (void)hipMalloc(&dA, 1024); (void)hipMalloc(&dB, 1024); (void)hipMalloc(&dC, 1024);
  (void)hipMemcpy(dA, hA, 1024, hipMemcpyHostToDevice); (void)hipMemcpy(dB, hB, 1024, hipMemcpyHostToDevice);
  for (int hyp = 0; hyp < 2; ++hyp) {
    hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, dA, dB, dC, hyp);
    (void)hipMemcpy(hC, dC, 1024, hipMemcpyDeviceToHost);
    double e = 0, et = 0;
    for (int m = 0; m < 16; ++m)
      for (int n = 0; n < 16; ++n) {
        double ref = 0, reft = 0;
        for (int k = 0; k < 16; ++k) { ref += hA[m * 16 + k] * hB[n * 16 + k]; }
        e = fmax(e, fabs(ref - hC[m * 16 + n]));
        for (int k = 0; k < 16; ++k) { reft += hA[n * 16 + k] * hB[m * 16 + k]; }  // transposed C
        et = fmax(et, fabs(reft - hC[m * 16 + n]));
      }
    printf("hypothesis %d (%s): max err %.3e  (transposed-C err %.3e)\n", hyp, hyp == 0 ? "k = 4g + j" : "k = g + 4j", e, et);
  }
  return 0;
}
