// One 16x16 output tile over K = 16 (one fp32 K-chunk of common.h): fp32 MFMA chain vs the split-bf16 form
// (MNIST_AMD_F32_SPLIT), against a host double reference.  hipcc --offload-arch=gfx950 -O3 -DMNIST_AMD_F32_SPLIT
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cmath>
#include <cstdlib>
#include "../../csrc/kernels/common.h"

__global__ void tile(const float* A, const float* B, float* C) {  // A [16][16] row-major (m, k), B [16][16] (n, k)
  const int l = threadIdx.x, row = l & 15, grp = l >> 4;
  Mma<float>::Frag a = Mma<float>::load(A + row * 16 + grp * 4), b = Mma<float>::load(B + row * 16 + grp * 4);
  f32x4 acc = zero4();
  Mma<float>::mma(acc, a, b);
  for (int i = 0; i < 4; ++i) C[(grp * 4 + i) * 16 + row] = acc[i];  // C[m][n]: row = 4 grp + i, col = lane & 15
}

int main() {
  float hA[256], hB[256], hC[256];
  srand(1);
  for (int i = 0; i < 256; ++i) { hA[i] = (rand() / (float)RAND_MAX) * 2 - 1; hB[i] = (rand() / (float)RAND_MAX) * 2 - 1; }
  float *dA, *dB, *dC;
  hipMalloc(&dA, 1024); hipMalloc(&dB, 1024); hipMalloc(&dC, 1024);
  hipMemcpy(dA, hA, 1024, hipMemcpyHostToDevice); hipMemcpy(dB, hB, 1024, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(tile, dim3(1), dim3(64), 0, 0, dA, dB, dC);
  hipMemcpy(hC, dC, 1024, hipMemcpyDeviceToHost);
  double maxerr = 0, maxref = 0;
  for (int m = 0; m < 16; ++m)
    for (int n = 0; n < 16; ++n) {
      double r = 0;
      for (int k = 0; k < 16; ++k) r += (double)hA[m * 16 + k] * hB[n * 16 + k];
      maxerr = fmax(maxerr, fabs(r - hC[m * 16 + n]));
      maxref = fmax(maxref, fabs(r));
    }
  printf("max abs err %.3e  (max |ref| %.3f)  C[0][0]=%f\n", maxerr, maxref, hC[0]);
  return maxerr < 1e-3 * maxref ? 0 : 1;
}
// Build and run (one GPU):  hipcc --offload-arch=gfx950 -O3 -std=c++17 -DMNIST_AMD_F32_SPLIT=2 \
//   scripts/diag/mfma_split_check.hip -o /tmp/split_check && /tmp/split_check
