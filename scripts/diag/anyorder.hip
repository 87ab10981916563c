// Does hipExtAnyOrderLaunch let two kernels of ONE stream overlap on gfx950 (no AQL barrier bit), eagerly and under
// stream capture?  Two 1-workgroup kernels that each hold for T us (bounded wall-clock spin).  Prints per-pair times:
// ~T = they overlapped, ~2T = serialized.   hipcc --offload-arch=gfx950 -O2 anyorder.hip -o anyorder
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

__global__ void hold(unsigned long long ticks, int* out) {
  const unsigned long long t0 = wall_clock64();
  while (wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(8);
  if (threadIdx.x == 0) out[blockIdx.x] = 1;
}

int main() {
  int* buf;
  CK(hipMalloc(&buf, 1024 * sizeof(int)));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  const unsigned long long T = 2000;  // 20 us at 100 MHz
  const int N = 50;
  for (int mode = 0; mode < 2; ++mode) {
    for (int trial = 0; trial < 2; ++trial) {
      CK(hipEventRecord(a, s));
      for (int i = 0; i < N; ++i) {
        hipLaunchKernelGGL(hold, dim3(1), dim3(64), 0, s, T, buf);
        hipExtLaunchKernelGGL(hold, dim3(1), dim3(64), 0, s, nullptr, nullptr, mode ? hipExtAnyOrderLaunch : 0u, T, buf + 1);
      }
      CK(hipEventRecord(b, s));
      CK(hipEventSynchronize(b));
      float ms;
      CK(hipEventElapsedTime(&ms, a, b));
      printf("eager   anyorder=%d: %.2f us per pair (one kernel holds 20 us)\n", mode, ms * 1000 / N);
    }
    // the same pairs captured into a graph
    hipGraph_t g;
    hipGraphExec_t ge;
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
    for (int i = 0; i < N; ++i) {
      hipLaunchKernelGGL(hold, dim3(1), dim3(64), 0, s, T, buf);
      hipExtLaunchKernelGGL(hold, dim3(1), dim3(64), 0, s, nullptr, nullptr, mode ? hipExtAnyOrderLaunch : 0u, T, buf + 1);
    }
    CK(hipStreamEndCapture(s, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    for (int trial = 0; trial < 2; ++trial) {
      CK(hipEventRecord(a, s));
      CK(hipGraphLaunch(ge, s));
      CK(hipEventRecord(b, s));
      CK(hipEventSynchronize(b));
      float ms;
      CK(hipEventElapsedTime(&ms, a, b));
      printf("graph   anyorder=%d: %.2f us per pair\n", mode, ms * 1000 / N);
    }
    CK(hipGraphExecDestroy(ge));
    CK(hipGraphDestroy(g));
  }
  CK(hipStreamDestroy(s));
  CK(hipFree(buf));
  return 0;
}
