// Fork / join cost between two streams, eager vs captured graph: K1 on s1; fork: K2 on s2 beside K3 on s1; join;
// K4 on s1.  Each kernel holds 20 us on one workgroup, so ideal = 3 x 20 us per iteration, serial = 4 x 20.
//   hipcc --offload-arch=gfx950 -O2 forkjoin_eager.hip -o forkjoin_eager.bin
#include <hip/hip_runtime.h>
#include <cstdio>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

__global__ void hold(unsigned long long ticks, int* out) {
  const unsigned long long t0 = wall_clock64();
  while (wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(8);
  if (threadIdx.x == 0) out[blockIdx.x] = 1;
}

int main() {
  int* buf;
  CK(hipMalloc(&buf, 1024 * sizeof(int)));
  hipStream_t s1, s2;
  CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
  hipEvent_t a, b, f, j;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  CK(hipEventCreateWithFlags(&f, hipEventDisableTiming));
  CK(hipEventCreateWithFlags(&j, hipEventDisableTiming));
  const unsigned long long T = 2000;
  const int N = 40;
  auto body = [&](bool fork) -> int {
    for (int i = 0; i < N; ++i) {
      hipLaunchKernelGGL(hold, dim3(1), dim3(64), 0, s1, T, buf);
      if (fork) {
        CK(hipEventRecord(f, s1));
        CK(hipStreamWaitEvent(s2, f, 0));
        hipLaunchKernelGGL(hold, dim3(1), dim3(64), 0, s2, T, buf + 1);
        CK(hipEventRecord(j, s2));
      } else {
        hipLaunchKernelGGL(hold, dim3(1), dim3(64), 0, s1, T, buf + 1);
      }
      hipLaunchKernelGGL(hold, dim3(1), dim3(64), 0, s1, T, buf + 2);
      if (fork) CK(hipStreamWaitEvent(s1, j, 0));
      hipLaunchKernelGGL(hold, dim3(1), dim3(64), 0, s1, T, buf + 3);
    }
    return 0;
  };
  for (int fork = 0; fork < 2; ++fork) {
    for (int trial = 0; trial < 2; ++trial) {
      CK(hipEventRecord(a, s1));
      if (body(fork)) return 1;
      CK(hipEventRecord(b, s1));
      CK(hipEventSynchronize(b));
      float ms;
      CK(hipEventElapsedTime(&ms, a, b));
      printf("eager fork=%d: %.2f us per iteration (ideal %s)\n", fork, ms * 1000 / N, fork ? "60" : "80");
    }
    hipGraph_t g;
    hipGraphExec_t ge;
    CK(hipStreamBeginCapture(s1, hipStreamCaptureModeGlobal));
    if (body(fork)) return 1;
    CK(hipStreamEndCapture(s1, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    for (int trial = 0; trial < 2; ++trial) {
      CK(hipEventRecord(a, s1));
      CK(hipGraphLaunch(ge, s1));
      CK(hipEventRecord(b, s1));
      CK(hipEventSynchronize(b));
      float ms;
      CK(hipEventElapsedTime(&ms, a, b));
      printf("graph fork=%d: %.2f us per iteration\n", fork, ms * 1000 / N);
    }
    CK(hipGraphExecDestroy(ge));
    CK(hipGraphDestroy(g));
  }
  CK(hipStreamDestroy(s1));
  CK(hipStreamDestroy(s2));
  CK(hipFree(buf));
  return 0;
}
