// Native RCCL communicator (the GPU data plane of the DDP gradient exchange).
//
// Replaces c10d ProcessGroupNCCL as used by the reference (ddp_tutorial_multi_gpu.py:133-134,
// DDP Reducer all-reduce per step; survey B1/N10).  One communicator per process/GPU; the
// 128-byte ncclUniqueId is produced by rank 0 and exchanged through the control-plane TCP
// store (parallel/comm.py).  Collectives are enqueued on caller-provided HIP streams so they
// can be overlapped with backward kernels and captured into the step's hipGraph.  Failure
// handling: ncclCommGetAsyncError polling with a deadline, then ncclCommAbort (survey §5.3).
#pragma once
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <string>
#include <vector>

class RcclComm {
 public:
  static std::string make_unique_id();  // 128 raw bytes
  RcclComm(const std::string& uid, int rank, int world, int device);
  ~RcclComm();
  RcclComm(const RcclComm&) = delete;
  RcclComm& operator=(const RcclComm&) = delete;

  void all_reduce_sum_f32(float* buf, size_t count, hipStream_t s);
  void broadcast_f32(float* buf, size_t count, int root, hipStream_t s);
  void all_reduce_max_f64(double* buf, size_t count, hipStream_t s);
  // Latency of ONE sum all-reduce of `count` floats at `buf`, as the step graph issues it: the call is
  // captured into its own hipGraph and replayed `warmup` + `iters` times back to back on `s`; returns the
  // `iters` per-replay times in ms (events between replays).  Collective: every rank must call it with
  // the same count, in the same order.  Waits through wait_stream (throws on an RCCL error / timeout).
  std::vector<float> time_all_reduce(float* buf, size_t count, int warmup, int iters, hipStream_t s,
                                     double timeout_s);
  // Returns "" if healthy, else the error string.  Non-blocking.
  std::string async_error();
  // Wait for `s` with async-error polling: "" once it drains, else the RCCL error or "timeout after …".
  // Does not abort: the caller decides (NativeTrainer.synchronize aborts, then raises).
  std::string wait_stream(hipStream_t s, double timeout_s);
  void abort();
  int rank() const { return rank_; }
  int world() const { return world_; }
  bool aborted() const { return aborted_; }
  static int version();

 private:
  ncclComm_t comm_ = nullptr;
  int rank_, world_;
  bool aborted_ = false;
};
