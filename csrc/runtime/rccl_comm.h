// Native RCCL communicator (the GPU data plane of the DDP gradient exchange).
//
// Replaces c10d ProcessGroupNCCL as used by the reference (ddp_tutorial_multi_gpu.py:133-134,
// DDP Reducer all-reduce per step; survey B1/N10).  One communicator per process/GPU; the
// 128-byte ncclUniqueId is produced by rank 0 and exchanged through the control-plane TCP
// store (parallel/comm.py).  Collectives are enqueued on caller-provided HIP streams so they
// can be overlapped with backward kernels and captured into the step's hipGraph.
//
// Failure handling (survey §5.3):
//   * bring-up is BOUNDED: the communicator is created non-blocking (ncclCommInitRankConfig,
//     config.blocking = 0) and its state is polled (ncclCommGetAsyncError) against a deadline; a rank
//     whose peers never arrive aborts the half-built communicator and throws "rank r: ... init did
//     not complete within T s" instead of hanging the whole job inside ncclCommInitRank;
//   * ncclCommGetAsyncError polling with a deadline on every host wait, then ncclCommAbort;
//   * destroy(): ncclCommFinalize (flush, polled against the deadline) -> ncclCommDestroy, called
//     in a fixed order at teardown (DistContext.finalize), abort if the flush does not complete.
#pragma once
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <functional>
#include <string>
#include <vector>

class RcclComm {
 public:
  static std::string make_unique_id();  // 128 raw bytes
  // init_timeout_s <= 0: no deadline.  MNIST_AMD_RCCL_BLOCKING=1 selects the blocking ncclCommInitRank
  // (escape hatch; unbounded).
  RcclComm(const std::string& uid, int rank, int world, int device, double init_timeout_s = 180.0);
  ~RcclComm();
  RcclComm(const RcclComm&) = delete;
  RcclComm& operator=(const RcclComm&) = delete;

  void all_reduce_sum_f32(float* buf, size_t count, hipStream_t s);
  void broadcast_f32(float* buf, size_t count, int root, hipStream_t s);
  void all_reduce_max_f64(double* buf, size_t count, hipStream_t s);
  // Latency of ONE sum all-reduce of `count` floats at `buf`, as the step graph issues it: `per_graph` calls are
  // captured back to back into one hipGraph (so the host's graph-launch rate, ~10 us per replay, does not set the
  // figure), replayed `warmup` + `iters` times on `s`; returns the `iters` per-call times in ms (events between
  // replays / per_graph).  Collective: every rank must call it with the same count, in the same order.  Waits
  // through wait_stream (throws on an RCCL error / timeout).
  std::vector<float> time_all_reduce(float* buf, size_t count, int warmup, int iters, hipStream_t s,
                                     double timeout_s, int per_graph = 1);
  // Capture probe of the pattern the SPLIT plan was built to avoid (ROCm 7.0 segfaulted in hipStreamEndCapture on a
  // related form): inside ONE captured graph a side stream runs the all-reduce, a THIRD stream waits on an event
  // recorded behind it and runs a kernel, the capturing stream joins that stream; the graph is instantiated and
  // replayed `replays` times.  Returns "" or what failed.  Collective (every rank, same count).
  std::string probe_cross_stream_capture(float* buf, size_t count, hipStream_t s, int replays, double timeout_s);
  // Returns "" if healthy, else the error string.  Non-blocking.
  std::string async_error();
  // Wait for `s` with async-error polling: "" once it drains, else the RCCL error or "timeout after …".
  // Does not abort: the caller decides (NativeTrainer.synchronize aborts, then raises).
  std::string wait_stream(hipStream_t s, double timeout_s);
  void abort();
  // Orderly teardown: flush (ncclCommFinalize, polled against `timeout_s`), then ncclCommDestroy.  On a
  // flush timeout / error the communicator is aborted instead.  Idempotent; the destructor calls it.
  // Returns "" or what went wrong.
  std::string destroy(double timeout_s);
  int rank() const { return rank_; }
  int world() const { return world_; }
  bool aborted() const { return aborted_; }
  bool destroyed() const { return comm_ == nullptr; }
  bool nonblocking() const { return nonblocking_; }
  double init_seconds() const { return init_s_; }
  static int version();

  // Deadline poll of an asynchronous RCCL state (init, finalize, a non-blocking enqueue): calls `query`
  // until it returns something other than ncclInProgress or `timeout_s` passes (<= 0: no deadline).
  // Returns the last status (ncclInProgress = timed out) and the seconds waited.  Static and
  // communicator-free, so the bounded-failure logic is testable without a GPU (tests/test_comm_init.py).
  static ncclResult_t poll_ready(const std::function<ncclResult_t()>& query, double timeout_s, double* waited_s);
  // What the constructor does with the poll result: "" on success, else the message it throws (the
  // `abort` callback has been run on a timeout / error).  Exposed for the fake-communicator test.
  static std::string init_outcome(ncclResult_t st, int rank, int world, double timeout_s, double waited_s,
                                  const std::function<void()>& abort);

 private:
  // a non-blocking call returned ncclInProgress: wait (deadline) until the communicator is ready again
  void settle(ncclResult_t r, const char* what);

  ncclComm_t comm_ = nullptr;
  int rank_, world_;
  bool aborted_ = false;
  bool nonblocking_ = false;
  double init_s_ = 0.0;
  double op_timeout_s_ = 600.0;
};
