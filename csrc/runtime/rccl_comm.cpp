#include "rccl_comm.h"

#include "../kernels/launch.h"

#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <future>
#include <memory>
#include <stdexcept>
#include <thread>

#include "hip_check.h"

#define NCCL_CHECK(x)                                                                        \
  do {                                                                                       \
    ncclResult_t r_ = (x);                                                                   \
    if (r_ != ncclSuccess && r_ != ncclInProgress)                                          \
      throw std::runtime_error(std::string("RCCL error: ") + ncclGetErrorString(r_) + " at " \
                               + __FILE__ + ":" + std::to_string(__LINE__));                 \
  } while (0)

namespace {
double env_seconds(const char* name, double def) {
  const char* e = std::getenv(name);
  return e && *e ? std::atof(e) : def;
}
bool env_on(const char* name) {
  const char* e = std::getenv(name);
  return e && *e && *e != '0';
}
// ncclCommAbort with a bound: an abort of a communicator whose bootstrap is still waiting for peers may
// itself wait on sockets.  It runs on a detached thread; after `bound_s` the caller goes on (the thread and
// the half-built communicator are leaked -- the process is about to fail anyway).
void bounded_abort(ncclComm_t c, double bound_s) {
  if (!c) return;
  auto done = std::make_shared<std::promise<void>>();
  std::future<void> f = done->get_future();
  std::thread([c, done] {
    ncclCommAbort(c);
    done->set_value();
  }).detach();
  f.wait_for(std::chrono::duration<double>(bound_s));
}
}  // namespace

std::string RcclComm::make_unique_id() {
  ncclUniqueId id;
  NCCL_CHECK(ncclGetUniqueId(&id));
  return std::string(reinterpret_cast<const char*>(&id), sizeof(id));
}

int RcclComm::version() {
  int v = 0;
  ncclGetVersion(&v);
  return v;
}

ncclResult_t RcclComm::poll_ready(const std::function<ncclResult_t()>& query, double timeout_s, double* waited_s) {
  const auto t0 = std::chrono::steady_clock::now();
  ncclResult_t st = ncclInProgress;
  for (int i = 0;; ++i) {
    st = query();
    const double el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    if (waited_s) *waited_s = el;
    if (st != ncclInProgress) return st;
    if (timeout_s > 0 && el > timeout_s) return ncclInProgress;
    // short sleeps first (a healthy init at W = 8 completes in well under a second), then 1 ms
    std::this_thread::sleep_for(std::chrono::microseconds(i < 200 ? 50 : 1000));
  }
}

std::string RcclComm::init_outcome(ncclResult_t st, int rank, int world, double timeout_s, double waited_s,
                                   const std::function<void()>& abort) {
  if (st == ncclSuccess) return "";
  if (abort) abort();
  if (st == ncclInProgress)
    return "rank " + std::to_string(rank) + " of " + std::to_string(world) +
           ": RCCL communicator init did not complete within " + std::to_string(timeout_s) +
           " s (peers missing or stalled; communicator aborted; MNIST_AMD_COMM_INIT_TIMEOUT sets the deadline)";
  return "rank " + std::to_string(rank) + " of " + std::to_string(world) + ": RCCL communicator init failed after " +
         std::to_string(waited_s) + " s: " + ncclGetErrorString(st) + " (communicator aborted)";
}

RcclComm::RcclComm(const std::string& uid, int rank, int world, int device, double init_timeout_s)
    : rank_(rank), world_(world) {
  if (uid.size() != sizeof(ncclUniqueId)) throw std::runtime_error("RcclComm: bad unique id size");
  op_timeout_s_ = env_seconds("MNIST_AMD_COMM_TIMEOUT", 600.0);
  ncclUniqueId id;
  std::memcpy(&id, uid.data(), sizeof(id));
  HIP_CHECK(hipSetDevice(device));
  const auto t0 = std::chrono::steady_clock::now();
  if (env_on("MNIST_AMD_RCCL_BLOCKING")) {
    NCCL_CHECK(ncclCommInitRank(&comm_, world, id, rank));
  } else {
    ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
    cfg.blocking = 0;
    nonblocking_ = true;
    ncclResult_t r = ncclCommInitRankConfig(&comm_, world, id, rank, &cfg);
    if (r != ncclSuccess && r != ncclInProgress) {
      if (comm_) bounded_abort(comm_, 10.0);
      comm_ = nullptr;
      throw std::runtime_error(init_outcome(r, rank, world, init_timeout_s, 0.0, nullptr));
    }
    double waited = 0.0;
    ncclComm_t c = comm_;
    const ncclResult_t st = poll_ready(
        [c] {
          ncclResult_t e = ncclInProgress;
          if (ncclCommGetAsyncError(c, &e) != ncclSuccess) return ncclInternalError;
          return e;
        },
        init_timeout_s, &waited);
    const std::string err = init_outcome(st, rank, world, init_timeout_s, waited, [c] { bounded_abort(c, 15.0); });
    if (!err.empty()) {
      comm_ = nullptr;
      aborted_ = true;
      throw std::runtime_error(err);
    }
  }
  init_s_ = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
}

RcclComm::~RcclComm() {
  try {
    destroy(op_timeout_s_);
  } catch (...) {
  }
}

void RcclComm::settle(ncclResult_t r, const char* what) {
  NCCL_CHECK(r);
  if (r != ncclInProgress) return;
  // non-blocking communicator: the call is still being enqueued (e.g. the first collective connecting the
  // peers); no further RCCL call on this communicator before it is ready
  double waited = 0.0;
  ncclComm_t c = comm_;
  const ncclResult_t st = poll_ready(
      [c] {
        ncclResult_t e = ncclInProgress;
        if (ncclCommGetAsyncError(c, &e) != ncclSuccess) return ncclInternalError;
        return e;
      },
      op_timeout_s_, &waited);
  if (st == ncclSuccess) return;
  abort();
  throw std::runtime_error("rank " + std::to_string(rank_) + ": RCCL " + what +
                           (st == ncclInProgress ? " did not complete its enqueue within " + std::to_string(op_timeout_s_) + " s"
                                                 : std::string(" failed: ") + ncclGetErrorString(st)) +
                           " (communicator aborted)");
}

void RcclComm::all_reduce_sum_f32(float* buf, size_t count, hipStream_t s) {
  if (count == 0) return;
  if (!comm_) throw std::runtime_error("RcclComm: communicator destroyed / aborted");
  settle(ncclAllReduce(buf, buf, count, ncclFloat32, ncclSum, comm_, s), "all_reduce");
}

void RcclComm::broadcast_f32(float* buf, size_t count, int root, hipStream_t s) {
  if (count == 0) return;
  if (!comm_) throw std::runtime_error("RcclComm: communicator destroyed / aborted");
  settle(ncclBroadcast(buf, buf, count, ncclFloat32, root, comm_, s), "broadcast");
}

void RcclComm::all_reduce_max_f64(double* buf, size_t count, hipStream_t s) {
  if (count == 0) return;
  if (!comm_) throw std::runtime_error("RcclComm: communicator destroyed / aborted");
  settle(ncclAllReduce(buf, buf, count, ncclFloat64, ncclMax, comm_, s), "all_reduce(max)");
}

std::vector<float> RcclComm::time_all_reduce(float* buf, size_t count, int warmup, int iters, hipStream_t s,
                                             double timeout_s, int per_graph) {
  if (count == 0 || iters <= 0) return {};
  if (!comm_) throw std::runtime_error("RcclComm: communicator destroyed / aborted");
  per_graph = std::max(1, per_graph);
  hipGraph_t g = nullptr;
  hipGraphExec_t ge = nullptr;
  HIP_CHECK(hipStreamBeginCapture(s, hipStreamCaptureModeRelaxed));
  ncclResult_t r = ncclSuccess;
  for (int i = 0; i < per_graph && (r == ncclSuccess || r == ncclInProgress); ++i)
    r = ncclAllReduce(buf, buf, count, ncclFloat32, ncclSum, comm_, s);
  HIP_CHECK(hipStreamEndCapture(s, &g));
  if (r != ncclSuccess && r != ncclInProgress) {
    hipGraphDestroy(g);
    NCCL_CHECK(r);
  }
  settle(r, "all_reduce (captured)");
  HIP_CHECK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  std::vector<hipEvent_t> ev(iters + 1);
  for (auto& e : ev) HIP_CHECK(hipEventCreate(&e));
  for (int i = 0; i < warmup; ++i) HIP_CHECK(hipGraphLaunch(ge, s));
  HIP_CHECK(hipEventRecord(ev[0], s));
  for (int i = 0; i < iters; ++i) {
    HIP_CHECK(hipGraphLaunch(ge, s));
    HIP_CHECK(hipEventRecord(ev[i + 1], s));
  }
  const std::string err = wait_stream(s, timeout_s);
  std::vector<float> out;
  if (err.empty()) {
    out.resize(iters);
    for (int i = 0; i < iters; ++i) {
      HIP_CHECK(hipEventElapsedTime(&out[i], ev[i], ev[i + 1]));
      out[i] /= float(per_graph);
    }
  }
  if (err.empty()) {
    for (auto& e : ev) hipEventDestroy(e);
    hipGraphExecDestroy(ge);
    hipGraphDestroy(g);
  }  // else: the replays may still be in flight -- leak rather than destroy under them; the caller aborts
  if (!err.empty()) throw std::runtime_error("time_all_reduce: " + err);
  return out;
}

std::string RcclComm::probe_cross_stream_capture(float* buf, size_t count, hipStream_t s, int replays,
                                                 double timeout_s) {
  if (!comm_) return "communicator destroyed / aborted";
  hipStream_t cs = nullptr, as = nullptr;
  hipEvent_t ev[3] = {nullptr, nullptr, nullptr};
  hipGraph_t g = nullptr;
  hipGraphExec_t ge = nullptr;
  std::string err;
  bool capturing = false;
  try {
    HIP_CHECK(hipStreamCreateWithFlags(&cs, hipStreamNonBlocking));
    HIP_CHECK(hipStreamCreateWithFlags(&as, hipStreamNonBlocking));
    for (auto& e : ev) HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    HIP_CHECK(hipStreamBeginCapture(s, hipStreamCaptureModeRelaxed));
    capturing = true;
    HIP_CHECK(hipEventRecord(ev[0], s));
    HIP_CHECK(hipStreamWaitEvent(cs, ev[0], 0));
    const ncclResult_t r = ncclAllReduce(buf, buf, count, ncclFloat32, ncclSum, comm_, cs);
    if (r != ncclSuccess && r != ncclInProgress) throw std::runtime_error(std::string("ncclAllReduce: ") + ncclGetErrorString(r));
    HIP_CHECK(hipEventRecord(ev[1], cs));          // recorded behind the captured collective ...
    HIP_CHECK(hipStreamWaitEvent(as, ev[1], 0));   // ... and waited on by another stream
    launch_spin(0.0, as);
    HIP_CHECK(hipGetLastError());
    HIP_CHECK(hipEventRecord(ev[2], as));
    HIP_CHECK(hipStreamWaitEvent(s, ev[2], 0));
    capturing = false;
    HIP_CHECK(hipStreamEndCapture(s, &g));
    settle(r, "all_reduce (captured, cross-stream probe)");
    HIP_CHECK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    for (int i = 0; i < replays; ++i) HIP_CHECK(hipGraphLaunch(ge, s));
    err = wait_stream(s, timeout_s);
  } catch (const std::exception& e) {
    err = e.what();
    if (capturing) {
      hipGraph_t g2 = nullptr;
      (void)hipStreamEndCapture(s, &g2);
      if (g2) hipGraphDestroy(g2);
    }
  }
  if (err.empty() || err.find("timeout") == std::string::npos) {  // (a stuck replay is leaked, not destroyed)
    if (ge) hipGraphExecDestroy(ge);
    if (g) hipGraphDestroy(g);
    for (auto& e : ev) if (e) hipEventDestroy(e);
    if (cs) hipStreamDestroy(cs);
    if (as) hipStreamDestroy(as);
  }
  return err;
}

std::string RcclComm::async_error() {
  if (!comm_) return aborted_ ? "communicator aborted" : "communicator destroyed";
  ncclResult_t e = ncclSuccess;
  if (ncclCommGetAsyncError(comm_, &e) != ncclSuccess) return "ncclCommGetAsyncError failed";
  if (e == ncclSuccess || e == ncclInProgress) return "";
  return ncclGetErrorString(e);
}

std::string RcclComm::wait_stream(hipStream_t s, double timeout_s) {
  auto t0 = std::chrono::steady_clock::now();
  for (;;) {
    hipError_t q = hipStreamQuery(s);
    if (q == hipSuccess) return "";
    if (q != hipErrorNotReady) HIP_CHECK(q);
    std::string err = async_error();
    if (!err.empty()) return err;
    double el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    if (timeout_s > 0 && el > timeout_s) return "timeout after " + std::to_string(timeout_s) + " s";
    std::this_thread::sleep_for(std::chrono::microseconds(50));
  }
}

void RcclComm::abort() {
  if (comm_ && !aborted_) {
    ncclComm_t c = comm_;
    comm_ = nullptr;
    aborted_ = true;
    bounded_abort(c, 15.0);
  }
}

std::string RcclComm::destroy(double timeout_s) {
  if (!comm_) return "";
  ncclComm_t c = comm_;
  ncclResult_t r = ncclCommFinalize(c);
  double waited = 0.0;
  if (r == ncclInProgress || (r == ncclSuccess && nonblocking_)) {
    r = poll_ready(
        [c] {
          ncclResult_t e = ncclInProgress;
          if (ncclCommGetAsyncError(c, &e) != ncclSuccess) return ncclInternalError;
          return e;
        },
        timeout_s, &waited);
  }
  if (r != ncclSuccess) {
    abort();
    return r == ncclInProgress ? "finalize did not complete within " + std::to_string(timeout_s) + " s (aborted)"
                               : std::string("finalize failed: ") + ncclGetErrorString(r) + " (aborted)";
  }
  comm_ = nullptr;
  ncclCommDestroy(c);
  return "";
}
