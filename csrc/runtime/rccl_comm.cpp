#include "rccl_comm.h"

#include <chrono>
#include <cstring>
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

RcclComm::RcclComm(const std::string& uid, int rank, int world, int device) : rank_(rank), world_(world) {
  if (uid.size() != sizeof(ncclUniqueId)) throw std::runtime_error("RcclComm: bad unique id size");
  ncclUniqueId id;
  std::memcpy(&id, uid.data(), sizeof(id));
  HIP_CHECK(hipSetDevice(device));
  NCCL_CHECK(ncclCommInitRank(&comm_, world, id, rank));
}

RcclComm::~RcclComm() {
  if (comm_ && !aborted_) ncclCommDestroy(comm_);
}

void RcclComm::all_reduce_sum_f32(float* buf, size_t count, hipStream_t s) {
  if (count == 0) return;
  NCCL_CHECK(ncclAllReduce(buf, buf, count, ncclFloat32, ncclSum, comm_, s));
}

void RcclComm::broadcast_f32(float* buf, size_t count, int root, hipStream_t s) {
  if (count == 0) return;
  NCCL_CHECK(ncclBroadcast(buf, buf, count, ncclFloat32, root, comm_, s));
}

void RcclComm::all_reduce_max_f64(double* buf, size_t count, hipStream_t s) {
  if (count == 0) return;
  NCCL_CHECK(ncclAllReduce(buf, buf, count, ncclFloat64, ncclMax, comm_, s));
}

std::vector<float> RcclComm::time_all_reduce(float* buf, size_t count, int warmup, int iters, hipStream_t s,
                                             double timeout_s) {
  if (count == 0 || iters <= 0) return {};
  hipGraph_t g = nullptr;
  hipGraphExec_t ge = nullptr;
  HIP_CHECK(hipStreamBeginCapture(s, hipStreamCaptureModeRelaxed));
  ncclResult_t r = ncclAllReduce(buf, buf, count, ncclFloat32, ncclSum, comm_, s);
  HIP_CHECK(hipStreamEndCapture(s, &g));
  if (r != ncclSuccess && r != ncclInProgress) {
    hipGraphDestroy(g);
    NCCL_CHECK(r);
  }
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
    for (int i = 0; i < iters; ++i) HIP_CHECK(hipEventElapsedTime(&out[i], ev[i], ev[i + 1]));
  }
  if (err.empty()) {
    for (auto& e : ev) hipEventDestroy(e);
    hipGraphExecDestroy(ge);
    hipGraphDestroy(g);
  }  // else: the replays may still be in flight -- leak rather than destroy under them; the caller aborts
  if (!err.empty()) throw std::runtime_error("time_all_reduce: " + err);
  return out;
}

std::string RcclComm::async_error() {
  if (!comm_) return "communicator not initialised";
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
    ncclCommAbort(comm_);
    aborted_ = true;
  }
}
