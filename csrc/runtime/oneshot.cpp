#include "oneshot.h"

#include <cstdio>

#include <cstdlib>
#include <cstring>
#include <stdexcept>

#include "../kernels/launch.h"
#include "hip_check.h"

OneShotAllReduce::OneShotAllReduce(int rank, int world, int device, int max_count, int nblk, double timeout_s)
    : rank_(rank), world_(world), device_(device), max_count_((max_count + 3) / 4 * 4), nblk_(nblk) {
  if (world < 1 || rank < 0 || rank >= world) throw std::invalid_argument("OneShotAllReduce: bad rank / world");
  if (nblk < 1 || max_count < 1) throw std::invalid_argument("OneShotAllReduce: bad sizes");
  timeout_ticks_ = (unsigned long long)(timeout_s * 1e8);  // wall_clock64: 100 MHz
  HIP_CHECK(hipSetDevice(device));
  data_bytes_ = (size_t)2 * world * max_count_ * sizeof(float);
  region_bytes_ = data_bytes_ + (size_t)world * nblk * sizeof(uint32_t);
  // uncached: peers' remote stores land in this HBM and the local reads see them without cache maintenance
  HIP_CHECK(hipExtMallocWithFlags(reinterpret_cast<void**>(&region_), region_bytes_, hipDeviceMallocUncached));
  HIP_CHECK(hipMemset(region_, 0, region_bytes_));
  HIP_CHECK(hipMalloc(&d_data_, world * sizeof(float*)));
  HIP_CHECK(hipMalloc(&d_flags_, world * sizeof(uint32_t*)));
  HIP_CHECK(hipMalloc(&d_local_, (nblk + 1) * sizeof(uint32_t)));
  HIP_CHECK(hipMemset(d_local_, 0, (nblk + 1) * sizeof(uint32_t)));
  HIP_CHECK(hipDeviceSynchronize());
  // test-only fault injection: "rank:call" -- this rank does not issue its call number `call` (0-based), so its
  // peers' flag waits run out (the latched-error path)
  if (const char* e = std::getenv("MNIST_AMD_ONESHOT_SKIP_CALL"); e && *e) {
    int r = -1;
    long long c = -1;
    if (std::sscanf(e, "%d:%lld", &r, &c) == 2 && r == rank_) skip_call_ = c;
  }
  if (world == 1) open_peers({});
}

OneShotAllReduce::~OneShotAllReduce() {
  for (void* p : opened_) (void)hipIpcCloseMemHandle(p);
  if (d_data_) (void)hipFree(d_data_);
  if (d_flags_) (void)hipFree(d_flags_);
  if (d_local_) (void)hipFree(d_local_);
  if (d_stamps_) (void)hipFree(d_stamps_);
  if (region_) (void)hipFree(region_);
}

std::string OneShotAllReduce::handle() const {
  hipIpcMemHandle_t h;
  HIP_CHECK(hipIpcGetMemHandle(&h, region_));
  return std::string(reinterpret_cast<const char*>(&h), sizeof(h));
}

void OneShotAllReduce::open_peers(const std::vector<std::string>& handles) {
  if (ready_) throw std::runtime_error("OneShotAllReduce: peers already opened");
  if (world_ > 1 && (int)handles.size() != world_) throw std::invalid_argument("open_peers: need one handle per rank");
  HIP_CHECK(hipSetDevice(device_));
  std::vector<float*> data(world_);
  std::vector<uint32_t*> flags(world_);
  for (int r = 0; r < world_; ++r) {
    char* base = region_;
    if (r != rank_) {
      if (handles[r].size() != sizeof(hipIpcMemHandle_t)) throw std::invalid_argument("open_peers: bad handle size");
      hipIpcMemHandle_t h;
      std::memcpy(&h, handles[r].data(), sizeof(h));
      void* p = nullptr;
      HIP_CHECK(hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess));
      opened_.push_back(p);
      base = static_cast<char*>(p);
    }
    data[r] = reinterpret_cast<float*>(base);
    flags[r] = reinterpret_cast<uint32_t*>(base + data_bytes_);
  }
  HIP_CHECK(hipMemcpy(d_data_, data.data(), world_ * sizeof(float*), hipMemcpyHostToDevice));
  HIP_CHECK(hipMemcpy(d_flags_, flags.data(), world_ * sizeof(uint32_t*), hipMemcpyHostToDevice));
  ready_ = true;
}

void OneShotAllReduce::all_reduce_sum_f32(float* buf, size_t count, hipStream_t s) {
  if (count == 0) return;
  if (!ready_) throw std::runtime_error("OneShotAllReduce: open_peers() first");
  if (count > (size_t)max_count_) throw std::invalid_argument("OneShotAllReduce: count exceeds max_count");
  if (reinterpret_cast<uintptr_t>(buf) % 16) throw std::invalid_argument("OneShotAllReduce: buffer not 16-byte aligned");
  if (calls_++ == skip_call_) return;  // fault injection (tests)
  launch_oneshot_allreduce(buf, (int)count, rank_, world_, max_count_, d_data_, d_flags_, d_local_, d_local_ + nblk_,
                           nblk_, timeout_ticks_, s, d_stamps_);
  HIP_CHECK(hipGetLastError());
}

std::string OneShotAllReduce::check() {
  uint32_t e = 0;
  HIP_CHECK(hipMemcpy(&e, d_local_ + nblk_, sizeof(e), hipMemcpyDeviceToHost));
  if (!e) return "";
  return "rank " + std::to_string(rank_) + ": one-shot all-reduce flag wait timed out (a peer did not arrive within " +
         std::to_string(timeout_ticks_ / 100000000ull) + " s); the error is latched: later calls and the parameter "
         "updates behind them are skipped";
}

void OneShotAllReduce::clear_error() {
  HIP_CHECK(hipMemset(d_local_ + nblk_, 0, sizeof(uint32_t)));
  HIP_CHECK(hipDeviceSynchronize());
}

void OneShotAllReduce::enable_stamps(bool on) {
  if (on && !d_stamps_) {
    HIP_CHECK(hipMalloc(&d_stamps_, (size_t)nblk_ * 4 * sizeof(unsigned long long)));
    HIP_CHECK(hipMemset(d_stamps_, 0, (size_t)nblk_ * 4 * sizeof(unsigned long long)));
  } else if (!on && d_stamps_) {
    HIP_CHECK(hipDeviceSynchronize());
    HIP_CHECK(hipFree(d_stamps_));
    d_stamps_ = nullptr;
  }
}

std::vector<unsigned long long> OneShotAllReduce::stamps() {
  std::vector<unsigned long long> out;
  if (!d_stamps_) return out;
  out.resize((size_t)nblk_ * 4);
  HIP_CHECK(hipMemcpy(out.data(), d_stamps_, out.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost));
  return out;
}
