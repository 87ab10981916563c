// One-shot all-reduce over xGMI peer memory (csrc/kernels/oneshot.hip): the alternative to RCCL's ring for
// the latency-bound per-step gradient all-reduce (survey §5.8-3; reference ddp_tutorial_multi_gpu.py:94).
//
// Every rank allocates ONE uncached device region -- receive slots [2 parities][world][max_count] f32 and
// flags [world][nblk] u32 -- and exports it with hipIpcGetMemHandle; the handles travel over the control
// plane (TCPStore, parallel/oneshot.py); every rank opens its peers' regions (hipIpcOpenMemHandle) and keeps a
// device table of the W bases.  all_reduce_sum_f32() is then ONE kernel launch on the caller's stream
// (graph-capturable, like the RCCL calls it replaces in the step graph).  Flag waits are bounded in the kernel
// (timeout -> LATCHED error word: that call writes no sum, every later call does nothing, the update kernels that
// take err_word() as their `skip` leave the parameters alone, and check() reports it).  Collective: every rank
// must issue the same calls in the same order on ONE stream.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <string>
#include <vector>

class OneShotAllReduce {
 public:
  OneShotAllReduce(int rank, int world, int device, int max_count, int nblk = 64, double timeout_s = 5.0);
  ~OneShotAllReduce();
  OneShotAllReduce(const OneShotAllReduce&) = delete;
  OneShotAllReduce& operator=(const OneShotAllReduce&) = delete;

  std::string handle() const;  // this rank's IPC handle (raw bytes)
  // handles[r] of every rank (own entry ignored): open the peers' regions, upload the pointer tables
  void open_peers(const std::vector<std::string>& handles);
  // in-place SUM over the ranks of `count` floats at `buf` (16-byte aligned, count <= max_count)
  void all_reduce_sum_f32(float* buf, size_t count, hipStream_t s);
  // "" if no flag wait timed out, else a message.  The device word stays latched (clear_error() re-arms it after
  // every rank has agreed to continue; tests only)
  std::string check();
  void clear_error();
  // the latched device error word (non-zero after a timeout): the `skip` operand of the update kernels
  const uint32_t* err_word() const { return d_local_ + nblk_; }
  // MNIST_AMD_STAMPS profiling: [nblk][4] wall-clock stamps of the most recent call (entry, pushed, flags seen,
  // summed); empty unless enabled
  void enable_stamps(bool on);
  std::vector<unsigned long long> stamps();
  long long calls() const { return calls_; }
  int rank() const { return rank_; }
  int world() const { return world_; }
  int max_count() const { return max_count_; }
  bool ready() const { return ready_; }

 private:
  int rank_, world_, device_, max_count_, nblk_;
  unsigned long long timeout_ticks_;
  bool ready_ = false;
  char* region_ = nullptr;          // own uncached region: data then flags
  size_t data_bytes_ = 0, region_bytes_ = 0;
  std::vector<void*> opened_;        // peers' mapped regions (closed in the destructor)
  float** d_data_ = nullptr;         // device [world] data bases
  uint32_t** d_flags_ = nullptr;     // device [world] flag bases
  uint32_t* d_local_ = nullptr;      // device: seq[nblk] then err
  unsigned long long* d_stamps_ = nullptr;
  long long calls_ = 0;              // host-issued calls (launches)
  long long skip_call_ = -1;         // fault injection (MNIST_AMD_ONESHOT_SKIP_CALL=rank:call): that call is not issued
};
