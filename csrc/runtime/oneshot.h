// One-shot all-reduce over xGMI peer memory (csrc/kernels/oneshot.hip): the alternative to RCCL's ring for
// the latency-bound per-step gradient all-reduce (survey §5.8-3; reference ddp_tutorial_multi_gpu.py:94).
//
// Every rank allocates ONE uncached device region -- receive slots [2 parities][world][max_count] f32 and
// flags [world][nblk] u32 -- and exports it with hipIpcGetMemHandle; the handles travel over the control
// plane (TCPStore, parallel/oneshot.py); every rank opens its peers' regions (hipIpcOpenMemHandle) and keeps a
// device table of the W bases.  all_reduce_sum_f32() is then ONE kernel launch on the caller's stream
// (graph-capturable, like the RCCL calls it replaces in the step graph).  Flag waits are bounded in the kernel
// (timeout -> error word, reported by check()).  Collective: every rank must issue the same calls in the same
// order on ONE stream.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <string>
#include <vector>

class OneShotAllReduce {
 public:
  OneShotAllReduce(int rank, int world, int device, int max_count, int nblk = 64, double timeout_s = 30.0);
  ~OneShotAllReduce();
  OneShotAllReduce(const OneShotAllReduce&) = delete;
  OneShotAllReduce& operator=(const OneShotAllReduce&) = delete;

  std::string handle() const;  // this rank's IPC handle (raw bytes)
  // handles[r] of every rank (own entry ignored): open the peers' regions, upload the pointer tables
  void open_peers(const std::vector<std::string>& handles);
  // in-place SUM over the ranks of `count` floats at `buf` (16-byte aligned, count <= max_count)
  void all_reduce_sum_f32(float* buf, size_t count, hipStream_t s);
  // "" if no flag wait timed out, else a message (the device error word is cleared)
  std::string check();
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
};
