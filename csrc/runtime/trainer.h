// Static-schedule training step: the whole forward/backward/all-reduce/update of one batch as a
// fixed list of stream-ordered launches (no autograd tape, survey N8), optionally captured into
// one hipGraph and replayed per step.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <map>
#include <stdexcept>
#include <memory>
#include <string>
#include <vector>

#include "../kernels/launch.h"
#include "oneshot.h"
#include "rccl_comm.h"

struct TrainerPtrs {
  uintptr_t images = 0, labels = 0, idx = 0, step = 0;
  uintptr_t params = 0, grad = 0, mom = 0, pack = 0;
  uintptr_t slab_fc = 0, slab_conv = 0, metrics = 0;
  uintptr_t xT = 0, h1T = 0, h2T = 0, dy1T = 0, dy2T = 0, dy3T = 0;
  uintptr_t p1 = 0, m1 = 0, p2 = 0, m2 = 0, dp2 = 0;
  uintptr_t z1p = 0;  // optional: enables the small-batch layer-1 split path
  uintptr_t stamps = 0;  // optional: per-block phase timestamps of the head kernel (profiling)
  uintptr_t xnext = 0, ynext = 0;  // optional: small-batch MLP look-ahead gather buffers (BatchRef)
  uintptr_t xb = 0;     // optional: LeNet [batch][784] uint8 pixel rows + [batch] labels in batch order (conv_fwd ->
                        // conv_bwd / head16)
};

// A gradient bucket = contiguous range of the flat grad slab, all-reduced as one RCCL call as
// soon as the bucket GROUP (`phase`) that holds it has been reduced.  Groups are numbered in backward-ready
// order and each covers whole gradient-producing units (model_job_begin: the FC layers, last to first; LeNet's
// conv range [0, conv_params) is always the last group): the default plan is two groups (LeNet FC | conv, MLP
// layers 2+3 | layer 1); a link-aware plan (parallel/ddp.py choose_bucket_groups) cuts the FC head into more.
struct Bucket {
  int p0, p1, phase;
};

// Multi-GPU step plans.  Both models' backward produces its gradients in two phases: phase 0 = the late
// layers (LeNet: the FC head [conv_params, n); MLP: layers 2+3 [W2, n)), phase 1 = the early ones (LeNet:
// conv [0, conv_params); MLP: layer 1 [0, W2)).  Every collective is issued on ONE comm stream, in the
// same order on every rank.
//   JOIN  : both phases' gradients are reduced, then ONE all-reduce of the coalesced slab, then one SGD.
//   SPLIT : phase 0's buckets go out on the comm stream as soon as they are reduced (LeNet: beside conv_bwd,
//           whose grid can be capped to leave whole CUs free for RCCL's kernels; MLP: beside the layer-1
//           weight gradient) and phase 0's parameters are updated right after them on the same stream;
//           phase 1's buckets follow its reduce, then its update (which also bumps the step counters).
//   OVERLAP (LeNet, one-shot data plane): the single-GPU concurrent schedule with an all-reduce inside each
//           branch -- aux: FC wgrad -> reduce -> one-shot AR(FC) -> FC update, beside conv_bwd; main: conv_bwd ->
//           reduce -> one-shot AR(conv) -> conv update + step bump; the aux branch is joined by the next step's
//           head like the local schedule.  Two one-shot instances (one per branch/stream, each with its own
//           slots, flags and sequence numbers); no RCCL call and no cross-stream event behind a collective.
enum class Plan : int { JOIN = 0, SPLIT = 1, OVERLAP = 2 };

class Trainer {
 public:
  static constexpr int MAX_GROUPS = 8;  // bucket groups of a plan (Bucket::phase < MAX_GROUPS)
  // LeNet training steps of B <= XB_MAX_B rows hand conv_bwd batch-ordered pixel rows (TrainerPtrs::xb)
  static constexpr int XB_MAX_B = 2048;
  Trainer(int model, int dtype, int batch, int ld_b, int fc_splits, const TrainerPtrs& p);
  ~Trainer();

  void set_comm(std::shared_ptr<RcclComm> c) { invalidate(); comm_ = std::move(c); }
  // Gradient data plane of the step's collectives: the one-shot xGMI all-reduce instead of RCCL (null: RCCL).
  // Works with or without an RCCL communicator attached (parameter broadcast then goes over the control plane).
  void set_oneshot(std::shared_ptr<OneShotAllReduce> o) { invalidate(); oneshot_ = std::move(o); }
  bool has_oneshot() const { return oneshot_ != nullptr; }
  // Plan::OVERLAP's two one-shot instances: FC range [conv_params, n) on the aux stream, conv range on main
  void set_overlap(std::shared_ptr<OneShotAllReduce> fc, std::shared_ptr<OneShotAllReduce> conv) {
    invalidate();
    ov_fc_ = std::move(fc);
    ov_conv_ = std::move(conv);
  }
  bool has_overlap() const { return ov_fc_ != nullptr && ov_conv_ != nullptr; }
  // Timing only (exposed-communication measurement): with a communicator attached, run the local
  // single-GPU schedule without any collective.  Cached graphs are keyed by it.
  void set_comm_enabled(bool on) { comm_enabled_ = on; }
  bool comm_enabled() const { return comm_enabled_; }
  void set_world(int w) { world_ = w; invalidate(); }
  void set_optimizer(float lr, float momentum) { lr_ = lr; momentum_ = momentum; invalidate(); }
  void set_dropout(float p, uint32_t seed) { drop_p_ = p; seed_ = seed; invalidate(); }
  // validated (contiguous groups in ready order on unit boundaries); graphs are cached per bucket plan
  void set_buckets(const std::vector<Bucket>& b);
  std::vector<Bucket> buckets() const { return buckets_; }
  // bucket groups in ready order: parameter range + the FC weight-gradient jobs that produce it (0: conv)
  struct Group {
    int p0, p1, mask;
  };
  std::vector<Group> groups() const;
  // Per-unit backward cost (us, median of `iters` eager launches on `stream` after `warmup`): the FC units in
  // ready order (each its own weight-gradient launch + reduce; LeNet fc3, fc2, fc1 / MLP layer 3, 2, 1), then all
  // FC units as ONE launch + reduce, then (LeNet) conv_bwd + its reduce.  Input of the bucket-plan model.
  std::vector<double> time_units(int iters, int warmup, uintptr_t stream);
  void set_plan(int p) {
    if (p < 0 || p > 2) throw std::invalid_argument("plan must be 0 (join), 1 (split) or 2 (overlap)");
    if (p == 2 && (model_ != ModelKind::LENET || !has_overlap()))
      throw std::invalid_argument("plan overlap: LeNet with two one-shot instances attached (set_overlap) only");
    plan_ = static_cast<Plan>(p);
  }
  int plan() const { return static_cast<int>(plan_); }
  // single-GPU LeNet schedule: FC wgrad + FC update on the aux stream beside conv_bwd (true) or serial
  void set_concurrent(bool on) { concurrent_ = on; }
  bool concurrent() const { return concurrent_; }
  // MLP, one GPU, one FC batch split: SGD as the wgrad kernel's epilogue (true) or wgrad + reduce_sgd
  void set_fuse_wgrad_sgd(bool on) { fuse_wgrad_sgd_ = on; invalidate(); }
  // LeNet bf16 (large batches): conv_fwd + FC head as ONE kernel (fwd_head_kernel, true) or the two
  // kernels (false).  Part of the graph-cache key, so a calibration can compare both.
  void set_fwd_head(bool on) { fwd_head_ = on; }
  bool fwd_head() const { return fwd_head_; }
  bool fwd_head_active(int B) const { return model_ == ModelKind::LENET && fwd_head_ && lenet_fwd_head_applies(dtype_, B); }
  bool fuse_wgrad_sgd() const { return fuse_wgrad_sgd_; }
  // conv_bwd workgroup target (0 = default); the grid actually used for the full batch is bwd_grid()
  void set_bwd_blocks(int n) {
    n = n < 0 ? 0 : n;
    if (lenet_conv_bwd_max_blocks(batch_, n) > max_conv_slabs_)
      throw std::invalid_argument("set_bwd_blocks: more conv_bwd workgroups than conv slab rows");
    bwd_blocks_ = n;
  }
  int bwd_blocks() const { return bwd_blocks_; }
  int bwd_grid() const;
  // The collectives one full-batch step issues under the current plan, in issue order.
  std::vector<Bucket> issued_collectives() const;
  bool has_comm() const { return comm_ != nullptr || oneshot_ != nullptr || has_overlap(); }
  int world() const { return world_; }
  // first parameter of backward phase 0 (see Plan): LeNet conv_params, MLP the layer-2 weight offset
  int phase_split() const;
  // Hold `stream` busy for `seconds` (bounded device spin; watchdog tests).
  void spin(double seconds, uintptr_t stream);

  void pack(uintptr_t stream);
  // re-gather the look-ahead buffers for the current device step (after the host set the counter)
  void prime_next(uintptr_t stream);
  // Full eager step for a batch of B rows (B <= batch).
  void train_step(int B, uintptr_t stream);
  // Phases (used by the torch.distributed comm path and by tests).
  void forward_backward(int B, uintptr_t stream);
  void reduce_grads(int B, uintptr_t stream);
  void optimizer_step(float gscale, uintptr_t stream);
  // Forward-only metrics over an explicit index vector (eval loop).
  void eval_batch(uintptr_t images, uintptr_t labels, uintptr_t idx, int B, uintptr_t metrics,
                  uintptr_t stream);

  // hipGraph of train_step(batch) under the current schedule (plan, concurrent, conv_bwd grid),
  // captured on `stream`, replayed by replay().  Graphs are cached per schedule.
  void capture(uintptr_t stream);
  void replay(uintptr_t stream);
  bool captured() const;
  // k consecutive full-batch steps in one hipGraph (one launch per k steps)
  void capture_multi(uintptr_t stream, int k);
  void replay_multi(uintptr_t stream);
  int multi_steps() const;  // k of the multi-step graph of the current schedule, 0 if none
  // graphs of n consecutive steps besides the k-step one (a run's remainder: 20 steps = 8 + 8 + 4), cached
  // per schedule like the others; multi_steps() is not changed
  void capture_n(uintptr_t stream, int n);
  bool has_graph(int n) const;
  void replay_n(uintptr_t stream, int n);
  void invalidate();        // drop every cached graph
  // teardown: drop the graphs (they captured collectives), drain the side streams, detach the communicator
  void release();
  // the cached single-step graph of the current schedule, one line per node: "index type deps" (diagnostics:
  // what the captured step looks like to the runtime -- kernel / event / memset / empty nodes and their edges)
  std::vector<std::string> graph_nodes() const;
  // final teardown at a point the caller chooses (NativeTrainer.close): release(), then the native streams, events
  // and device counters are destroyed while the HIP runtime is certainly alive (not from a destructor that may run
  // during interpreter shutdown, after torch's own HIP teardown).  Idempotent; the object is unusable afterwards.
  void destroy();

  int nparam() const { return nparam_; }
  int pack_size() const;
  int conv_slabs() const;
  int conv_params() const;
  int fc_splits() const { return fc_splits_; }
  int fc_ld() const { return fc_ld_; }

 private:
  BatchRef batch_ref(int B) const;
  HeadBuffers head_buffers(float* metrics) const;
  // MLP bf16 training: the head hands the batch's raw uint8 rows to the layer-1 weight gradient instead of a
  // bf16 X^T, unless the step's wgrad is the SGD-fused one (no LDS staging) or no row buffer was given
  // B > 0: the buffers of a training step of B rows (cb.xb set when conv_fwd_kernel writes batch-ordered rows)
  LenetConvBuffers conv_buffers(int B = 0) const;
  int fc_splits_for(int B) const;  // FC weight-gradient batch splits used for B rows
  // defer_join: (single GPU, concurrent schedule, inside a multi-step graph) leave the aux branch (FC
  // wgrad + FC update) un-joined at the end of the step; the NEXT step's head waits for it instead.
  void launch_step(int B, hipStream_t s, bool defer_join = false);
  void launch_lenet_comm_tail(int B, int nslab, int splits, hipStream_t s);
  // Plan::SPLIT (LeNet) after the fork: the FC groups' weight gradients + reduces on the aux stream, each group's
  // buckets and update on the comm stream as soon as it is reduced; then the conv group behind conv_bwd
  void launch_lenet_split_tail(int B, int nslab, hipStream_t s, const HeadBuffers& hb, int hrows);
  // Plan::OVERLAP after the fork (conv_bwd launched on s, nothing yet on aux); returns with the aux branch open
  void launch_lenet_overlap(int B, int nslab, hipStream_t s, const HeadBuffers& hb, int hrows);
  void launch_mlp_comm_tail(int B, hipStream_t s, const HeadBuffers& hb, int hrows);
  // comm stream: wait for `ready`, all-reduce group `g`'s buckets, update its parameter range
  void comm_phase(int g, hipEvent_t ready, bool bump);
  bool use_comm() const { return (comm_ || oneshot_ || has_overlap()) && comm_enabled_; }
  // the attached communicator was aborted (also after release() dropped it)
  bool comm_aborted() const { return comm_was_aborted_ || (comm_ && comm_->aborted()); }
  // the update kernels' skip word: the one-shot data plane's latched error (oneshot.hip), none with RCCL
  const uint32_t* dp_skip() const { return oneshot_ ? oneshot_->err_word() : nullptr; }
  void sync_own_streams();
  struct GraphSlot {
    hipGraph_t graph = nullptr;
    hipGraphExec_t exec = nullptr;
  };
  void capture_into(hipStream_t s, int nsteps, hipGraph_t* graph, hipGraphExec_t* exec);
  static void drop(GraphSlot& g);
  uint64_t schedule_key(int nsteps) const;
  const GraphSlot* find_graph(int nsteps) const;
  std::vector<Bucket> coalesced_buckets() const;
  void all_reduce(const std::vector<Bucket>& bs, int phase, hipStream_t s);

  ModelKind model_;
  DType dtype_;
  int batch_, ldb_, fc_splits_, nparam_;
  int fc_ld_ = 0;  // FC slab row stride: nparam rounded up to 4 floats (16-byte aligned rows for the wide slab stores)
  TrainerPtrs p_;
  float lr_ = 0.01f, momentum_ = 0.f, drop_p_ = 0.2f;
  uint32_t seed_ = 1234;
  int world_ = 1;
  Plan plan_ = Plan::JOIN;
  bool concurrent_ = true;
  bool fuse_wgrad_sgd_ = true;
  bool fwd_head_ = true;
  bool comm_enabled_ = true;
  bool destroyed_ = false;  // destroy() ran
  bool comm_was_aborted_ = false;  // release() dropped an aborted communicator
  hipStream_t last_stream_ = nullptr;  // stream of the last graph launch / capture (drained by invalidate)
  int bwd_blocks_ = 0;
  int max_conv_slabs_ = 0;  // rows of the conv slab (lenet_conv_bwd_max_blocks(batch) at the default target)
  std::shared_ptr<RcclComm> comm_;
  std::shared_ptr<OneShotAllReduce> oneshot_;
  std::shared_ptr<OneShotAllReduce> ov_fc_, ov_conv_;
  std::vector<Bucket> buckets_;
  int bucket_id_ = 0;                              // index of buckets_ in bucket_plans_ (graph-cache key)
  std::vector<std::vector<Bucket>> bucket_plans_;  // every bucket plan installed so far
  hipStream_t comm_stream_ = nullptr;
  hipStream_t aux_stream_ = nullptr;  // concurrent FC wgrad branch (fork/join inside the step graph)
  std::vector<hipEvent_t> events_;
  bool aux_pending_ = false;  // the aux branch of the previous step is not joined yet (events_[5])
  std::map<uint64_t, GraphSlot> graphs_;
  int multi_k_ = 0;
  int zero_step_dev_ = 0;
  int32_t* zero_counter_ = nullptr;  // device {0,0} for eval batch addressing
};
