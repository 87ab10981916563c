// Static-schedule step orchestration (see trainer.h).
//
// Kernel sequence of one data-parallel step (reference CS5, survey §3; kernel IDs of §2.6):
//   LeNet, no comm : conv_fwd -> head(fwd+loss+dgrad) -> { conv_bwd  ||  wgrad(FC) -> reduce+sgd(FC) on aux }
//                    -> reduce+sgd(conv) + step bump (fused reduce/SGD/pack kernels)
//   LeNet, comm    : conv_fwd -> head -> { conv_bwd -> reduce(conv)  ||  wgrad(FC) -> reduce(FC) on aux }
//                    then Plan::JOIN  : ONE all-reduce of the coalesced slab -> sgd_pack
//                      or Plan::OVERLAP: one-shot AR + update inside each branch (aux: FC, main: conv)
//                      or Plan::SPLIT : comm stream: AR(FC buckets) as soon as reduce(FC) is done (beside
//                                       conv_bwd) -> update(FC range); then AR(conv buckets) after
//                                       reduce(conv) -> update(conv range) + step bump
//   MLP, no comm   : head -> wgrad(+SGD epilogue) or wgrad -> reduce_sgd
//   MLP, comm      : JOIN : head -> wgrad -> reduce -> ONE all-reduce -> sgd_pack
//                    SPLIT: head -> wgrad(layers 2+3) -> reduce -> [comm: AR -> update(layers 2+3)]
//                                -> wgrad(layer 1) -> reduce -> [comm: AR -> update(layer 1) + bump]
// conv_bwd's one-round grid (2 blocks/CU) is LDS-bound and leaves VGPR room on every SIMD, which the
// FC wgrad (no LDS) fills: running the two concurrently hides most of the wgrad (-6% step time on
// one MI355X).  MNIST_AMD_CONCURRENT=0 restores the serial single-GPU schedule.  Which multi-GPU plan
// runs is chosen at start-up by timing the candidates (NativeTrainer.autotune_plan, parallel/ddp.py
// choose_plan); MNIST_AMD_MG_SCHED=join|split overrides it.
// All launches are allocation- and sync-free; capture() records the sequence (all streams, RCCL
// included) into one hipGraph, so a training step costs one hipGraphLaunch on the host.
#include "trainer.h"

#include <algorithm>
#include <cstdio>
#include <functional>
#include <cstdlib>
#include <stdexcept>
#include <string>

#include "hip_check.h"

namespace {
bool sync_debug() {
  static const bool on = [] {
    const char* e = std::getenv("MNIST_AMD_SYNC_DEBUG");
    return e && *e && *e != '0';
  }();
  return on;
}
void post_launch(hipStream_t s) {
  HIP_CHECK(hipGetLastError());
  if (sync_debug()) {
    hipStreamCaptureStatus st;
    HIP_CHECK(hipStreamIsCapturing(s, &st));
    if (st == hipStreamCaptureStatusNone) HIP_CHECK(hipStreamSynchronize(s));
  }
}
// MNIST_AMD_CONCURRENT: initial value of the single-GPU schedule (0 = serial, otherwise FC wgrad ||
// conv_bwd); set_concurrent() changes it at run time (NativeTrainer.autotune_plan times both)
int concurrent_mode() {
  static const int m = [] {
    const char* e = std::getenv("MNIST_AMD_CONCURRENT");
    return e ? std::atoi(e) : 1;
  }();
  return m;
}
// (Measured and removed: conv_bwd as two concurrent halves on two streams -- bitwise equal, but 0.184 vs
// 0.157 ms/step: the halves contend for the same LDS bandwidth.)
// XCD-contiguous work mapping of conv_fwd / head / conv_bwd / FC wgrad (common.h xcd_unit), always on
constexpr int xcd_map() { return 1; }
// Deferred aux-branch join inside multi-step graphs: the next step's head joins the FC branch
constexpr bool defer_join() { return true; }
// MNIST_AMD_TRACE=1: log every orchestration call of a step to stderr (host-side debugging)
void trace(const char* what) {
  static const bool on = [] {
    const char* e = std::getenv("MNIST_AMD_TRACE");
    return e && *e == '1';
  }();
  if (on) { std::fputs(what, stderr); std::fputc('\n', stderr); std::fflush(stderr); }
}
// Diagnostic phase-skipping masks (launch.h ABLATED): honoured only by an ablation build; the normal build
// refuses a set variable (a stale MNIST_AMD_ABLATE on a box must not train on skipped phases unnoticed)
int ablation_mask(const char* var) {
  const char* e = std::getenv(var);
  const int m = e && *e ? std::atoi(e) : 0;
#ifndef MNIST_AMD_ABLATION_BUILD
  if (m != 0)
    throw std::runtime_error(std::string(var) + " is set, but this build has no ablation switches (they skip kernel "
                             "phases and give wrong results): unset it, or build with -DMNIST_AMD_ABLATION_BUILD "
                             "(scripts/ablate.sh)");
#endif
  return m;
}
inline hipStream_t S(uintptr_t s) { return reinterpret_cast<hipStream_t>(s); }
template <typename P> P* ptr(uintptr_t v) { return reinterpret_cast<P*>(v); }
}  // namespace

Trainer::Trainer(int model, int dtype, int batch, int ld_b, int fc_splits, const TrainerPtrs& p)
    : model_(static_cast<ModelKind>(model)), dtype_(static_cast<DType>(dtype)), batch_(batch), ldb_(ld_b),
      fc_splits_(fc_splits), p_(p) {
  if (model != 0 && model != 1) throw std::invalid_argument("model must be 0 (mlp) or 1 (lenet5)");
  if (dtype != 0 && dtype != 1) throw std::invalid_argument("dtype must be 0 (fp32) or 1 (bf16)");
  if (batch <= 0) throw std::invalid_argument("batch must be positive");
  if (ld_b < ((batch + 63) / 64) * 64) throw std::invalid_argument("ld_b must be >= batch rounded up to 64");
  nparam_ = model_nparam(model_);
  fc_ld_ = (nparam_ + 3) / 4 * 4;
  max_conv_slabs_ = model_ == ModelKind::LENET ? lenet_conv_bwd_max_blocks(batch_, 0) : 0;
  concurrent_ = concurrent_mode() != 0;
  const int ps = model_phase_split(model_);  // default buckets: one per backward phase (see Plan)
  set_buckets({{ps, nparam_, 0}, {0, ps, 1}});
  HIP_CHECK(hipStreamCreateWithFlags(&comm_stream_, hipStreamNonBlocking));
  HIP_CHECK(hipStreamCreateWithFlags(&aux_stream_, hipStreamNonBlocking));
  events_.resize(6 + MAX_GROUPS);  // [6 + g]: group g reduced (SPLIT)
  for (auto& e : events_) HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  HIP_CHECK(hipMalloc(&zero_counter_, 2 * sizeof(int32_t)));
  HIP_CHECK(hipMemset(zero_counter_, 0, 2 * sizeof(int32_t)));
}

Trainer::~Trainer() { destroy(); }

void Trainer::destroy() {
  if (destroyed_) return;  // (the destructor after an explicit destroy(): touches nothing)
  invalidate();
  // after an abort a replay may still sit in a collective that never completes: its graph execs (leaked by
  // invalidate), streams and events stay alive rather than being destroyed under it (the process is failing)
  if (comm_aborted()) return;
  sync_own_streams();
  for (auto& e : events_) if (e) hipEventDestroy(e);
  events_.clear();
  if (comm_stream_) hipStreamDestroy(comm_stream_);
  if (aux_stream_) hipStreamDestroy(aux_stream_);
  if (zero_counter_) hipFree(zero_counter_);
  comm_stream_ = aux_stream_ = last_stream_ = nullptr;
  zero_counter_ = nullptr;
  comm_.reset();
  oneshot_.reset();
  ov_fc_.reset();
  ov_conv_.reset();
  destroyed_ = true;
}

void Trainer::release() {
  // teardown order (DistContext.finalize): every graph that captured a collective is dropped -- after its
  // replays drained -- before the communicator is destroyed, then the communicator reference is released
  invalidate();
  if (!comm_aborted()) {
    (void)hipStreamSynchronize(comm_stream_);
    (void)hipStreamSynchronize(aux_stream_);
  }
  // remembered past the reset below: destroy() / sync_own_streams() must still see that a replay may be stuck in an
  // aborted collective (advisor, round 5: after close() -> release() they found comm_ null and synchronised anyway)
  if (comm_ && comm_->aborted()) comm_was_aborted_ = true;
  comm_.reset();
  oneshot_.reset();
  ov_fc_.reset();
  ov_conv_.reset();
  if (plan_ == Plan::OVERLAP) plan_ = Plan::JOIN;
}

int Trainer::fc_splits_for(int B) const {
  // the batch-split count launch_head_wgrad actually uses for B rows (wg::make_args)
  const int KC = dtype_ == DType::BF16 ? 32 : 16;
  const int Bp = (B + KC - 1) / KC * KC;
  int splits = std::max(1, std::min(fc_splits_, Bp / KC));
  const int rlen = ((Bp + splits - 1) / splits + KC - 1) / KC * KC;
  return (Bp + rlen - 1) / rlen;
}

void Trainer::set_buckets(const std::vector<Bucket>& b) {
  // groups: contiguous ranges in backward-ready order (group 0 ends at nparam, each next one ends where the previous
  // starts, the last starts at 0), every boundary a unit boundary (model_job_begin; LeNet: the conv range is the
  // last group on its own)
  if (b.empty()) throw std::invalid_argument("set_buckets: no buckets");
  int ng = 0;
  for (const Bucket& x : b) {
    if (x.p0 < 0 || x.p1 > nparam_ || x.p0 >= x.p1) throw std::invalid_argument("set_buckets: bad bucket range");
    if (x.phase < 0 || x.phase >= MAX_GROUPS) throw std::invalid_argument("set_buckets: group index out of range");
    ng = std::max(ng, x.phase + 1);
  }
  std::vector<int> bounds = {0, nparam_};
  for (int j = 0; j < 4; ++j) bounds.push_back(model_job_begin(model_, j));
  const int cp = model_conv_params(model_);
  auto on_bound = [&](int p) { return std::find(bounds.begin(), bounds.end(), p) != bounds.end(); };
  int end = nparam_;
  for (int g = 0; g < ng; ++g) {
    std::vector<Bucket> mine;
    for (const Bucket& x : b) if (x.phase == g) mine.push_back(x);
    if (mine.empty()) throw std::invalid_argument("set_buckets: empty bucket group " + std::to_string(g));
    std::sort(mine.begin(), mine.end(), [](const Bucket& u, const Bucket& v) { return u.p0 < v.p0; });
    for (size_t i = 1; i < mine.size(); ++i)
      if (mine[i].p0 != mine[i - 1].p1) throw std::invalid_argument("set_buckets: group " + std::to_string(g) + " is not contiguous");
    const int p0 = mine.front().p0, p1 = mine.back().p1;
    if (p1 != end) throw std::invalid_argument("set_buckets: groups must tile [0, nparam) in backward-ready order");
    if (!on_bound(p0)) throw std::invalid_argument("set_buckets: group boundary " + std::to_string(p0) + " splits a layer");
    if (cp > 0 && p0 < cp && p1 > cp) throw std::invalid_argument("set_buckets: a group mixes conv and FC gradients");
    end = p0;
  }
  if (end != 0) throw std::invalid_argument("set_buckets: groups must cover [0, nparam)");
  buckets_ = b;
  // graphs are cached per bucket plan (schedule_key), so a calibration can interleave several plans
  auto it = std::find_if(bucket_plans_.begin(), bucket_plans_.end(), [&](const std::vector<Bucket>& v) {
    return v.size() == b.size() && std::equal(v.begin(), v.end(), b.begin(), [](const Bucket& x, const Bucket& y) {
             return x.p0 == y.p0 && x.p1 == y.p1 && x.phase == y.phase;
           });
  });
  if (it == bucket_plans_.end()) {
    if (bucket_plans_.size() >= 255) throw std::invalid_argument("set_buckets: too many distinct bucket plans");
    bucket_plans_.push_back(b);
    it = bucket_plans_.end() - 1;
  }
  bucket_id_ = static_cast<int>(it - bucket_plans_.begin());
}

std::vector<Trainer::Group> Trainer::groups() const {
  int ng = 0;
  for (const Bucket& x : buckets_) ng = std::max(ng, x.phase + 1);
  std::vector<Group> out(ng, Group{nparam_, 0, 0});
  for (const Bucket& x : buckets_) {
    out[x.phase].p0 = std::min(out[x.phase].p0, x.p0);
    out[x.phase].p1 = std::max(out[x.phase].p1, x.p1);
  }
  for (Group& g : out)
    for (int j = 0; j < 3; ++j)
      if (model_job_begin(model_, j) >= g.p0 && model_job_begin(model_, j + 1) <= g.p1) g.mask |= 1 << j;
  return out;
}

std::vector<double> Trainer::time_units(int iters, int warmup, uintptr_t stream) {
  hipStream_t s = S(stream);
  const int B = batch_;
  const HeadBuffers hb = head_buffers(ptr<float>(p_.metrics));
  const float scale = 1.0f / float(B);
  const int hrows = head_rows_per_block(model_, dtype_, batch_);
  float* g = ptr<float>(p_.grad);
  // (the operand buffers hold the last step's activations / gradients: the values do not matter for timing,
  //  grad is overwritten -- callers save and restore training state around this)
  std::vector<std::function<void()>> units;
  for (int j = 2; j >= 0; --j)  // ready order: the last FC layer first
    units.push_back([=] {
      const int sp = launch_head_wgrad(model_, dtype_, hb, B, fc_splits_, ptr<float>(p_.slab_fc), fc_ld_, s, hrows,
                                       nullptr, 1 << j);
      launch_reduce(ptr<const float>(p_.slab_fc), fc_ld_, sp, model_job_begin(model_, j), model_job_begin(model_, j + 1),
                    scale, g, s);
    });
  units.push_back([=] {
    const int sp = launch_head_wgrad(model_, dtype_, hb, B, fc_splits_, ptr<float>(p_.slab_fc), fc_ld_, s, hrows, nullptr, 7);
    launch_reduce(ptr<const float>(p_.slab_fc), fc_ld_, sp, model_job_begin(model_, 0), nparam_, scale, g, s);
  });
  if (model_ == ModelKind::LENET)
    units.push_back([=] {
      int nslab = 0;
      launch_lenet_conv_bwd(dtype_, batch_ref(B), conv_buffers(B), &nslab, s, bwd_blocks_);
      launch_reduce(ptr<const float>(p_.slab_conv), model_conv_params(model_), nslab, 0, model_conv_params(model_), scale, g, s);
    });
  hipEvent_t e0, e1;
  HIP_CHECK(hipEventCreate(&e0));
  HIP_CHECK(hipEventCreate(&e1));
  std::vector<double> out;
  for (auto& u : units) {
    for (int i = 0; i < warmup; ++i) u();
    std::vector<float> ts;
    for (int i = 0; i < iters; ++i) {
      HIP_CHECK(hipEventRecord(e0, s));
      u();
      HIP_CHECK(hipEventRecord(e1, s));
      HIP_CHECK(hipEventSynchronize(e1));
      float ms = 0.f;
      HIP_CHECK(hipEventElapsedTime(&ms, e0, e1));
      ts.push_back(ms);
    }
    HIP_CHECK(hipGetLastError());
    std::sort(ts.begin(), ts.end());
    out.push_back(ts.empty() ? 0.0 : 1000.0 * ts[ts.size() / 2]);
  }
  hipEventDestroy(e0);
  hipEventDestroy(e1);
  return out;
}

std::vector<std::string> Trainer::graph_nodes() const {
  std::vector<std::string> out;
  const GraphSlot* g = find_graph(1);
  if (!g || !g->graph) return out;
  size_t n = 0;
  HIP_CHECK(hipGraphGetNodes(g->graph, nullptr, &n));
  std::vector<hipGraphNode_t> nodes(n);
  HIP_CHECK(hipGraphGetNodes(g->graph, nodes.data(), &n));
  for (size_t i = 0; i < n; ++i) {
    hipGraphNodeType t;
    HIP_CHECK(hipGraphNodeGetType(nodes[i], &t));
    size_t nd = 0;
    HIP_CHECK(hipGraphNodeGetDependencies(nodes[i], nullptr, &nd));
    std::vector<hipGraphNode_t> deps(nd);
    if (nd) HIP_CHECK(hipGraphNodeGetDependencies(nodes[i], deps.data(), &nd));
    std::string line = std::to_string(i) + " type=" + std::to_string(static_cast<int>(t));
    if (t == hipGraphNodeTypeKernel) {
      hipKernelNodeParams kp{};
      if (hipGraphKernelNodeGetParams(nodes[i], &kp) == hipSuccess)
        line += " grid=" + std::to_string(kp.gridDim.x) + "x" + std::to_string(kp.gridDim.y) + " block=" +
                std::to_string(kp.blockDim.x);
    }
    line += " deps=";
    for (size_t d = 0; d < nd; ++d)
      for (size_t j = 0; j < n; ++j)
        if (nodes[j] == deps[d]) line += std::to_string(j) + ",";
    out.push_back(line);
  }
  return out;
}

int Trainer::pack_size() const { return model_pack_size(model_); }
int Trainer::phase_split() const { return model_phase_split(model_); }
int Trainer::conv_params() const { return model_conv_params(model_); }
int Trainer::conv_slabs() const { return model_ == ModelKind::LENET ? lenet_conv_bwd_blocks(batch_, bwd_blocks_) : 0; }

void Trainer::sync_own_streams() {
  // a replay of a cached graph may still be running on the stream it was launched on and on its forked
  // aux / comm branches: drain those (not the whole device, which would also wait on other trainers'
  // and other libraries' work).  After an abort a collective may never complete: nothing is waited for.
  if (comm_aborted()) return;
  if (last_stream_) (void)hipStreamSynchronize(last_stream_);
  (void)hipStreamSynchronize(aux_stream_);
  (void)hipStreamSynchronize(comm_stream_);
}

void Trainer::invalidate() {
  if (graphs_.empty()) return;
  if (comm_aborted()) {
    // a replay may be stuck in an aborted collective: leak the graph execs (as RcclComm::time_all_reduce
    // does) instead of destroying them under it
    graphs_.clear();
    multi_k_ = 0;
    return;
  }
  // configuration changes only, never in the step loop
  sync_own_streams();
  for (auto& kv : graphs_) drop(kv.second);
  graphs_.clear();
}

BatchRef Trainer::batch_ref(int B) const {
  BatchRef br;
  br.images = ptr<const uint8_t>(p_.images);
  br.labels = ptr<const uint8_t>(p_.labels);
  br.idx_epoch = ptr<const int32_t>(p_.idx);
  br.step_ptr = ptr<const int32_t>(p_.step);
  br.batch_stride = batch_;
  br.B = B;
  br.xnext = ptr<uint8_t>(p_.xnext);
  br.ynext = ptr<uint8_t>(p_.ynext);
  br.xcd = xcd_map();
  return br;
}

void Trainer::prime_next(uintptr_t stream) {
  if (!p_.xnext) return;
  launch_gather_next(batch_ref(batch_), S(stream));
  post_launch(S(stream));
}

HeadBuffers Trainer::head_buffers(float* metrics) const {
  HeadBuffers hb;
  hb.params = ptr<const float>(p_.params);
  hb.pack = ptr<const void>(p_.pack);
  hb.xin = ptr<const void>(p_.p2);
  hb.xT = ptr<void>(p_.xT);
  hb.h1T = ptr<void>(p_.h1T);
  hb.h2T = ptr<void>(p_.h2T);
  hb.dy1T = ptr<void>(p_.dy1T);
  hb.dy2T = ptr<void>(p_.dy2T);
  hb.dy3T = ptr<void>(p_.dy3T);
  hb.dx = ptr<void>(p_.dp2);
  hb.metrics = metrics;
  hb.z1p = ptr<float>(p_.z1p);
  hb.stamps = ptr<unsigned long long>(p_.stamps);
  hb.ldB = ldb_;
  hb.seed = seed_;
  hb.drop_p = drop_p_;
  hb.xcd = xcd_map();
  hb.ablate = ablation_mask("MNIST_AMD_HEAD_ABLATE");
  return hb;
}

LenetConvBuffers Trainer::conv_buffers(int B) const {
  LenetConvBuffers cb;
  // a training step of B rows whose forward is conv_fwd_kernel (not the fused forward + head) hands conv_bwd
  // its pixel rows in batch order (small batches only: there the index chain is conv_bwd's start-up latency)
  if (B > 0 && B <= XB_MAX_B && p_.xb && !fwd_head_active(B)) {
    cb.xb = ptr<uint8_t>(p_.xb);                          // [batch][784] pixel rows
    cb.yb = ptr<uint8_t>(p_.xb) + (size_t)batch_ * 784;   // then [batch] labels
  }
  cb.params = ptr<const float>(p_.params);
  cb.pack = ptr<const void>(p_.pack);
  cb.p1 = ptr<void>(p_.p1);
  cb.m1 = ptr<uint8_t>(p_.m1);
  cb.p2 = ptr<void>(p_.p2);
  cb.m2 = ptr<uint8_t>(p_.m2);
  cb.dp2 = ptr<const void>(p_.dp2);
  cb.slab = ptr<float>(p_.slab_conv);
  cb.ablate = ablation_mask("MNIST_AMD_ABLATE");
  // stamps layout: launch.h STAMP_* (the conv kernels address their rows relative to STAMP_CONV_BWD)
  cb.stamps = p_.stamps ? ptr<unsigned long long>(p_.stamps) + STAMP_CONV_BWD * 16 : nullptr;
  return cb;
}

void Trainer::pack(uintptr_t stream) {
  launch_pack(model_, dtype_, ptr<const float>(p_.params), ptr<void>(p_.pack), nparam_, S(stream));
  post_launch(S(stream));
}

void Trainer::forward_backward(int B, uintptr_t stream) {
  hipStream_t s = S(stream);
  if (B <= 0 || B > batch_) throw std::invalid_argument("forward_backward: bad batch size");
  const BatchRef br = batch_ref(B);
  HeadBuffers hb = head_buffers(ptr<float>(p_.metrics));
  if (model_ == ModelKind::LENET) hb.yb = conv_buffers(B).yb;  // (small batches: labels from conv_fwd_kernel)
  int hrows = 0;
  if (model_ == ModelKind::LENET) {
    if (fwd_head_active(B)) hrows = launch_lenet_fwd_head(dtype_, br, conv_buffers(B), hb, s);
    if (!hrows) launch_lenet_conv_fwd(dtype_, true, br, conv_buffers(B), s);
    post_launch(s);
  }
  if (!hrows) {
    if (model_ == ModelKind::LENET) hrows = launch_lenet_head16(dtype_, br, hb, s);
    if (!hrows) hrows = launch_head(model_, dtype_, true, br, hb, head_rows_per_block(model_, dtype_, batch_), s);
    post_launch(s);
  }
  launch_head_wgrad(model_, dtype_, hb, B, fc_splits_, ptr<float>(p_.slab_fc), fc_ld_, s, hrows);
  post_launch(s);
  if (model_ == ModelKind::LENET) {
    launch_lenet_conv_bwd(dtype_, br, conv_buffers(B), nullptr, s, bwd_blocks_);
    post_launch(s);
  }
}

void Trainer::reduce_grads(int B, uintptr_t stream) {
  hipStream_t s = S(stream);
  const float scale = 1.0f / float(B);
  const int cp = model_conv_params(model_);
  const HeadBuffers hb = head_buffers(ptr<float>(p_.metrics));
  (void)hb;
  const int splits = fc_splits_for(B);
  launch_reduce(ptr<const float>(p_.slab_fc), fc_ld_, splits, cp, nparam_, scale, ptr<float>(p_.grad), s);
  post_launch(s);
  if (cp > 0) {
    launch_reduce(ptr<const float>(p_.slab_conv), cp, lenet_conv_bwd_blocks(B, bwd_blocks_), 0, cp, scale, ptr<float>(p_.grad), s);
    post_launch(s);
  }
}

void Trainer::optimizer_step(float gscale, uintptr_t stream) {
  launch_sgd_pack(model_, dtype_, ptr<float>(p_.params), ptr<const float>(p_.grad), ptr<float>(p_.mom),
                  ptr<void>(p_.pack), nparam_, lr_, momentum_, gscale, ptr<int32_t>(p_.step), S(stream));
  post_launch(S(stream));
}

int Trainer::bwd_grid() const {
  return model_ == ModelKind::LENET ? lenet_conv_bwd_blocks(batch_, bwd_blocks_) : 0;
}

void Trainer::spin(double seconds, uintptr_t stream) {
  launch_spin(seconds, S(stream));
  post_launch(S(stream));
}

void Trainer::all_reduce(const std::vector<Bucket>& bs, int phase, hipStream_t s) {
  for (const Bucket& b : bs)
    if (phase < 0 || b.phase == phase) {
      float* g = ptr<float>(p_.grad) + b.p0;
      if (oneshot_) oneshot_->all_reduce_sum_f32(g, size_t(b.p1 - b.p0), s);
      else if (comm_) comm_->all_reduce_sum_f32(g, size_t(b.p1 - b.p0), s);
      else throw std::logic_error("all_reduce: no RCCL communicator or one-shot instance for this plan");
    }
}

std::vector<Bucket> Trainer::issued_collectives() const {
  std::vector<Bucket> out;
  if (!use_comm()) return out;
  if (plan_ == Plan::OVERLAP) {  // aux stream's FC range, main stream's conv range
    const int cp = model_conv_params(model_);
    return {{cp, nparam_, 0}, {0, cp, 1}};
  }
  if (plan_ == Plan::SPLIT) {  // group by group in ready order (LeNet: the conv group after the FC ones)
    const int ng = static_cast<int>(groups().size());
    for (int g = 0; g < ng; ++g)
      for (const Bucket& b : buckets_) if (b.phase == g) out.push_back(b);
    return out;
  }
  return coalesced_buckets();
}

void Trainer::launch_step(int B, hipStream_t s, bool defer_join) {
  if (B <= 0 || B > batch_) throw std::invalid_argument("train_step: bad batch size");
  const BatchRef br = batch_ref(B);
  HeadBuffers hb = head_buffers(ptr<float>(p_.metrics));
  if (model_ == ModelKind::LENET) hb.yb = conv_buffers(B).yb;  // (small batches: labels from conv_fwd_kernel)
  const float scale = 1.0f / float(B);
  const int cp = model_conv_params(model_);
  const bool comm = use_comm();
  last_stream_ = s;
  // deferred join of the previous step's aux branch: the head overwrites the activations its FC wgrad
  // read and reads the FC weights its FC update wrote (conv_fwd touches neither, so with separate
  // kernels it runs without waiting: the join's cross-queue latency is off the conv_bwd -> conv update ->
  // conv_fwd chain; the fused forward + head kernel contains the head, so it joins first)
  auto join_aux = [&] {
    if (aux_pending_) {
      HIP_CHECK(hipStreamWaitEvent(s, events_[5], 0));
      aux_pending_ = false;
    }
  };
  int hrows = 0;
  if (model_ == ModelKind::LENET) {
    if (fwd_head_active(B)) {
      join_aux();
      hrows = launch_lenet_fwd_head(dtype_, br, conv_buffers(B), hb, s);
    } else {
      launch_lenet_conv_fwd(dtype_, true, br, conv_buffers(B), s);
    }
    post_launch(s);
  }
  join_aux();
  if (!hrows) {
    if (model_ == ModelKind::LENET) hrows = launch_lenet_head16(dtype_, br, hb, s);
    if (!hrows) hrows = launch_head(model_, dtype_, true, br, hb, head_rows_per_block(model_, dtype_, batch_), s);
    post_launch(s);
  }

  if (model_ == ModelKind::LENET && (comm || concurrent_)) {
    // fork: conv_bwd on the main stream (enqueued first, so its one-round grid is dispatched whole:
    // measured wgrad-first 0.1692 ms/step, conv_bwd-first 0.1565, serial 0.1671), the FC wgrad (no LDS,
    // 320 small blocks) on the aux stream beside it
    HIP_CHECK(hipEventRecord(events_[4], s));
    HIP_CHECK(hipStreamWaitEvent(aux_stream_, events_[4], 0));
    int nslab = 0;
    launch_lenet_conv_bwd(dtype_, br, conv_buffers(B), &nslab, s, bwd_blocks_);
    post_launch(s);
    if (comm && plan_ == Plan::OVERLAP) {
      launch_lenet_overlap(B, nslab, s, hb, hrows);
      // like the local schedule: the FC branch is joined by the next step's head inside a multi-step graph
      if (defer_join) aux_pending_ = true;
      else HIP_CHECK(hipStreamWaitEvent(s, events_[5], 0));
      return;
    }
    if (comm && plan_ == Plan::SPLIT) {
      launch_lenet_split_tail(B, nslab, s, hb, hrows);
      return;
    }
    if (comm) {
      const int splits =
          launch_head_wgrad(model_, dtype_, hb, B, fc_splits_, ptr<float>(p_.slab_fc), fc_ld_, aux_stream_, hrows);
      post_launch(aux_stream_);
      launch_lenet_comm_tail(B, nslab, splits, s);
      return;
    }
    // single GPU: the FC update follows the FC wgrad on the aux stream (it touches only FC parameters
    // and FC operand images); the conv update + step bump follows the join.  With ONE batch split the
    // update is the wgrad kernel's epilogue (small batches: one kernel and one boundary less on the aux
    // branch; bitwise equal to wgrad -> reduce_sgd)
    int splits = 1;
    if (fc_splits_ == 1 && fuse_wgrad_sgd_) {
      const SgdFuse f{scale, lr_, momentum_, ptr<float>(p_.params), ptr<float>(p_.grad),
                      momentum_ != 0.f ? ptr<float>(p_.mom) : nullptr, ptr<void>(p_.pack), nullptr};
      launch_head_wgrad(model_, dtype_, hb, B, 1, ptr<float>(p_.slab_fc), fc_ld_, aux_stream_, hrows, &f);
      post_launch(aux_stream_);
    } else {
      splits = launch_head_wgrad(model_, dtype_, hb, B, fc_splits_, ptr<float>(p_.slab_fc), fc_ld_, aux_stream_, hrows);
      post_launch(aux_stream_);
      launch_reduce_sgd(model_, dtype_, ptr<const float>(p_.slab_conv), cp, nslab, ptr<const float>(p_.slab_fc),
                        fc_ld_, splits, cp, cp, nparam_, scale, ptr<float>(p_.params), ptr<float>(p_.grad),
                        ptr<float>(p_.mom), ptr<void>(p_.pack), lr_, momentum_, nullptr, aux_stream_);
      post_launch(aux_stream_);
    }
    HIP_CHECK(hipEventRecord(events_[5], aux_stream_));
    // the conv update touches only conv parameters / operand images and the step counters (which no aux
    // kernel reads): with defer_join it follows conv_bwd directly, the join moves to the next head
    if (defer_join) aux_pending_ = true;
    else HIP_CHECK(hipStreamWaitEvent(s, events_[5], 0));
    launch_reduce_sgd(model_, dtype_, ptr<const float>(p_.slab_conv), cp, nslab, ptr<const float>(p_.slab_fc),
                      fc_ld_, splits, cp, 0, cp, scale, ptr<float>(p_.params), ptr<float>(p_.grad),
                      ptr<float>(p_.mom), ptr<void>(p_.pack), lr_, momentum_, ptr<int32_t>(p_.step), s);
    post_launch(s);
    return;
  }

  if (model_ == ModelKind::MLP && comm) {
    launch_mlp_comm_tail(B, s, hb, hrows);
    return;
  }
  if (model_ == ModelKind::MLP && fc_splits_ == 1 && fuse_wgrad_sgd_) {
    // one GPU, one batch split: the SGD update is the wgrad kernel's epilogue (no reduce_sgd kernel)
    const SgdFuse f{scale, lr_, momentum_, ptr<float>(p_.params), ptr<float>(p_.grad),
                    momentum_ != 0.f ? ptr<float>(p_.mom) : nullptr,  // as launch_reduce_sgd
                    ptr<void>(p_.pack), ptr<int32_t>(p_.step)};
    launch_head_wgrad(model_, dtype_, hb, B, 1, ptr<float>(p_.slab_fc), fc_ld_, s, hrows, &f);
    post_launch(s);
    return;
  }
  if (model_ == ModelKind::LENET && fc_splits_ == 1 && fuse_wgrad_sgd_) {
    // serial single-GPU schedule, one FC batch split (small batches): the FC update is the wgrad kernel's
    // epilogue (it touches only FC parameters / operand images, which conv_bwd does not read), and the closing
    // reduce + SGD covers the conv parameters only (bitwise equal to wgrad -> reduce_sgd over all of them)
    const SgdFuse f{scale, lr_, momentum_, ptr<float>(p_.params), ptr<float>(p_.grad),
                    momentum_ != 0.f ? ptr<float>(p_.mom) : nullptr, ptr<void>(p_.pack), nullptr};
    // ... as extra workgroups of the conv_bwd launch (one kernel instead of two; the FC wgrad + update as its own
    // kernel before conv_bwd measured 31.0 vs 25.8 us per B = 128 step, profiles/r4_session2/NOTES.md)
    const int nslab = launch_lenet_conv_bwd_fc(dtype_, br, conv_buffers(B), hb, f, s, bwd_blocks_);
    post_launch(s);
    launch_reduce_sgd(model_, dtype_, ptr<const float>(p_.slab_conv), cp, nslab, ptr<const float>(p_.slab_fc),
                      fc_ld_, 1, cp, 0, cp, scale, ptr<float>(p_.params), ptr<float>(p_.grad), ptr<float>(p_.mom),
                      ptr<void>(p_.pack), lr_, momentum_, ptr<int32_t>(p_.step), s);
    post_launch(s);
    return;
  }
  const int splits = launch_head_wgrad(model_, dtype_, hb, B, fc_splits_, ptr<float>(p_.slab_fc), fc_ld_, s, hrows);
  post_launch(s);
  int nslab = 0;
  if (model_ == ModelKind::LENET) {  // serial single-GPU schedule (MNIST_AMD_CONCURRENT=0)
    launch_lenet_conv_bwd(dtype_, br, conv_buffers(B), &nslab, s, bwd_blocks_);
    post_launch(s);
  }
  // no communicator: ONE fused reduce + SGD + pack kernel (2 boundaries fewer than reduce -> sgd)
  launch_reduce_sgd(model_, dtype_, ptr<const float>(p_.slab_conv), cp, nslab, ptr<const float>(p_.slab_fc),
                    fc_ld_, splits, cp, 0, nparam_, scale, ptr<float>(p_.params), ptr<float>(p_.grad),
                    ptr<float>(p_.mom), ptr<void>(p_.pack), lr_, momentum_, ptr<int32_t>(p_.step), s);
  post_launch(s);
}

// Comm stream: wait for phase `phase`'s reduced gradients, all-reduce its buckets, then update that
// phase's parameter range (and operand images) with the 1/W average folded in.  Everything stays on the
// comm stream, so no other stream waits on an event recorded behind a captured RCCL call mid-step.
void Trainer::comm_phase(int g, hipEvent_t ready, bool bump) {
  HIP_CHECK(hipStreamWaitEvent(comm_stream_, ready, 0));
  all_reduce(buckets_, g, comm_stream_);
  const Group gr = groups().at(g);
  launch_sgd_pack_range(model_, dtype_, ptr<float>(p_.params), ptr<const float>(p_.grad), ptr<float>(p_.mom),
                        ptr<void>(p_.pack), gr.p0, gr.p1, lr_, momentum_, 1.0f / float(world_),
                        bump ? ptr<int32_t>(p_.step) : nullptr, comm_stream_, dp_skip());
  post_launch(comm_stream_);
}

// MLP with a communicator (after the head).  JOIN: the whole weight gradient, one all-reduce, one update.
// SPLIT: layers 2+3 first (their buckets and update go out on the comm stream), then layer 1's 784-deep
// weight gradient -- the largest GEMM of the step -- runs beside that all-reduce.
void Trainer::launch_mlp_comm_tail(int B, hipStream_t s, const HeadBuffers& hb, int hrows) {
  const float scale = 1.0f / float(B);
  const int ps = model_phase_split(model_);
  float* g = ptr<float>(p_.grad);
  float* slab = ptr<float>(p_.slab_fc);
  if (plan_ == Plan::JOIN) {
    const int splits = launch_head_wgrad(model_, dtype_, hb, B, fc_splits_, slab, fc_ld_, s, hrows);
    post_launch(s);
    launch_reduce(slab, fc_ld_, splits, 0, nparam_, scale, g, s);
    post_launch(s);
    all_reduce(coalesced_buckets(), -1, s);
    launch_sgd_pack(model_, dtype_, ptr<float>(p_.params), g, ptr<float>(p_.mom), ptr<void>(p_.pack), nparam_, lr_,
                    momentum_, 1.0f / float(world_), ptr<int32_t>(p_.step), s, dp_skip());
    post_launch(s);
    return;
  }
  // SPLIT: the bucket groups in ready order (default: layers 2+3, then layer 1), each one's weight gradient and
  // reduce on the main stream, its buckets + update on the comm stream beside the next group's weight gradient
  (void)ps;
  const std::vector<Group> gs = groups();
  for (size_t k = 0; k < gs.size(); ++k) {
    const int splits = launch_head_wgrad(model_, dtype_, hb, B, fc_splits_, slab, fc_ld_, s, hrows, nullptr, gs[k].mask);
    post_launch(s);
    launch_reduce(slab, fc_ld_, splits, gs[k].p0, gs[k].p1, scale, g, s);
    post_launch(s);
    HIP_CHECK(hipEventRecord(events_[6 + k], s));
    comm_phase(static_cast<int>(k), events_[6 + k], k + 1 == gs.size());
  }
  HIP_CHECK(hipEventRecord(events_[0], comm_stream_));
  HIP_CHECK(hipStreamWaitEvent(s, events_[0], 0));
}

// LeNet with a communicator, after the fork (conv_bwd on `s`, FC wgrad on the aux stream).
// Every collective is issued on ONE stream per plan (JOIN: main, SPLIT: comm), in a fixed order, so all
// ranks enqueue the same RCCL sequence.
void Trainer::launch_lenet_comm_tail(int B, int nslab, int splits, hipStream_t s) {
  const float scale = 1.0f / float(B), gs = 1.0f / float(world_);
  const int cp = model_conv_params(model_);
  float* g = ptr<float>(p_.grad);
  launch_reduce(ptr<const float>(p_.slab_fc), fc_ld_, splits, cp, nparam_, scale, g, aux_stream_);
  post_launch(aux_stream_);
  HIP_CHECK(hipEventRecord(events_[5], aux_stream_));
  if (plan_ == Plan::JOIN) {
    launch_reduce(ptr<const float>(p_.slab_conv), cp, nslab, 0, cp, scale, g, s);
    post_launch(s);
    HIP_CHECK(hipStreamWaitEvent(s, events_[5], 0));
    all_reduce(coalesced_buckets(), -1, s);
    launch_sgd_pack(model_, dtype_, ptr<float>(p_.params), g, ptr<float>(p_.mom), ptr<void>(p_.pack), nparam_, lr_,
                    momentum_, gs, ptr<int32_t>(p_.step), s, dp_skip());
    post_launch(s);
    return;
  }
  throw std::logic_error("launch_lenet_comm_tail: JOIN only (SPLIT: launch_lenet_split_tail)");
}

// SPLIT: the FC bucket groups in ready order (default: ONE group, the whole FC head; a link-aware plan: e.g.
// fc3 + fc2, then fc1), each one's weight gradient (its job mask) and reduce on the aux stream beside conv_bwd;
// the comm stream sends a group's buckets as soon as it is reduced and updates its range right behind them; the
// conv buckets follow reduce(conv), then the conv update (+ step bump).  Per-parameter arithmetic is that of the
// one-group form (same tiles, splits, reduce tree), so every bucket plan gives bitwise-identical parameters.
// (A graph where another stream waits on an event recorded behind a captured RCCL call made hipStreamEndCapture
// segfault on ROCm 7.0's runtime, so only the main stream consumes the comm stream's completion, once, at the
// end of the step.)
void Trainer::launch_lenet_split_tail(int B, int nslab, hipStream_t s, const HeadBuffers& hb, int hrows) {
  const float scale = 1.0f / float(B);
  const int cp = model_conv_params(model_);
  float* g = ptr<float>(p_.grad);
  const std::vector<Group> gs = groups();
  int conv_g = -1;
  for (size_t k = 0; k < gs.size(); ++k) {
    if (gs[k].mask == 0) {  // the conv group (set_buckets: the last one)
      conv_g = static_cast<int>(k);
      continue;
    }
    trace("split: FC group wgrad + reduce (aux), AR + update (comm)");
    const int splits = launch_head_wgrad(model_, dtype_, hb, B, fc_splits_, ptr<float>(p_.slab_fc), fc_ld_, aux_stream_,
                                         hrows, nullptr, gs[k].mask);
    post_launch(aux_stream_);
    launch_reduce(ptr<const float>(p_.slab_fc), fc_ld_, splits, gs[k].p0, gs[k].p1, scale, g, aux_stream_);
    post_launch(aux_stream_);
    HIP_CHECK(hipEventRecord(events_[6 + k], aux_stream_));
    comm_phase(static_cast<int>(k), events_[6 + k], false);
  }
  if (conv_g < 0) throw std::logic_error("launch_lenet_split_tail: no conv bucket group");
  trace("split: reduce(conv)");
  launch_reduce(ptr<const float>(p_.slab_conv), cp, nslab, 0, cp, scale, g, s);
  post_launch(s);
  HIP_CHECK(hipEventRecord(events_[1], s));
  trace("split: comm AR(conv) + update(conv)");
  comm_phase(conv_g, events_[1], true);
  HIP_CHECK(hipEventRecord(events_[0], comm_stream_));
  HIP_CHECK(hipStreamWaitEvent(s, events_[0], 0));
  // the FC branch ended with an event the comm stream waited for, and the comm stream is joined above
  trace("split: done");
}

// Plan::OVERLAP (see trainer.h): each branch reduces its slab, all-reduces its range with its own one-shot
// instance and updates it (1/W folded into the update).  Same reduce trees and update kernels as JOIN, so at
// world 1 it is bitwise the local step.
void Trainer::launch_lenet_overlap(int B, int nslab, hipStream_t s, const HeadBuffers& hb, int hrows) {
  const float scale = 1.0f / float(B), gs = 1.0f / float(world_);
  const int cp = model_conv_params(model_);
  float* g = ptr<float>(p_.grad);
  const int splits =
      launch_head_wgrad(model_, dtype_, hb, B, fc_splits_, ptr<float>(p_.slab_fc), fc_ld_, aux_stream_, hrows);
  post_launch(aux_stream_);
  launch_reduce(ptr<const float>(p_.slab_fc), fc_ld_, splits, cp, nparam_, scale, g, aux_stream_);
  post_launch(aux_stream_);
  ov_fc_->all_reduce_sum_f32(g + cp, size_t(nparam_ - cp), aux_stream_);
  launch_sgd_pack_range(model_, dtype_, ptr<float>(p_.params), g, ptr<float>(p_.mom), ptr<void>(p_.pack), cp, nparam_,
                        lr_, momentum_, gs, nullptr, aux_stream_, ov_fc_->err_word());
  post_launch(aux_stream_);
  HIP_CHECK(hipEventRecord(events_[5], aux_stream_));
  launch_reduce(ptr<const float>(p_.slab_conv), cp, nslab, 0, cp, scale, g, s);
  post_launch(s);
  ov_conv_->all_reduce_sum_f32(g, size_t(cp), s);
  launch_sgd_pack_range(model_, dtype_, ptr<float>(p_.params), g, ptr<float>(p_.mom), ptr<void>(p_.pack), 0, cp, lr_,
                        momentum_, gs, ptr<int32_t>(p_.step), s, ov_conv_->err_word());
  post_launch(s);
}

std::vector<Bucket> Trainer::coalesced_buckets() const {
  // buckets sorted by offset; a bucket that starts where the previous one ends and belongs to a
  // different backward phase is merged into it (splits within a phase came from an explicit cap)
  std::vector<Bucket> b = buckets_, out;
  std::sort(b.begin(), b.end(), [](const Bucket& x, const Bucket& y) { return x.p0 < y.p0; });
  for (const Bucket& x : b) {
    if (!out.empty() && out.back().p1 == x.p0 && out.back().phase != x.phase) {
      out.back().p1 = x.p1;
      out.back().phase = x.phase;
    } else {
      out.push_back(x);
    }
  }
  return out;
}

void Trainer::train_step(int B, uintptr_t stream) { launch_step(B, S(stream)); }

void Trainer::eval_batch(uintptr_t images, uintptr_t labels, uintptr_t idx, int B, uintptr_t metrics,
                         uintptr_t stream) {
  hipStream_t s = S(stream);
  if (B <= 0) return;
  if (B > batch_) throw std::invalid_argument("eval_batch: B exceeds the trainer batch capacity");
  BatchRef br;
  br.images = ptr<const uint8_t>(images);
  br.labels = ptr<const uint8_t>(labels);
  br.idx_epoch = ptr<const int32_t>(idx);
  br.step_ptr = zero_counter_;
  br.batch_stride = 0;
  br.B = B;
  HeadBuffers hb = head_buffers(ptr<float>(metrics));
  if (model_ == ModelKind::LENET) {
    launch_lenet_conv_fwd(dtype_, false, br, conv_buffers(), s);
    post_launch(s);
  }
  launch_head(model_, dtype_, false, br, hb, head_rows_per_block(model_, dtype_, batch_), s);
  post_launch(s);
}

void Trainer::capture_into(hipStream_t s, int nsteps, hipGraph_t* graph, hipGraphExec_t* exec) {
  trace("capture: begin");
  HIP_CHECK(hipStreamBeginCapture(s, hipStreamCaptureModeRelaxed));
  try {
    // steps inside one graph leave their aux branch to the next step's head; the last one joins it
    aux_pending_ = false;
    for (int i = 0; i < nsteps; ++i) launch_step(batch_, s, defer_join() && i + 1 < nsteps);
    if (aux_pending_) throw std::logic_error("capture: aux branch left un-joined");
  } catch (...) {
    aux_pending_ = false;
    hipGraph_t g = nullptr;
    hipStreamEndCapture(s, &g);
    if (g) hipGraphDestroy(g);
    throw;
  }
  trace("capture: end");
  HIP_CHECK(hipStreamEndCapture(s, graph));
  trace("capture: instantiate");
  HIP_CHECK(hipGraphInstantiate(exec, *graph, nullptr, nullptr, 0));
  // device-side resources of the executable graph are set up now (setup time), not by its first launch
  HIP_CHECK(hipGraphUpload(*exec, s));
  trace("capture: done");
}

void Trainer::drop(GraphSlot& g) {
  if (g.exec) hipGraphExecDestroy(g.exec);
  if (g.graph) hipGraphDestroy(g.graph);
  g = GraphSlot{};
}

// Graphs are cached per (schedule, steps): switching plan / concurrent / conv_bwd grid selects a
// different cached graph instead of re-capturing, so a calibration can interleave the candidates'
// replays back to back; anything that changes the kernels' arguments clears the cache (invalidate).
uint64_t Trainer::schedule_key(int nsteps) const {
  return (static_cast<uint64_t>(nsteps) << 40) | (static_cast<uint64_t>(bucket_id_ & 255) << 32) |
         (static_cast<uint64_t>(bwd_blocks_) << 8) |
         (static_cast<uint64_t>(fwd_head_) << 4) | (static_cast<uint64_t>(comm_enabled_) << 3) | (static_cast<uint64_t>(concurrent_) << 2) |
         static_cast<uint64_t>(plan_);
}

const Trainer::GraphSlot* Trainer::find_graph(int nsteps) const {
  auto it = graphs_.find(schedule_key(nsteps));
  return it == graphs_.end() || !it->second.exec ? nullptr : &it->second;
}

void Trainer::capture(uintptr_t stream) {
  GraphSlot& g = graphs_[schedule_key(1)];
  if (g.exec) HIP_CHECK(hipStreamSynchronize(S(stream)));  // re-capture: the old exec may be in flight
  drop(g);
  capture_into(S(stream), 1, &g.graph, &g.exec);
}

// k consecutive steps in ONE graph: consecutive steps are plain stream-order edges inside it, so the
// per-launch gap between graphs is paid once per k steps; the device step counter addresses every
// step's batch, so the graph stays valid for any k-step window.
void Trainer::capture_multi(uintptr_t stream, int k) {
  if (k < 2) throw std::invalid_argument("capture_multi: k must be >= 2");
  GraphSlot& g = graphs_[schedule_key(k)];
  if (g.exec) HIP_CHECK(hipStreamSynchronize(S(stream)));
  drop(g);
  capture_into(S(stream), k, &g.graph, &g.exec);
  multi_k_ = k;
}

void Trainer::capture_n(uintptr_t stream, int n) {
  if (n < 2) throw std::invalid_argument("capture_n: n must be >= 2");
  GraphSlot& g = graphs_[schedule_key(n)];
  if (g.exec) HIP_CHECK(hipStreamSynchronize(S(stream)));
  drop(g);
  capture_into(S(stream), n, &g.graph, &g.exec);
}

bool Trainer::has_graph(int n) const { return find_graph(n) != nullptr; }

void Trainer::replay_n(uintptr_t stream, int n) {
  const GraphSlot* g = find_graph(n);
  if (!g) throw std::runtime_error("replay_n: no captured graph of that many steps for the current schedule");
  last_stream_ = S(stream);
  HIP_CHECK(hipGraphLaunch(g->exec, S(stream)));
  if (sync_debug()) HIP_CHECK(hipStreamSynchronize(S(stream)));
}

int Trainer::multi_steps() const { return multi_k_ > 1 && find_graph(multi_k_) ? multi_k_ : 0; }

bool Trainer::captured() const { return find_graph(1) != nullptr; }

void Trainer::replay(uintptr_t stream) {
  const GraphSlot* g = find_graph(1);
  if (!g) throw std::runtime_error("replay: no captured graph for the current schedule");
  last_stream_ = S(stream);
  HIP_CHECK(hipGraphLaunch(g->exec, S(stream)));
  if (sync_debug()) HIP_CHECK(hipStreamSynchronize(S(stream)));
}

void Trainer::replay_multi(uintptr_t stream) {
  const GraphSlot* g = multi_k_ > 1 ? find_graph(multi_k_) : nullptr;
  if (!g) throw std::runtime_error("replay_multi: no captured multi-step graph for the current schedule");
  last_stream_ = S(stream);
  HIP_CHECK(hipGraphLaunch(g->exec, S(stream)));
  if (sync_debug()) HIP_CHECK(hipStreamSynchronize(S(stream)));
}
