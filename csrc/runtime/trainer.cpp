// Static-schedule step orchestration (see trainer.h).
//
// Kernel sequence of one data-parallel step (reference CS5, survey §3; kernel IDs of §2.6):
//   LeNet, 1 GPU : conv_fwd -> head(fwd+loss+dgrad) -> wgrad(FC) -> conv_bwd -> reduce+sgd+pack (fused)
//   LeNet, W > 1 : conv_fwd -> head -> conv_bwd -> reduce(conv) -> [RCCL conv bucket on the comm
//                  stream] || wgrad(FC) -> reduce(FC) -> [RCCL FC bucket] -> join -> sgd_pack
//   MLP          : head -> wgrad -> reduce -> [RCCL bucket] -> join -> sgd_pack
// Why conv_bwd goes first with W > 1: its one-round grid (2 blocks/CU) fills every CU's register
// file for the kernel's whole life, so no collective can be co-resident with it; the conv bucket's
// all-reduce instead overlaps the FC wgrad/reduce (320 small blocks leave CUs free), and only the FC
// bucket (236.5 KB) remains exposed before the update.
// All launches are allocation- and sync-free; capture() records the sequence (both streams,
// RCCL included) into one hipGraph, so a training step costs one hipGraphLaunch on the host.
#include "trainer.h"

#include <cstdlib>
#include <stdexcept>

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
  const int cp = model_conv_params(model_);
  if (cp > 0) {
    buckets_.push_back({cp, nparam_, 0});
    buckets_.push_back({0, cp, 1});
  } else {
    buckets_.push_back({0, nparam_, 0});
  }
  HIP_CHECK(hipStreamCreateWithFlags(&comm_stream_, hipStreamNonBlocking));
  events_.resize(4);
  for (auto& e : events_) HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  HIP_CHECK(hipMalloc(&zero_counter_, 2 * sizeof(int32_t)));
  HIP_CHECK(hipMemset(zero_counter_, 0, 2 * sizeof(int32_t)));
}

Trainer::~Trainer() {
  if (exec_) hipGraphExecDestroy(exec_);
  if (graph_) hipGraphDestroy(graph_);
  for (auto& e : events_) hipEventDestroy(e);
  if (comm_stream_) hipStreamDestroy(comm_stream_);
  if (zero_counter_) hipFree(zero_counter_);
}

int Trainer::pack_size() const { return model_pack_size(model_); }
int Trainer::conv_params() const { return model_conv_params(model_); }
int Trainer::conv_slabs() const { return model_ == ModelKind::LENET ? lenet_conv_bwd_blocks(batch_) : 0; }

void Trainer::invalidate() {
  if (exec_) { hipGraphExecDestroy(exec_); exec_ = nullptr; }
  if (graph_) { hipGraphDestroy(graph_); graph_ = nullptr; }
}

BatchRef Trainer::batch_ref(int B) const {
  BatchRef br;
  br.images = ptr<const uint8_t>(p_.images);
  br.labels = ptr<const uint8_t>(p_.labels);
  br.idx_epoch = ptr<const int32_t>(p_.idx);
  br.step_ptr = ptr<const int32_t>(p_.step);
  br.batch_stride = batch_;
  br.B = B;
  return br;
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
  hb.ldB = ldb_;
  hb.seed = seed_;
  hb.drop_p = drop_p_;
  return hb;
}

LenetConvBuffers Trainer::conv_buffers() const {
  LenetConvBuffers cb;
  cb.params = ptr<const float>(p_.params);
  cb.pack = ptr<const void>(p_.pack);
  cb.p1 = ptr<void>(p_.p1);
  cb.m1 = ptr<uint8_t>(p_.m1);
  cb.p2 = ptr<void>(p_.p2);
  cb.m2 = ptr<uint8_t>(p_.m2);
  cb.dp2 = ptr<const void>(p_.dp2);
  cb.slab = ptr<float>(p_.slab_conv);
  static const int ablate = [] {
    const char* e = std::getenv("MNIST_AMD_ABLATE");
    return e ? std::atoi(e) : 0;
  }();
  cb.ablate = ablate;
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
  const HeadBuffers hb = head_buffers(ptr<float>(p_.metrics));
  if (model_ == ModelKind::LENET) {
    launch_lenet_conv_fwd(dtype_, true, br, conv_buffers(), s);
    post_launch(s);
  }
  const int hrows = launch_head(model_, dtype_, true, br, hb, head_rows_per_block(model_, dtype_, batch_), s);
  post_launch(s);
  launch_head_wgrad(model_, dtype_, hb, B, fc_splits_, ptr<float>(p_.slab_fc), nparam_, s, hrows);
  post_launch(s);
  if (model_ == ModelKind::LENET) {
    launch_lenet_conv_bwd(dtype_, br, conv_buffers(), nullptr, s);
    post_launch(s);
  }
}

void Trainer::reduce_grads(int B, uintptr_t stream) {
  hipStream_t s = S(stream);
  const float scale = 1.0f / float(B);
  const int cp = model_conv_params(model_);
  const HeadBuffers hb = head_buffers(ptr<float>(p_.metrics));
  (void)hb;
  // the split count actually used by launch_head_wgrad for this B
  const int KC = dtype_ == DType::BF16 ? 32 : 16;
  const int Bp = (B + KC - 1) / KC * KC;
  int splits = std::max(1, std::min(fc_splits_, Bp / KC));
  const int rlen = ((Bp + splits - 1) / splits + KC - 1) / KC * KC;
  splits = (Bp + rlen - 1) / rlen;
  launch_reduce(ptr<const float>(p_.slab_fc), nparam_, splits, cp, nparam_, scale, ptr<float>(p_.grad), s);
  post_launch(s);
  if (cp > 0) {
    launch_reduce(ptr<const float>(p_.slab_conv), cp, lenet_conv_bwd_blocks(B), 0, cp, scale, ptr<float>(p_.grad), s);
    post_launch(s);
  }
}

void Trainer::optimizer_step(float gscale, uintptr_t stream) {
  launch_sgd_pack(model_, dtype_, ptr<float>(p_.params), ptr<const float>(p_.grad), ptr<float>(p_.mom),
                  ptr<void>(p_.pack), nparam_, lr_, momentum_, gscale, ptr<int32_t>(p_.step), S(stream));
  post_launch(S(stream));
}

void Trainer::comm_phase(int phase, hipStream_t s) {
  if (!comm_) return;  // an attached communicator is always used (world 1 included: tests RCCL-in-graph)
  hipStream_t cs = s;
  if (overlap_) {
    HIP_CHECK(hipEventRecord(events_[phase], s));
    HIP_CHECK(hipStreamWaitEvent(comm_stream_, events_[phase], 0));
    cs = comm_stream_;
  }
  for (const Bucket& b : buckets_)
    if (b.phase == phase) comm_->all_reduce_sum_f32(ptr<float>(p_.grad) + b.p0, size_t(b.p1 - b.p0), cs);
}

void Trainer::launch_step(int B, hipStream_t s) {
  if (B <= 0 || B > batch_) throw std::invalid_argument("train_step: bad batch size");
  const BatchRef br = batch_ref(B);
  const HeadBuffers hb = head_buffers(ptr<float>(p_.metrics));
  const float scale = 1.0f / float(B);
  const int cp = model_conv_params(model_);
  if (model_ == ModelKind::LENET) {
    launch_lenet_conv_fwd(dtype_, true, br, conv_buffers(), s);
    post_launch(s);
  }
  const int hrows = launch_head(model_, dtype_, true, br, hb, head_rows_per_block(model_, dtype_, batch_), s);
  post_launch(s);
  if (comm_ && model_ == ModelKind::LENET) {
    // Multi-GPU order: conv backward FIRST, its (small) bucket all-reduce on the side stream then
    // overlaps the FC wgrad + reduce below.  conv_bwd's 2 blocks/CU fill every CU's register file
    // for the kernel's whole life, so a collective queued "behind" it could not start until it ended.
    int nslab = 0;
    launch_lenet_conv_bwd(dtype_, br, conv_buffers(), &nslab, s);
    post_launch(s);
    launch_reduce(ptr<const float>(p_.slab_conv), cp, nslab, 0, cp, scale, ptr<float>(p_.grad), s);
    post_launch(s);
    comm_phase(1, s);
  }
  const int splits = launch_head_wgrad(model_, dtype_, hb, B, fc_splits_, ptr<float>(p_.slab_fc), nparam_, s, hrows);
  post_launch(s);
  if (!comm_) {
    // single GPU: conv backward, then ONE fused reduce + SGD + pack kernel (2 boundaries fewer)
    int nslab = 0;
    if (model_ == ModelKind::LENET) {
      launch_lenet_conv_bwd(dtype_, br, conv_buffers(), &nslab, s);
      post_launch(s);
    }
    launch_reduce_sgd(model_, dtype_, ptr<const float>(p_.slab_conv), cp, nslab, ptr<const float>(p_.slab_fc),
                      nparam_, splits, cp, nparam_, scale, ptr<float>(p_.params), ptr<float>(p_.grad),
                      ptr<float>(p_.mom), ptr<void>(p_.pack), lr_, momentum_, ptr<int32_t>(p_.step), s);
    post_launch(s);
    return;
  }
  launch_reduce(ptr<const float>(p_.slab_fc), nparam_, splits, cp, nparam_, scale, ptr<float>(p_.grad), s);
  post_launch(s);
  comm_phase(0, s);
  if (comm_ && overlap_) {
    HIP_CHECK(hipEventRecord(events_[2], comm_stream_));
    HIP_CHECK(hipStreamWaitEvent(s, events_[2], 0));
  }
  launch_sgd_pack(model_, dtype_, ptr<float>(p_.params), ptr<const float>(p_.grad), ptr<float>(p_.mom),
                  ptr<void>(p_.pack), nparam_, lr_, momentum_, 1.0f / float(world_), ptr<int32_t>(p_.step), s);
  post_launch(s);
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

void Trainer::capture(uintptr_t stream) {
  invalidate();
  hipStream_t s = S(stream);
  HIP_CHECK(hipStreamBeginCapture(s, hipStreamCaptureModeRelaxed));
  try {
    launch_step(batch_, s);
  } catch (...) {
    hipGraph_t g = nullptr;
    hipStreamEndCapture(s, &g);
    if (g) hipGraphDestroy(g);
    throw;
  }
  HIP_CHECK(hipStreamEndCapture(s, &graph_));
  HIP_CHECK(hipGraphInstantiate(&exec_, graph_, nullptr, nullptr, 0));
}

void Trainer::replay(uintptr_t stream) {
  if (!exec_) throw std::runtime_error("replay: no captured graph");
  HIP_CHECK(hipGraphLaunch(exec_, S(stream)));
  if (sync_debug()) HIP_CHECK(hipStreamSynchronize(S(stream)));
}
