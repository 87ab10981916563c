// Host-side launch interface of the HIP kernels (all launches are stream-ordered,
// allocation-free and synchronisation-free, so the whole step is hipGraph-capturable).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

enum class ModelKind : int { MLP = 0, LENET = 1 };
enum class DType : int { F32 = 0, BF16 = 1 };

// Batch addressing shared by all kernels of a step: the rows of the current step are
// idx_epoch[*step_ptr * batch_stride + r], r < B.  A device-side step counter (bumped
// by the optimizer kernel) keeps captured graphs valid across steps.
struct BatchRef {
  const uint8_t* images;     // [N][784] uint8, HBM-resident dataset
  const uint8_t* labels;     // [N]
  const int32_t* idx_epoch;  // this rank's sample order for the epoch
  const int32_t* step_ptr;   // device step counter
  int32_t batch_stride;      // regular batch size
  int32_t B;                 // rows in this batch (<= batch_stride)
  // Small-batch MLP training (layer-1 split path): the batch's samples gathered one step AHEAD, by the
  // previous step's head kernel (or launch_gather_next after the step counter is set): [batch][784]
  // raw pixels and [batch] labels of step step_ptr[0].  step_ptr[2] = number of loaded indices.
  // Null: every kernel gathers through idx_epoch itself.
  uint8_t* xnext = nullptr;
  uint8_t* ynext = nullptr;
  // XCD-contiguous work mapping (xcd_unit in common.h): conv_fwd, the head and conv_bwd give XCD x the
  // same contiguous eighth of the batch, so a kernel reads what the previous one wrote from its own L2
  int32_t xcd = 0;
};

// Gather the rows of the CURRENT step (step_ptr[0]) into br.xnext / br.ynext (primes the look-ahead
// after the step counter was set from the host).
void launch_gather_next(const BatchRef& br, hipStream_t s);

struct HeadBuffers {
  const float* params;   // fp32 master slab
  const void* pack;      // packed T operands
  const void* xin;       // LeNet: p2 [B][K0P] (T); MLP: unused (gather)
  void* xT;              // [K0P][ldB]  layer-1 input, transposed (wgrad operand)
  void* h1T;             // [N1P][ldB]
  void* h2T;             // [N2P][ldB]
  void* dy1T;            // [N1P][ldB]
  void* dy2T;            // [N2P][ldB]
  void* dy3T;            // [16][ldB]
  void* dx;              // LeNet: dp2 [B][K0P]
  float* metrics;        // [head grid][4]: per-workgroup [loss_sum, correct, count, 0] (metric_rows(batch) rows)
  float* z1p;            // [L1_KSPLIT][N1P][ldB] fp32 layer-1 partial sums (small-batch split path) or null
  unsigned long long* stamps;  // optional phase timestamps [block][16] (MNIST_AMD_STAMPS profiling) or null
  int32_t ldB;
  uint32_t seed;
  float drop_p;
  int32_t xcd = 0;       // the head kernel used the XCD-contiguous row mapping (BatchRef::xcd)
  int32_t ablate = 0;    // diagnostics only (MNIST_AMD_HEAD_ABLATE): bit 0 = skip the X^T stores (wrong wgrad)
  const uint8_t* yb = nullptr;  // LeNet head16: this step's labels in batch order (LenetConvBuffers::yb) or null
};

struct LenetConvBuffers {
  const float* params;
  const void* pack;
  void* p1;              // [B][196][8] T  pool1 output (NHWC, C padded to 8)
  uint8_t* m1;           // [B][196][8]    pool1 argmax(2b)|relu-positive(bit 2)
  void* p2;              // [B][K0P=416] T pool2 output (NCHW flatten), cols >=400 zero
  uint8_t* m2;           // [B][400]
  const void* dp2;       // [B][416] T   (backward input)
  float* slab;           // conv partial grads, row per workgroup: [G][2572]
  // optional [B][784] u8: this step's pixel rows in batch order, written by conv_fwd_kernel (training) and read
  // by conv_bwd instead of re-gathering them through the sample index (small batches: the index chain
  // step counter -> index -> pixels was conv_bwd's start-up latency); null = gather by index
  uint8_t* xb = nullptr;
  uint8_t* yb = nullptr;  // [B] u8: the labels in batch order, written with xb (read by the head16 head)
  int ablate = 0;        // diagnostics only: bitmask of phases to skip (timing ablation, wrong results)
  unsigned long long* stamps = nullptr;  // optional phase timestamps (profiling): fwd [block][16], bwd [block][16]
};

// Timing-ablation switches (MNIST_AMD_ABLATE / MNIST_AMD_HEAD_ABLATE: skip kernel phases, WRONG results).
// Compiled in only by an ablation build (-DMNIST_AMD_ABLATION_BUILD, scripts/ablate.sh); in the normal
// build every ABLATED() is a constant false and the runtime refuses the variables instead of silently
// training on skipped phases.
#ifdef MNIST_AMD_ABLATION_BUILD
#define ABLATED(flags, bit) (((flags) & (bit)) != 0)
#else
#define ABLATED(flags, bit) false
#endif

// MNIST_AMD_STAMPS profiling buffer: [STAMP_ROWS][16] uint64 wall-clock stamps, one row per workgroup,
// each kernel in its own row range (scripts/stamps.py reads the same layout)
constexpr int STAMP_HEAD = 0;          // head workgroups            [0, 1024)
constexpr int STAMP_CONV_BWD = 1024;   // conv_bwd MODE 0/1 blocks   [1024, 1536), MODE 2 blocks [1536, 2048)
constexpr int STAMP_CONV_FWD = 2048;   // conv_fwd                   [2048, 3072)
constexpr int STAMP_WGRAD = 3072;      // grouped FC wgrad           [3072, 3584)
constexpr int STAMP_L1 = 3584;         // layer-1 K-split GEMM       [3584, 4096)
constexpr int STAMP_HEAD_ARRIVE = 4096;  // head: per-wave softmax-barrier arrival, slot = wave [4096, 4608)
constexpr int STAMP_BWD_HWLOC = 4608;  // conv_bwd MODE 0: workgroup hardware location, slot 0 [4608, 5120)
constexpr int STAMP_ROWS = 5120;

int head_rows_per_block(ModelKind m, DType t, int B);
// rows of a metrics buffer: one per head workgroup of any batch <= B (16-row tiles at the smallest)
constexpr int metric_rows(int B) { return (B + 31) / 32 * 2; }
// Small batches (B <= L1_SPLIT_MAX_B) run layer 1 as a separate many-workgroup GEMM split L1_KSPLIT
// ways over K (the head kernel alone would put the whole 784-deep GEMM on B/16 CUs).
constexpr int L1_KSPLIT = 4;
constexpr int L1_SPLIT_MAX_B = 1024;

// returns the batch rows per workgroup it used
int launch_head(ModelKind m, DType t, bool train, const BatchRef& br, const HeadBuffers& hb,
                 int rows_per_block, hipStream_t s);

// Grouped weight-gradient GEMM over the batch (split-K over rows): writes S slabs, returns S.
// Optional SGD epilogue of the weight-gradient GEMM (one GPU, ONE batch split: each output element is
// the whole gradient): g = scale * dW, momentum, parameter, packed operand images and the device step
// counters updated in place -- the separate reduce + SGD kernel and its boundary disappear.  Bitwise
// equal to the wgrad -> reduce_sgd pair (a one-slab reduce is scale * dW).
struct SgdFuse {
  float scale, lr, momentum;
  float* params;
  float* grad;
  float* mom;
  void* pack;
  int32_t* step_ptr;
};

// job_mask: which layers' weight gradients to compute (bit l = layer l+1; 7 = all three).  A subset
// writes only those layers' slab columns (the MLP's SPLIT plan sends layers 2+3 while layer 1 computes).
int launch_head_wgrad(ModelKind m, DType t, const HeadBuffers& hb, int B, int splits, float* slab,
                      int slab_ld, hipStream_t s, int head_rows = 0, const SgdFuse* fuse = nullptr,
                      int job_mask = 7);

void launch_lenet_conv_fwd(DType t, bool train, const BatchRef& br, const LenetConvBuffers& cb,
                           hipStream_t s);
// LeNet training forward + FC head (fwd, softmax-CE, dgrad) in one kernel (lenet.hip fwd_head_kernel):
// replaces launch_lenet_conv_fwd + launch_head for bf16 batches B >= 4096, B % 16 == 0 (Trainer::set_fwd_head(false)
// selects the two kernels).  Returns the head-rows value for launch_head_wgrad's XCD-aware mapping (32: the fused
// kernel's 16-row units give each XCD the same contiguous eighth of the batch as 32-row head tiles), or 0
// when it does not apply (the caller launches the two kernels).
int launch_lenet_fwd_head(DType t, const BatchRef& br, const LenetConvBuffers& cb, const HeadBuffers& hb,
                          hipStream_t s);
bool lenet_fwd_head_applies(DType t, int B);
// LeNet training head alone as the 16-row register-B head (lenet.hip head16_kernel) on the pool2 rows of
// conv_fwd: bf16, B <= 2048.  Returns launch_head's rows value, or 0 when it
// does not apply (the caller launches launch_head).
int launch_lenet_head16(DType t, const BatchRef& br, const HeadBuffers& hb, hipStream_t s);
// target_blocks: workgroup count to aim for (0 = default, one full round of 2 blocks per CU); each
// block walks ceil(B / target) images, so a smaller target leaves whole CUs free (for RCCL kernels).
void launch_lenet_conv_bwd(DType t, const BatchRef& br, const LenetConvBuffers& cb, int* nslab_out,
                           hipStream_t s, int target_blocks = 0);
// Small batches (one GPU, one FC batch split): conv_bwd + the FC weight gradient with its SGD update (as
// launch_head_wgrad with `fuse`) in ONE kernel; returns the conv slab count (the conv update follows).
int launch_lenet_conv_bwd_fc(DType t, const BatchRef& br, const LenetConvBuffers& cb, const HeadBuffers& hb,
                             const SgdFuse& fuse, hipStream_t s, int target_blocks = 0);
int lenet_conv_bwd_blocks(int B, int target_blocks = 0);
int lenet_conv_bwd_max_blocks(int B, int target_blocks = 0);  // slab rows needed for any batch <= B

// One-shot all-reduce over xGMI peer memory (oneshot.hip; host side csrc/runtime/oneshot.h): in-place SUM of
// `count` floats at buf; peer_data / peer_flags are device tables of every rank's receive region.
void launch_oneshot_allreduce(float* buf, int count, int rank, int world, int max_count, float* const* peer_data,
                              uint32_t* const* peer_flags, uint32_t* seq, uint32_t* err, int nblk,
                              unsigned long long timeout_ticks, hipStream_t s, unsigned long long* stamps = nullptr);

// grad[p] = scale * sum_s slab[s][p]  for p in [p0, p1)
void launch_reduce(const float* slab, int slab_ld, int nslab, int p0, int p1, float scale, float* grad,
                   hipStream_t s);

// SGD (+momentum) on the flat fp32 slab, then re-pack operands; optionally bumps the step counter.
// `skip`: optional device word (a one-shot all-reduce's latched error, oneshot.hip): when it reads non-zero the
// parameters and momentum are left as they are (the gradient may hold a partial sum); the step counter still moves.
void launch_sgd_pack(ModelKind m, DType t, float* params, const float* grad, float* mom, void* pack,
                     int nparam, float lr, float momentum, float gscale, int32_t* step_ptr,
                     hipStream_t s, const uint32_t* skip = nullptr);
// Same, over the parameter range [p0, p1) only (per-bucket updates of the split multi-GPU plan).
void launch_sgd_pack_range(ModelKind m, DType t, float* params, const float* grad, float* mom, void* pack, int p0,
                           int p1, float lr, float momentum, float gscale, int32_t* step_ptr, hipStream_t s,
                           const uint32_t* skip = nullptr);
void launch_pack(ModelKind m, DType t, const float* params, void* pack, int nparam, hipStream_t s);
// Bounded device busy-wait (watchdog tests).
void launch_spin(double seconds, hipStream_t s);
// Fused gradient reduce + SGD + pack + step bump (no all-reduce between them: single-GPU runs).
void launch_reduce_sgd(ModelKind m, DType t, const float* slab_a, int lda, int na, const float* slab_b, int ldb,
                       int nb, int split, int p0, int n, float scale, float* params, float* grad, float* mom,
                       void* pack, float lr, float momentum, int32_t* step_ptr, hipStream_t s);  // params [p0, n)

void launch_gather_normalize(DType t, const BatchRef& br, void* out, int ld, hipStream_t s);

// model geometry queried by the host runtime
int model_nparam(ModelKind m);
int model_conv_params(ModelKind m);
// first parameter of backward phase 0 (the late layers, whose gradients backward produces first):
// LeNet: conv_params (phase 0 = FC head); MLP: the layer-2 weight (phase 0 = layers 2+3)
int model_phase_split(ModelKind m);
int model_pack_size(ModelKind m);
// First parameter of FC weight-gradient job j (0: first FC layer, 1: second, 2: third; 3: nparam): the
// launch_head_wgrad job-mask bit j computes exactly the gradients [model_job_begin(j), model_job_begin(j + 1))
int model_job_begin(ModelKind m, int job);
