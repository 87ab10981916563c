// Fused fully-connected head: forward, softmax cross-entropy, and backward (dgrad) in ONE
// kernel per R-row tile of the batch, plus the grouped weight-gradient GEMM.
//
// Replaces, for the reference MLP (ddp_tutorial_cpu.py:43-53, step loop :70-78), the ATen
// sequence addmm -> relu -> native_dropout -> addmm -> relu -> mm -> _log_softmax ->
// nll_loss -> nll_loss_backward -> _log_softmax_backward -> mm x2 -> threshold_backward ->
// addmm-backward ... (survey §2.6 K1..K13) and, for LeNet-5, its three Linear layers.
// All activations of a tile stay in LDS; the only HBM traffic is the input tile, the packed
// weights (L2 resident) and the transposed activations/gradients that the wgrad GEMM needs.
//
// Per tile (4 waves, R = 16*MT rows):
//   stage X -> LDS (MLP: gather dataset[idx[r]] + normalise, fused; LeNet: pool2 rows)
//   H1 = relu(X W1^T + b1) [dropout]      H2 = relu(H1 W2^T + b2)      Z = H2 W3^T [+ b3]
//   loss/acc + dZ = softmax(Z) - onehot(y)         (1/B applied by the gradient reduce)
//   dH2 = (dZ W3) * [H2>0]    dH1 = (dH2 W2) * [H1>0] (/keep)    [LeNet] dX = dH1 W1
// Every product is a 16x16 MFMA tile loop (common.h); epilogues fuse bias, ReLU, dropout
// masks, padding and the transposed global stores.
#include <algorithm>
#include <cstdlib>
#include <stdexcept>
#include <type_traits>

#include "common.h"
#include "launch.h"
#include "models.h"
#include "wgrad.h"

namespace {
using wg::WgArgs;
using wg::WgJob;
using wg::wgrad_sgd_tile;

// fp32 products as exact 3-part bf16 splits (common.h Mma<float>::mma_s: three 16x16x32 bf16 MFMAs per 16-k
// chunk, 48 cycles, instead of 4 x 32 for v_mfma_f32_16x16x4_f32; ~2^-24 relative, every fp32 tolerance test
// passes): the weight-gradient GEMMs (wg_mma; the MLP's from B = 4096, wgrad_launch) and the head's products at
// row tiles of >= 32 (head_mma<T, true>; the compiler hoists the cut of the B fragment the row tiles share).
// Measured against exact fp32 MFMA (profiles/r5_session1/hsplit, hsplit2): weight gradient -2 % LeNet fp32
// B=8192, -3 % B=1024, -6 % MLP fp32 B=8192 (+6 % at B=1024); the head split another -3 % on the MLP at B=8192
// but +6 % (MLP) / +1.5 % (LeNet) at B=128 (16-row tiles, l1_split_kernel).
#ifndef MNIST_AMD_HEAD_SPLIT
#define MNIST_AMD_HEAD_SPLIT 1
#endif
#ifndef MNIST_AMD_WGRAD_SPLIT
#define MNIST_AMD_WGRAD_SPLIT 1
#endif
template <typename T, bool SPLIT = true, typename F>
DEV void head_mma(f32x4& acc, const F& a, const F& b) {
  if constexpr (sizeof(T) == 4 && SPLIT && MNIST_AMD_HEAD_SPLIT) Mma<float>::mma_s(acc, a, b);
  else Mma<T>::mma(acc, a, b);
}
template <typename T, bool SPLIT = true, typename F>
DEV void wg_mma(f32x4& acc, const F& a, const F& b) {
  if constexpr (sizeof(T) == 4 && SPLIT && MNIST_AMD_WGRAD_SPLIT) Mma<float>::mma_s(acc, a, b);
  else Mma<T>::mma(acc, a, b);
}

template <typename T, class H, int MT, bool PRE = false>
struct HeadSmem {
  static constexpr int R = MT * 16;
  // fp32 (one k per MFMA input register): the dgrad products read W2 / W3 themselves with a k-strided
  // access, so their transposed images are not staged (FT) and the weights fit in LDS next to the tile
  static constexpr bool FT = sizeof(T) == 4;
  static constexpr int PX = H::K0P + 8;
  static constexpr int XROWS = PRE ? 0 : R;  // PRE: layer 1 ran in l1_split_kernel, X is never staged
  static constexpr int P1 = H::N1P + 8;
  static constexpr int P2 = H::N2P + 8;
  static constexpr int PD = H::NCK + 8;
  static constexpr int OFF_X = 0;
  static constexpr int OFF_H1 = rup(OFF_X + XROWS * PX * (int)sizeof(T), 16);
  static constexpr int OFF_H2 = rup(OFF_H1 + R * P1 * (int)sizeof(T), 16);
  static constexpr int OFF_D = rup(OFF_H2 + R * P2 * (int)sizeof(T), 16);
  static constexpr int OFF_L = rup(OFF_D + R * PD * (int)sizeof(T), 16);
  static constexpr int OFF_I = OFF_L + R * 16 * 4;
  static constexpr int OFF_LAB = OFF_I + R * 4;                       // [R] int labels of the tile
  static constexpr int OFF_B = OFF_LAB + R * 4;                       // fp32 biases b1 [N1P] | b2 [N2P] | b3 [16]
  static constexpr int OFF_PART = OFF_B + (H::N1P + H::N2P + 16) * 4;  // [16 waves][4] f32 metric partials
  static constexpr int BASE_END = rup(OFF_PART + 16 * 4 * 4, 16);
  // Layer-2/3 weights (forward and dgrad operand images) staged once per workgroup, rows padded by 8
  // elements (<= 2-way ds_read_b128 conflicts), when they fit beside the activations: every phase
  // after L1 then reads its B operand from LDS instead of waiting on an L2/MALL round trip.
  // (FT: pitch = 4 mod 8 dwords, so the 4 k-rows a k-strided fragment spans land on different banks)
  static constexpr int PW2 = H::N1P + (FT ? 4 : 8), PW2T = H::N2P + 8, PW3 = H::N2P + (FT ? 4 : 8),
                       PW3T = H::NCK + 8;
  static constexpr int OFF_W2 = BASE_END;                                          // [N2P][PW2]
  static constexpr int OFF_W2T = rup(OFF_W2 + H::N2P * PW2 * (int)sizeof(T), 16);  // [N1P][PW2T] (not FT)
  static constexpr int OFF_W3 = rup(OFF_W2T + (FT ? 0 : H::N1P * PW2T * (int)sizeof(T)), 16); // [16][PW3]
  static constexpr int OFF_W3T = rup(OFF_W3 + 16 * PW3 * (int)sizeof(T), 16);      // [N2P][PW3T] (not FT)
  static constexpr int W_END = rup(OFF_W3T + (FT ? 0 : H::N2P * PW3T * (int)sizeof(T)), 16);
  static constexpr bool WLDS = W_END <= 160 * 1024;
  static constexpr int TOTAL = WLDS ? W_END : BASE_END;
  static constexpr bool FITS = TOTAL <= 160 * 1024;
};

// store 4 consecutive-row values of one column into a transposed [col][ldB] buffer
template <typename T>
DEV void store_col4(T* base, float a, float b, float c, float d) {
  if constexpr (sizeof(T) == 2) {
    bf16x4 v; v[0] = (bf16)a; v[1] = (bf16)b; v[2] = (bf16)c; v[3] = (bf16)d;
    *reinterpret_cast<bf16x4*>(base) = v;
  } else {
    *reinterpret_cast<f32x4*>(base) = f32x4{a, b, c, d};
  }
}

// MFMA B fragment whose KV consecutive k values sit `pitch` elements apart (one k per row)
template <typename T>
DEV typename Mma<T>::Frag load_kstrided(const T* p, int pitch) {
  typename Mma<T>::Frag f;
#pragma unroll
  for (int j = 0; j < Mma<T>::KV; ++j) Mma<T>::set(f, j, to_f(p[j * pitch]));
  return f;
}

// copy a [ROWS][COLS] T matrix (COLS a multiple of 16 B) into LDS with row pitch PITCH, in two halves:
// load() issues the thread's global loads into registers, store() writes them to LDS -- so a kernel can
// issue the loads of several matrices (and of its input tile) before the first LDS store: one memory
// round trip for the whole staging phase instead of one per matrix
template <typename T, int NT, int ROWS, int COLS, int PITCH>
struct RowStager {
  static constexpr int VE = 16 / (int)sizeof(T), CV = COLS / VE, N = ROWS * CV, IT = (N + NT - 1) / NT;
  // native vector registers (HIP's uint4 class kept the member array on the scratch stack)
  u32x4 v[IT];
  DEV void load(const T* src, int tid) {
#pragma unroll
    for (int i = 0; i < IT; ++i) {
      const int e = min(tid + i * NT, N - 1);
      v[i] = *reinterpret_cast<const u32x4*>(src + (e / CV) * COLS + (e % CV) * VE);
    }
  }
  DEV void store(T* dst, int tid) const {
#pragma unroll
    for (int i = 0; i < IT; ++i) {
      const int e = tid + i * NT;
      if (e < N) *reinterpret_cast<u32x4*>(dst + (e / CV) * PITCH + (e % CV) * VE) = v[i];
    }
  }
};

// Phase timeline of one workgroup (measured with MNIST_AMD_STAMPS, LeNet bf16 B=8192, 64-row tiles,
// 16 waves; before this layout every phase was dominated by its B-operand fetch from L2/MALL):
//   stage X + W2/W3 images + biases (one barrier; idx and the first L1 operands are in flight with it)
//   L1 -> L2 -> L3 -> softmax-CE -> dH2 -> dH1 -> dX, one barrier each; the dX operands (W1^T, the
//   largest) are fetched into registers while softmax, dH2 and dH1 run.
template <typename T, class H, int MT, bool TRAIN, bool PRE, int NWV = 4>
__global__ __launch_bounds__(NWV * 64) void head_kernel(BatchRef br, HeadBuffers hb) {
  using S = HeadSmem<T, H, MT, PRE>;
  using M = Mma<T>;
  using Frag = typename M::Frag;
  constexpr int R = S::R, KV = M::KV, KC = M::KC, NTH = NWV * 64;
  constexpr bool HSP = !PRE && MT >= 2;  // fp32: products as 3-part bf16 splits (head_mma)
  static_assert(S::FITS, "head tile does not fit in LDS");
  __shared__ __attribute__((aligned(16))) char smem[S::TOTAL];
  T* sX = reinterpret_cast<T*>(smem + S::OFF_X);
  T* sH1 = reinterpret_cast<T*>(smem + S::OFF_H1);
  T* sH2 = reinterpret_cast<T*>(smem + S::OFF_H2);
  T* sD = reinterpret_cast<T*>(smem + S::OFF_D);
  float* sLog = reinterpret_cast<float*>(smem + S::OFF_L);
  int* sIdx = reinterpret_cast<int*>(smem + S::OFF_I);
  int* sLab = reinterpret_cast<int*>(smem + S::OFF_LAB);
  float* sB1 = reinterpret_cast<float*>(smem + S::OFF_B);
  float* sB2 = sB1 + H::N1P;
  float* sB3 = sB2 + H::N2P;
  float* sPart = reinterpret_cast<float*>(smem + S::OFF_PART);

  const int tid = threadIdx.x, lane = tid & 63, w = wave_id();
  const int row = lane & 15, grp = lane >> 4;
  const int r0 = xcd_unit(blockIdx.x, gridDim.x, br.xcd) * R;  // rows conv_fwd wrote on this XCD
  const int B = br.B;
  // The device step counters are read where they are needed, not here: a scalar load issued at the top
  // made every later scalar-operand wait (lgkmcnt(0)) -- the first weight loads included -- wait for it.
  // (Exception: the MLP head gathers and draws dropout masks with them early on, so for it -- the model
  //  with the dropout / look-ahead paths -- both counters are still read here.)
  auto batch_idx = [&] { return br.idx_epoch + (size_t)br.step_ptr[0] * br.batch_stride; };
  constexpr bool EARLY_STEP = H::GATHER || H::DROPOUT;
  const int step_early = EARLY_STEP ? br.step_ptr[0] : 0;
  const int gstep_early = EARLY_STEP ? br.step_ptr[1] : 0;
  const T* pack = reinterpret_cast<const T*>(hb.pack);
  const float* prm = hb.params;
  const int ldB = hb.ldB;

  // optional per-phase wall-clock stamps (MNIST_AMD_STAMPS; thread 0, one vector store each)
  auto stamp = [&](int k) {
    if (hb.stamps && tid == 0 && blockIdx.x < 1024) hb.stamps[blockIdx.x * 16 + k] = wall_clock64();
  };
  stamp(0);

  // B operands of each phase: LDS images when they fit (WLDS), else -- WX: a model without an input
  // gradient (the MLP), whose X tile is dead after layer 1 -- the same images staged into the X region
  // after layer 1 (loads issued before it), else the packed global copies
  constexpr bool WX = !S::WLDS && !PRE && !H::DX && S::W_END - S::OFF_W2 <= S::OFF_H1 - S::OFF_X;
  constexpr bool WIN = S::WLDS || WX;            // B operands of layers 2/3 and their dgrads from LDS
  constexpr int WOFF = WX ? S::OFF_X - S::OFF_W2 : 0;  // where the weight images live
  const T* bW2 = WIN ? reinterpret_cast<const T*>(smem + WOFF + S::OFF_W2) : pack + H::F2;
  const T* bW2T = WIN ? reinterpret_cast<const T*>(smem + WOFF + S::OFF_W2T) : pack + H::F2T;
  const T* bW3 = WIN ? reinterpret_cast<const T*>(smem + WOFF + S::OFF_W3) : pack + H::F3;
  const T* bW3T = WIN ? reinterpret_cast<const T*>(smem + WOFF + S::OFF_W3T) : pack + H::F3T;
  constexpr int LW2 = WIN ? S::PW2 : H::N1P, LW2T = WIN ? S::PW2T : H::N2P;
  constexpr int LW3 = WIN ? S::PW3 : H::N2P, LW3T = WIN ? S::PW3T : H::NCK;

  // ---- PRE: this thread's layer-1 partial sums (written by l1_split_kernel), issued first: their
  //      latency overlaps the weight staging instead of following it
  constexpr int PE = PRE ? (H::N1P * R + NTH - 1) / NTH : 1;
  float zpre[PE][L1_KSPLIT];
  if constexpr (PRE) {
#pragma unroll
    for (int j = 0; j < PE; ++j) {
      const int e = min(tid + j * NTH, H::N1P * R - 1), n = e / R, rg = r0 + e % R;
#pragma unroll
      for (int q = 0; q < L1_KSPLIT; ++q) zpre[j][q] = hb.z1p[((size_t)q * H::N1P + n) * ldB + rg];
    }
  }

  // ---- L1 operands of this wave's first n-tile: issued first, in flight during the staging.
  //      KS1: with at least two waves per layer-1 n-tile, the 784/400-deep K is split in two halves
  //      (wave w: n-tile w % NT1, half w / NT1); the second half's accumulators are added through LDS.
  //      Halves each wave's chain of B-fragment fetches (the MLP's 25-chunk layer 1 ran on 8 of the 16
  //      waves, 10.4 us of a 23 us head).
  constexpr int NT1 = H::N1P / 16, KCH1 = H::K0P / KC;
  constexpr bool KS1 = !PRE && NWV >= 2 * NT1 && NT1 * MT * 64 * 16 <= R * S::PX * (int)sizeof(T);
  constexpr int KH1 = KS1 ? (KCH1 + 1) / 2 : KCH1;  // chunks of the first half (per-wave chunk count bound)
  constexpr bool PF1 = !PRE && KH1 <= 16;  // <= 64 VGPRs of prefetched fragments
  const int l1_nt = KS1 ? w % NT1 : w, l1_half = KS1 ? w / NT1 : 0;
  const int l1_k0 = l1_half * KH1, l1_k1 = KS1 ? (l1_half ? KCH1 : KH1) : KCH1;
  const bool l1_live = KS1 ? (NWV == 2 * NT1 || w < 2 * NT1) : w < NT1;  // constant true when every wave works
  Frag b1pre[PF1 ? KH1 : 1];
  auto prefetch_b1 = [&] {
    if constexpr (PF1) {
      if (l1_live) {
        const T* bp = pack + H::FM1 + (l1_nt * KCH1 * 64 + lane) * KV;  // fragment-major W1 (models.h)
#pragma unroll
        for (int kc = 0; kc < KH1; ++kc) b1pre[kc] = M::load(bp + min(l1_k0 + kc, KCH1 - 1) * 64 * KV);
      }
    }
  };
  // (the gathering head issues them after its pixel loads: vmcnt counts in order, so prefetched W1
  //  fragments issued first would make the gather's conversion wait for all of W1)
  if constexpr (!H::GATHER) prefetch_b1();

  // ---- look-ahead (MLP training): this step's pixels / labels come from xnext / ynext (gathered by the
  //      previous step, in batch-row order), and this kernel gathers the NEXT step's rows of its tile into
  //      xnext / ynext (consumed by the next l1_split / head; this step's l1_split -- small batches -- has
  //      already read xnext, and without it this kernel read its own rows during the staging: a workgroup
  //      only ever touches its own rows)
  constexpr bool LOOK = H::GATHER && TRAIN;
  const bool look = LOOK && br.xnext != nullptr;  // uniform
  constexpr int GCH = R * 49, GIT2 = LOOK ? (GCH + NTH - 1) / NTH : 1;  // 16-byte chunks of the tile's rows
  int gidx[GIT2];

  // ---- staging: indices, weights, biases (+ the input tile; the MLP gather needs sIdx first)
  //      Every global load of the phase is issued before the first LDS / global store (the stores of
  //      one matrix used to wait for its loads before the next matrix's loads were issued, and the
  //      input tile's loads could not move above the previous row's xT global stores): one round trip.
  // (the tile's sample indices: the MLP gather needs them in LDS before its X gather; with a staged
  //  input tile only the labels need them, and the last wave loads both after the barrier -- the
  //  step counter -> index chain in wave 0 held its weight loads back and made it the barrier's straggler)
  if (look) {
    if (tid < R) sLab[tid] = (r0 + tid < B) ? (int)br.ynext[r0 + tid] : 0;
  } else if (H::GATHER && tid < R) {
    sIdx[tid] = (r0 + tid < B) ? br.idx_epoch[(size_t)step_early * br.batch_stride + r0 + tid] : -1;
  }
  RowStager<T, NTH, H::N2P, H::N1P, S::PW2> st_w2;
  RowStager<T, NTH, H::N1P, H::N2P, S::PW2T> st_w2t;
  RowStager<T, NTH, H::N2P, H::NCK, S::PW3T> st_w3t;
  RowStager<T, NTH, 16, H::N2P, S::PW3> st_w3;
  constexpr bool STW_T = TRAIN && !S::FT;  // transposed W2 / W3 images staged
  if constexpr (S::WLDS) {
    st_w2.load(pack + H::F2, tid);
    if constexpr (STW_T) {
      st_w2t.load(pack + H::F2T, tid);
      st_w3t.load(pack + H::F3T, tid);
    }
    st_w3.load(pack + H::F3, tid);
  }
  constexpr int NBIAS = H::N1P + H::N2P + 16, ITB = (NBIAS + NTH - 1) / NTH;
  // branch-free (a load inside a lane-divergent branch is followed by vmcnt(0) at the branch join, which
  // serialised the staging loads): every lane loads a clamped address, the value is selected at use
  float bias_v[ITB];
  auto bias_src = [](int e, bool& live) {
    int q;
    if (e < H::N1P) { live = e < H::N1; q = H::B1 + min(e, H::N1 - 1); }
    else if (e < H::N1P + H::N2P) { live = e - H::N1P < H::N2; q = H::B2 + min(e - H::N1P, H::N2 - 1); }
    else if constexpr (H::BIAS3) { live = e < NBIAS && e - H::N1P - H::N2P < H::NC; q = H::B3 + min(max(e - H::N1P - H::N2P, 0), H::NC - 1); }
    else { live = false; q = H::B1; }  // no layer-3 bias: any in-range address, value unused
    return q;
  };
#pragma unroll
  for (int i = 0; i < ITB; ++i) {
    bool live;
    const int q = bias_src(tid + i * NTH, live);
    bias_v[i] = prm[q];
  }
  // input tile rows (LeNet: pool2 rows written by conv_fwd), loaded with the weights.  A thread owns one
  // 16-byte k-chunk of 4 consecutive rows, so its xT (transposed) stores are 4 rows wide: one 4-element
  // store per k instead of four 1-element stores (16 lanes of a k cover the 64-row line)
  constexpr bool XROW = !PRE && !H::GATHER;
  constexpr int XVE = 16 / (int)sizeof(T), XCH = H::K0P / XVE, NXE = (R / 4) * XCH,
                ITX = XROW ? (NXE + NTH - 1) / NTH : 1;
  u32x4 xv[ITX][4];
  if constexpr (XROW) {
    const T* xin = reinterpret_cast<const T*>(hb.xin);
#pragma unroll
    for (int i = 0; i < ITX; ++i) {
      const int e = tid + i * NTH, r = (e % (R / 4)) * 4, k = (e / (R / 4)) * XVE;
#pragma unroll
      for (int q = 0; q < 4; ++q)  // branch-free: clamped row / chunk, rows past the batch zeroed at use
        xv[i][q] = *reinterpret_cast<const u32x4*>(xin + (size_t)min(r0 + r + q, B - 1) * H::K0P + min(k, H::K0P - XVE));
    }
  }
  stamp(9);  // every staging load issued
  if constexpr (S::WLDS) {
    st_w2.store(reinterpret_cast<T*>(smem + S::OFF_W2), tid);
    if constexpr (STW_T) {
      st_w2t.store(reinterpret_cast<T*>(smem + S::OFF_W2T), tid);
      st_w3t.store(reinterpret_cast<T*>(smem + S::OFF_W3T), tid);
    }
    st_w3.store(reinterpret_cast<T*>(smem + S::OFF_W3), tid);
  }
#pragma unroll
  for (int i = 0; i < ITB; ++i) {
    bool live;
    (void)bias_src(tid + i * NTH, live);
    if (tid + i * NTH < NBIAS) sB1[tid + i * NTH] = live ? bias_v[i] : 0.f;
  }
  stamp(10);  // weights + biases stored (their loads have arrived)
  // look-ahead indices: issued after every load the staging barrier waits for (in-order vmcnt)
  if constexpr (LOOK) {
    if (look) {
      const int nidx = br.step_ptr[2], step = step_early;
#pragma unroll
      for (int j = 0; j < GIT2; ++j) {
        const int e = tid + j * NTH, r = e / 49;
        const int g = (step + 1) * br.batch_stride + r0 + r;
        gidx[j] = (e < GCH && r0 + r < br.batch_stride && g < nidx) ? br.idx_epoch[g] : -1;
      }
    }
  }
  if constexpr (H::GATHER && !PRE) __syncthreads();

  // ---------------------------------------------------------------- stage the input tile
  // (PRE: layer 1 already ran in l1_split_kernel, which also wrote xT; X itself is not needed)
  if constexpr (PRE) {
  } else if constexpr (H::GATHER && sizeof(T) == 2) {
    // bf16: one work item = one 8-pixel chunk of 4 consecutive rows: four 8-byte image loads (all items' loads
    // issued before any conversion), four 16-byte LDS stores and eight 4-row-wide xT stores.  (16-pixel items left
    // 6 of the 16 waves with the whole gather -- 392 items -- and the rest waiting at the staging barrier.)
    static_assert(H::K0 % 8 == 0 && H::K0P % 8 == 0 && R % 4 == 0, "gather chunking");
    constexpr int GC = H::K0P / 8, NGI = (R / 4) * GC, ITG = (NGI + NTH - 1) / NTH;
    T* xT = reinterpret_cast<T*>(hb.xT);
    u32x2 px[ITG][4];
#pragma unroll
    for (int i = 0; i < ITG; ++i) {
      const int e = min(tid + i * NTH, NGI - 1), r = (e % (R / 4)) * 4, c = e / (R / 4);
#pragma unroll
      for (int q = 0; q < 4; ++q) {  // branch-free: padding chunks / rows past the batch read row 0, zeroed at use
        // (look-ahead: the tile's own rows of xnext, contiguous; else the dataset rows by sample index)
        const uint8_t* src = look ? br.xnext + (size_t)(r0 + r + q) * 784 : br.images + (size_t)max(sIdx[r + q], 0) * 784;
        px[i][q] = *reinterpret_cast<const u32x2*>(src + min(c, H::K0 / 8 - 1) * 8);
      }
    }
    // pinned order: pixel loads, then the W1 prefetch, then the conversion (which then waits for the
    // pixels only -- the scheduler otherwise hoisted the prefetch above them and sank the pixel loads into
    // the conversion, one wait per row)
    __builtin_amdgcn_sched_barrier(0);
    prefetch_b1();
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int i = 0; i < ITG; ++i) {
      // threads past the last item convert the (clamped) last item again and skip the stores: no branch
      // around the loads' consumers
      const int eu = tid + i * NTH, e = min(eu, NGI - 1), r = (e % (R / 4)) * 4, c = e / (R / 4);
      const bool item = eu < NGI;
      u32x4 pk[4];  // row q's 8 pixels as 8 bf16
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const bool live = (look ? r0 + r + q < B : sIdx[r + q] >= 0) && c < H::K0 / 8;
        const uint32_t lm = live ? 0xFFFFFFFFu : 0u;  // the row's pixels or zeros, applied to packed pairs
        typedef __attribute__((ext_vector_type(2))) float f32x2;
        uint32_t d[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {  // pixel pairs: one v_cvt_pk_bf16_f32 each, computed unconditionally
          const uint32_t wv = px[i][q][k >> 1];
          const float a = mnist_norm((wv >> (16 * (k & 1))) & 255u), b = mnist_norm((wv >> (16 * (k & 1) + 8)) & 255u);
          d[k] = __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2{a, b}), bf16x2)) & lm;
        }
        pk[q] = u32x4{d[0], d[1], d[2], d[3]};
        if (item) *reinterpret_cast<u32x4*>(sX + (r + q) * S::PX + c * 8) = pk[q];
      }
      if (TRAIN && item && !ABLATED(hb.ablate, 1)) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {  // pixel j of the 4 rows: halfword j of each row, one v_perm_b32 per pair
          const int wd = j >> 1;
          const uint32_t lo = pack_half16(pk[0][wd], pk[1][wd], j & 1);
          const uint32_t hi = pack_half16(pk[2][wd], pk[3][wd], j & 1);
          *reinterpret_cast<u32x2*>(xT + (size_t)(c * 8 + j) * ldB + r0 + r) = u32x2{lo, hi};
        }
      }
    }
    stamp(11);  // gathered tile converted and stored to LDS, xT stores issued
  } else if constexpr (H::GATHER) {
    // fp32: one work item = one 8-pixel chunk of 4 consecutive rows (as bf16): four 8-byte image loads (all items'
    // loads issued before any conversion), 16-byte LDS stores, and 4-row-wide xT stores (one per pixel)
    static_assert(H::K0 % 8 == 0 && H::K0P % 8 == 0 && R % 4 == 0, "gather chunking");
    constexpr int GC = H::K0P / 8, NGI = (R / 4) * GC, ITG = (NGI + NTH - 1) / NTH;
    T* xT = reinterpret_cast<T*>(hb.xT);
    u32x2 px[ITG][4];
#pragma unroll
    for (int i = 0; i < ITG; ++i) {
      const int e = min(tid + i * NTH, NGI - 1), r = (e % (R / 4)) * 4, c = e / (R / 4);
#pragma unroll
      for (int q = 0; q < 4; ++q) {  // branch-free: padding chunks / rows past the batch read row 0, zeroed at use
        // (look-ahead: the tile's own rows of xnext, contiguous; else the dataset rows by sample index)
        const uint8_t* src = look ? br.xnext + (size_t)(r0 + r + q) * 784 : br.images + (size_t)max(sIdx[r + q], 0) * 784;
        px[i][q] = *reinterpret_cast<const u32x2*>(src + min(c, H::K0 / 8 - 1) * 8);
      }
    }
    // pinned order: pixel loads, then the W1 prefetch, then the conversion (which then waits for the
    // pixels only -- the scheduler otherwise hoisted the prefetch above them and sank the pixel loads into
    // the conversion, one wait per row)
    __builtin_amdgcn_sched_barrier(0);
    prefetch_b1();
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int i = 0; i < ITG; ++i) {
      // threads past the last item convert the (clamped) last item again and skip the stores: no branch
      // around the loads' consumers
      const int eu = tid + i * NTH, e = min(eu, NGI - 1), r = (e % (R / 4)) * 4, c = e / (R / 4);
      const bool item = eu < NGI;
      {
#pragma unroll
        for (int j0 = 0; j0 < 8; j0 += 4) {  // fp32: 4 pixels at a time (one 16-byte LDS store per row)
          float v[4][4];
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const bool live = (look ? r0 + r + q < B : sIdx[r + q] >= 0) && c < H::K0 / 8;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              const float nv = mnist_norm((px[i][q][(j0 + j) >> 2] >> (8 * ((j0 + j) & 3))) & 255u);
              v[q][j] = live ? nv : 0.f;
            }
            if (item) *reinterpret_cast<f32x4*>(sX + (r + q) * S::PX + c * 8 + j0) = f32x4{v[q][0], v[q][1], v[q][2], v[q][3]};
          }
          if (TRAIN && item) {
#pragma unroll
            for (int j = 0; j < 4; ++j)
              store_col4<T>(xT + (size_t)(c * 8 + j0 + j) * ldB + r0 + r, v[0][j], v[1][j], v[2][j], v[3][j]);
          }
        }
      }
    }
    stamp(11);  // gathered tile converted and stored to LDS, xT stores issued
  } else {
    T* xT = reinterpret_cast<T*>(hb.xT);
    // element j of a 16-byte chunk, as raw bits (register extracts: a pointer-punned read of the chunk
    // array put it on the scratch stack)
    auto word = [](const u32x4& v, int w) { return v[w]; };
#pragma unroll
    for (int i = 0; i < ITX; ++i) {
      const int e = tid + i * NTH, r = (e % (R / 4)) * 4, k = (e / (R / 4)) * XVE;
      if (e < NXE) {
        u32x4 rv[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          rv[q] = r0 + r + q < B ? xv[i][q] : u32x4{0u, 0u, 0u, 0u};
          *reinterpret_cast<u32x4*>(sX + (r + q) * S::PX + k) = rv[q];
        }
        if constexpr (TRAIN) {
#pragma unroll
          for (int j = 0; j < XVE; ++j) {
            T* dst = xT + (size_t)(k + j) * ldB + r0 + r;
            if constexpr (sizeof(T) == 2) {
              const int w = j >> 1;
              const uint32_t lo = pack_half16(word(rv[0], w), word(rv[1], w), j & 1);
              const uint32_t hi = pack_half16(word(rv[2], w), word(rv[3], w), j & 1);
              *reinterpret_cast<u32x2*>(dst) = u32x2{lo, hi};
            } else {
              *reinterpret_cast<u32x4*>(dst) = u32x4{word(rv[0], j), word(rv[1], j), word(rv[2], j), word(rv[3], j)};
            }
          }
        }
      }
    }
    stamp(11);  // input tile stored to LDS, xT stores issued
  }
  __syncthreads();
  stamp(1);
  // labels: fetched by the LAST threads of the block (idle in L1 when NWV > NT1), used after 3 barriers
  const int gstep = EARLY_STEP ? gstep_early : br.step_ptr[1];  // dropout stream (see batch_idx)
  if (!look) {
    const int t = tid - (NTH - R);
    if (t >= 0) {
      const int id = H::GATHER ? sIdx[t] : ((r0 + t < B) ? batch_idx()[r0 + t] : -1);
      sLab[t] = id >= 0 ? (int)br.labels[id] : 0;
    }
  }
  // look-ahead: the next step's pixels / labels (indices were loaded during the staging)
  uint4 gv[GIT2];
  int glab[GIT2];
  if constexpr (LOOK) {
    if (look) {
#pragma unroll
      for (int j = 0; j < GIT2; ++j) {
        const int e = tid + j * NTH, c = e % 49;
        gv[j] = gidx[j] >= 0 ? *reinterpret_cast<const uint4*>(br.images + (size_t)gidx[j] * 784 + c * 16)
                             : make_uint4(0, 0, 0, 0);
        glab[j] = (gidx[j] >= 0 && c == 0) ? (int)br.labels[gidx[j]] : 0;
      }
    }
  }

  const float keep_scale = H::DROPOUT ? 1.0f / (1.0f - hb.drop_p) : 1.0f;
  const uint32_t drop_thr = H::DROPOUT ? (uint32_t)(hb.drop_p * 4294967295.0f) : 0u;

  if constexpr (WX) {  // weight images for after layer 1 (issued after the label loads: in-order vmcnt)
    st_w2.load(pack + H::F2, tid);
    if constexpr (STW_T) {
      st_w2t.load(pack + H::F2T, tid);
      st_w3t.load(pack + H::F3T, tid);
    }
    st_w3.load(pack + H::F3, tid);
  }
  // ---------------------------------------------------------------- L1: H1 = relu(X W1^T + b1)
  if constexpr (PRE) {
    // sum the L1_KSPLIT partial products in a fixed order, then the same bias/ReLU/dropout epilogue
    T* h1T = reinterpret_cast<T*>(hb.h1T);
#pragma unroll
    for (int j = 0; j < PE; ++j) {
      const int e = tid + j * NTH;
      if (e >= H::N1P * R) break;
      const int n = e / R, r = e % R, rg = r0 + r;
      float z = 0.f;
#pragma unroll
      for (int q = 0; q < L1_KSPLIT; ++q) z += zpre[j][q];
      float x = fmaxf(z + sB1[n], 0.f);
      if constexpr (H::DROPOUT && TRAIN) {
        const uint32_t h = hash4(hb.seed, (uint32_t)gstep, (uint32_t)rg, (uint32_t)n);
        x = (h >= drop_thr) ? x * keep_scale : 0.f;
      }
      if (n >= H::N1 || rg >= B) x = 0.f;
      sH1[r * S::P1 + n] = to_t<T>(x);
      if constexpr (TRAIN) h1T[(size_t)n * ldB + rg] = to_t<T>(x);
    }
  } else {
    T* h1T = reinterpret_cast<T*>(hb.h1T);
    const T* ap = sX + row * S::PX + grp * KV;
    constexpr int NJ1 = KS1 ? 1 : (NT1 + NWV - 1) / NWV;
#pragma unroll
    for (int j = 0; j < NJ1; ++j) {
      const int nt = KS1 ? l1_nt : w + j * NWV;
      const bool live = KS1 ? l1_live : nt < NT1;
      if (!KS1 && !live) break;
      f32x4 acc[MT];
#pragma unroll
      for (int m = 0; m < MT; ++m) acc[m] = zero4();
      if (live) {
        const T* bp = pack + H::FM1 + (nt * KCH1 * 64 + lane) * KV;  // fragment-major W1 (models.h)
#pragma unroll
        for (int kk = 0; kk < KH1; ++kk) {
          const int kc = l1_k0 + kk;
          if (kc >= l1_k1) break;  // wave-uniform (second half of an odd chunk count)
          const Frag b = (PF1 && j == 0) ? b1pre[PF1 ? kk : 0] : M::load(bp + kc * 64 * KV);
#pragma unroll
          for (int m = 0; m < MT; ++m) head_mma<T, HSP>(acc[m], M::load(ap + m * 16 * S::PX + kc * KC), b);
        }
      }
      if constexpr (KS1) {
        // second-half waves hand their partial sums to the first-half wave of the same n-tile through the
        // X region (every wave has finished reading X at the first barrier; every wave passes both)
        f32x4* red = reinterpret_cast<f32x4*>(smem + S::OFF_X);
        __syncthreads();
        if (live && l1_half == 1) {
#pragma unroll
          for (int m = 0; m < MT; ++m) red[(nt * MT + m) * 64 + lane] = acc[m];
        }
        __syncthreads();
        if (!live || l1_half == 1) continue;
#pragma unroll
        for (int m = 0; m < MT; ++m) acc[m] += red[(nt * MT + m) * 64 + lane];
      }
      const int n = nt * 16 + row;
      const float bias = sB1[n];
#pragma unroll
      for (int m = 0; m < MT; ++m) {
        float v[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int r = m * 16 + grp * 4 + i, rg = r0 + r;
          float x = fmaxf(acc[m][i] + bias, 0.f);
          if constexpr (H::DROPOUT && TRAIN) {
            const uint32_t h = hash4(hb.seed, (uint32_t)gstep, (uint32_t)rg, (uint32_t)n);
            x = (h >= drop_thr) ? x * keep_scale : 0.f;
          }
          if (n >= H::N1 || rg >= B) x = 0.f;
          sH1[r * S::P1 + n] = to_t<T>(x);
          v[i] = to_f(to_t<T>(x));
        }
        if constexpr (TRAIN)
          store_col4<T>(h1T + (size_t)n * ldB + r0 + m * 16 + grp * 4, v[0], v[1], v[2], v[3]);
      }
    }
  }
  __syncthreads();
  if constexpr (WX) {  // the X tile is dead: the weight images land in its place (loads issued before L1)
    T* wb = reinterpret_cast<T*>(smem + WOFF + S::OFF_W2);
    st_w2.store(wb, tid);
    if constexpr (STW_T) {
      st_w2t.store(reinterpret_cast<T*>(smem + WOFF + S::OFF_W2T), tid);
      st_w3t.store(reinterpret_cast<T*>(smem + WOFF + S::OFF_W3T), tid);
    }
    st_w3.store(reinterpret_cast<T*>(smem + WOFF + S::OFF_W3), tid);
    __syncthreads();
  }
  stamp(2);
  // ---------------------------------------------------------------- L2: H2 = relu(H1 W2^T + b2)
  {
    constexpr int NT = H::N2P / 16, KCH = H::N1P / KC;
    T* h2T = reinterpret_cast<T*>(hb.h2T);
    for (int nt = w; nt < NT; nt += NWV) {
      f32x4 acc[MT];
#pragma unroll
      for (int m = 0; m < MT; ++m) acc[m] = zero4();
      const T* bp = bW2 + (nt * 16 + row) * LW2 + grp * KV;
      const T* ap = sH1 + row * S::P1 + grp * KV;
#pragma unroll
      for (int kc = 0; kc < KCH; ++kc) {
        const Frag b = M::load(bp + kc * KC);
#pragma unroll
        for (int m = 0; m < MT; ++m) head_mma<T, HSP>(acc[m], M::load(ap + m * 16 * S::P1 + kc * KC), b);
      }
      const int n = nt * 16 + row;
      const float bias = sB2[n];
#pragma unroll
      for (int m = 0; m < MT; ++m) {
        float v[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int r = m * 16 + grp * 4 + i, rg = r0 + r;
          float x = fmaxf(acc[m][i] + bias, 0.f);
          if (n >= H::N2 || rg >= B) x = 0.f;
          sH2[r * S::P2 + n] = to_t<T>(x);
          v[i] = to_f(to_t<T>(x));
        }
        if constexpr (TRAIN)
          store_col4<T>(h2T + (size_t)n * ldB + r0 + m * 16 + grp * 4, v[0], v[1], v[2], v[3]);
      }
    }
  }
  __syncthreads();
  stamp(3);

  // ---------------------------------------------------------------- L3: logits = H2 W3^T (+ b3)
  {
    constexpr int KCH = H::N2P / KC;
    for (int m = w; m < MT; m += NWV) {
      f32x4 acc = zero4();
      const T* bp = bW3 + row * LW3 + grp * KV;
      const T* ap = sH2 + (m * 16 + row) * S::P2 + grp * KV;
      for (int kc = 0; kc < KCH; ++kc) head_mma<T, HSP>(acc, M::load(ap + kc * KC), M::load(bp + kc * KC));
      const int c = row;
      const float bias = sB3[c];
#pragma unroll
      for (int i = 0; i < 4; ++i) sLog[(m * 16 + grp * 4 + i) * 16 + c] = acc[i] + bias;
    }
  }
  __syncthreads();
  stamp(4);

  // ---- dX operands (W1^T, [K0 rows][N1P]): the first two n-tiles of this wave, fetched now so the
  //      L2/MALL latency hides behind softmax, dH2 and dH1.  (Their issue -- 128 wave-loads per CU --
  //      occupies the CU's memory pipeline for ~1.5 us wherever it is placed: issued at the start of layer 2
  //      the softmax phase drops 2.5 -> 1.0 us and layer 2 grows 1.0 -> 2.8 us.)
  constexpr int NTX = rup(H::K0, 16) / 16, KCHX = H::N1P / KC, PXT = KCHX <= 4 ? 2 : 1;  // <= 32 VGPRs
  Frag bx[H::DX && TRAIN ? PXT : 1][KCHX];
  auto prefetch_dx = [&] {
    if constexpr (H::DX && TRAIN) {
#pragma unroll
      for (int j = 0; j < PXT; ++j) {
        const int nt = w + j * NWV;
        if (nt < NTX) {
          const T* bp = pack + H::F1T + (nt * 16 + row) * H::N1P + grp * KV;
#pragma unroll
          for (int kc = 0; kc < KCHX; ++kc) bx[j][kc] = M::load(bp + kc * KC);
        }
      }
    }
  };

  prefetch_dx();
  stamp(12);  // dX operand loads issued

  // ---------------------------------------------------------------- softmax cross-entropy
  // Every thread takes one (row, class) pair: t -> r = t >> 4, c = t & 15, so a row is one 16-lane
  // group and its max / first argmax (ATen tie order) / exp-sum are xor-shuffle reductions.  dZ goes
  // to LDS here; its transposed copy for the wgrad GEMM is stored in the dH2 phase.
  {
    float loss = 0.f, corr = 0.f, cnt = 0.f;
    for (int t = tid; t < R * 16; t += NTH) {
      const int r = t >> 4, c = t & 15, rg = r0 + r;
      const bool valid = rg < B;
      const float z = c < H::NC ? sLog[r * 16 + c] : -INFINITY;
      // row reductions over the 16 lanes of the row with DPP (the ds_bpermute shuffles were the phase)
      const float mx = row16_max(z);
      const int am = row16_min(z == mx ? c : 16);
      const float e = c < H::NC ? __expf(z - mx) : 0.f;
      const float se = row16_sum(e);
      const int y = sLab[r];
      const float zy = sLog[r * 16 + y];
      if (c == 0 && valid) {
        loss += mx + __logf(se) - zy;
        corr += (am == y) ? 1.f : 0.f;
        cnt += 1.f;
      }
      if constexpr (TRAIN) {
        const float d = (valid && c < H::NC) ? e / se - (c == y ? 1.f : 0.f) : 0.f;
        sD[r * S::PD + c] = to_t<T>(d);
        sD[r * S::PD + 16 + c] = to_t<T>(0.f);  // K padding of the dH2 product (NCK = 32)
      }
    }
    stamp(13);  // softmax rows done (before the metric reductions)
    // only the class-0 lane of each 16-lane row accumulates (lanes 0, 16, 32, 48: c = lane & 15 in every
    // iteration), so the wave total is those four lanes -- bitwise what wave_sum gives (its row sums add
    // zeros), without its three dependent DPP chains
    static_assert(NTH % 16 == 0, "class index = lane & 15 in every softmax iteration");
    auto rows4 = [](float v) { return (lane_f(v, 0) + lane_f(v, 16)) + (lane_f(v, 32) + lane_f(v, 48)); };
    loss = rows4(loss);
    corr = rows4(corr);
    cnt = rows4(cnt);
    if (lane == 0) {
      sPart[w * 4 + 0] = loss;
      sPart[w * 4 + 1] = corr;
      sPart[w * 4 + 2] = cnt;
    }
  }
  // tile totals -> this workgroup's own row of hb.metrics ([grid][4], summed on the host when read):
  // a plain read-modify-write, no atomics.  (Three float atomics per workgroup on the same three words
  // were serialised at the memory side behind the kernel's last stores and held the kernel's end --
  // and the next kernel's start -- back by several us; a fixed row per workgroup is also deterministic.)
  auto flush_metrics = [&] {
    if (tid == 0) {
      float a = 0.f, b = 0.f, c = 0.f;
      for (int i = 0; i < NWV; ++i) {
        a += sPart[i * 4 + 0];
        b += sPart[i * 4 + 1];
        c += sPart[i * 4 + 2];
      }
      float* m = hb.metrics + (size_t)blockIdx.x * 4;
      const f32x4 old = *reinterpret_cast<const f32x4*>(m);
      *reinterpret_cast<f32x4*>(m) = f32x4{old[0] + a, old[1] + b, old[2] + c, 0.f};
    }
  };
  stamp(14);  // metric partials stored (before the barrier)
  // per-wave arrival at the softmax barrier (profiling stamps, own row range, one slot per wave)
  if (hb.stamps && lane == 0 && w < 16 && blockIdx.x < 512)
    hb.stamps[(STAMP_HEAD_ARRIVE + blockIdx.x) * 16 + w] = wall_clock64();
  __syncthreads();
  stamp(5);
  if constexpr (!TRAIN) {
    flush_metrics();
    return;
  }

  // ---------------------------------------------------------------- dH2 = (dZ W3) * [H2 > 0]
  {
    // (FT: B[k = c][n] = W3[c][n] read k-strided from the W3 image; the zero dZ columns c >= 16
    //  contribute nothing, so only the 16 staged rows are read)
    constexpr bool TW3 = S::FT && WIN;
    constexpr int NT = H::N2P / 16, KCH = (TW3 ? H::NCP : H::NCK) / KC;
    T* dy2T = reinterpret_cast<T*>(hb.dy2T);
    for (int nt = w; nt < NT; nt += NWV) {
      f32x4 acc[MT];
#pragma unroll
      for (int m = 0; m < MT; ++m) acc[m] = zero4();
      const T* bp = TW3 ? bW3 + grp * KV * LW3 + nt * 16 + row : bW3T + (nt * 16 + row) * LW3T + grp * KV;
      const T* ap = sD + row * S::PD + grp * KV;
#pragma unroll
      for (int kc = 0; kc < KCH; ++kc) {
        const Frag b = TW3 ? load_kstrided<T>(bp + kc * KC * LW3, LW3) : M::load(bp + kc * KC);
#pragma unroll
        for (int m = 0; m < MT; ++m) head_mma<T, HSP>(acc[m], M::load(ap + m * 16 * S::PD + kc * KC), b);
      }
      const int n = nt * 16 + row;
#pragma unroll
      for (int m = 0; m < MT; ++m) {
        float v[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int r = m * 16 + grp * 4 + i;
          T* h = &sH2[r * S::P2 + n];
          const float x = to_f(*h) > 0.f ? acc[m][i] : 0.f;
          *h = to_t<T>(x);  // in place: H2 becomes dH2
          v[i] = to_f(to_t<T>(x));
        }
        store_col4<T>(dy2T + (size_t)n * ldB + r0 + m * 16 + grp * 4, v[0], v[1], v[2], v[3]);
      }
    }
    // dZ^T for the wgrad GEMM (coalesced along the batch; waves without a dH2 tile go first)
    T* dy3T = reinterpret_cast<T*>(hb.dy3T);
    for (int e = tid; e < H::NCP * R; e += NTH) {
      const int c = e / R, r = e % R;
      dy3T[(size_t)c * ldB + r0 + r] = sD[r * S::PD + c];
    }
  }
  __syncthreads();
  stamp(6);

  // ---------------------------------------------------------------- dH1 = (dH2 W2) * [H1 > 0] / keep
  {
    constexpr bool TW2 = S::FT && WIN;  // B[k = n2][n = n1] = W2[n2][n1], k-strided from the W2 image
    constexpr int NT = H::N1P / 16, KCH = H::N2P / KC;
    T* dy1T = reinterpret_cast<T*>(hb.dy1T);
    for (int nt = w; nt < NT; nt += NWV) {
      f32x4 acc[MT];
#pragma unroll
      for (int m = 0; m < MT; ++m) acc[m] = zero4();
      const T* bp = TW2 ? bW2 + grp * KV * LW2 + nt * 16 + row : bW2T + (nt * 16 + row) * LW2T + grp * KV;
      const T* ap = sH2 + row * S::P2 + grp * KV;
#pragma unroll
      for (int kc = 0; kc < KCH; ++kc) {
        const Frag b = TW2 ? load_kstrided<T>(bp + kc * KC * LW2, LW2) : M::load(bp + kc * KC);
#pragma unroll
        for (int m = 0; m < MT; ++m) head_mma<T, HSP>(acc[m], M::load(ap + m * 16 * S::P2 + kc * KC), b);
      }
      const int n = nt * 16 + row;
#pragma unroll
      for (int m = 0; m < MT; ++m) {
        float v[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int r = m * 16 + grp * 4 + i;
          T* h = &sH1[r * S::P1 + n];
          const float x = to_f(*h) > 0.f ? acc[m][i] * keep_scale : 0.f;
          *h = to_t<T>(x);  // in place: H1 becomes dH1
          v[i] = to_f(to_t<T>(x));
        }
        store_col4<T>(dy1T + (size_t)n * ldB + r0 + m * 16 + grp * 4, v[0], v[1], v[2], v[3]);
      }
    }
  }

  // ---------------------------------------------------------------- dX = dH1 W1 (LeNet: into pool2 grads)
  if constexpr (H::DX) {
    __syncthreads();
    stamp(7);
    T* dx = reinterpret_cast<T*>(hb.dx);
    const T* ap = sH1 + row * S::P1 + grp * KV;
#pragma unroll
    for (int j = 0; j < (NTX + NWV - 1) / NWV; ++j) {
      const int nt = w + j * NWV;
      if (nt >= NTX) break;
      f32x4 acc[MT];
#pragma unroll
      for (int m = 0; m < MT; ++m) acc[m] = zero4();
      const T* bp = pack + H::F1T + (nt * 16 + row) * H::N1P + grp * KV;
#pragma unroll
      for (int kc = 0; kc < KCHX; ++kc) {
        const Frag b = j < PXT ? bx[j < PXT ? j : 0][kc] : M::load(bp + kc * KC);
#pragma unroll
        for (int m = 0; m < MT; ++m) head_mma<T, HSP>(acc[m], M::load(ap + m * 16 * S::P1 + kc * KC), b);
      }
      const int k = nt * 16 + row;
#pragma unroll
      for (int m = 0; m < MT; ++m) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int rg = r0 + m * 16 + grp * 4 + i;
          if (rg < B) dx[(size_t)rg * H::K0P + k] = to_t<T>(acc[m][i]);
        }
      }
    }
  }
  if constexpr (LOOK) {
    if (look) {  // ordered after every read of this step's ynext by the softmax barrier
#pragma unroll
      for (int j = 0; j < GIT2; ++j) {
        const int e = tid + j * NTH, r = e / 49, c = e % 49;
        if (gidx[j] >= 0) {
          *reinterpret_cast<uint4*>(br.xnext + (size_t)(r0 + r) * 784 + c * 16) = gv[j];
          if (c == 0) br.ynext[r0 + r] = (uint8_t)glab[j];
        }
      }
    }
  }
  stamp(8);
  if (hb.stamps && tid == 0 && blockIdx.x < 1024) hb.stamps[blockIdx.x * 16 + 15] = hw_location();
  flush_metrics();
}

// ====================================================================================
// Small-batch layer 1: Z1 partial[q] = X[:, Kq] W1[:, Kq]^T over a (16-row tile, 64-column group,
// K quarter) grid, so a B=128 step spreads the 784-deep GEMM over 64 workgroups instead of 8.
// The X tile (gathered + normalised for the MLP, pool2 rows for LeNet) is staged once in LDS and
// shared by the 4 waves (one 16-column tile each); the n-group-0 blocks also write X^T for the
// wgrad GEMM.  Partials are stored transposed, [q][n][ldB], one 16-byte store per lane.
// ====================================================================================
template <typename T, class H, bool TRAIN>
__global__ __launch_bounds__(256) void l1_split_kernel(BatchRef br, HeadBuffers hb) {
  using M = Mma<T>;
  constexpr int KV = M::KV, KC = M::KC;
  constexpr int KCH = H::K0P / KC, QCH = (KCH + L1_KSPLIT - 1) / L1_KSPLIT;
  constexpr int XP = QCH * KC + 8;
  __shared__ __attribute__((aligned(16))) T sX[16 * XP];
  const int tid = threadIdx.x, lane = tid & 63, w = wave_id(), row = lane & 15, grp = lane >> 4;
  const int r0 = blockIdx.x * 16, ng = blockIdx.y, q = blockIdx.z;
  const int lin = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);
  auto stamp = [&](int k) {
    if (hb.stamps && tid == 0 && lin < 512) hb.stamps[(STAMP_L1 + lin) * 16 + k] = wall_clock64();
  };
  stamp(0);
  const int c0 = q * QCH, c1 = min(KCH, c0 + QCH);
  if (c0 >= c1) return;  // uniform per block
  const int k0 = c0 * KC, klen = (c1 - c0) * KC;
  const int B = br.B, ldB = hb.ldB;
  T* xT = reinterpret_cast<T*>(hb.xT);
  const bool write_xT = TRAIN && ng == 0;
  // this wave's W1 fragments of the K range, issued first: their latency hides behind the X gather
  using Frag = typename M::Frag;
  const int nt = ng * 4 + w;
  const bool has_nt = nt * 16 < H::N1P;  // wave-uniform
  const T* pack = reinterpret_cast<const T*>(hb.pack);
  const T* bp = pack + H::FM1 + ((size_t)min(nt, H::N1P / 16 - 1) * KCH * 64 + lane) * KV;  // fragment-major W1
  Frag bpre[QCH];
#pragma unroll
  for (int i = 0; i < QCH; ++i) bpre[i] = M::load(bp + (size_t)min(c0 + i, KCH - 1) * 64 * KV);  // clamped: unused past c1

  // MLP gather: a thread's row is tid & 15 in every iteration, so its sample index is loaded ONCE and
  // every pixel load of the thread is issued before the first conversion (one idx -> pixels latency
  // chain instead of one per iteration); addresses are clamped, invalid values masked at use
  constexpr int GIT = (16 * (QCH * KC / 8) + 255) / 256;
  uint2 gu[H::GATHER ? GIT : 1];
  if constexpr (H::GATHER) {
    // training with the look-ahead: the rows were gathered into xnext by the previous step's head
    const uint8_t* src;
    if (TRAIN && br.xnext) {
      src = br.xnext + (size_t)(r0 + (tid & 15)) * 784;
    } else {
      const int32_t* idx = br.idx_epoch + (size_t)br.step_ptr[0] * br.batch_stride;
      src = br.images + (size_t)idx[min(r0 + (tid & 15), B - 1)] * 784;
    }
#pragma unroll
    for (int it = 0; it < GIT; ++it) {
      const int k = k0 + ((tid + it * 256) >> 4) * 8;
      gu[it] = *reinterpret_cast<const uint2*>(src + min(k, H::K0 - 8));
    }
  }
#pragma unroll
  for (int it = 0; it < (H::GATHER ? GIT : (16 * (QCH * KC / 8) + 255) / 256); ++it) {
    const int e = tid + it * 256;
    if (e >= 16 * (klen / 8)) break;
    const int r = e & 15, kk = (e >> 4) * 8, k = k0 + kk, rg = r0 + r;
    float v[8];
    if constexpr (H::GATHER) {
      const uint2 u = gu[H::GATHER ? it : 0];
      const bool in = rg < B && k < H::K0;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        v[j] = in ? mnist_norm((u.x >> (8 * j)) & 255u) : 0.f;
        v[j + 4] = in ? mnist_norm((u.y >> (8 * j)) & 255u) : 0.f;
      }
    } else {
      const T* xin = reinterpret_cast<const T*>(hb.xin);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = rg < B ? to_f(xin[(size_t)rg * H::K0P + k + j]) : 0.f;
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) sX[r * XP + kk + j] = to_t<T>(v[j]);
    if (write_xT) {
#pragma unroll
      for (int j = 0; j < 8; ++j) xT[(size_t)(k + j) * ldB + rg] = to_t<T>(v[j]);
    }
  }
  __syncthreads();
  stamp(1);

  if (!has_nt) return;
  const T* ap = sX + row * XP + grp * KV;
  // two accumulators (even / odd chunks): half the dependent-MFMA chain
  f32x4 acc0 = zero4(), acc1 = zero4();
#pragma unroll
  for (int i = 0; i < QCH; ++i) {
    if (c0 + i < c1) {  // uniform: only the last K range is shorter
      if (i & 1) head_mma<T, false>(acc1, M::load(ap + i * KC), bpre[i]);
      else head_mma<T, false>(acc0, M::load(ap + i * KC), bpre[i]);
    }
  }
  f32x4 acc;
#pragma unroll
  for (int j = 0; j < 4; ++j) acc[j] = acc0[j] + acc1[j];
  float* out = hb.z1p + ((size_t)q * H::N1P + nt * 16 + row) * ldB + r0 + grp * 4;
  *reinterpret_cast<f32x4*>(out) = acc;
  stamp(2);
}

// ====================================================================================
// Grouped weight-gradient GEMM:  dW[n][k] = sum_r dY^T[n][r] * X^T[k][r]  (+ bias column k == K)
// Both operands are stored row = feature, contiguous batch, so each lane's K-chunk fragment is
// one 16-byte load.  A 64x64 output block per workgroup (each wave 32x32 = 2x2 MFMA tiles);
// the batch is split over gridDim.y, each split writes its own fp32 slab row (deterministic).
// ====================================================================================
template <typename T, int WD>
__global__ __launch_bounds__(256) void wgrad_kernel(WgArgs<T> a) {
  using M = Mma<T>;
  using Frag = typename M::Frag;
  constexpr int KV = M::KV, KC = M::KC;
  const int lane = threadIdx.x & 63, w = wave_id(), row = lane & 15, grp = lane >> 4;
  const int lin = blockIdx.y * gridDim.x + blockIdx.x;  // profiling stamps: [0] start, [1] end
  if (a.stamps && threadIdx.x == 0 && lin < 512) a.stamps[(STAMP_WGRAD + lin) * 16] = wall_clock64();
  int tile, split, nsteps, x = 0, m0 = 0, spc = 1, sh = 0, rs = 0;
  if (a.xcd_ch == 0) {
    tile = blockIdx.x;
    split = blockIdx.y;
    rs = split * a.rlen;
    nsteps = (min(rs + a.rlen, a.Bp) - rs + KC - 1) / KC;
  } else {
    const int L = blockIdx.x, q = L >> 3;
    x = L & 7;
    tile = q / a.sx;
    const int sub = q % a.sx;
    split = x * a.sx + sub;
    const int mx = a.contig ? a.nch / 8 : (x < a.nch ? (a.nch - x + 7) / 8 : 0);  // chunks owned by XCD x
    m0 = sub * mx / a.sx;
    const int m1 = (sub + 1) * mx / a.sx;
    spc = a.xcd_ch / KC;  // a power of two (wgrad_launch): steps -> chunks by shift and mask, no division
    sh = __builtin_ctz(spc);
    nsteps = (m1 - m0) * spc;
  }
  auto step_row = [&](int st) -> int {  // first batch row of step st (may be >= Bp: skipped)
    if (a.xcd_ch == 0) return rs + st * KC;
    const int m = m0 + (st >> sh);
    return (a.contig ? x * (a.nch / 8) + m : x + 8 * m) * a.xcd_ch + (st & (spc - 1)) * KC;
  };
  int j = 0;
  while (j + 1 < a.njobs && tile >= a.job[j + 1].blk_begin) ++j;
  const WgJob<T>& J = a.job[j];
  const int lb = tile - J.blk_begin;
  const int bn = lb / J.nblk_k, bk = lb % J.nblk_k;
  const int n0 = bn * 64 + (w >> 1) * 32, k0 = bk * 64 + (w & 1) * 32;
  const int Kb = J.K + (J.bias ? 1 : 0);
  if (n0 >= J.N || k0 >= Kb) return;
  const bool nv1 = n0 + 16 < J.NP;

  f32x4 acc[2][2];
#pragma unroll
  for (int mi = 0; mi < 2; ++mi)
#pragma unroll
    for (int ni = 0; ni < 2; ++ni) acc[mi][ni] = zero4();

  Frag ones;
#pragma unroll
  for (int q = 0; q < KV; ++q) M::set(ones, q, 1.f);
  const Frag zf = M::zero();

  const T* ap0 = J.dyT + (size_t)(n0 + row) * a.ldB + grp * KV;
  const T* ap1 = J.dyT + (size_t)(n0 + 16 + row) * a.ldB + grp * KV;
  const int kk0 = k0 + row, kk1 = k0 + 16 + row;
  const T* bp0 = J.xT + (size_t)min(kk0, J.K > 0 ? J.K - 1 : 0) * a.ldB + grp * KV;
  const T* bp1 = J.xT + (size_t)min(kk1, J.K > 0 ? J.K - 1 : 0) * a.ldB + grp * KV;
  const int sel0 = kk0 < J.K ? 0 : (kk0 == J.K && J.bias ? 1 : 2);
  const int sel1 = kk1 < J.K ? 0 : (kk1 == J.K && J.bias ? 1 : 2);

  // software pipeline: a ring of WD K-steps' fragments (four per step) is in flight while the oldest one
  // computes (one step of look-ahead left every wave waiting a full L2 round trip per 32-row step)
  Frag ra0[WD], ra1[WD], rb0[WD], rb1[WD];
  auto fetch = [&](int d, int rc) {
    ra0[d] = M::load(ap0 + rc);
    ra1[d] = nv1 ? M::load(ap1 + rc) : zf;
    rb0[d] = M::load(bp0 + rc);
    rb1[d] = M::load(bp1 + rc);
  };
#pragma unroll
  for (int d = 0; d < WD; ++d) {
    const int rc = d < nsteps ? step_row(d) : a.Bp;
    if (rc < a.Bp) fetch(d, rc);
  }
  for (int st0 = 0; st0 < nsteps; st0 += WD) {
#pragma unroll
    for (int d = 0; d < WD; ++d) {
      const int st = st0 + d;
      if (st >= nsteps || step_row(st) >= a.Bp) break;  // rows past the (padded) batch: nothing left
      const Frag a0 = ra0[d], a1 = ra1[d];
      const Frag b0 = sel0 == 0 ? rb0[d] : (sel0 == 1 ? ones : zf);
      const Frag b1 = sel1 == 0 ? rb1[d] : (sel1 == 1 ? ones : zf);
      const int rn = st + WD < nsteps ? step_row(st + WD) : a.Bp;
      if (rn < a.Bp) fetch(d, rn);
      wg_mma<T>(acc[0][0], a0, b0);
      wg_mma<T>(acc[0][1], a0, b1);
      wg_mma<T>(acc[1][0], a1, b0);
      wg_mma<T>(acc[1][1], a1, b1);
    }
  }

  float* out = a.slab + (size_t)split * a.slab_ld + J.out_off;
  // output element (mi, ni, i) -> parameter index within the job (slab rows are laid out by parameter
  // index), -1 for padding
  int qi[2][2][4];
#pragma unroll
  for (int mi = 0; mi < 2; ++mi)
#pragma unroll
    for (int ni = 0; ni < 2; ++ni) {
      const int k = k0 + ni * 16 + row;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int n = n0 + mi * 16 + grp * 4 + i;
        qi[mi][ni][i] = n >= J.N ? -1 : (k < J.K ? n * J.K + k : (k == J.K && J.bias ? J.N * J.K + n : -1));
      }
    }
#pragma unroll
  for (int mi = 0; mi < 2; ++mi)
#pragma unroll
    for (int ni = 0; ni < 2; ++ni)
#pragma unroll
      for (int i = 0; i < 4; ++i)
        if (qi[mi][ni][i] >= 0) out[qi[mi][ni][i]] = acc[mi][ni][i];
  if (a.stamps && threadIdx.x == 0 && lin < 512) a.stamps[(STAMP_WGRAD + lin) * 16 + 1] = wall_clock64();
}

// Batch rows of a wgrad workgroup's K-steps (wgrad_kernel's split / XCD-aware mapping, see WgArgs).
struct WgRows {
  int xcd_ch, rs, m0, spc, x, contig, nch, sh;  // spc = 1 << sh steps per chunk (a power of two: wgrad_launch)
  DEV int operator()(int st, int KC) const {  // first batch row of step st (monotonic in st)
    if (xcd_ch == 0) return rs + st * KC;
    const int m = m0 + (st >> sh);  // (was st / spc: ~30 scalar instructions per call, in every K-step's loads)
    return (contig ? x * (nch / 8) + m : x + 8 * m) * xcd_ch + (st & (spc - 1)) * KC;
  }
};

// LDS-staged variant of wgrad_kernel (same tiles, splits, step order and slab layout; every output element
// is the same MFMA chain, so the results are bitwise those of wgrad_kernel): the workgroup stages the 64-row
// dY^T tile and the 64-row X^T tile of SUB (2) consecutive 32-row K-steps per interval, and each wave reads its
// 32x32 operands from LDS (in wgrad_kernel every fragment is fetched by two waves straight from L2).
//  * loads: interval i's 16-byte chunks are issued two intervals ahead into one of two register slots (slot
//    i & 1, statically alternated by a two-way unrolled loop), so two intervals of loads are in flight behind
//    the MFMAs; ONE LDS buffer (20 KB at SUB 2), written between two barriers (a double-buffered SUB-4
//    version -- 72 KB, two workgroups per CU -- ran the MLP's 560-workgroup grid in two rounds).
//    (Measured and removed in round 5: the layer-1 B operand as the raw uint8 batch rows the head wrote,
//    normalised in registers and read with transposing LDS reads -- 35.5 vs 33.2 us per MLP bf16 step;
//    profiles/r4_session2/ab_mlp8k_raw_rows.txt.)
// Rows padded by 32 B (conflict-free ds_read_b128 fragment reads).  LDS use keeps it to the schedules where
// nothing LDS-heavy runs beside it (the MLP; LeNet's FC wgrad runs beside conv_bwd on the LDS-free kernel).
template <typename T, int SUB, bool SPL>
DEV void wgrad_lds_body(const WgArgs<T>& a, const int j, const WgRows rows, const int nsteps, const int tile,
                        const int split, T* sa, T* sb) {
  const WgJob<T>& J = a.job[j];
  using M = Mma<T>;
  using Frag = typename M::Frag;
  constexpr int KV = M::KV, KC = M::KC;
  constexpr int PE = (SUB * 64 + 32) / (int)sizeof(T);  // row pitch (elements): SUB steps x 64 B + 32 B pad
  const int tid = threadIdx.x, lane = tid & 63, w = wave_id(), row = lane & 15, grp = lane >> 4;
  const int nint = (nsteps + SUB - 1) / SUB;  // barrier intervals (block-uniform)
  const int lb = tile - J.blk_begin;
  const int bn = lb / J.nblk_k, bk = lb % J.nblk_k;
  const int nb0 = bn * 64, kb0 = bk * 64;
  const int n0 = nb0 + (w >> 1) * 32, k0 = kb0 + (w & 1) * 32;
  const int Kb = J.K + (J.bias ? 1 : 0);
  const bool wave_live = n0 < J.N && k0 < Kb;  // waves without outputs still stage and sync

  // staging role: tile row sr = tid / 4, 16-byte chunk sc = tid % 4 of each step's KC elements
  const int sr = tid >> 2, sc = tid & 3;
  const bool a_ok = nb0 + sr < J.NP, b_ok = kb0 + sr < J.K;
  const T* asrc = J.dyT + (size_t)min(nb0 + sr, J.NP - 1) * a.ldB + sc * KV;
  const T* bsrc = J.xT + (size_t)min(kb0 + sr, J.K > 0 ? J.K - 1 : 0) * a.ldB + sc * KV;
  const u32x4 z4 = u32x4{0u, 0u, 0u, 0u};
  struct Slot {
    u32x4 ra[SUB], rb[SUB];
  };
  auto fetch = [&](int it, Slot& d) {  // straight-line loads of interval it (steps past nsteps re-read the last)
#pragma unroll
    for (int q = 0; q < SUB; ++q) {
      const int rc = rows(min(it * SUB + q, nsteps - 1), KC);
      d.ra[q] = *reinterpret_cast<const u32x4*>(asrc + rc);
      d.rb[q] = *reinterpret_cast<const u32x4*>(bsrc + rc);
    }
  };
  auto stage = [&](const Slot& d) {
#pragma unroll
    for (int q = 0; q < SUB; ++q) {
      *reinterpret_cast<u32x4*>(&sa[sr * PE + q * KC + sc * KV]) = a_ok ? d.ra[q] : z4;
      *reinterpret_cast<u32x4*>(&sb[sr * PE + q * KC + sc * KV]) = b_ok ? d.rb[q] : z4;
    }
  };

  f32x4 acc[2][2];
#pragma unroll
  for (int mi = 0; mi < 2; ++mi)
#pragma unroll
    for (int ni = 0; ni < 2; ++ni) acc[mi][ni] = zero4();
  Frag ones;
#pragma unroll
  for (int q = 0; q < KV; ++q) M::set(ones, q, 1.f);
  const Frag zf = M::zero();
  const int kk0 = k0 + row, kk1 = k0 + 16 + row;
  const int sel0 = kk0 < J.K ? 0 : (kk0 == J.K && J.bias ? 1 : 2);
  const int sel1 = kk1 < J.K ? 0 : (kk1 == J.K && J.bias ? 1 : 2);
  const int ao0 = (n0 - nb0 + row) * PE + grp * KV, ao1 = ao0 + 16 * PE;
  const int bo0 = (k0 - kb0 + row) * PE + grp * KV, bo1 = bo0 + 16 * PE;
  // B columns past K: the bias column reads ones, the padding zeros -- loop-invariant per lane, applied as a
  // vector select (a select between whole fragments was lowered to an indexed scratch array)
  const bool use0 = sel0 == 0, use1 = sel1 == 0;
  const Frag alt0 = sel0 == 1 ? ones : zf, alt1 = sel1 == 1 ? ones : zf;
  auto compute = [&](int it) {
    const int nq = min(SUB, nsteps - it * SUB);  // live steps of this interval (block-uniform)
#pragma unroll
    for (int q = 0; q < SUB; ++q) {
      if (q < nq) {
        const Frag a0 = M::load(&sa[ao0 + q * KC]), a1 = M::load(&sa[ao1 + q * KC]);
        const Frag f0 = M::load(&sb[bo0 + q * KC]), f1 = M::load(&sb[bo1 + q * KC]);
        Frag b0, b1;
        b0.v = use0 ? f0.v : alt0.v;
        b1.v = use1 ? f1.v : alt1.v;
        wg_mma<T, SPL>(acc[0][0], a0, b0);
        wg_mma<T, SPL>(acc[0][1], a0, b1);
        wg_mma<T, SPL>(acc[1][0], a1, b0);
        wg_mma<T, SPL>(acc[1][1], a1, b1);
      }
    }
  };

  Slot s0, s1;
  if (nint > 0) {
    fetch(0, s0);
    if (nint > 1) fetch(1, s1);
    stage(s0);
  }
  __syncthreads();
  // interval it: slot `cur` (interval it, staged before the barrier) takes interval it + 2's loads; then interval
  // it's MFMAs; then, between two barriers, interval it + 1 (slot `nxt`) is staged
  auto body = [&](int it, Slot& cur, Slot& nxt) {
    if (it + 2 < nint) fetch(it + 2, cur);
    compute(it);
    if (it + 1 < nint) {
      __syncthreads();  // every wave has read interval it from the buffer
      stage(nxt);
      __syncthreads();
    }
  };
  for (int it = 0; it < nint; it += 2) {  // unrolled by two: the slots alternate statically (no register copies)
    body(it, s0, s1);
    if (it + 1 < nint) body(it + 1, s1, s0);
  }
  if (!wave_live) return;

  float* out = a.slab + (size_t)split * a.slab_ld + J.out_off;
#pragma unroll
  for (int mi = 0; mi < 2; ++mi)
#pragma unroll
    for (int ni = 0; ni < 2; ++ni) {
      const int k = k0 + ni * 16 + row;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int n = n0 + mi * 16 + grp * 4 + i;
        const int q = n >= J.N ? -1 : (k < J.K ? n * J.K + k : (k == J.K && J.bias ? J.N * J.K + n : -1));
        if (q >= 0) out[q] = acc[mi][ni][i];
      }
    }
}

template <typename T, int SUB, bool SPL>
__global__ __launch_bounds__(256) void wgrad_lds_kernel(WgArgs<T> a) {
  constexpr int KC = Mma<T>::KC;
  constexpr int TILE = 64 * ((SUB * 64 + 32) / (int)sizeof(T));
  __shared__ __attribute__((aligned(16))) T lds[2][TILE];  // [A = dY^T, B = X^T]
  const int lin = blockIdx.y * gridDim.x + blockIdx.x;
  if (a.stamps && threadIdx.x == 0 && lin < 512) a.stamps[(STAMP_WGRAD + lin) * 16] = wall_clock64();
  int tile, split, nsteps;
  WgRows rows{a.xcd_ch, 0, 0, 1, 0, a.contig, a.nch, 0};
  if (a.xcd_ch == 0) {
    tile = blockIdx.x;
    split = blockIdx.y;
    rows.rs = split * a.rlen;
    nsteps = (min(rows.rs + a.rlen, a.Bp) - rows.rs + KC - 1) / KC;
  } else {
    const int L = blockIdx.x, q = L >> 3;
    rows.x = L & 7;
    tile = q / a.sx;
    const int sub = q % a.sx;
    split = rows.x * a.sx + sub;
    const int mx = a.contig ? a.nch / 8 : (rows.x < a.nch ? (a.nch - rows.x + 7) / 8 : 0);
    rows.m0 = sub * mx / a.sx;
    const int m1 = (sub + 1) * mx / a.sx;
    rows.spc = a.xcd_ch / KC;
    rows.sh = __builtin_ctz(rows.spc);
    nsteps = (m1 - rows.m0) * rows.spc;
  }
  while (nsteps > 0 && rows(nsteps - 1, KC) >= a.Bp) --nsteps;  // steps past the (padded) batch
  nsteps = __builtin_amdgcn_readfirstlane(nsteps);
  int j = 0;
  while (j + 1 < a.njobs && tile >= a.job[j + 1].blk_begin) ++j;
  wgrad_lds_body<T, SUB, SPL>(a, j, rows, nsteps, tile, split, lds[0], lds[1]);
  if (a.stamps && threadIdx.x == 0 && lin < 512) a.stamps[(STAMP_WGRAD + lin) * 16 + 1] = wall_clock64();
}

template <typename T, class Model>
__global__ __launch_bounds__(256) void wgrad_sgd_kernel(WgArgs<T> a) {
  wgrad_sgd_tile<T, Model>(a, blockIdx.x);
}

// ====================================================================================
// Large-batch weight gradient with split-K INSIDE the workgroup (round 6; replaces wgrad_kernel /
// wgrad_lds_kernel from B >= SK_MIN_B).  Same 64x64 output blocks, batch splits and slab layout as wgrad_kernel,
// but each of the 4 waves computes the WHOLE 64x64 block (4x4 MFMA tiles, 64 accumulators) over every 4th
// K-step of the workgroup's batch range, and the four partial blocks are summed through LDS in a fixed order
// ((w0 + w1) + (w2 + w3)) before the one slab row is written.  Against wgrad_kernel (four 32x32 quadrants per
// block, every fragment fetched by two waves): half the L2 -> CU fragment traffic, 16 instead of 4 MFMAs per
// 8 fragment loads, and a quarter of the dependent K-steps per wave -- SK_PF steps (8 x SK_PF fragments) are
// issued before the first MFMA, so a whole 512-row split is ONE memory round trip per wave (LeNet-5 / MLP at
// B = 8192, 16 splits).  Round-5 counters of wgrad_kernel: 15.9 us at 1.9 % MFMA busy, latency-bound
// (profiles/r5_session1/pmc_table_final.md).
// fp32 (SPL): the 4 A and 4 B fragments of a K-step are cut into bf16 hi / mid / lo parts ONCE and reused by the
// 16 products (Mma<float>::mma_pp), instead of a cut per product.
constexpr int SK_MIN_B = 2048;  // smallest batch on the split-K-in-workgroup kernel
// PF: K-steps per wave whose fragments are in flight together (8 x PF 16-byte loads per lane)
template <typename T, bool SPL, int PF>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(PF > 2 || (sizeof(T) == 4 && SPL) ? 2 : 3))) void wgrad_sk_kernel(WgArgs<T> a) {
  using M = Mma<T>;
  using Frag = typename M::Frag;
  constexpr int KV = M::KV, KC = M::KC;
  constexpr bool CUT = sizeof(T) == 4 && SPL;
  constexpr int TP = 68;  // row pitch (floats) of the reduced 64x64 block in LDS: 16-byte rows, spread banks
  __shared__ __attribute__((aligned(16))) f32x4 red[2][16][64];  // 32 KB: two waves' partial blocks at a time
  const int lane = threadIdx.x & 63, w = wave_id(), row = lane & 15, grp = lane >> 4;
  const int L = blockIdx.x;
  if (a.stamps && threadIdx.x == 0 && L < 512) a.stamps[(STAMP_WGRAD + L) * 16] = wall_clock64();
  int tile, split;
  if (a.xcd_ch > 0) {  // XCD-aware: workgroup L runs on XCD L % 8 and takes a split of that XCD's batch rows
    const int x = L & 7, q = L >> 3;
    tile = q / a.sx;
    split = x * a.sx + q % a.sx;
  } else {
    const int ns = (a.Bp + a.rlen - 1) / a.rlen;
    tile = L / ns;
    split = L % ns;
  }
  const int rs = split * a.rlen, re = min(rs + a.rlen, a.Bp);
  const int nsteps = (re - rs) / KC;                      // K-steps of this workgroup (block-uniform)
  const int nw = nsteps > w ? (nsteps - w + 3) / 4 : 0;  // this wave's: steps w, w + 4, ...
  int j = 0;
  while (j + 1 < a.njobs && tile >= a.job[j + 1].blk_begin) ++j;
  const WgJob<T>& J = a.job[j];
  const int lb = tile - J.blk_begin;
  const int bn = lb / J.nblk_k, bk = lb % J.nblk_k;
  const int n0 = bn * 64, k0 = bk * 64;
  // Operand fragments by raw buffer loads whose resource ends at the operand's last real row (dY^T: N rows, X^T:
  // K rows): padding rows read as zeros WITHOUT memory traffic (LeNet's 10-row fc3 gradient in a 64-row block no
  // longer pulls 54 dead rows).  Branch-free body: every load is issued and all 16 MFMAs of a K-step run; the bias
  // column (k == K) reads ones by a per-lane select.  (Branching around the padding tiles' loads and MFMAs had put
  // 261 conditional branches into the loop.)
  const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc(const_cast<T*>(J.dyT), (short)0,
                                                                      J.N * a.ldB * (int)sizeof(T), 0x00020000);
  const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc(const_cast<T*>(J.xT), (short)0,
                                                                      J.K * a.ldB * (int)sizeof(T), 0x00020000);
  int ao[4], bo[4];
  bool ones_col[4];
  Frag ones;
#pragma unroll
  for (int q = 0; q < KV; ++q) M::set(ones, q, 1.f);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    ao[i] = ((n0 + 16 * i + row) * a.ldB + rs + grp * KV) * (int)sizeof(T);
    const int kk = k0 + 16 * i + row;
    bo[i] = (kk * a.ldB + rs + grp * KV) * (int)sizeof(T);
    ones_col[i] = kk == J.K && J.bias;
  }
  auto ld = [&](const __amdgpu_buffer_rsrc_t& r, int voff, int soff) {
    Frag f;
    f.v = __builtin_bit_cast(decltype(f.v), __builtin_amdgcn_raw_buffer_load_b128(r, voff, soff, 0));
    return f;
  };
  f32x4 acc[4][4];
#pragma unroll
  for (int mi = 0; mi < 4; ++mi)
#pragma unroll
    for (int ni = 0; ni < 4; ++ni) acc[mi][ni] = zero4();

  // K-step groups: every fragment of PF steps is issued before the first MFMA (the sched_barrier keeps hipcc
  // from sinking each load next to its use -- it had turned the group into one load + vmcnt(0) per 4 MFMAs); a
  // group's steps past this wave's count re-read its last step and multiply zero A fragments
  const Frag zf = M::zero();
  for (int g = 0; g < nw; g += PF) {
    Frag fa[PF][4], fb[PF][4];
#pragma unroll
    for (int p = 0; p < PF; ++p) {
      const int soff = (w + 4 * min(g + p, nw - 1)) * KC * (int)sizeof(T);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        fa[p][i] = ld(ra, ao[i], soff);
        fb[p][i] = ld(rb, bo[i], soff);
      }
    }
    __builtin_amdgcn_sched_barrier(0);
    const bool full = g + PF <= nw;  // wave-uniform
#pragma unroll
    for (int p = 0; p < PF; ++p) {
      Frag av[4], b[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        av[i].v = (full || g + p < nw) ? fa[p][i].v : zf.v;
        b[i].v = ones_col[i] ? ones.v : fb[p][i].v;
      }
      if constexpr (CUT) {
        u32x2 ah[4], am[4], al[4], bh[4], bm[4], bl[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          Mma<float>::split3(av[i].v, ah[i], am[i], al[i]);
          Mma<float>::split3(b[i].v, bh[i], bm[i], bl[i]);
        }
#pragma unroll
        for (int mi = 0; mi < 4; ++mi)
#pragma unroll
          for (int ni = 0; ni < 4; ++ni) Mma<float>::mma_pp(acc[mi][ni], ah[mi], am[mi], al[mi], bh[ni], bm[ni], bl[ni]);
      } else {
#pragma unroll
        for (int mi = 0; mi < 4; ++mi)
#pragma unroll
          for (int ni = 0; ni < 4; ++ni) M::mma(acc[mi][ni], av[mi], b[ni]);
      }
    }
  }
  if (a.stamps && threadIdx.x == 0 && L < 512) a.stamps[(STAMP_WGRAD + L) * 16 + 1] = wall_clock64();
  // fixed-order sum of the four waves' partial blocks, (w0 + w2) + (w1 + w3), through 32 KB of LDS
  if (w >= 2) {
#pragma unroll
    for (int t = 0; t < 16; ++t) red[w - 2][t][lane] = acc[t >> 2][t & 3];
  }
  __syncthreads();
  if (w < 2) {
#pragma unroll
    for (int t = 0; t < 16; ++t) acc[t >> 2][t & 3] += red[w][t][lane];
  }
  __syncthreads();
  if (w == 1) {
#pragma unroll
    for (int t = 0; t < 16; ++t) red[0][t][lane] = acc[t >> 2][t & 3];
  }
  __syncthreads();
  // wave 0 completes the sum, then lays the block out row-major ([n][k], pitch TP: 17 KB, over both buffers --
  // it has read buffer 0 into registers first, and nothing reads buffer 1 any more) ...
  static_assert(64 * TP * 4 <= (int)sizeof(red), "the row-major block must fit the reduction buffers");
  float* tileb = reinterpret_cast<float*>(&red[0][0][0]);
  if (w == 0) {
#pragma unroll
    for (int t = 0; t < 16; ++t) acc[t >> 2][t & 3] += red[0][t][lane];
#pragma unroll
    for (int mi = 0; mi < 4; ++mi)
#pragma unroll
      for (int ni = 0; ni < 4; ++ni)
#pragma unroll
        for (int i = 0; i < 4; ++i) tileb[(mi * 16 + grp * 4 + i) * TP + ni * 16 + row] = acc[mi][ni][i];
  }
  __syncthreads();
  // ... and all 256 threads write the slab row as 16-byte stores: weight (n, k..k+3) at n * K + k (K % 4 == 0 for
  // every layer, and slab rows / job offsets are 16-byte aligned: Trainer::fc_ld), the bias column k == K at
  // N * K + n; padding rows / columns get an offset past the resource end, which the hardware drops
  const int nout = J.N * J.K + (J.bias ? J.N : 0);  // this job's parameters
  const __amdgpu_buffer_rsrc_t rs_out = __builtin_amdgcn_make_buffer_rsrc(
      a.slab + (size_t)split * a.slab_ld + J.out_off, (short)0, nout * 4, 0x00020000);
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int c = threadIdx.x + 256 * e, n = c >> 4, kc = (c & 15) * 4;
    const f32x4 v = *reinterpret_cast<const f32x4*>(&tileb[n * TP + kc]);
    const bool ok = (n0 + n < J.N) & (k0 + kc < J.K);
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), rs_out,
                                           ok ? ((n0 + n) * J.K + k0 + kc) * 4 : 0x7FFFFFF0, 0, 0);
  }
  if (J.bias && J.K >= k0 && J.K < k0 + 64 && threadIdx.x < 64) {
    const int n = threadIdx.x;
    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(tileb[n * TP + (J.K - k0)]), rs_out,
                                          n0 + n < J.N ? (J.N * J.K + n0 + n) * 4 : 0x7FFFFFF0, 0, 0);
  }
  if (a.stamps && threadIdx.x == 0 && L < 512) {
    a.stamps[(STAMP_WGRAD + L) * 16 + 2] = wall_clock64();
    a.stamps[(STAMP_WGRAD + L) * 16 + 3] = hw_location() + 1;  // (+1: never 0, marks the 3-phase stamp set)
  }
}

// MNIST_AMD_WGRAD_SK_PF: K-steps in flight per wave (2 or 4)
int wgrad_sk_pf() {
  static const int v = [] {
    const char* e = std::getenv("MNIST_AMD_WGRAD_SK_PF");
    return e && *e == '4' ? 4 : 2;
  }();
  return v;
}
// MNIST_AMD_WGRAD_SK=1: the split-K-in-workgroup kernel from SK_MIN_B in every schedule (opt-in A/B).  Measured (profiles/r6_session1/NOTES.md): LeNet bf16
// B=8192 ~9.7 us span vs 15.9 us for wgrad_kernel alone, but beside conv_bwd its 32 KB of LDS per workgroup cannot
// co-reside with conv_bwd's two 71 KB workgroups (the concurrent step 0.1068 vs 0.0975 ms); the MLP's LDS-staged
// wgrad_lds_kernel stays faster (32.2 vs 35.6 us per step)
int wgrad_sk_mode() {
  static const int m = [] {
    const char* e = std::getenv("MNIST_AMD_WGRAD_SK");
    return e && *e ? (*e == '1' ? 1 : 0) : -1;
  }();
  return m;
}

// wgrad_kernel keeps ONE ring slot of K-step fragments per wave (the next step's fragments fetched while this
// one computes: two / four steps ahead measured within noise / 0.3-1.6 % slower on both models).  The
// LDS-staged weight gradient (wgrad_lds_kernel) is used for the MLP, whose wgrad runs alone on the chip; the
// LeNet wgrad runs beside conv_bwd, which holds the LDS.
constexpr int WGRAD_DEPTH = 1;
// 32-row K-steps per LDS interval, measured on the MLP at B = 8192 (1000 steps, same box, bitwise-equal
// parameters; profiles/r4_session2/ab_mlp8k_wgrad_sub.txt): SUB 1 / 2 / 3 / 4 = 34.9 / 33.2 / 34.1 / 34.9 us
// per step (the round-3 kernel -- one step per barrier, 6 workgroups per CU -- 34.1-34.6)
#ifndef MNIST_AMD_WGRAD_SUB
#define MNIST_AMD_WGRAD_SUB 2
#endif
constexpr int WGRAD_SUB = MNIST_AMD_WGRAD_SUB;  // wgrad_lds_kernel: 32-row K-steps staged per barrier interval

template <typename T, class H, class Model>
int wgrad_launch(const HeadBuffers& hb, int B, int splits, float* slab, int slab_ld, int xcd_ch, hipStream_t s,
                 const SgdFuse* fuse, int job_mask) {
  int blk = 0;
  WgArgs<T> a = wg::make_args<T, H, Model>(hb, B, splits, slab, slab_ld, fuse, job_mask, &blk);
  constexpr int KC = Mma<T>::KC;
  const bool lds_stage = std::is_same<Model, MlpModel>::value;
  // fp32 MLP weight gradient as 3-part bf16 splits from B = 4096 on (MLP fp32 B=8192 -6 %, but B=1024 +6 %:
  // profiles/r5_session1/hsplit2); no effect for bf16 (wg_mma)
  const bool spl = B >= 4096;
  const int skm = wgrad_sk_mode();
  // (off by default: on the chosen schedules the LDS-free wgrad_kernel runs beside conv_bwd, and giving the serial
  //  candidate a different kernel would end the bitwise equality of the single-GPU schedules)
  const bool sk = skm == 1;
  if (!fuse && B >= SK_MIN_B && sk) {
    // split-K-in-workgroup kernel over contiguous batch splits; with a split count that divides over the 8 XCDs,
    // XCD x takes splits [x * S / 8, (x + 1) * S / 8) -- the batch rows the XCD-contiguous head (xcd_unit) wrote
    // there (a bijection either way; only the L2 locality depends on the head's mapping)
    a.xcd_ch = splits % 8 == 0 ? 1 : 0;
    a.sx = splits / 8;
    // LeNet fp32: products as 3-part bf16 splits (as wgrad_kernel's wg_mma); MLP fp32 from B = 4096 (as wgrad_lds)
    const bool cut = std::is_same<Model, MlpModel>::value ? spl : true;
    const dim3 grid(blk * splits);
    if (sizeof(T) == 2 && wgrad_sk_pf() == 4) {  // (fp32: 2; at 4 the cut parts spill)
      if (cut) hipLaunchKernelGGL((wgrad_sk_kernel<T, true, 4>), grid, dim3(256), 0, s, a);
      else hipLaunchKernelGGL((wgrad_sk_kernel<T, false, 4>), grid, dim3(256), 0, s, a);
    } else {
      if (cut) hipLaunchKernelGGL((wgrad_sk_kernel<T, true, 2>), grid, dim3(256), 0, s, a);
      else hipLaunchKernelGGL((wgrad_sk_kernel<T, false, 2>), grid, dim3(256), 0, s, a);
    }
    return splits;
  }
  // XCD-aware mapping when the head's row tiling is known and the split count divides over 8 XCDs
  // (steps per row chunk xcd_ch / KC must be a power of two: the kernels map steps to rows by shift and mask)
  if (!fuse && xcd_ch > 0 && xcd_ch % KC == 0 && ((xcd_ch / KC) & (xcd_ch / KC - 1)) == 0 && splits % 8 == 0) {
    a.xcd_ch = xcd_ch;
    a.nch = (a.Bp + xcd_ch - 1) / xcd_ch;
    a.sx = splits / 8;
    const int head_grid = (rup(B, 32) + xcd_ch - 1) / xcd_ch;  // head_launch_mtw's grid
    a.contig = hb.xcd && head_grid % 8 == 0 && a.nch == head_grid;
    if (lds_stage && spl) hipLaunchKernelGGL((wgrad_lds_kernel<T, WGRAD_SUB, true>), dim3(blk * splits), dim3(256), 0, s, a);
    else if (lds_stage) hipLaunchKernelGGL((wgrad_lds_kernel<T, WGRAD_SUB, false>), dim3(blk * splits), dim3(256), 0, s, a);
    else hipLaunchKernelGGL((wgrad_kernel<T, WGRAD_DEPTH>), dim3(blk * splits), dim3(256), 0, s, a);
  } else if (a.fuse) {
    hipLaunchKernelGGL((wgrad_sgd_kernel<T, Model>), dim3(blk), dim3(256), 0, s, a);
  } else {
    if (lds_stage && spl) hipLaunchKernelGGL((wgrad_lds_kernel<T, WGRAD_SUB, true>), dim3(blk, splits), dim3(256), 0, s, a);
    else if (lds_stage) hipLaunchKernelGGL((wgrad_lds_kernel<T, WGRAD_SUB, false>), dim3(blk, splits), dim3(256), 0, s, a);
    else hipLaunchKernelGGL((wgrad_kernel<T, WGRAD_DEPTH>), dim3(blk, splits), dim3(256), 0, s, a);
  }
  return splits;
}

template <typename T, class H, int MT, int NWV>
void head_launch_mtw(bool train, const BatchRef& br, const HeadBuffers& hb, hipStream_t s) {
  const int rows = rup(br.B, 32);
  const int grid = (rows + MT * 16 - 1) / (MT * 16);
  if (train)
    hipLaunchKernelGGL((head_kernel<T, H, MT, true, false, NWV>), dim3(grid), dim3(NWV * 64), 0, s, br, hb);
  else
    hipLaunchKernelGGL((head_kernel<T, H, MT, false, false, NWV>), dim3(grid), dim3(NWV * 64), 0, s, br, hb);
}

// 16 waves per head workgroup (swept 4 / 8 / 16 at B=8192: 16 waves, 4 per SIMD, best by 3 % step time)
template <typename T, class H, int MT>
void head_launch_mt(bool train, const BatchRef& br, const HeadBuffers& hb, hipStream_t s) {
  head_launch_mtw<T, H, MT, 16>(train, br, hb, s);
}

// small-batch path: layer-1 split GEMM, then the head with 16-row tiles consuming the partials;
// with only B/16 workgroups, each gets SPLIT_NWV waves so every N-tile of a layer has its own wave
#ifndef SPLIT_NWV
#define SPLIT_NWV 16  // swept 4 / 8 / 16: 40.8 / 37.4 / 36.7 us per MLP fp32 B=128 step
#endif
template <typename T, class H, int NWV>
void head_launch_split_w(bool train, const BatchRef& br, const HeadBuffers& hb, hipStream_t s) {
  const int mt = (br.B + 15) / 16;
  const dim3 g1(mt, (H::N1P / 16 + 3) / 4, L1_KSPLIT);
  const int grid = (rup(br.B, 32) + 15) / 16;
  if (train) {
    hipLaunchKernelGGL((l1_split_kernel<T, H, true>), g1, dim3(256), 0, s, br, hb);
    hipLaunchKernelGGL((head_kernel<T, H, 1, true, true, NWV>), dim3(grid), dim3(NWV * 64), 0, s, br, hb);
  } else {
    hipLaunchKernelGGL((l1_split_kernel<T, H, false>), g1, dim3(256), 0, s, br, hb);
    hipLaunchKernelGGL((head_kernel<T, H, 1, false, true, NWV>), dim3(grid), dim3(NWV * 64), 0, s, br, hb);
  }
}

template <typename T, class H>
void head_launch_split(bool train, const BatchRef& br, const HeadBuffers& hb, hipStream_t s) {
  head_launch_split_w<T, H, SPLIT_NWV>(train, br, hb, s);
}

// returns the batch rows per workgroup actually used (the wgrad kernel's XCD-aware mapping needs it)
template <typename T, class H>
int head_launch_t(bool train, const BatchRef& br, const HeadBuffers& hb, int rows, hipStream_t s) {
  // the split layer 1 pays for its extra launch on the 784-deep MLP layer and, for fp32 (matrix rate 1/8 of
  // bf16: the 16-row head is matrix-bound on its 8 CUs), on LeNet's 400-deep one: LeNet fp32 B=128 46.9 -> 44.4 us,
  // B=1024 122.3 -> 112.8 us (profiles/r4_session2/ab_lenet_f32_l1_split.txt); LeNet bf16 keeps layer 1 in the head
  constexpr bool split_l1 = H::K0 >= 512 || sizeof(T) == 4;
  if (hb.z1p && br.B <= L1_SPLIT_MAX_B && split_l1) {
    head_launch_split<T, H>(train, br, hb, s);
    return 16;
  }
  if (rows <= 16) {
    head_launch_mt<T, H, 1>(train, br, hb, s);
    return 16;
  }
  if (rows <= 32 || !HeadSmem<T, H, 4>::FITS) {
    if constexpr (HeadSmem<T, H, 2>::FITS) {
      head_launch_mt<T, H, 2>(train, br, hb, s);
      return 32;
    } else {
      head_launch_mt<T, H, 1>(train, br, hb, s);
      return 16;
    }
  }
  if constexpr (HeadSmem<T, H, 4>::FITS) head_launch_mt<T, H, 4>(train, br, hb, s);
  return 64;
}

// Rows of the CURRENT step (step_ptr[0]) -> xnext / ynext: primes the look-ahead after the host set the
// step counter (set_epoch_indices); every training step's head keeps it one step ahead after that.
__global__ __launch_bounds__(256) void gather_next_kernel(BatchRef br) {
  const int e = blockIdx.x * 256 + threadIdx.x, r = e / 49, c = e % 49;
  if (r >= br.batch_stride) return;
  const int g = br.step_ptr[0] * br.batch_stride + r;
  const bool valid = g < br.step_ptr[2];
  const int gi = valid ? br.idx_epoch[g] : 0;
  const uint4 v = valid ? *reinterpret_cast<const uint4*>(br.images + (size_t)gi * 784 + c * 16) : make_uint4(0, 0, 0, 0);
  *reinterpret_cast<uint4*>(br.xnext + (size_t)r * 784 + c * 16) = v;
  if (c == 0) br.ynext[r] = valid ? br.labels[gi] : 0;
}

}  // namespace

void launch_gather_next(const BatchRef& br, hipStream_t s) {
  if (!br.xnext || br.batch_stride <= 0) return;
  hipLaunchKernelGGL(gather_next_kernel, dim3((br.batch_stride * 49 + 255) / 256), dim3(256), 0, s, br);
}

int head_rows_per_block(ModelKind m, DType t, int B) {
  if (B <= 256) return 16;
  if (t == DType::F32) return 32;
  // MLP bf16, B=8192: 32-row tiles (256 workgroups, every CU) 34.8 us per step vs 38.8-39.3 with 64-row
  // tiles on 128 CUs (same box, 1000-step bench, Dropout 0.2)
  if (m == ModelKind::MLP) return 32;
  // LeNet bf16, 16-wave workgroups: 32-row tiles = 256 workgroups at B=8192, every CU (0.1143-0.1150 ms
  // per step vs 0.1184-0.1186 with 64-row tiles on 128 CUs, same box; before the head's end-of-kernel
  // atomics were removed the 64-row tiles had measured 0.5 % faster)
  return 32;
}

int launch_head(ModelKind m, DType t, bool train, const BatchRef& br, const HeadBuffers& hb, int rows,
                hipStream_t s) {
  if (m == ModelKind::MLP) {
    if (t == DType::F32) return head_launch_t<float, MlpModel::Head>(train, br, hb, rows, s);
    return head_launch_t<bf16, MlpModel::Head>(train, br, hb, rows, s);
  }
  if (t == DType::F32) return head_launch_t<float, LenetModel::Head>(train, br, hb, rows, s);
  return head_launch_t<bf16, LenetModel::Head>(train, br, hb, rows, s);
}

int launch_head_wgrad(ModelKind m, DType t, const HeadBuffers& hb, int B, int splits, float* slab,
                      int slab_ld, hipStream_t s, int head_rows, const SgdFuse* fuse, int job_mask) {
  // head_rows: batch rows per head workgroup for this B (0 = unknown: contiguous split mapping)
  if (m == ModelKind::MLP) {
    if (t == DType::F32)
      return wgrad_launch<float, MlpModel::Head, MlpModel>(hb, B, splits, slab, slab_ld, head_rows, s, fuse, job_mask);
    return wgrad_launch<bf16, MlpModel::Head, MlpModel>(hb, B, splits, slab, slab_ld, head_rows, s, fuse, job_mask);
  }
  if (t == DType::F32)
    return wgrad_launch<float, LenetModel::Head, LenetModel>(hb, B, splits, slab, slab_ld, head_rows, s, fuse, job_mask);
  return wgrad_launch<bf16, LenetModel::Head, LenetModel>(hb, B, splits, slab, slab_ld, head_rows, s, fuse, job_mask);
}
