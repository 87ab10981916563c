// Grouped FC weight-gradient GEMM: argument blocks and the SGD-fused tile body, shared by the head kernels
// (head.hip: wgrad_kernel / wgrad_lds_kernel / wgrad_sgd_kernel) and LeNet's small-batch conv_bwd + FC-update
// kernel (lenet.hip), which runs the SGD-fused FC tiles as extra workgroups of the conv_bwd grid.
#pragma once
#include <algorithm>
#include <stdexcept>
#include <type_traits>

#include "common.h"
#include "launch.h"
#include "models.h"

namespace wg {

// ====================================================================================
// Grouped weight-gradient GEMM:  dW[n][k] = sum_r dY^T[n][r] * X^T[k][r]  (+ bias column k == K)
// Both operands are stored row = feature, contiguous batch, so each lane's K-chunk fragment is
// one 16-byte load.  A 64x64 output block per workgroup (each wave 32x32 = 2x2 MFMA tiles);
// the batch is split over gridDim.y, each split writes its own fp32 slab row (deterministic).
// ====================================================================================
template <typename T>
struct WgJob {
  const T* dyT;
  const T* xT;
  int N, K, NP, bias, out_off, nblk_k, blk_begin;
};
template <typename T>
struct WgArgs {
  WgJob<T> job[3];
  int njobs, ldB, rlen, Bp, slab_ld;
  // XCD-aware mode (xcd_ch > 0): 1-D grid; workgroup L runs on XCD L % 8 (round-robin dispatch) and
  // reads only the batch rows the head kernel wrote from that XCD -- row chunks c = x, x+8, ... of
  // xcd_ch rows (= head rows per workgroup) -- so its operands hit the XCD's own L2.
  // contig: the head used the XCD-contiguous mapping (xcd_unit), so XCD x wrote chunks
  // [x * nch / 8, (x + 1) * nch / 8) instead of x, x + 8, ...
  int xcd_ch, nch, sx, contig;  // chunk rows, chunk count, splits per XCD
  float* slab;
  SgdFuse sgd;          // used when fuse != 0 (then splits == 1)
  int fuse;
  unsigned long long* stamps;  // optional phase stamps (MNIST_AMD_STAMPS): slots [STAMP_WGRAD + block][16]
};

// Weight-gradient GEMM + SGD update for one GPU and ONE batch split (small batches), one 32x32 output tile
// (`tile`) per 4-wave workgroup (waves >= 4 of a larger workgroup idle): every output
// element is the whole gradient, so the update is the epilogue -- g = scale * dW, momentum, parameter,
// packed operand images, device step counters -- and the separate reduce + SGD kernel disappears
// (bitwise equal to wgrad -> reduce_sgd: a one-slab reduce is (0 + dW) * scale).  One 16x16 output tile
// per wave and a 32x32 tile per block: few MFMAs and few memory operations per wave, so the whole K
// range is prefetched at once and the epilogue's stores stay within one wave's outstanding-operation
// budget (the 32x32-per-wave variant stalled on it).
template <typename T, class Model>
DEV void wgrad_sgd_tile(const WgArgs<T>& a, int tile) {
  using M = Mma<T>;
  using Frag = typename M::Frag;
  constexpr int KV = M::KV, KC = M::KC, FPS = 8;
  const int lane = threadIdx.x & 63, w = wave_id(), row = lane & 15, grp = lane >> 4;
  auto stamp = [&](int k) {
    if (a.stamps && threadIdx.x == 0 && tile < 512) a.stamps[(STAMP_WGRAD + tile) * 16 + k] = wall_clock64();
  };
  stamp(0);
  if (a.sgd.step_ptr && tile == 0 && threadIdx.x == 0) {
    a.sgd.step_ptr[0] += 1;  // nothing after the head reads the batch counter in this step
    a.sgd.step_ptr[1] += 1;
  }
  int j = 0;
  while (j + 1 < a.njobs && tile >= a.job[j + 1].blk_begin) ++j;
  const WgJob<T>& J = a.job[j];
  const int lb = tile - J.blk_begin;
  const int bn = lb / J.nblk_k, bk = lb % J.nblk_k;
  const int n0 = bn * 32 + (w >> 1) * 16, k0 = bk * 32 + (w & 1) * 16;
  const int Kb = J.K + (J.bias ? 1 : 0);
  if (n0 >= J.N || k0 >= Kb) return;  // wave-uniform
  const int nsteps = a.Bp / KC;

  const T* ap = J.dyT + (size_t)(n0 + row) * a.ldB + grp * KV;  // rows < NP (zero padded)
  const int kk = k0 + row;
  const T* bp = J.xT + (size_t)min(kk, J.K > 0 ? J.K - 1 : 0) * a.ldB + grp * KV;
  const int sel = kk < J.K ? 0 : (kk == J.K && J.bias ? 1 : 2);
  Frag ones;
#pragma unroll
  for (int q = 0; q < KV; ++q) M::set(ones, q, 1.f);
  const Frag zf = M::zero();

  // the first FPS K-steps' fragments, then the SGD operands (the MFMAs wait only for the former)
  Frag fa[FPS], fb[FPS];
#pragma unroll
  for (int st = 0; st < FPS; ++st) {
    const int rc = min(st, nsteps - 1) * KC;
    fa[st] = M::load(ap + rc);
    fb[st] = M::load(bp + rc);
  }
  int pidx[4];
  float pv[4], mv[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int n = n0 + grp * 4 + i;
    const int q = n >= J.N ? -1 : (kk < J.K ? n * J.K + kk : (kk == J.K && J.bias ? J.N * J.K + n : -1));
    pidx[i] = q < 0 ? -1 : J.out_off + q;
    const int p = max(pidx[i], 0);
    pv[i] = a.sgd.params[p];
    mv[i] = a.sgd.mom ? a.sgd.mom[p] : 0.f;
  }
  f32x4 acc = zero4();
#pragma unroll
  for (int st = 0; st < FPS; ++st)
    if (st < nsteps) M::mma(acc, fa[st], sel == 0 ? fb[st] : (sel == 1 ? ones : zf));
  for (int st = FPS; st < nsteps; ++st) {  // longer batches: the rest, one step at a time
    const Frag x = M::load(ap + st * KC), y = M::load(bp + st * KC);
    M::mma(acc, x, sel == 0 ? y : (sel == 1 ? ones : zf));
  }
  stamp(1);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    if (pidx[i] < 0) continue;
    const int p = pidx[i];
    float g = (0.f + acc[i]) * a.sgd.scale;  // = reduce_sgd over one slab
    a.sgd.grad[p] = g;
    if (a.sgd.mom) {
      const float b = a.sgd.momentum * mv[i] + g;
      a.sgd.mom[p] = b;
      g = b;
    }
    const float nv = pv[i] - a.sgd.lr * g;
    a.sgd.params[p] = nv;
    Packer<Model, T>::pack(p, nv, reinterpret_cast<T*>(a.sgd.pack));
  }
  stamp(2);
}


// The jobs (one per layer in job_mask) and split geometry of one grouped weight gradient; *blocks = output
// tiles of BT x BT (BT = 32 with the SGD epilogue, else 64), *splits = batch splits actually used.
template <typename T, class H, class Model>
WgArgs<T> make_args(const HeadBuffers& hb, int B, int& splits, float* slab, int slab_ld, const SgdFuse* fuse,
                    int job_mask, int* blocks) {
  WgArgs<T> a{};
  const int BT = fuse ? 32 : 64;
  int nj = 0;
  auto mk = [&](int layer, const void* dy, const void* x, int N, int K, int NP, bool bias, int off, int& blk) {
    if (!(job_mask >> layer & 1)) return;
    WgJob<T>& J = a.job[nj++];
    J.dyT = reinterpret_cast<const T*>(dy);
    J.xT = reinterpret_cast<const T*>(x);
    J.N = N; J.K = K; J.NP = NP; J.bias = bias ? 1 : 0; J.out_off = off;
    J.nblk_k = (K + (bias ? 1 : 0) + BT - 1) / BT;
    J.blk_begin = blk;
    blk += ((N + BT - 1) / BT) * J.nblk_k;
  };
  int blk = 0;
  mk(0, hb.dy1T, hb.xT, H::N1, H::K0, H::N1P, true, H::W1, blk);
  mk(1, hb.dy2T, hb.h1T, H::N2, H::N1, H::N2P, true, H::W2, blk);
  mk(2, hb.dy3T, hb.h2T, H::NC, H::N2, H::NCP, H::BIAS3, H::W3, blk);
  if (nj == 0) throw std::invalid_argument("wgrad: empty job mask");
  a.njobs = nj;
  a.ldB = hb.ldB;
  constexpr int KC = Mma<T>::KC;
  a.Bp = rup(B, KC);
  splits = std::max(1, std::min(splits, a.Bp / KC));
  a.rlen = rup((a.Bp + splits - 1) / splits, KC);
  splits = (a.Bp + a.rlen - 1) / a.rlen;
  if (fuse) {
    if (splits != 1) throw std::invalid_argument("wgrad with the SGD epilogue needs one batch split");
    a.sgd = *fuse;
    a.fuse = 1;
  }
  a.slab = slab;
  a.slab_ld = slab_ld;
  a.stamps = hb.stamps;
  a.xcd_ch = 0;
  *blocks = blk;
  return a;
}

}  // namespace wg
