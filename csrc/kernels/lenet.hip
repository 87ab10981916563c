// LeNet-5 convolution trunk on CDNA4 matrix cores.
//
//   conv_fwd : gather(idx) + Normalize -> Conv2d(1,6,5,pad 2) + bias + ReLU + MaxPool2d(2)
//              -> Conv2d(6,16,5) + bias + ReLU + MaxPool2d(2) -> pool2 [B][400] (NCHW flatten)
//   conv_bwd : pool2 grads -> (pool2 argmax, ReLU mask) -> conv2 wgrad + bias grad
//              -> conv2 dgrad -> (pool1 argmax, ReLU mask) -> conv1 wgrad + bias grad
// One workgroup walks IPB images; each image lives entirely in LDS (padded 32x32 input,
// 14x14x8 pool1 map, 10x10x16 conv2 grads), so the only HBM traffic is the uint8 pixels,
// the pooled outputs/grads, 1-byte pool codes, and the packed weights.
//
// Implicit GEMM with pooling folded into the M ordering: output rows are ordered
// m = pooled_position*4 + window_element, so in the 16x16 MFMA C layout
// (row = (lane>>4)*4 + i) lane group g holds the four window elements of ONE pooled
// output in its 4 accumulator registers: 2x2 max-pool, argmax and ReLU are pure
// register epilogue work.  Channels of pool1 are padded 6->8 (NHWC) so an im2col fragment
// of conv2 (8 contiguous k = one tap, 8 channels) is a single 16-byte LDS read.
// Weight gradients are accumulated in MFMA accumulators across all images of the
// workgroup; bias gradients come out of the same GEMMs through an all-ones column.
// Pool code byte: bits 0-1 argmax window element (first max, raster order, as ATen),
// bit 2 = pooled pre-activation > 0 (ReLU passes the gradient).
#include <algorithm>

#include "common.h"
#include "launch.h"
#include "models.h"

namespace {

using L = LenetModel;
constexpr int K0P = L::Head::K0P;  // 416

template <typename T>
struct FwdSmem {
  static constexpr int OFF_X = 0;                                  // [32][32] padded input
  static constexpr int OFF_P1 = rup(32 * 32 * (int)sizeof(T), 16);  // [196][8]
  static constexpr int TOTAL = rup(OFF_P1 + 196 * 8 * (int)sizeof(T), 16);
};

// Stage dataset image `s` normalised into the zero-padded 32x32 LDS tile (cooperative).
template <typename T>
DEV void stage_image(T* xpad, const uint8_t* images, int s, bool valid) {
  for (int e = threadIdx.x; e < 32 * 32; e += blockDim.x) xpad[e] = to_t<T>(0.f);
  __syncthreads();
  if (valid) {
    const uint8_t* img = images + (size_t)s * 784;
    for (int e = threadIdx.x; e < 196; e += blockDim.x) {  // 196 x 4 pixels
      const uint32_t u = *reinterpret_cast<const uint32_t*>(img + e * 4);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int k = e * 4 + j, y = k / 28, x = k % 28;
        xpad[(y + 2) * 32 + x + 2] = to_t<T>(mnist_norm((u >> (8 * j)) & 255u));
      }
    }
  }
}

template <typename T, bool TRAIN>
__global__ __launch_bounds__(256) void conv_fwd_kernel(BatchRef br, LenetConvBuffers cb, int ipb) {
  using M = Mma<T>;
  using Frag = typename M::Frag;
  using S = FwdSmem<T>;
  constexpr int KV = M::KV, KC = M::KC;
  __shared__ __attribute__((aligned(16))) char smem[S::TOTAL];
  T* xpad = reinterpret_cast<T*>(smem + S::OFF_X);
  T* p1s = reinterpret_cast<T*>(smem + S::OFF_P1);
  const int lane = threadIdx.x & 63, w = wave_id(), row = lane & 15, grp = lane >> 4;
  const int32_t* idx = br.idx_epoch + (size_t)br.step_ptr[0] * br.batch_stride;
  const T* pack = reinterpret_cast<const T*>(cb.pack);
  const float* prm = cb.params;

  // ---- per-lane constants: conv1 B fragments + tap offsets, conv2 B fragments
  constexpr int C1CH = 32 / KC;          // conv1 K = 32 (25 taps + pad)
  constexpr int C2CH = (25 * 8 + KC - 1) / KC;  // conv2 K = 25 taps x 8 ch (7 bf16 / 13 f32 chunks)
  Frag b1[C1CH];
  int koff1[C1CH][KV];
#pragma unroll
  for (int kc = 0; kc < C1CH; ++kc) {
    b1[kc] = M::load(pack + L::C1 + row * 32 + kc * KC + grp * KV);
#pragma unroll
    for (int j = 0; j < KV; ++j) {
      const int k = kc * KC + grp * KV + j;
      koff1[kc][j] = k < 25 ? (k / 5) * 32 + (k % 5) : 0;
    }
  }
  Frag b2[C2CH];
#pragma unroll
  for (int kc = 0; kc < C2CH; ++kc) b2[kc] = M::load(pack + L::C2F + row * 224 + kc * KC + grp * KV);
  const float bias1 = row < 6 ? prm[L::CB1 + row] : 0.f;
  const float bias2 = prm[L::CB2 + row];

  for (int t = 0; t < ipb; ++t) {
    const int b = blockIdx.x * ipb + t;
    const bool valid = b < br.B;
    stage_image<T>(xpad, br.images, valid ? idx[b] : 0, valid);
    __syncthreads();

    // ---- conv1 + bias + ReLU + maxpool: 49 M-tiles (4 pooled outputs x 4 window elems each)
    for (int mt = w; mt < 49; mt += 4) {
      const int q = row >> 2, e = row & 3;
      const int p = mt * 4 + q, py = p / 14, px = p % 14;
      const int base = (2 * py + (e >> 1)) * 32 + 2 * px + (e & 1);
      f32x4 acc = zero4();
#pragma unroll
      for (int kc = 0; kc < C1CH; ++kc) {
        Frag a;
#pragma unroll
        for (int j = 0; j < KV; ++j) M::set(a, j, to_f(xpad[base + koff1[kc][j]]));
        M::mma(acc, a, b1[kc]);
      }
      // lane: channel n = row, pooled position pp = mt*4 + grp, window elems in acc[0..3]
      const int n = row, pp = mt * 4 + grp;
      float mx = acc[0];
      int am = 0;
#pragma unroll
      for (int i = 1; i < 4; ++i)
        if (acc[i] > mx) { mx = acc[i]; am = i; }
      const float pre = mx + bias1;
      const float v = (n < 6) ? fmaxf(pre, 0.f) : 0.f;
      if (n < 8) {
        p1s[pp * 8 + n] = to_t<T>(v);
        if (TRAIN && valid) {
          reinterpret_cast<T*>(cb.p1)[((size_t)b * 196 + pp) * 8 + n] = to_t<T>(v);
          cb.m1[((size_t)b * 196 + pp) * 8 + n] = (n < 6) ? (uint8_t)(am | (pre > 0.f ? 4 : 0)) : 0;
        }
      }
    }
    __syncthreads();

    // ---- conv2 + bias + ReLU + maxpool: 100 rows (25 pooled x 4) = 7 M-tiles, N = 16
    for (int mt = w; mt < 7; mt += 4) {
      const int q = row >> 2, e = row & 3;
      const int p = min(mt * 4 + q, 24), py = p / 5, px = p % 5;
      const int base = ((2 * py + (e >> 1)) * 14 + 2 * px + (e & 1)) * 8;
      f32x4 acc = zero4();
#pragma unroll
      for (int kc = 0; kc < C2CH; ++kc) {
        int pos, c0;
        if constexpr (KV == 8) { pos = kc * 4 + grp; c0 = 0; }
        else { pos = kc * 2 + (grp >> 1); c0 = (grp & 1) * 4; }
        pos = min(pos, 24);
        const int kh = pos / 5, kw = pos % 5;
        M::mma(acc, M::load(p1s + base + (kh * 14 + kw) * 8 + c0), b2[kc]);
      }
      const int n = row, pp = mt * 4 + grp;
      if (pp < 25) {
        float mx = acc[0];
        int am = 0;
#pragma unroll
        for (int i = 1; i < 4; ++i)
          if (acc[i] > mx) { mx = acc[i]; am = i; }
        const float pre = mx + bias2;
        if (valid) {
          reinterpret_cast<T*>(cb.p2)[(size_t)b * K0P + n * 25 + pp] = to_t<T>(fmaxf(pre, 0.f));
          if (TRAIN) cb.m2[(size_t)b * 400 + n * 25 + pp] = (uint8_t)(am | (pre > 0.f ? 4 : 0));
        }
      }
    }
    __syncthreads();
  }
}

// ====================================================================================
template <typename T>
struct BwdSmem {
  static constexpr int OFF_X = 0;                                        // [32][32] T
  static constexpr int OFF_P1 = rup(OFF_X + 32 * 32 * (int)sizeof(T), 16);  // [196][8] T
  static constexpr int OFF_M1 = rup(OFF_P1 + 196 * 8 * (int)sizeof(T), 16); // [196][8] u8
  static constexpr int OFF_DY = rup(OFF_M1 + 196 * 8, 16);                 // [100][16] T
  static constexpr int OFF_DYT = rup(OFF_DY + 100 * 16 * (int)sizeof(T), 16);  // [16][128] T
  static constexpr int OFF_DP1 = rup(OFF_DYT + 16 * 128 * (int)sizeof(T), 16); // [196][8] f32
  static constexpr int OFF_RED = rup(OFF_DP1 + 196 * 8 * 4, 16);           // [4][2][256] f32
  static constexpr int TOTAL = rup(OFF_RED + 4 * 2 * 256 * 4, 16);
};

template <typename T>
__global__ __launch_bounds__(256) void conv_bwd_kernel(BatchRef br, LenetConvBuffers cb, int ipb) {
  using M = Mma<T>;
  using Frag = typename M::Frag;
  using S = BwdSmem<T>;
  constexpr int KV = M::KV, KC = M::KC;
  __shared__ __attribute__((aligned(16))) char smem[S::TOTAL];
  T* xpad = reinterpret_cast<T*>(smem + S::OFF_X);
  T* p1s = reinterpret_cast<T*>(smem + S::OFF_P1);
  uint8_t* m1s = reinterpret_cast<uint8_t*>(smem + S::OFF_M1);
  T* dys = reinterpret_cast<T*>(smem + S::OFF_DY);
  T* dyT = reinterpret_cast<T*>(smem + S::OFF_DYT);
  float* dp1 = reinterpret_cast<float*>(smem + S::OFF_DP1);
  float* red = reinterpret_cast<float*>(smem + S::OFF_RED);
  const int tid = threadIdx.x, lane = tid & 63, w = wave_id(), row = lane & 15, grp = lane >> 4;
  const int32_t* idx = br.idx_epoch + (size_t)br.step_ptr[0] * br.batch_stride;
  const T* pack = reinterpret_cast<const T*>(cb.pack);
  const T* dp2 = reinterpret_cast<const T*>(cb.dp2);

  constexpr int W2CH = 128 / KC;              // conv2 wgrad reduction over 100 (->128) positions
  constexpr int D2CH = (400 + KC - 1) / KC;   // conv2 dgrad K = 25 taps x 16 ch (13 bf16 / 25 f32)
  constexpr int W1CH = (784 + KC - 1) / KC;   // conv1 wgrad over 784 positions (25 bf16 / 49 f32)

  f32x4 accW2[4];   // conv2 wgrad tiles nt = w + 4*i (13 tiles over kcol = tap*8 + c, + bias col 200)
  f32x4 accW1[2];   // conv1 wgrad partial (this wave's share of the positions), kcol = tap, bias col 25
#pragma unroll
  for (int i = 0; i < 4; ++i) accW2[i] = zero4();
  accW1[0] = zero4();
  accW1[1] = zero4();

  for (int t = 0; t < ipb; ++t) {
    const int b = blockIdx.x * ipb + t;
    const bool valid = b < br.B;
    stage_image<T>(xpad, br.images, valid ? idx[b] : 0, valid);
    // pool1 activations + codes, zeroed grads
    {
      constexpr int P1V = 196 * 8 * (int)sizeof(T) / 16, M1V = 196 * 8 / 16;
      const uint4* psrc = reinterpret_cast<const uint4*>(reinterpret_cast<const T*>(cb.p1) + (size_t)b * 196 * 8);
      const uint4* msrc = reinterpret_cast<const uint4*>(cb.m1 + (size_t)b * 196 * 8);
      const uint4 z = make_uint4(0, 0, 0, 0);
      for (int e = tid; e < P1V; e += 256) reinterpret_cast<uint4*>(p1s)[e] = valid ? psrc[e] : z;
      for (int e = tid; e < M1V; e += 256) reinterpret_cast<uint4*>(m1s)[e] = valid ? msrc[e] : z;
    }
    for (int e = tid; e < 100 * 16; e += 256) dys[e] = to_t<T>(0.f);
    for (int e = tid; e < 16 * 128; e += 256) dyT[e] = to_t<T>(0.f);
    __syncthreads();
    // ---- scatter pool2 grads through argmax + ReLU mask into conv2 pre-activation grads
    if (valid) {
      for (int e = tid; e < 400; e += 256) {
        const int n = e / 25, p = e % 25;
        const uint8_t code = cb.m2[(size_t)b * 400 + e];
        if (code & 4) {
          const int win = code & 3, py = p / 5, px = p % 5;
          const int pos = (2 * py + (win >> 1)) * 10 + 2 * px + (win & 1);
          const T g = dp2[(size_t)b * K0P + e];
          dys[pos * 16 + n] = g;
          dyT[n * 128 + pos] = g;
        }
      }
    }
    __syncthreads();

    // ---- conv2 wgrad: dW2[n][tap*8+c] += sum_m dY2[m][n] * im2col(p1)[m][tap*8+c]
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int nt = w + 4 * i;
      if (nt >= 13) break;
      const int kcol = nt * 16 + row;
      const int tap = min(kcol >> 3, 24), c = kcol & 7;
      const int toff = ((tap / 5) * 14 + tap % 5) * 8 + c;
      const float sel = kcol < 200 ? 0.f : (kcol == 200 ? 1.f : -1.f);  // 0: data, 1: bias col, -1: zero
      for (int kc = 0; kc < W2CH; ++kc) {
        const Frag a = M::load(dyT + row * 128 + kc * KC + grp * KV);
        Frag bf;
#pragma unroll
        for (int j = 0; j < KV; ++j) {
          const int m = kc * KC + grp * KV + j;
          const int mm = min(m, 99), oh = mm / 10, ow = mm % 10;
          float x = to_f(p1s[(oh * 14 + ow) * 8 + toff]);
          if (sel != 0.f) x = (sel > 0.f && m < 100) ? 1.f : 0.f;
          M::set(bf, j, x);
        }
        M::mma(accW2[i], a, bf);
      }
    }

    // ---- conv2 dgrad: dP1[q][c] = sum_{tap,n} dY2[q - tap][n] * W2[n][c][tap]
    for (int mt = w; mt < 13; mt += 4) {
      const int q = mt * 16 + row;
      const int qy = q / 14, qx = q % 14;
      f32x4 acc = zero4();
      for (int kc = 0; kc < D2CH; ++kc) {
        int tap, n0;
        if constexpr (KV == 8) { tap = kc * 2 + (grp >> 1); n0 = (grp & 1) * 8; }
        else { tap = kc; n0 = grp * 4; }
        const int oy = qy - tap / 5, ox = qx - tap % 5;
        Frag a = M::zero();
        if (q < 196 && tap < 25 && oy >= 0 && oy < 10 && ox >= 0 && ox < 10) a = M::load(dys + (oy * 10 + ox) * 16 + n0);
        M::mma(acc, a, M::load(pack + L::C2D + row * 416 + kc * KC + grp * KV));
      }
      const int c = row;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int qq = mt * 16 + grp * 4 + i;
        if (c < 8 && qq < 196) dp1[qq * 8 + c] = c < 6 ? acc[i] : 0.f;
      }
    }
    __syncthreads();

    // ---- conv1 wgrad: dW1[n][tap] += sum_{m1} dY1[m1][n] * xpad-im2col[m1][tap]; m1 = pp*4 + e
    for (int kc = w; kc < W1CH; kc += 4) {
      Frag a;
      const int n = row;
#pragma unroll
      for (int j = 0; j < KV; ++j) {
        const int m1 = kc * KC + grp * KV + j;
        const int pp = m1 >> 2, e = m1 & 3;
        float v = 0.f;
        if (n < 6 && pp < 196) {
          const uint8_t code = m1s[pp * 8 + n];
          if ((code & 4) && (code & 3) == e) v = dp1[pp * 8 + n];
        }
        M::set(a, j, v);
      }
#pragma unroll
      for (int nt = 0; nt < 2; ++nt) {
        const int kcol = nt * 16 + row;
        const int tap = min(kcol, 24);
        const int toff = (tap / 5) * 32 + tap % 5;
        Frag bf;
#pragma unroll
        for (int j = 0; j < KV; ++j) {
          const int m1 = kc * KC + grp * KV + j;
          const int pp = min(m1 >> 2, 195), e = m1 & 3;
          const int base = (2 * (pp / 14) + (e >> 1)) * 32 + 2 * (pp % 14) + (e & 1);
          float x = to_f(xpad[base + toff]);
          if (kcol >= 25) x = (kcol == 25 && (m1 >> 2) < 196) ? 1.f : 0.f;
          M::set(bf, j, x);
        }
        M::mma(accW1[nt], a, bf);
      }
    }
    __syncthreads();
  }

  // ---- write this workgroup's partial gradients (slab row = blockIdx.x)
  float* out = cb.slab + (size_t)blockIdx.x * L::CONV_PARAMS;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int nt = w + 4 * i;
    if (nt >= 13) break;
    const int kcol = nt * 16 + row;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int n = grp * 4 + r;
      if (kcol < 200) {
        const int tap = kcol >> 3, c = kcol & 7;
        if (c < 6) out[L::CW2 + n * 150 + c * 25 + tap] = accW2[i][r];
      } else if (kcol == 200) {
        out[L::CB2 + n] = accW2[i][r];
      }
    }
  }
#pragma unroll
  for (int nt = 0; nt < 2; ++nt)
#pragma unroll
    for (int r = 0; r < 4; ++r) red[(w * 2 + nt) * 256 + (grp * 4 + r) * 16 + row] = accW1[nt][r];
  __syncthreads();
  for (int e = tid; e < 512; e += 256) {
    const int nt = e >> 8, ix = e & 255, n = ix >> 4, kcol = nt * 16 + (ix & 15);
    const float v = (red[(0 * 2 + nt) * 256 + ix] + red[(1 * 2 + nt) * 256 + ix]) +
                    (red[(2 * 2 + nt) * 256 + ix] + red[(3 * 2 + nt) * 256 + ix]);
    if (n < 6) {
      if (kcol < 25) out[L::CW1 + n * 25 + kcol] = v;
      else if (kcol == 25) out[L::CB1 + n] = v;
    }
  }
}

}  // namespace

static int fwd_ipb(int B) { return std::max(1, (B + 1023) / 1024); }
static int bwd_ipb(int B) { return std::max(1, (B + 255) / 256); }

int lenet_conv_bwd_blocks(int B) {
  const int ipb = bwd_ipb(B);
  return (B + ipb - 1) / ipb;
}

void launch_lenet_conv_fwd(DType t, bool train, const BatchRef& br, const LenetConvBuffers& cb, hipStream_t s) {
  if (br.B <= 0) return;
  const int ipb = fwd_ipb(br.B), grid = (br.B + ipb - 1) / ipb;
  if (t == DType::F32) {
    if (train) hipLaunchKernelGGL((conv_fwd_kernel<float, true>), dim3(grid), dim3(256), 0, s, br, cb, ipb);
    else hipLaunchKernelGGL((conv_fwd_kernel<float, false>), dim3(grid), dim3(256), 0, s, br, cb, ipb);
  } else {
    if (train) hipLaunchKernelGGL((conv_fwd_kernel<bf16, true>), dim3(grid), dim3(256), 0, s, br, cb, ipb);
    else hipLaunchKernelGGL((conv_fwd_kernel<bf16, false>), dim3(grid), dim3(256), 0, s, br, cb, ipb);
  }
}

void launch_lenet_conv_bwd(DType t, const BatchRef& br, const LenetConvBuffers& cb, int* nslab_out, hipStream_t s) {
  const int ipb = bwd_ipb(br.B), grid = (br.B + ipb - 1) / ipb;
  if (nslab_out) *nslab_out = grid;
  if (br.B <= 0) return;
  if (t == DType::F32) hipLaunchKernelGGL(conv_bwd_kernel<float>, dim3(grid), dim3(256), 0, s, br, cb, ipb);
  else hipLaunchKernelGGL(conv_bwd_kernel<bf16>, dim3(grid), dim3(256), 0, s, br, cb, ipb);
}
