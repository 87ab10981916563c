// Parameter-slab and packed-operand layouts of the two networks.
//
// Master weights live in ONE flat fp32 slab in torch ``state_dict`` order (so
// ``model.pt`` is written from views of it, keys/shapes of survey §0.1):
//   MLP   (reference create_model, ddp_tutorial_cpu.py:43-53):
//         0.weight[128,784] 0.bias[128] 3.weight[128,128] 3.bias[128] 5.weight[10,128]  = 118,272
//   LeNet-5 (north-star model; nn.Sequential indices 0,3,7,9,11):
//         0.weight[6,1,5,5] 0.bias[6] 3.weight[16,6,5,5] 3.bias[16] 7.weight[120,400]
//         7.bias[120] 9.weight[84,120] 9.bias[84] 11.weight[10,84] 11.bias[10]            = 61,706
// Gradients use the same layout (one flat slab = one DDP bucket space).
//
// The MFMA kernels never read the master slab for GEMM operands: the optimizer
// kernel re-packs every updated weight, in the compute dtype T, into the exact
// operand layouts the kernels consume (zero padded to MFMA tile multiples):
//   F*  [NP][KP]  forward  B operand (row n, contiguous k)
//   F*t [KP][NP]  dgrad    B operand (row k_in, contiguous n_out)
//   C1  [16][64]  conv1 B operand, k = kh*8 + kw (kw padded 5->8: one tap row = 8 contiguous k)
//   C2f [16][224] conv2 forward B operand, k = (kh*5+kw)*8 + c   (channels padded 6->8)
//   C2d [16][416] conv2 dgrad B operand, row = c, k' = (kh*5+kw)*16 + n
// so every fragment fetch is one 16-byte vector load and no kernel converts or
// transposes weights on the fly.
#pragma once
#include "common.h"

constexpr int rup(int x, int m) { return (x + m - 1) / m * m; }

// Three-layer fully connected head: K0 -> N1 (relu[,dropout]) -> N2 (relu) -> NC.
template <int K0_, int N1_, int N2_, bool BIAS3_, bool DROPOUT_, bool GATHER_, bool DX_,
          int W1_, int B1_, int W2_, int B2_, int W3_, int B3_, int PACK0_>
struct HeadDims {
  static constexpr int K0 = K0_, N1 = N1_, N2 = N2_, NC = 10;
  static constexpr int K0P = rup(K0, 32), N1P = rup(N1, 32), N2P = rup(N2, 32), NCP = 16, NCK = 32;
  static constexpr bool BIAS3 = BIAS3_, DROPOUT = DROPOUT_, GATHER = GATHER_, DX = DX_;
  // master-slab offsets (fp32 elements)
  static constexpr int W1 = W1_, B1 = B1_, W2 = W2_, B2 = B2_, W3 = W3_, B3 = B3_;
  // packed-operand offsets (T elements)
  static constexpr int F1 = PACK0_;
  static constexpr int F1T = F1 + N1P * K0P;
  static constexpr int F2 = F1T + (DX ? K0P * N1P : 0);
  static constexpr int F2T = F2 + N2P * N1P;
  static constexpr int F3 = F2T + N1P * N2P;
  static constexpr int F3T = F3 + NCP * N2P;
  // W1 (and, DX models, W1^T) also in FRAGMENT-MAJOR order for the layer-1 / dX products of the head
  // kernels (head.hip, lenet.hip): the B fragment of (n-tile t, K-chunk c) is 64 lanes x KV contiguous
  // elements, so one wave load reads whole cache lines (the row-major images touch 16 half-used lines
  // per fragment; fwd_head_kernel layer 1: 5.6 -> 3.2 us)
  //   FM1 [N1P/16][K0P/KC][64][KV]: lane (g, r) of fragment (t, c) = W1[16t + r][c*KC + g*KV .. +KV)
  //   FM1T[K0R/16][N1P/KC][64][KV]: lane (g, r) of fragment (t, c) = W1[c*KC + g*KV .. +KV)[16t + r]
  static constexpr int K0R = rup(K0, 16);
  static constexpr int FM1 = F3T + N2P * NCK;
  static constexpr int FM1T = FM1 + N1P * K0P;
  static constexpr int PACK_END = FM1T + (DX ? K0R * N1P : 0);
};

struct MlpModel {
  using Head = HeadDims<784, 128, 128, false, true, true, false,
                        0, 100352, 100480, 116864, 116992, -1, 0>;
  static constexpr int NPARAM = 118272;
  static constexpr int PACK_SIZE = Head::PACK_END;
  static constexpr int CONV_PARAMS = 0;
};

struct LenetModel {
  static constexpr int CW1 = 0, CB1 = 150, CW2 = 156, CB2 = 2556;
  static constexpr int C1 = 0;                 // [16][64]
  static constexpr int C2F = C1 + 16 * 64;     // [16][224]
  static constexpr int C2D = C2F + 16 * 224;   // [16][416]
  static constexpr int CONV_PACK_END = C2D + 16 * 416;
  using Head = HeadDims<400, 120, 84, true, false, false, true,
                        2572, 50572, 50692, 60772, 60856, 61696, CONV_PACK_END>;
  static constexpr int NPARAM = 61706;
  static constexpr int PACK_SIZE = Head::PACK_END;
  static constexpr int CONV_PARAMS = 2572;     // conv1 + conv2 params precede the head
  // activation geometry
  static constexpr int P1POS = 196, P1C = 8;   // pool1 output 14x14, channels padded 6->8
  static constexpr int P2 = 400;               // pool2 output 16x5x5, NCHW-flattened
};

// ------------------------------------------------------------------ packing
// Write the packed copies of master parameter `p` (value v).  One thread per parameter.
template <class H, typename T>
DEV void pack_head_param(int p, float v, T* pack) {
  if (p >= H::W1 && p < H::B1) {
    int q = p - H::W1, n = q / H::K0, k = q % H::K0;
    pack[H::F1 + n * H::K0P + k] = to_t<T>(v);
    constexpr int KV = Mma<T>::KV, KC = Mma<T>::KC;
    const int kk = k % KC, nn = n % KC;
    pack[H::FM1 + (((n >> 4) * (H::K0P / KC) + k / KC) * 64 + (kk / KV) * 16 + (n & 15)) * KV + kk % KV] = to_t<T>(v);
    if (H::DX) {
      pack[H::F1T + k * H::N1P + n] = to_t<T>(v);
      pack[H::FM1T + (((k >> 4) * (H::N1P / KC) + n / KC) * 64 + (nn / KV) * 16 + (k & 15)) * KV + nn % KV] = to_t<T>(v);
    }
  } else if (p >= H::W2 && p < H::B2) {
    int q = p - H::W2, n = q / H::N1, k = q % H::N1;
    pack[H::F2 + n * H::N1P + k] = to_t<T>(v);
    pack[H::F2T + k * H::N2P + n] = to_t<T>(v);
  } else if (p >= H::W3 && p < H::W3 + H::NC * H::N2) {
    int q = p - H::W3, n = q / H::N2, k = q % H::N2;
    pack[H::F3 + n * H::N2P + k] = to_t<T>(v);
    pack[H::F3T + k * H::NCK + n] = to_t<T>(v);
  }
}

template <class Model, typename T> struct Packer;

template <typename T> struct Packer<MlpModel, T> {
  static DEV void pack(int p, float v, T* pack) { pack_head_param<MlpModel::Head, T>(p, v, pack); }
};

template <typename T> struct Packer<LenetModel, T> {
  static DEV void pack(int p, float v, T* pack) {
    using L = LenetModel;
    if (p < L::CB1) {                     // conv1.weight [6][1][5][5]
      int n = p / 25, k = p % 25;
      pack[L::C1 + n * 64 + (k / 5) * 8 + k % 5] = to_t<T>(v);
    } else if (p >= L::CW2 && p < L::CB2) {  // conv2.weight [16][6][5][5]
      int q = p - L::CW2, n = q / 150, r = q % 150, c = r / 25, pos = r % 25;
      pack[L::C2F + n * 224 + pos * 8 + c] = to_t<T>(v);
      pack[L::C2D + c * 416 + pos * 16 + n] = to_t<T>(v);
    } else if (p >= L::CONV_PARAMS) {
      pack_head_param<L::Head, T>(p, v, pack);
    }
  }
};
