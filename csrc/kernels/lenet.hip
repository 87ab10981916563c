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
#include <cstdlib>
#include <algorithm>
#include <type_traits>

#include "common.h"
#include "launch.h"
#include "models.h"
#include "wgrad.h"

namespace {

using L = LenetModel;
constexpr int K0P = L::Head::K0P;  // 416
// pool1 activations / codes handed from conv_fwd to conv_bwd through HBM, channel-major with rows
// padded 14 -> 16 (CHW16), the layout conv_bwd stages into LDS with 16-byte stores; channel pitches
// padded so conv_fwd's per-lane epilogue stores hit distinct LDS banks (lane = channel fastest)
#ifndef MNIST_AMD_F32_C2SPLIT
#define MNIST_AMD_F32_C2SPLIT 1  // fp32 conv2 forward on pre-split operand images (FwdSmem::SPL)
#endif
constexpr int P1CP = 232;            // pool1 value channel pitch (elements), >= 14 * 16
constexpr int P1IMG = 6 * P1CP;      // elements per image in cb.p1
constexpr int M1CP = 240;            // pool1 code channel pitch (bytes), multiple of 16
constexpr int M1IMG = 6 * M1CP;      // bytes per image in cb.m1

// p 16-byte aligned; 16-byte stores, scalar tail; by threads tid of nth (default: the whole workgroup)
template <typename T>
DEV void zero_lds(T* p, int n, int tid = -1, int nth = 0) {
  if (tid < 0) { tid = threadIdx.x; nth = blockDim.x; }
  const int nv = n * (int)sizeof(T) / 16;
  for (int e = tid; e < nv; e += nth) reinterpret_cast<uint4*>(p)[e] = make_uint4(0, 0, 0, 0);
  for (int e = nv * 16 / (int)sizeof(T) + tid; e < n; e += nth) p[e] = to_t<T>(0.f);
}

// The sample indices of a workgroup's images, loaded ONCE at kernel start: lane l of every wave holds
// idx[first + l] and an image's index is read with v_readlane.  A per-image index load made the
// image-row loads that depend on it wait (s_waitcnt vmcnt(0)) in the middle of every image.  The
// launchers cap a workgroup at MAX_IPB = 64 images (one per lane).
constexpr int MAX_IPB = 64;
struct BlockIdx {
  int v;
  DEV BlockIdx(const int32_t* idx, int first, int count, int B) {  // idx null: unused (all zero)
    const int l = threadIdx.x & 63;
    v = (idx && l < count && first + l < B) ? idx[first + l] : 0;
  }
  DEV int operator[](int t) const { return __builtin_amdgcn_readlane(v, t); }
};

// MFMA fragment of KV ones (bias-gradient column) / zeros
template <typename T>
DEV typename Mma<T>::Frag ones_frag() {
  typename Mma<T>::Frag f;
#pragma unroll
  for (int j = 0; j < Mma<T>::KV; ++j) Mma<T>::set(f, j, 1.f);
  return f;
}

// ====================================================================================
// forward
// LDS: xs8[s][y][x] = xpad[y][x+s] for s = 0..7 (8 shifted copies of the zero-padded 32x32
// input) so that any run of KV consecutive taps of one kernel row, starting at any column, is
// an ALIGNED 16-byte read: conv1's im2col A fragment with k = kh*8 + kw is one ds_read_b128.
// (Measured alternative: ONE un-shifted copy read with under-aligned ds_read_b128 -- legal on
// gfx950 -- makes the stage 1 store/thread instead of 32, but conv_fwd goes 50 -> 120 us: the
// under-aligned 16-byte LDS reads are far slower than the extra stores.)
template <typename T>
struct FwdSmem {
  static constexpr int XP = 1048;  // plane pitch (32x32 + pad): 2-way worst-case conflicts (was 8-way at 1024)
  // shifted planes: a K-chunk run of taps starting at column x is at column x & ~(NPL-1) of plane x & (NPL-1) --
  // bf16, 4 planes: 8 taps = an 8-byte aligned pair of 8-byte reads (Mma::load8); fp32, 2 planes: 4 taps = an
  // 8-byte aligned pair of 8-byte reads.  (Was 8 planes with every read 16-byte aligned: more LDS and staging
  // stores per image.  bf16 with 2 planes -- 4-byte reads -- measured 3.8 % slower at B=1024, neutral at 8192.)
  static constexpr int NPL = sizeof(T) == 2 ? 4 : 2;
  static constexpr int OFF_XS = 0;                                        // [NPL][XP] T
  static constexpr int XTAIL = 64;  // zeroed tail: conv1's all-zero kernel row kh' = 7 reads 1 row past the last plane
  // SPL (fp32): conv2's operands as pre-split bf16 images -- pool1 as three [196][8] planes (hi, mid, lo) written
  // by conv1's epilogue, W2 as three [16][W2P] planes staged once -- read by Mma<float>::mma_pp: three 16x16x32
  // bf16 MFMAs per 16-k chunk (48 cycles) instead of four v_mfma_f32_16x16x4_f32 (128), with no cut at use
  static constexpr bool SPL = sizeof(T) == 4 && MNIST_AMD_F32_C2SPLIT;
  static constexpr int OFF_P1 = rup((NPL * XP + XTAIL) * (int)sizeof(T), 16);  // [196][8] T   pool1 output (conv2 im2col)
  static constexpr int P1_BYTES = SPL ? 3 * 196 * 8 * 2 : 196 * 8 * (int)sizeof(T);
  static constexpr int OFF_P1C = rup(OFF_P1 + P1_BYTES, 16);                  // [6][P1CP] T pool1, CHW16 (-> HBM)
  static constexpr int OFF_M1 = rup(OFF_P1C + P1IMG * (int)sizeof(T), 16);    // [6][M1CP] u8 pool1 codes, CHW16
  static constexpr int OFF_P2 = rup(OFF_M1 + M1IMG, 16);                  // [400] T      pool2 output (NCHW)
  static constexpr int OFF_M2 = rup(OFF_P2 + 400 * (int)sizeof(T), 16);   // [400] u8     pool2 codes
  static constexpr int W2P = 232;                                          // C2F row pitch (224 + 8)
  // conv2's B operand: registers for bf16 (7 chunks = 28 VGPRs), an LDS image for f32 (13 chunks)
  static constexpr bool W2LDS = sizeof(T) != 2;
  // junk words: the epilogue stores of lanes without an output (padding columns / channels) go here instead of
  // being branched around -- branch-free epilogues let the compiler count lgkmcnt exactly, so a tile's MFMAs do
  // not wait for the previous tile's epilogue stores (a store inside an exec-masked branch forced lgkmcnt(0))
  // The junk area covers every per-tile offset of the conv1 epilogue (6 tiles x 2*14*8 elements beyond a lane's
  // base) plus the 64 lanes' bases, so an invalid lane's store address is its own junk base plus the SAME
  // immediate offset a valid lane uses.
  static constexpr int JUNK_BYTES = rup((6 * 2 * 14 * 8 + 64) * (int)sizeof(T), 16);
  static constexpr int OFF_JUNK = rup(OFF_M2 + 400, 16);                   // junk stores
  static constexpr int OFF_W2 = OFF_JUNK + JUNK_BYTES;                     // [16][W2P] T  conv2 B operand
  static constexpr int W2_BYTES = SPL ? 3 * 16 * W2P * 2 : 16 * W2P * (int)sizeof(T);
  static constexpr int TOTAL = W2LDS ? rup(OFF_W2 + W2_BYTES, 16) : OFF_W2;
};

// Coalesced 16-byte copy of a staged LDS image to global memory (both 16-byte aligned).  STREAM: the
// output is read only after another kernel has run (pool1 -> conv_bwd), so it is stored non-temporally
// and is not left dirty in L2 for the kernel-end write-back; pool2 (read by the very next kernel) is not.
template <bool STREAM = false>
DEV void copy_out16(void* dst, const void* src, int bytes, int tid, int nth) {
  for (int e = tid; e < bytes / 16; e += nth) {
    const uint4 v = reinterpret_cast<const uint4*>(src)[e];
    if constexpr (STREAM) st_stream16(reinterpret_cast<uint4*>(dst) + e, v);
    else reinterpret_cast<uint4*>(dst)[e] = v;
  }
}

// The image loop of the forward pass, run by 4 waves (local thread ids 0..255) over the images
// [first, first + ipb) in the LDS region `smem` (FwdSmem layout).  conv_fwd_kernel runs one such stream
// per workgroup; fwd_head_kernel runs two (one per 4-wave half) and then the FC head on their rows.
// XROWS (fwd_head_kernel): pool2 of image t goes to row xrow0 + t of the head's LDS input tile `xrows`
// (row pitch XPITCH, zero for images past the batch) instead of global memory.
// NW = 8 (fp32 conv_fwd_kernel): the same image stream on 8 waves -- waves 4-7 take conv1's tiles 4..6 and
// conv2's M-tiles one per wave -- so the fp32 matrix pipe has 4 waves per SIMD to switch between (two
// 512-thread workgroups per CU at the same LDS footprint)
template <typename T, bool TRAIN, bool XROWS = false, int XPITCH = 0, int NW = 4>
DEV void conv_fwd_images(const BatchRef& br, const LenetConvBuffers& cb, int first, int ipb, char* smem, int tid,
                         int w, bool stamper, T* xrows) {
  static_assert(NW == 4 || NW == 8, "conv_fwd_images: 4 or 8 waves");
  constexpr int NT = NW * 64;
  const int wc = w & 3, hh = NW == 8 ? (w >> 2) : 0;  // column group of conv1's tiles, tile half (8 waves)
  using M = Mma<T>;
  using Frag = typename M::Frag;
  using S = FwdSmem<T>;
  constexpr int KV = M::KV, KC = M::KC;
  T* xs = reinterpret_cast<T*>(smem + S::OFF_XS);
  T* p1s = reinterpret_cast<T*>(smem + S::OFF_P1);
  T* p1c = reinterpret_cast<T*>(smem + S::OFF_P1C);
  uint8_t* m1s = reinterpret_cast<uint8_t*>(smem + S::OFF_M1);
  T* p2s = reinterpret_cast<T*>(smem + S::OFF_P2);
  uint8_t* m2s = reinterpret_cast<uint8_t*>(smem + S::OFF_M2);
  const int lane = tid & 63, row = lane & 15, grp = lane >> 4;
  const BlockIdx bidx(br.idx_epoch + (size_t)br.step_ptr[0] * br.batch_stride, first, ipb, br.B);
  const T* pack = reinterpret_cast<const T*>(cb.pack);
  const float* prm = cb.params;
  // optional wall-clock stamps (profiling): [0] start, [1] setup, 3 per image for images 0..3, [14] loop end
  auto stamp = [&](int k) {
    if (cb.stamps && stamper && blockIdx.x < 1024) cb.stamps[(STAMP_CONV_FWD - STAMP_CONV_BWD + blockIdx.x) * 16 + k] = wall_clock64();
  };
  stamp(0);

  // software pipeline: image t+1's pixels are in flight (registers) while image t computes
  // Stage mapping: thread (y, g, h), y = 2..29 padded row, g = 8-column group, h = plane half.
  // It fetches the dword-aligned 20-byte window [8g-4, 8g+16) of image row y-2 (pixel at padded
  // column 8g+i is window byte i+2), normalises its 16 pixels once, and writes planes 4h..4h+3 as
  // ALIGNED 16-byte stores: xs[s][y][8g..8g+7] = xpad[y][8g+s..8g+s+7].  Rows 0,1,30,31 stay zero.
  struct Raw { uint32_t d[5], lab; };
  const int sy = 2 + (tid >> 3), sg = (tid >> 1) & 3, sh = tid & 1;
  // Branch-free: every lane issues the same 5 loads, addresses clamped into the image; the words are
  // kept raw (selecting on a loaded value right after the load made the wave wait for it).  Words
  // loaded for out-of-image columns only feed pixels the stage masks (`in`), lanes >= 224 do not
  // stage, and images past the batch are masked with `valid`.
  auto fetch = [&](int t) -> Raw {  // software pipeline: image t+1's bytes are in flight during image t
    Raw r;
    const bool live = t < ipb && first + t < br.B;  // wave-uniform
#pragma unroll
    for (int k = 0; k < 5; ++k) r.d[k] = 0u;
    r.lab = 0u;
    if (NW == 4 || w < 4) {  // (8 waves: the staging threads are waves 0-3; wave-uniform)
      const uint8_t* rowp = br.images + (size_t)bidx[live ? t : 0] * 784 + min(sy - 2, 27) * 28;
#pragma unroll
      for (int k = 0; k < 5; ++k) r.d[k] = *reinterpret_cast<const uint32_t*>(rowp + min(max(8 * sg - 4 + 4 * k, 0), 24));
      if constexpr (TRAIN && !XROWS) r.lab = br.labels[bidx[live ? t : 0]];  // (batch-ordered labels, cb.yb)
    }
    return r;
  };
  Raw u_next = fetch(0);  // issued before the setup below, so its latency overlaps it

  constexpr int C1CH = 64 / KC;                 // conv1 K = 5 rows x 8 (kw padded)
  constexpr int C2CH = (25 * 8 + KC - 1) / KC;  // conv2 K = 25 taps x 8 ch (7 bf16 / 13 f32 chunks)
  // conv1's B operand lives in registers, and so does conv2's for bf16 (7 chunks; the kernel stays
  // well under 128 VGPRs, 4 waves per SIMD: the whole 1024-block grid co-resident)
  T* w2s = reinterpret_cast<T*>(smem + S::OFF_W2);  // (f32 only)
  // (SPL) the hi / mid / lo planes of pool1 and W2
  uint16_t* const p1h = reinterpret_cast<uint16_t*>(smem + S::OFF_P1);
  uint16_t* const p1m = p1h + 196 * 8;
  uint16_t* const p1l = p1m + 196 * 8;
  uint16_t* const w2h = reinterpret_cast<uint16_t*>(smem + S::OFF_W2);
  uint16_t* const w2m = w2h + 16 * S::W2P;
  uint16_t* const w2l = w2m + 16 * S::W2P;
  // conv1 B operand for TWO pooled rows per tile: column (r, c) = (row >> 3, row & 7), k = kh'*8 + kw
  // with kh' = kh + 2r in 0..7, so B[(kh', kw)][(r, c)] = W1[c][kh' - 2r][kw] (zero outside 0..4)
  // (a lane's KV k-values never straddle a kernel row, so each fragment is one 16-byte load or zero)
  Frag b1[C1CH];
  {
    const int r1 = row >> 3, c1 = row & 7;
#pragma unroll
    for (int kc = 0; kc < C1CH; ++kc) {
      const int k0 = kc * KC + grp * KV, kh = (k0 >> 3) - 2 * r1;
      b1[kc] = (c1 < 6 && kh >= 0 && kh <= 4) ? M::load(pack + L::C1 + c1 * 64 + kh * 8 + (k0 & 7)) : M::zero();
    }
  }
  Frag b2r[S::W2LDS ? 1 : C2CH];
  if constexpr (S::SPL) {
    // every thread's W2 loads issued before its first cut / LDS store (clamped, branch-free): ONE memory round
    // trip for the workgroup's W2 staging instead of one per loop trip -- at B = 128 each workgroup stages W2 for
    // a single image, so this prologue is on the step's critical path (round 5: 7.6 -> 8.4 us conv_fwd fp32)
    constexpr int NV = 16 * 224 / 4, IT = (NV + NT - 1) / NT;
    f32x4 wv[IT];
#pragma unroll
    for (int i = 0; i < IT; ++i) {
      const int e = min(tid + i * NT, NV - 1), r = e / 56, c = (e % 56) * 4;
      wv[i] = *reinterpret_cast<const f32x4*>(pack + L::C2F + r * 224 + c);
    }
#pragma unroll
    for (int i = 0; i < IT; ++i) {
      const int e = tid + i * NT, r = e / 56, c = (e % 56) * 4;
      if (e < NV) {
        u32x2 h, m, l;
        Mma<float>::split3(wv[i], h, m, l);
        *reinterpret_cast<u32x2*>(w2h + r * S::W2P + c) = h;
        *reinterpret_cast<u32x2*>(w2m + r * S::W2P + c) = m;
        *reinterpret_cast<u32x2*>(w2l + r * S::W2P + c) = l;
      }
    }
  } else if constexpr (S::W2LDS) {
    constexpr int VE = 16 / (int)sizeof(T);
    for (int e = tid; e < 16 * 224 / VE; e += NT) {
      const int r = e / (224 / VE), c = (e % (224 / VE)) * VE;
      *reinterpret_cast<uint4*>(w2s + r * S::W2P + c) = *reinterpret_cast<const uint4*>(pack + L::C2F + r * 224 + c);
    }
  } else {
#pragma unroll
    for (int kc = 0; kc < C2CH; ++kc) b2r[kc] = M::load(pack + L::C2F + row * 224 + kc * KC + grp * KV);
  }
  const float bias1 = (row & 7) < 6 ? prm[L::CB1 + (row & 7)] : 0.f;
  const float bias2 = prm[L::CB2 + row];

  // conv1 tiling: tile (t, w) = pooled rows 2t, 2t+1 (t = 0..6) x pooled columns 4w..4w+3 (grid padded
  // 14->16); M row = pooled column * 4 + window element, N = (pooled-row parity r, channel c) -- 12 of
  // 16 columns live instead of 6 -- and K = 7 kernel-row offsets x 8 taps (2 bf16 chunks, as before).
  // Since 2*4w is a multiple of 8, the shifted-copy plane and column of every fragment are lane
  // constants: A(t, kc) = c1base[kc] + 128*t.
  int c1base[C1CH];
  {
    const int q = row >> 2, e = row & 3, xt = 2 * q + (e & 1);
#pragma unroll
    for (int kc = 0; kc < C1CH; ++kc) {
      const int k0 = kc * KC + grp * KV;
      const int khp = k0 >> 3, xx = xt + (k0 & 7);
      c1base[kc] = (xx & (S::NPL - 1)) * S::XP + ((e >> 1) + khp) * 32 + 8 * wc + (xx & ~(S::NPL - 1));
    }
  }
  const bool c1valid = 4 * wc + grp < 14;  // column group 3, lane groups 2-3: padding columns 14, 15
  auto c1_load = [&](int off) {  // conv1 A fragment at an 8-byte aligned address (FwdSmem::NPL): two 8-byte reads
    if constexpr (sizeof(T) == 2) {
      return M::load8(xs + off);
    } else {
      typename M::Frag f;
      const u32x2 lo = *reinterpret_cast<const u32x2*>(xs + off), hi = *reinterpret_cast<const u32x2*>(xs + off + 2);
      f.v = __builtin_bit_cast(f32x4, u32x4{lo[0], lo[1], hi[0], hi[1]});
      return f;
    }
  };
  // Branch-free epilogues: a lane without an output (padding column / channel) stores into the junk area.  Each
  // store address is a per-lane base (real or junk, chosen ONCE) plus a per-tile immediate offset, so the 7
  // tiles' stores need 3 address registers, not 21, and no exec-masked branch breaks the lgkmcnt counting.
  char* junk = smem + S::OFF_JUNK + (int)sizeof(T) * lane;
  const int n1 = row & 7;
  const bool st1 = c1valid && n1 < 6;
  T* const e1_p1s = c1valid ? p1s + ((row >> 3) * 14 + 4 * wc + grp) * 8 + n1 : reinterpret_cast<T*>(junk);
  // (SPL: the three planes; a junk lane's three stores all go to its junk base)
  const int e1_i = ((row >> 3) * 14 + 4 * wc + grp) * 8 + n1;
  uint16_t* const e1_h = c1valid ? p1h + e1_i : reinterpret_cast<uint16_t*>(junk);
  uint16_t* const e1_m = c1valid ? p1m + e1_i : reinterpret_cast<uint16_t*>(junk);
  uint16_t* const e1_l = c1valid ? p1l + e1_i : reinterpret_cast<uint16_t*>(junk);
  T* const e1_p1c = st1 ? p1c + n1 * P1CP + (row >> 3) * 16 + 4 * wc + grp : reinterpret_cast<T*>(junk);
  uint8_t* const e1_m1s = st1 ? m1s + n1 * M1CP + (row >> 3) * 16 + 4 * wc + grp : reinterpret_cast<uint8_t*>(junk);
  auto c1_epi = [&](int t, const f32x4& acc) {  // pool + bias + ReLU, staged in LDS (pooled row 2t + r)
    float mx = acc[0];
    int am = 0;
#pragma unroll
    for (int i = 1; i < 4; ++i)
      if (acc[i] > mx) { mx = acc[i]; am = i; }
    const float pre = mx + bias1;
    // (padding channels n1 = 6, 7: zero weights and zero bias give pre = 0 exactly, so ReLU stores the 0 the
    //  conv2 im2col rows need without a select)
    const T v = to_t<T>(fmaxf(pre, 0.f));
    if constexpr (S::SPL) {
      uint16_t h, m, l;
      Mma<float>::split3_1(v, h, m, l);
      e1_h[t * 2 * 14 * 8] = h;
      e1_m[t * 2 * 14 * 8] = m;
      e1_l[t * 2 * 14 * 8] = l;
    } else {
      e1_p1s[t * 2 * 14 * 8] = v;
    }
    if (TRAIN) {
      e1_p1c[t * 2 * 16] = v;
      e1_m1s[t * 2 * 16] = (uint8_t)(am | (pre > 0.f ? 4 : 0));
    }
  };
  auto c2_base = [&](int mt) {  // im2col row of tile mt for this lane: pooled position x window element
    const int q = row >> 2, e = row & 3;
    const int p = min(mt * 4 + q, 24), py = p / 5, px = p % 5;
    return ((2 * py + (e >> 1)) * 14 + 2 * px + (e & 1)) * 8;
  };
  auto c2_a = [&](int base, int kc) {  // A fragment of K-chunk kc (8 taps x 8 channels ... per lane group)
    int pos, c0;
    if constexpr (KV == 8) { pos = kc * 4 + grp; c0 = 0; }
    else { pos = kc * 2 + (grp >> 1); c0 = (grp & 1) * 4; }
    pos = min(pos, 24);
    const int kh = pos / 5, kw = pos % 5;
    return M::load(p1s + base + (kh * 14 + kw) * 8 + c0);
  };
  // NT tiles (1 or 2) sharing the B fragments, next chunk's A fragments in flight during this chunk's
  // MFMAs (the rolled-up form waited for every A read before its MFMA).  (Measured: reading every A fragment
  // of the tiles first -- 14 reads in flight, 56 VGPRs -- pushed the fused kernel past 128 VGPRs into
  // scratch spills inside the image loop.)
  struct SplitA { u32x2 h, m, l; };
  auto c2_as = [&](int base, int kc) {  // (SPL) the A fragment's three parts: 4 channels of one tap per lane
    const int pos = min(kc * 2 + (grp >> 1), 24), c0 = (grp & 1) * 4;
    const int i = base + ((pos / 5) * 14 + pos % 5) * 8 + c0;
    return SplitA{*reinterpret_cast<const u32x2*>(p1h + i), *reinterpret_cast<const u32x2*>(p1m + i),
                  *reinterpret_cast<const u32x2*>(p1l + i)};
  };
  auto c2_acc = [&](auto ntc, const int* mts, f32x4* acc) {
    constexpr int NT = decltype(ntc)::value;
    if constexpr (S::SPL) {
      int base[NT];
      SplitA a[NT];
#pragma unroll
      for (int j = 0; j < NT; ++j) {
        base[j] = c2_base(mts[j]);
        a[j] = c2_as(base[j], 0);
      }
      const int bo = row * S::W2P + grp * KV;
#pragma unroll 1  // (fully unrolled, the training kernel spilled 26 VGPRs at its 128-register bound)
      for (int kc = 0; kc < C2CH; ++kc) {
        SplitA an[NT];
#pragma unroll
        for (int j = 0; j < NT; ++j) an[j] = kc + 1 < C2CH ? c2_as(base[j], kc + 1) : a[j];
        const int bi = bo + kc * KC;
        const u32x2 bh = *reinterpret_cast<const u32x2*>(w2h + bi), bm = *reinterpret_cast<const u32x2*>(w2m + bi),
                    bl = *reinterpret_cast<const u32x2*>(w2l + bi);
#pragma unroll
        for (int j = 0; j < NT; ++j) Mma<float>::mma_pp(acc[j], a[j].h, a[j].m, a[j].l, bh, bm, bl);
#pragma unroll
        for (int j = 0; j < NT; ++j) a[j] = an[j];
      }
      return;
    }
    int base[NT];
    Frag a[NT];
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      base[j] = c2_base(mts[j]);
      a[j] = c2_a(base[j], 0);
    }
#pragma unroll
    for (int kc = 0; kc < C2CH; ++kc) {
      Frag an[NT];
#pragma unroll
      for (int j = 0; j < NT; ++j) an[j] = kc + 1 < C2CH ? c2_a(base[j], kc + 1) : a[j];
      Frag b;
      if constexpr (S::W2LDS) b = M::load(w2s + row * S::W2P + kc * KC + grp * KV);
      else b = b2r[kc];
#pragma unroll
      for (int j = 0; j < NT; ++j) M::mma(acc[j], a[j], b);
#pragma unroll
      for (int j = 0; j < NT; ++j) a[j] = an[j];
    }
  };
  auto c2_epi = [&](int t, bool valid, int mt, const f32x4& acc) {  // branch-free: pp >= 25 stores to junk
    const int n = row, pp = min(mt * 4 + grp, 24);
    const bool live = mt * 4 + grp < 25;
    float mx = acc[0];
    int am = 0;
#pragma unroll
    for (int i = 1; i < 4; ++i)
      if (acc[i] > mx) { mx = acc[i]; am = i; }
    const float pre = mx + bias2;
    if constexpr (XROWS) *(live ? xrows + t * XPITCH + n * 25 + pp : reinterpret_cast<T*>(junk)) = to_t<T>(valid ? fmaxf(pre, 0.f) : 0.f);
    else *(live ? p2s + n * 25 + pp : reinterpret_cast<T*>(junk)) = to_t<T>(fmaxf(pre, 0.f));
    *(live ? m2s + n * 25 + pp : reinterpret_cast<uint8_t*>(junk)) = (uint8_t)(am | (pre > 0.f ? 4 : 0));
  };
  auto flush_p2 = [&](int bprev) {  // previous image's pool2 outputs -> HBM (16-byte stores)
    if (bprev >= 0 && bprev < br.B) {
      if constexpr (!XROWS) copy_out16(reinterpret_cast<T*>(cb.p2) + (size_t)bprev * K0P, p2s, 400 * (int)sizeof(T), tid, NT);
      if (TRAIN) copy_out16(cb.m2 + (size_t)bprev * 400, m2s, 400, tid, NT);
    }
  };

  // bf16 staging: the lane's window (image columns 8 sg - 2 + i, i < 12) leaves the image only as whole pixel pairs --
  // pair 0 when sg = 0 (columns -2, -1), pairs 3..5 when sg = 3 (columns 28..33): two loop-invariant masks
  const uint32_t keep_sg0 = sg == 0 ? 0u : 0xFFFFFFFFu, keep_sg3 = sg == 3 ? 0u : 0xFFFFFFFFu;
  zero_lds<T>(xs, S::NPL * S::XP + S::XTAIL, tid, NT);
  if (TRAIN) {
    zero_lds<T>(p1c, P1IMG, tid, NT);
    zero_lds<uint8_t>(m1s, M1IMG, tid, NT);
  }
  // b1 / b2r / biases are loop-invariant registers loaded from global memory above (image 0's pixels
  // are also in flight and consumed right after this barrier anyway)
  wait_vm_all();
  __syncthreads();
  stamp(1);
  for (int t = 0; t < ipb; ++t) {
    const int b = first + t;
    const bool valid = b < br.B;
    const Raw u = u_next;
    // this image's pixel rows in batch order for conv_bwd (cb.xb): columns 8sg .. 8sg+7 of row sy - 2 are the
    // window's words 1 and 2 (word 2 of sg = 3 is a clamped duplicate)
    if (TRAIN && !XROWS && cb.xb && valid && tid < 224 && sh == 0) {
      uint8_t* d = cb.xb + (size_t)b * 784 + (sy - 2) * 28 + 8 * sg;
      *reinterpret_cast<uint32_t*>(d) = u.d[1];
      if (sg < 3) *reinterpret_cast<uint32_t*>(d + 4) = u.d[2];
      if (tid == 0) cb.yb[b] = (uint8_t)u.lab;
    }
    // ---- stage: normalise once, 4 aligned 16-byte plane stores per thread
    if (tid < 224 && !ABLATED(cb.ablate, 1)) {
      auto pixel = [&](int i) { return mnist_norm((u.d[(i + 2) >> 2] >> (8 * ((i + 2) & 3))) & 255u); };
      T* dst = xs + sy * 32 + 8 * sg;
      if constexpr (sizeof(T) == 2) {
        // packed pairs D[k] = (v[2k], v[2k+1]), each ONE v_cvt_pk_bf16_f32, the zero padding (0 AFTER normalising)
        // applied to the pair by the lane's loop-invariant mask and the image's `valid`; E = window for this
        // thread's plane half (sh); even planes are dword-aligned slices of E, odd planes one alignbyte per dword
        typedef __attribute__((ext_vector_type(2))) float f32x2;
        const uint32_t vm = valid ? 0xFFFFFFFFu : 0u;
        const uint32_t m0 = keep_sg0 & vm, m3 = keep_sg3 & vm;
        uint32_t D[6], E[6];
#pragma unroll
        for (int k = 0; k < 6; ++k)
          D[k] = __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2{pixel(2 * k), pixel(2 * k + 1)}), bf16x2)) &
                 (k == 0 ? m0 : (k >= 3 ? m3 : vm));
        const uint32_t msk = 0u - (uint32_t)sh;  // bit blend: a ?: select here becomes scratch-indexed D
        // 4 planes: this thread writes planes 2 sh, 2 sh + 1 (window E = D shifted by sh dwords = 2 sh taps)
#pragma unroll
        for (int j = 0; j < 5; ++j) E[j] = (D[j] & ~msk) | (D[j + 1] & msk);
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          uint4 o;
          uint32_t* ov = reinterpret_cast<uint32_t*>(&o);
#pragma unroll
          for (int j = 0; j < 4; ++j) ov[j] = q == 0 ? E[j] : __builtin_amdgcn_alignbyte(E[j + 1], E[j], 2);
          *reinterpret_cast<uint4*>(dst + (2 * sh + q) * S::XP) = o;
        }
      } else {
        float f[16];
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const bool in = valid && (unsigned)(8 * sg - 2 + i) < 28u;  // zero padding is 0 AFTER normalising
          f[i] = in ? pixel(i) : 0.f;
        }
        // bit blend instead of `sh ? f[i + 1] : f[i]`: hipcc turned that select into a lane-indexed
        // load of f[] from scratch memory (80 B/lane of scratch traffic per image); plane sh
        const uint32_t msk = 0u - (uint32_t)sh;
        {
          constexpr int q = 0;
          float o[8];
#pragma unroll
          for (int i = 0; i < 8; ++i)
            o[i] = __builtin_bit_cast(float, (__builtin_bit_cast(uint32_t, f[i + q]) & ~msk) |
                                                 (__builtin_bit_cast(uint32_t, f[i + 1 + q]) & msk));
          float* d = reinterpret_cast<float*>(dst) + sh * S::XP;
          *reinterpret_cast<f32x4*>(d) = f32x4{o[0], o[1], o[2], o[3]};
          *reinterpret_cast<f32x4*>(d + 4) = f32x4{o[4], o[5], o[6], o[7]};
        }
      }
    }
    __syncthreads();
    if (t < 4) stamp(2 + 3 * t);
    // next image's pixels (and the previous image's pool2 flush) are issued here, a whole conv1 +
    // conv2 before their consumer, with no global operation in between
    u_next = fetch(t + 1);
    flush_p2(t > 0 ? b - 1 : -1);

    // ---- conv1 + bias + ReLU + maxpool: 7 two-row tiles per wave
    if (!ABLATED(cb.ablate, 2)) {
      // software pipeline: tile t+1's fragments are loaded and tile t's MFMAs issued BEFORE tile
      // t-1's epilogue (the compiler cannot hoist xs loads over the epilogue's p1s stores itself)
      // Tile t+1 starts 4 input rows below tile t and K spans 8 rows, so its first half of K chunks
      // (rows kh' = 0..3) IS tile t's second half (kh' = 4..7): c1base[kc + C1CH/2] = c1base[kc] + 128.
      // Only the second half is read per tile (8 instead of 14 A reads per wave and image, bf16).
      constexpr int HC = C1CH / 2;
      // tiles [T0, T1) of this wave's column group (4 waves: all 7; 8 waves: 0..3 / 4..6 by tile half)
      auto conv1_tiles = [&](auto t0c, auto t1c) {
        constexpr int T0 = decltype(t0c)::value, T1 = decltype(t1c)::value;
        Frag fa[C1CH];
#pragma unroll
        for (int kc = 0; kc < C1CH; ++kc) fa[kc] = c1_load(c1base[kc] + T0 * 128);
        f32x4 prev = zero4();
#pragma unroll
        for (int t = T0; t < T1; ++t) {
          f32x4 acc = zero4();
#pragma unroll
          for (int kc = 0; kc < C1CH; ++kc) {
            // fp32: conv1's products as exact 3-part bf16 splits on 16x16x32 MFMAs (Mma<float>::mma_s; the cut of the
            // loop-invariant weights hoisted): 3 x 16 instead of 4 x 32 MFMA cycles per chunk on the convolution
            // whose K is 61 % padding (LeNet fp32 B=8192 0.4028 -> 0.3830 ms, profiles/r5_session1/f32conv1/).
            // conv2: both operands pre-split in LDS (FwdSmem::SPL; B alone pre-split was neutral); conv_bwd's streamed
            // operands slower.
            if constexpr (sizeof(T) == 4) Mma<float>::mma_s(acc, fa[kc], b1[kc]);
            else M::mma(acc, fa[kc], b1[kc]);
          }
          if (t + 1 < T1) {
#pragma unroll
            for (int kc = 0; kc < HC; ++kc) fa[kc] = fa[kc + HC];
#pragma unroll
            for (int kc = HC; kc < C1CH; ++kc) fa[kc] = c1_load(c1base[kc] + (t + 1) * 128);
          }
          if (t > T0) c1_epi(t - 1, prev);
          prev = acc;
        }
        c1_epi(T1 - 1, prev);
      };
      if constexpr (NW == 4) {
        conv1_tiles(std::integral_constant<int, 0>{}, std::integral_constant<int, 7>{});
      } else if (hh == 0) {  // (wave-uniform)
        conv1_tiles(std::integral_constant<int, 0>{}, std::integral_constant<int, 4>{});
      } else {
        conv1_tiles(std::integral_constant<int, 4>{}, std::integral_constant<int, 7>{});
      }
    }
    __syncthreads();
    if (t < 4) stamp(3 + 3 * t);

    // ---- pool1 -> HBM for the backward pass (16-byte stores), overlapped with conv2
    if (TRAIN && valid && !ABLATED(cb.ablate, 1024)) {
      copy_out16<true>(reinterpret_cast<T*>(cb.p1) + (size_t)b * P1IMG, p1c, P1IMG * (int)sizeof(T), tid, NT);
      copy_out16<true>(cb.m1 + (size_t)b * M1IMG, m1s, M1IMG, tid, NT);
    }
    // ---- conv2 + bias + ReLU + maxpool: 100 rows (25 pooled x 4) = 7 M-tiles, N = 16
    if (!ABLATED(cb.ablate, 4)) {
      if constexpr (NW == 8) {  // one M-tile per wave (wave 7: none)
        if (w < 7) {
          const int mts[1] = {w};
          f32x4 acc[1] = {zero4()};
          c2_acc(std::integral_constant<int, 1>{}, mts, acc);
          c2_epi(t, valid, w, acc[0]);
        }
      } else if (w < 3) {  // waves 0-2: tiles (2w, 2w+1) as a pair; wave 3: tile 6
        const int mts[2] = {2 * w, 2 * w + 1};
        f32x4 acc[2] = {zero4(), zero4()};
        c2_acc(std::integral_constant<int, 2>{}, mts, acc);
        c2_epi(t, valid, 2 * w, acc[0]);
        c2_epi(t, valid, 2 * w + 1, acc[1]);
      } else {
        const int mts[1] = {6};
        f32x4 acc[1] = {zero4()};
        c2_acc(std::integral_constant<int, 1>{}, mts, acc);
        c2_epi(t, valid, 6, acc[0]);
      }
    }
    __syncthreads();
    if (t < 4) stamp(4 + 3 * t);
  }
  stamp(14);
  if (cb.stamps && stamper && blockIdx.x < 1024) cb.stamps[(STAMP_CONV_FWD - STAMP_CONV_BWD + blockIdx.x) * 16 + 15] = hw_location();
  flush_p2(first + ipb - 1);
}

template <typename T, bool TRAIN, int NW = 4>
// (f32, 4 waves: its ~64 KB of LDS allows 2 workgroups per CU anyway, so it may use up to 256 VGPRs instead of
//  spilling; 8 waves: 2 x 8 waves per CU, 128 VGPRs)
__global__ __launch_bounds__(NW * 64) __attribute__((amdgpu_waves_per_eu(sizeof(T) == 2 || NW == 8 ? 4 : 2))) void conv_fwd_kernel(BatchRef br, LenetConvBuffers cb, int ipb) {
  __shared__ __attribute__((aligned(16))) char smem[FwdSmem<T>::TOTAL];
  const int unit = xcd_unit(blockIdx.x, gridDim.x, br.xcd);  // this workgroup's images: [unit * ipb, +ipb)
  conv_fwd_images<T, TRAIN, false, 0, NW>(br, cb, unit * ipb, ipb, smem, threadIdx.x, wave_id(), threadIdx.x == 0, nullptr);
}

// ====================================================================================
// forward + FC head in ONE kernel (LeNet-5 training, large batches)
// A 512-thread workgroup owns 16 consecutive batch rows = one 16-row MFMA tile of the head.  Its two
// 4-wave halves each run the conv_fwd image loop over 8 of the rows (the same per-image code and LDS
// layout as conv_fwd_kernel, so per CU the conv work keeps 16 waves in flight), writing pool2 straight
// into the head's LDS input tile.  The 8 waves then run the whole head on the tile:
//   L1 (wave w: n-tile w) -> L2 -> L3 -> softmax-CE + metrics -> dH2 -> dH1 -> dX (= pool2 grads)
// B operands come straight from the L2-resident packed weights into registers, each phase's fragments
// issued one or more phases ahead (a 16-row tile reads every weight fragment exactly once, so an LDS copy
// would buy nothing).  This removes the head kernel, its kernel boundary, the pool2 HBM round trip and
// the head's per-workgroup weight staging (replaces head_kernel's LeNet path at B >= FH_MIN_B; the FC
// wgrad reads the same transposed activations / gradients the head wrote).
// Reference: the forward/loss/backward of ddp_tutorial_multi_gpu.py:72-79 for the LeNet-5 model.
constexpr int FH_MIN_B = 4096;
// LDS of the 16-row register-B head (head16_tile): the input tile X, and the small per-phase tiles
template <typename T>
struct Head16Smem {
  using H = LenetModel::Head;
  static constexpr int PX = H::K0P + 8, P1 = H::N1P + 8, P2 = H::N2P + 8, PD = H::NCK + 8;
  static constexpr int X_BYTES = rup(16 * PX * (int)sizeof(T), 16);           // [16][PX] T input tile
  static constexpr int OFF_H1 = 0;                                               // [16][P1] T
  static constexpr int OFF_H2 = rup(OFF_H1 + 16 * P1 * (int)sizeof(T), 16);      // [16][P2] T
  static constexpr int OFF_D = rup(OFF_H2 + 16 * P2 * (int)sizeof(T), 16);       // [16][PD] T  dZ
  static constexpr int OFF_L = rup(OFF_D + 16 * PD * (int)sizeof(T), 16);        // [16][16] f32 logits
  static constexpr int OFF_LAB = OFF_L + 16 * 16 * 4;                            // [16] int
  static constexpr int OFF_PART = OFF_LAB + 16 * 4;                              // [8][4] f32
  static constexpr int OFF_DX = rup(OFF_PART + 8 * 4 * 4, 16);                   // [16][PX] T dX tile
  static constexpr int HEAD_END = rup(OFF_DX + 16 * PX * (int)sizeof(T), 16);
};
template <typename T>
struct FwdHeadSmem : Head16Smem<T> {
  static constexpr int HALF = FwdSmem<T>::TOTAL;  // one conv image stream
  static constexpr int OFF_X = 2 * HALF;           // head input tile (pool2 rows)
  static constexpr int TOTAL = OFF_X + Head16Smem<T>::X_BYTES;
  // after the image loops the two conv regions are dead: the head's small tiles live there
  static_assert(Head16Smem<T>::HEAD_END <= 2 * HALF, "head tiles must fit in the dead conv regions");
};

template <typename T>
DEV void head16_tile(const BatchRef& br, const HeadBuffers& hb, char* ht, T* sX, int r0, int tile);

template <typename T>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(4))) void fwd_head_kernel(BatchRef br, LenetConvBuffers cb,
                                                                                           HeadBuffers hb) {
  using H = LenetModel::Head;
  using S = FwdHeadSmem<T>;
  using M = Mma<T>;
  using Frag = typename M::Frag;
  constexpr int KV = M::KV, KC = M::KC;
  static_assert(sizeof(T) == 2, "fwd_head_kernel: bf16 operand layout");
  __shared__ __attribute__((aligned(16))) char smem[S::TOTAL];
  T* sX = reinterpret_cast<T*>(smem + S::OFF_X);
  const int tid = threadIdx.x, lane = tid & 63, w = wave_id(), row = lane & 15, grp = lane >> 4;
  const int half = w >> 2;  // wave-uniform (an SGPR: the image stream's addresses stay scalar)
  const int r0 = xcd_unit(blockIdx.x, gridDim.x, br.xcd) * 16;  // this workgroup's batch rows [r0, r0 + 16)
  const int B = br.B;
  // the head tile's padding columns (400..415) must be zero: cleared once, before the loop's first barrier
  for (int e = tid; e < 16 * S::PX * (int)sizeof(T) / 16; e += 512) reinterpret_cast<uint4*>(sX)[e] = make_uint4(0, 0, 0, 0);
  conv_fwd_images<T, true, true, S::PX>(br, cb, r0 + 8 * half, 8, smem + half * S::HALF, tid & 255, w & 3, tid == 0,
                                        sX + 8 * half * S::PX);
  head16_tile<T>(br, hb, smem, sX, r0, blockIdx.x);  // its first barrier: every pool2 row is in sX, the conv regions dead
}

// The 16-row register-B head (fwd_head_kernel after its conv loops; head16_kernel): 8 waves, X in sX
// (rows past the batch zero), the small per-phase tiles at `ht` (Head16Smem offsets).  The caller does NOT
// barrier after writing sX: the first weight fragments are issued, THEN the block barrier (their latency
// overlaps the wait for the slowest wave), and only then is LDS at `ht` written (it may alias the caller's
// dead buffers).
// `tile` = this head tile's index (its metrics row and stamp slots)
template <typename T>
DEV void head16_tile(const BatchRef& br, const HeadBuffers& hb, char* ht, T* sX, int r0, int tile) {
  using H = LenetModel::Head;
  using S = Head16Smem<T>;
  using M = Mma<T>;
  using Frag = typename M::Frag;
  constexpr int KV = M::KV, KC = M::KC;
  static_assert(sizeof(T) == 2, "head16_tile: bf16 operand layout");
  const int tid = threadIdx.x, lane = tid & 63, w = wave_id(), row = lane & 15, grp = lane >> 4;
  const int B = br.B;
  // optional head-phase stamps (profiling; the head's own row range): [0] X ready, [9] X^T stored,
  // [1] L1, [2] L2, [3] L3, [4] softmax, [5] dH2, [6] dH1, [7] dX, [8] end
  auto hstamp = [&](int k) {
    if (hb.stamps && tid == 0 && tile < 1024) hb.stamps[tile * 16 + k] = wall_clock64();
  };

  T* sH1 = reinterpret_cast<T*>(ht + S::OFF_H1);
  T* sH2 = reinterpret_cast<T*>(ht + S::OFF_H2);
  T* sD = reinterpret_cast<T*>(ht + S::OFF_D);
  T* sDX = reinterpret_cast<T*>(ht + S::OFF_DX);
  float* sLog = reinterpret_cast<float*>(ht + S::OFF_L);
  int* sLab = reinterpret_cast<int*>(ht + S::OFF_LAB);
  float* sPart = reinterpret_cast<float*>(ht + S::OFF_PART);
  const T* pack = reinterpret_cast<const T*>(hb.pack);
  const float* prm = hb.params;
  const int ldB = hb.ldB;
  constexpr int KCH1 = H::K0P / KC, KCH2 = H::N1P / KC, KCH3 = H::N2P / KC, KCHX = H::N1P / KC;
  constexpr int NT2 = H::N2P / 16, NTX = H::K0 / 16, XJ = (NTX + 7) / 8;  // dX: tiles w + 8j
  static_assert(H::N1P / 16 == 8, "one layer-1 n-tile per wave");

  // ---- the B fragments of L1, L2 and dH2 for this wave, issued now (L1's first: in-order
  //      vmcnt lets L1 start while the rest is in flight); biases and labels with them
  Frag b1[KCH1], b2[KCH2], b3[KCH3], bd2, bd1[KCH3];
  {  // fragment-major W1 (models.h FM1): each fragment is one contiguous 1 KB (bf16) wave load
    const T* p = pack + H::FM1 + (w * KCH1 * 64 + lane) * KV;
#pragma unroll
    for (int kc = 0; kc < KCH1; ++kc) b1[kc] = M::load(p + kc * 64 * KV);
  }
  const int w2 = min(w, NT2 - 1);  // waves 6, 7 have no L2 / dH2 tile: they load (and ignore) tile 5
  {
    const T* p = pack + H::F2 + (w2 * 16 + row) * H::N1P + grp * KV;
#pragma unroll
    for (int kc = 0; kc < KCH2; ++kc) b2[kc] = M::load(p + kc * KC);
  }
  bd2 = M::load(pack + H::F3T + (w2 * 16 + row) * H::NCK + grp * KV);
  const int n1 = w * 16 + row, n2 = w2 * 16 + row;
  const float bias1 = prm[H::B1 + min(n1, H::N1 - 1)], bias2 = prm[H::B2 + min(n2, H::N2 - 1)];
  const float bias3 = prm[H::B3 + min(row, H::NC - 1)];
  int lab = 0;
  if (tid >= 512 - 16) {  // labels of the tile (the last wave: its L2 tile is a dummy)
    const int t = tid - (512 - 16), rg = r0 + t;
    if (hb.yb) {  // batch-ordered labels from conv_fwd_kernel (small batches): no index chain
      lab = rg < B ? (int)hb.yb[rg] : 0;
    } else {
      const int id = rg < B ? br.idx_epoch[(size_t)br.step_ptr[0] * br.batch_stride + rg] : -1;
      lab = id >= 0 ? (int)br.labels[id] : 0;
    }
  }
  // sX complete (caller), `ht` free: a raw barrier after the LDS writes drained -- __syncthreads() would also
  // wait (vmcnt(0)) for the weight fragments just issued
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  hstamp(0);
  if (tid >= 512 - 16) sLab[tid - (512 - 16)] = lab;

  // ---- X^T for the wgrad GEMM (only the wgrad kernel reads it: stored by waves 4-7 while waves 0-3 run
  //      the softmax): item = (8-column chunk, 4-row quad), 4 rows read as 16-byte LDS chunks and written
  //      as 4-row (8-byte) column stores
  auto store_xT = [&](int t0, int nth) {
    T* xT = reinterpret_cast<T*>(hb.xT);
    constexpr int NCH = H::K0P / 8;
    for (int e = tid - t0; e < NCH * 4; e += nth) {
      const int c = e >> 2, rq = (e & 3) * 4;
      u32x4 v[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) v[q] = *reinterpret_cast<const u32x4*>(sX + (rq + q) * S::PX + c * 8);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int wd = j >> 1;
        const uint32_t lo = pack_half16(v[0][wd], v[1][wd], j & 1);  // one v_perm_b32 each
        const uint32_t hi = pack_half16(v[2][wd], v[3][wd], j & 1);
        *reinterpret_cast<u32x2*>(xT + (size_t)(c * 8 + j) * ldB + r0 + rq) = u32x2{lo, hi};
      }
    }
  };
  hstamp(9);
  auto store4 = [&](T* base, const float* v) {  // 4 consecutive rows of one column of a [col][ldB] buffer
    bf16x4 q;
#pragma unroll
    for (int i = 0; i < 4; ++i) q[i] = (bf16)v[i];
    *reinterpret_cast<bf16x4*>(base) = q;
  };

  // ---------------------------------------------------------------- L1: H1 = relu(X W1^T + b1)
  {
    f32x4 acc = zero4();
    const T* ap = sX + row * S::PX + grp * KV;
#pragma unroll
    for (int kc = 0; kc < KCH1; ++kc) M::mma(acc, M::load(ap + kc * KC), b1[kc]);
    float v[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int r = grp * 4 + i;
      float x = fmaxf(acc[i] + bias1, 0.f);
      if (n1 >= H::N1 || r0 + r >= B) x = 0.f;
      sH1[r * S::P1 + n1] = to_t<T>(x);
      v[i] = to_f(to_t<T>(x));
    }
    store4(reinterpret_cast<T*>(hb.h1T) + (size_t)n1 * ldB + r0 + grp * 4, v);
  }
  {  // L3's fragments (used by wave 7 only) and the dX fragments (W1^T, the largest operand): issued now
     // that L1's registers are free; they arrive during L2 .. dH1
    const T* p = pack + H::F3 + row * H::N2P + grp * KV;
#pragma unroll
    for (int kc = 0; kc < KCH3; ++kc) b3[kc] = M::load(p + kc * KC);
  }
  Frag bx[XJ][KCHX];
#pragma unroll
  for (int j = 0; j < XJ; ++j) {
    const int nt = min(w + 8 * j, NTX - 1);
    const T* p = pack + H::FM1T + (nt * KCHX * 64 + lane) * KV;  // fragment-major W1^T (models.h FM1T)
#pragma unroll
    for (int kc = 0; kc < KCHX; ++kc) bx[j][kc] = M::load(p + kc * 64 * KV);
  }
  __syncthreads();
  hstamp(1);

  // ---------------------------------------------------------------- L2: H2 = relu(H1 W2^T + b2)
  if (w < NT2) {
    f32x4 acc = zero4();
    const T* ap = sH1 + row * S::P1 + grp * KV;
#pragma unroll
    for (int kc = 0; kc < KCH2; ++kc) M::mma(acc, M::load(ap + kc * KC), b2[kc]);
    float v[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int r = grp * 4 + i;
      float x = fmaxf(acc[i] + bias2, 0.f);
      if (n2 >= H::N2 || r0 + r >= B) x = 0.f;
      sH2[r * S::P2 + n2] = to_t<T>(x);
      v[i] = to_f(to_t<T>(x));
    }
    store4(reinterpret_cast<T*>(hb.h2T) + (size_t)n2 * ldB + r0 + grp * 4, v);
  }
  __syncthreads();
  hstamp(2);

  // ---------------------------------------------------------------- L3: logits = H2 W3^T + b3
  if (w == 7) {
    f32x4 acc = zero4();
    const T* ap = sH2 + row * S::P2 + grp * KV;
#pragma unroll
    for (int kc = 0; kc < KCH3; ++kc) M::mma(acc, M::load(ap + kc * KC), b3[kc]);
#pragma unroll
    for (int i = 0; i < 4; ++i) sLog[(grp * 4 + i) * 16 + row] = acc[i] + bias3;
  }
  __syncthreads();
  hstamp(3);

  // ---------------------------------------------------------------- softmax cross-entropy (waves 0-3)
  {  // dH1's fragments (two phases ahead; issued here to keep L1..L3 under the register budget)
    const T* p = pack + H::F2T + (w * 16 + row) * H::N2P + grp * KV;
#pragma unroll
    for (int kc = 0; kc < KCH3; ++kc) bd1[kc] = M::load(p + kc * KC);
  }
  if (tid < 256) {
    const int r = tid >> 4, c = tid & 15, rg = r0 + r;
    const bool valid = rg < B;
    const float z = c < H::NC ? sLog[r * 16 + c] : -INFINITY;
    const float mx = row16_max(z);
    const int am = row16_min(z == mx ? c : 16);
    const float e = c < H::NC ? __expf(z - mx) : 0.f;
    const float se = row16_sum(e);
    const int y = sLab[r];
    const float zy = sLog[r * 16 + y];
    float loss = 0.f, corr = 0.f, cnt = 0.f;
    if (c == 0 && valid) {
      loss = mx + __logf(se) - zy;
      corr = (am == y) ? 1.f : 0.f;
      cnt = 1.f;
    }
    const float d = (valid && c < H::NC) ? e / se - (c == y ? 1.f : 0.f) : 0.f;
    sD[r * S::PD + c] = to_t<T>(d);
    sD[r * S::PD + 16 + c] = to_t<T>(0.f);  // K padding of the dH2 product (NCK = 32)
    auto rows4 = [](float v) { return (lane_f(v, 0) + lane_f(v, 16)) + (lane_f(v, 32) + lane_f(v, 48)); };
    loss = rows4(loss);
    corr = rows4(corr);
    cnt = rows4(cnt);
    if (lane == 0) {
      sPart[w * 4 + 0] = loss;
      sPart[w * 4 + 1] = corr;
      sPart[w * 4 + 2] = cnt;
    }
  } else {
    store_xT(256, 256);
  }
  __syncthreads();
  hstamp(4);

  // ---------------------------------------------------------------- dH2 = (dZ W3) * [H2 > 0]
  if (w < NT2) {
    f32x4 acc = zero4();
    M::mma(acc, M::load(sD + row * S::PD + grp * KV), bd2);
    float v[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      T* h = &sH2[(grp * 4 + i) * S::P2 + n2];
      const float x = to_f(*h) > 0.f ? acc[i] : 0.f;
      *h = to_t<T>(x);  // in place: H2 becomes dH2
      v[i] = to_f(to_t<T>(x));
    }
    store4(reinterpret_cast<T*>(hb.dy2T) + (size_t)n2 * ldB + r0 + grp * 4, v);
  } else {  // waves 6, 7: dZ^T for the wgrad GEMM
    T* dy3T = reinterpret_cast<T*>(hb.dy3T);
    const int e = tid - NT2 * 64, c = e >> 3, rq = (e & 7) * 2;  // 128 threads: (class, row pair)
    dy3T[(size_t)c * ldB + r0 + rq] = sD[rq * S::PD + c];
    dy3T[(size_t)c * ldB + r0 + rq + 1] = sD[(rq + 1) * S::PD + c];
  }
  __syncthreads();
  hstamp(5);

  // ---------------------------------------------------------------- dH1 = (dH2 W2) * [H1 > 0]
  {
    f32x4 acc = zero4();
    const T* ap = sH2 + row * S::P2 + grp * KV;
#pragma unroll
    for (int kc = 0; kc < KCH3; ++kc) M::mma(acc, M::load(ap + kc * KC), bd1[kc]);
    float v[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      T* h = &sH1[(grp * 4 + i) * S::P1 + n1];
      const float x = to_f(*h) > 0.f ? acc[i] : 0.f;
      *h = to_t<T>(x);  // in place: H1 becomes dH1
      v[i] = to_f(to_t<T>(x));
    }
    store4(reinterpret_cast<T*>(hb.dy1T) + (size_t)n1 * ldB + r0 + grp * 4, v);
  }
  __syncthreads();
  hstamp(6);

  // ---------------------------------------------------------------- dX = dH1 W1 -> pool2 grads
  {
    const T* ap = sH1 + row * S::P1 + grp * KV;
    Frag a[KCHX];
#pragma unroll
    for (int kc = 0; kc < KCHX; ++kc) a[kc] = M::load(ap + kc * KC);
#pragma unroll
    for (int j = 0; j < XJ; ++j) {
      const int nt = w + 8 * j;
      if (nt >= NTX) break;
      f32x4 acc = zero4();
#pragma unroll
      for (int kc = 0; kc < KCHX; ++kc) M::mma(acc, a[kc], bx[j][kc]);
#pragma unroll
      for (int i = 0; i < 4; ++i) sDX[(grp * 4 + i) * S::PX + nt * 16 + row] = to_t<T>(acc[i]);
    }
  }
  if (tid == 0) {  // tile metric totals -> this workgroup's own metrics row (summed on the host)
    float a = 0.f, b = 0.f, c = 0.f;
    for (int i = 0; i < 4; ++i) {
      a += sPart[i * 4 + 0];
      b += sPart[i * 4 + 1];
      c += sPart[i * 4 + 2];
    }
    float* m = hb.metrics + (size_t)tile * 4;
    const f32x4 old = *reinterpret_cast<const f32x4*>(m);
    *reinterpret_cast<f32x4*>(m) = f32x4{old[0] + a, old[1] + b, old[2] + c, 0.f};
  }
  __syncthreads();
  hstamp(7);
  {  // dX rows -> HBM as whole 16-byte chunks (400 columns = 50 chunks per row)
    T* dx = reinterpret_cast<T*>(hb.dx);
    for (int e = tid; e < 16 * 50; e += 512) {
      const int r = e / 50, c = e - 50 * r;
      if (r0 + r < B)
        *reinterpret_cast<uint4*>(dx + (size_t)(r0 + r) * H::K0P + c * 8) = *reinterpret_cast<const uint4*>(sDX + r * S::PX + c * 8);
    }
  }
  hstamp(8);
}

// LeNet bf16 head alone (the 16-row register-B head of fwd_head_kernel on pool2 rows from conv_fwd_kernel):
// small batches, where the LDS-staged head_kernel spends most of its time staging weights for 8 tiles.
template <typename T>
__global__ __launch_bounds__(512) void head16_kernel(BatchRef br, HeadBuffers hb) {
  using S = Head16Smem<T>;
  using H = LenetModel::Head;
  __shared__ __attribute__((aligned(16))) char smem[S::X_BYTES + S::HEAD_END];
  T* sX = reinterpret_cast<T*>(smem);
  const int tid = threadIdx.x;
  const int r0 = xcd_unit(blockIdx.x, gridDim.x, br.xcd) * 16;
  const T* xin = reinterpret_cast<const T*>(hb.xin);
  constexpr int CH = H::K0P * (int)sizeof(T) / 16;  // 16-byte chunks per row (52)
  constexpr int IT = (16 * CH + 511) / 512;
  // every load issued (branch-free, clamped row) before the first LDS store: one memory round trip
  u32x4 xv[IT];
#pragma unroll
  for (int i = 0; i < IT; ++i) {
    const int e = min(tid + 512 * i, 16 * CH - 1), r = e / CH, c = e - CH * r;
    xv[i] = reinterpret_cast<const u32x4*>(xin + (size_t)min(r0 + r, br.B - 1) * H::K0P)[c];
  }
#pragma unroll
  for (int i = 0; i < IT; ++i) {
    const int e = tid + 512 * i, r = e / CH, c = e - CH * r;
    if (e < 16 * CH)
      *reinterpret_cast<u32x4*>(sX + r * S::PX + c * (16 / (int)sizeof(T))) = r0 + r < br.B ? xv[i] : u32x4{0u, 0u, 0u, 0u};
  }
  head16_tile<T>(br, hb, smem + S::X_BYTES, sX, r0, blockIdx.x);  // barriers before reading sX
}

// (A single-launch small-batch forward + head -- conv_fwd per image pair, pool2 rows handed to the 16-row
// group's last-arriving workgroup -- measured SLOWER than conv_fwd + head16 at B = 128: 27.2-33.1 vs 25.7 us per
// step, bitwise-equal parameters; profiles/r4_session2/ab_lenet_b128_fwd_head_small.txt.  Removed in round 5.)

// ====================================================================================
// backward
// LDS images chosen so that every MFMA operand fragment is ONE aligned 16-byte read:
//   XS  [5][32][32]     xs[kw][y][x]  = xpad[y][x+kw]          conv1 wgrad B (im2col^T rows), + a ones plane
//   P1T [5][6][14][PW]  p1t[kw][c][y][x] = pool1[y][x+kw][c]   conv2 wgrad B (rows PW = 16 (bf16) / 12 (fp32) wide)
//   DY2T[16][10*16]     (fp32 only) conv2 pre-act grad, channel-major, rows padded 10->16   conv2 wgrad A
//   DYS [18][18][16]    same grad, position-major (NHWC), zero border of 4 so the full-correlation
//                       dgrad reads it without bounds checks                     conv2 dgrad A
//                       (bf16: also the conv2 wgrad A operand, read with transposing ds_read_b64_tr_b16)
//   W2  [16][496]       packed conv2 dgrad operand (C2d) for two output rows     conv2 dgrad B
//   DY1T[8][28*32]      conv1 pre-act grad, channel-major, rows padded 28->32    conv1 wgrad A
//                       (zero prefix + >= one zero image row after each channel: the wgrad reads
//                       rows y - 1 .. y + 1 of it, see phase C)
// The pool1 un-pooling (argmax + ReLU) is fused into the conv2-dgrad epilogue, which writes DY1T
// directly; pool2 un-pooling is a cooperative scatter.  Both scatters write every position of
// their map (2x2 windows tile it), so nothing but the padding is ever zero-filled.
template <typename T>
struct BwdSmem {
  // pitches padded so the fragment reads and the un-pooling scatters are <= 2-way bank
  // conflicted (measured 60% conflict cycles with the unpadded 1024/224/160/896 pitches)
  // W2R: conv2 dgrad B operand for TWO output rows per tile, [16 = (r, c)][30 taps x 16 ch + pad]
  // (pitches from scripts/lds_model.py, a bank model of every LDS access of this kernel that matches
  //  the measured SQ_LDS_BANK_CONFLICT share: 38.5 % modelled vs 38.9 % measured at 488/1048/240/176/912)
  // XP / D1P / ONES and the phase-C lane maps below: conflict-free A reads and 1.5-way B reads in the
  // conv1 wgrad (scripts/lds_model.py C2 model; 616 -> 290 LDS cycles per image for that phase)
  static constexpr int W2P = 496, XP = 1048, P1P = 240, D2P = 168, D1P = 944;
  // conv2 wgrad K: position p = y * PW + x of the 10 x 10 output (x >= 10 padding).  fp32: PW = 12, 120 positions =
  // 8 chunks instead of 10 (its phase B is MFMA-bound: LeNet fp32 B=8192 0.4139 -> 0.4015 ms), every kernel-row
  // shift (kh * PW elements) still 16-byte aligned.  bf16 keeps 16 (5 chunks): at 12 -- 4 chunks, 8-byte B reads,
  // per-lane transposed-read addresses -- B=8192 went 0.1011 -> 0.1086 ms (profiles/r5_session1/pw12/)
  static constexpr int PW = sizeof(T) == 4 ? 12 : 16;
  static constexpr int D1PRE = 32;  // zero elements before channel 0 of DY1T (row y - 1 of the first row)
  // XS: 5 shifted planes, then an all-ones plane at ONES (bias-gradient column; its position sets the
  // bank of that column); P1T has 32 planes (30 + zero + ones): padding / bias-gradient columns read a
  // constant plane instead of branching per lane
  static constexpr int ONES = 5 * XP + 120, ONES_N = 944;
  static constexpr int XS_N = ONES + ONES_N, PPL = 32;
  static constexpr int OFF_XS = 0;
  static constexpr int OFF_P1T = rup(OFF_XS + XS_N * (int)sizeof(T), 16);
  // TRA (bf16): the conv2 wgrad reads its A operand (channel-major dY2) straight from the position-major
  // DYS image with ds_read_b64_tr_b16 (transposing LDS reads), so there is no DY2T image and no second
  // un-pooling scatter
  static constexpr bool TRA = sizeof(T) == 2;
  static constexpr bool DY2 = !TRA;
  static constexpr int OFF_DY2T = rup(OFF_P1T + PPL * P1P * (int)sizeof(T), 16);
  static constexpr int OFF_DYS = rup(OFF_DY2T + (DY2 ? 16 * D2P * (int)sizeof(T) : 0), 16);  // [18][18][16] zero-padded
  static constexpr int OFF_W2 = rup(OFF_DYS + 18 * 18 * 16 * (int)sizeof(T), 16);
  static constexpr int OFF_DY1T = rup(OFF_W2 + 16 * W2P * (int)sizeof(T), 16);
  static constexpr int OFF_M1 = rup(OFF_DY1T + (D1PRE + 8 * D1P) * (int)sizeof(T), 16);  // [6][M1CP] u8 pool1 codes
  static constexpr int TOTAL = rup(OFF_M1 + M1IMG, 16);
  static constexpr int OFF_RED = OFF_XS;  // [NW][256] f32 scratch after the image loop
  static_assert(8 * 256 * 4 <= XS_N * (int)sizeof(T), "reduction scratch must fit in the aliased XS region");
  static_assert(D1P >= 928 && 4 * XP + 4 * 32 + 928 <= ONES, "phase C reads stay inside zeroed rows");
  static_assert(14 * PW <= P1P && 4 * PW + 128 <= P1P && 128 <= D2P, "conv2 wgrad reads stay inside their (zeroed) planes");
};

// Per-image thread roles and the phase-B work split of conv_bwd_kernel, by workgroup size (NW waves).
// NW = 4 (256 threads, the round-1..3 layout): every wave stages, every wave computes both GEMMs of phase B.
// NW = 8 (512 threads, two workgroups = 16 waves per CU at the same LDS footprint): the staging roles and the
// two phase-B GEMMs are on DIFFERENT waves -- waves 0-3 the conv2 dgrad (row pairs {2,2,2,1}), waves 4-7 the
// conv2 wgrad (tiles {3,3,2,2}) -- so twice as many independent LDS / MFMA chains are in flight per CU and the
// longest per-wave chain of a phase is 30 MFMAs instead of 45.
template <typename T, int NW>
struct BwdRoles {
  static constexpr int NT = NW * 64;
  static constexpr bool W8 = NW == 8;
  // phase A staging roles (thread ranges)
  static constexpr int XS_T0 = 0, XS_N = 112;                 // input row y, column chunk -> 5 XS planes
  static constexpr int M1_T0 = W8 ? 128 : 112, M1_N = M1IMG / 16;  // 16-byte chunks of the pool1 codes
  static constexpr int P1_T0 = W8 ? 256 : 128, P1_N = 84;     // pool1 row (c, y) -> 5 shifted P1T rows
  static constexpr int DS_T0 = W8 ? 312 : 0, DS_N = 200;      // bf16 pool2 un-pooling: (channel pair, position)
  static constexpr int F_T0 = W8 ? 112 : 0, F_ITEMS = W8 ? 1 : 2;  // f32 un-pooling: items per thread
  // waves that load each role's next-image inputs (wave-uniform: a wave without the role issues none)
  static DEV bool loads_px(int w) { return !W8 || w < 2; }
  static DEV bool loads_m1(int w) { return !W8 || (w >= 2 && w < 4); }
  static DEV bool loads_p1(int w) { return !W8 || (w >= 4 && w < 6); }
  static DEV bool loads_p2(int w) { return !W8 || (sizeof(T) == 2 ? w >= 4 : w >= 1); }
  // phase B: dgrad row pairs [q0, q0 + np) of 7 (np = 0: no dgrad on this wave); wgrad tiles [n0w, n0w + nw)
  // (Measured: putting the dgrad on waves 0-1 {4, 3} and the wgrad on waves 2-3 {5, 5}, or the wgrad on one wave --
  // fewer waves reading each shared fragment -- made phase B 14 / 32 % slower: the per-wave chains, not the LDS
  // bandwidth, bound it; profiles/r5_session1/roles/)
  static constexpr int NPMAX = 2;  // most dgrad row pairs on a wave
  static DEV int dg_np(int w) { return W8 ? (w < 3 ? 2 : (w == 3 ? 1 : 0)) : (w < 3 ? 2 : 1); }
  static DEV int dg_q0(int w) { return W8 ? (w < 4 ? 2 * w : 0) : 2 * w; }
  // The wgrad tiles go {2, 2, 2, 4} against the dgrad row pairs {2, 2, 2, 1} (waves w and w + 4 of the 8-wave
  // layout share SIMD w % 4): a dgrad tile is 3x a wgrad tile's MFMAs (fp32: 120 vs 40 v_mfma_f32_16x16x4_f32;
  // bf16: 15 vs 5 16x16x32), so per SIMD 320 / 320 / 320 / 280 fp32 MFMAs (was {3, 3, 2, 2}: 360 / 360 / 320 / 200)
  // and the longest per-wave bf16 chain (4 waves) is 40 MFMAs instead of 45.
  static constexpr bool BAL = !W8 || sizeof(T) == 4;
  static constexpr int NWT = BAL ? 4 : 3;  // wgrad accumulators per wave
  static DEV int wg_nw(int w) {
    if (W8 && BAL) return w < 4 ? 0 : (w < 7 ? 2 : 4);
    if (W8) return w < 4 ? 0 : (w < 6 ? 3 : 2);
    return w < 3 ? 2 : 4;
  }
  static DEV int wg_n0(int w) {
    if (W8 && BAL) return w < 4 ? 0 : 2 * (w - 4);
    if (W8) return w < 4 ? 0 : (w < 6 ? 3 * (w - 4) : 6 + 2 * (w - 6));
    return 2 * w;
  }
};

// phase-B LDS prefetch distance (chunks of fragments in flight ahead of the MFMAs).  LeNet bf16 B=8192, 2000
// steps (profiles/r4_session2/ab_conv_bwd_pd.txt): PD 1 / 2 / 3 = 0.1038-0.1041 / 0.1024-0.1034 / 0.1036-0.1038
// ms/step, bitwise-equal parameters; fp32 unchanged (0.439 ms).  Re-measured on the round-6 kernels (two boxes,
// profiles/r6_session1/ab_bwd_pd.txt): PD 3 0.0966-0.0971 vs PD 2 0.0970-0.0974 ms; PD 1 / 4 / 5 no better; fp32
// unchanged (0.370 ms).
#ifndef MNIST_AMD_BWD_PD
#define MNIST_AMD_BWD_PD 3
#endif
constexpr int BWD_PD = MNIST_AMD_BWD_PD;
// One conv_bwd workgroup: block `blk` of `nblk` (the conv_bwd part of the grid).
template <typename T, int NW>
DEV void conv_bwd_block(const BatchRef br, const LenetConvBuffers cb, const int ipb, const int blk, const int nblk) {
  using M = Mma<T>;
  using Frag = typename M::Frag;
  using S = BwdSmem<T>;
  using R = BwdRoles<T, NW>;
  constexpr int KV = M::KV, KC = M::KC, NT = R::NT;
  __shared__ __attribute__((aligned(16))) char smem[S::TOTAL];
  T* xs = reinterpret_cast<T*>(smem + S::OFF_XS);
  T* p1t = reinterpret_cast<T*>(smem + S::OFF_P1T);
  T* dy2t = reinterpret_cast<T*>(smem + S::OFF_DY2T);
  T* dys = reinterpret_cast<T*>(smem + S::OFF_DYS);
  T* w2 = reinterpret_cast<T*>(smem + S::OFF_W2);
  T* dy1t = reinterpret_cast<T*>(smem + S::OFF_DY1T) + S::D1PRE;  // channel 0 row 0
  uint8_t* m1s = reinterpret_cast<uint8_t*>(smem + S::OFF_M1);
  float* red = reinterpret_cast<float*>(smem + S::OFF_RED);
  const int tid = threadIdx.x, lane = tid & 63, w = wave_id(), row = lane & 15, grp = lane >> 4;
  const int unit = xcd_unit(blk, nblk, br.xcd);  // images [unit * ipb, +ipb), slab row unit
  // pixel rows: batch-ordered copy from conv_fwd (cb.xb: no index chain in front of the first image), else
  // gathered through the sample index
  const uint8_t* const xb = cb.xb;
  const BlockIdx bidx(xb ? nullptr : br.idx_epoch + (size_t)br.step_ptr[0] * br.batch_stride, unit * ipb, ipb, br.B);
  const T* pack = reinterpret_cast<const T*>(cb.pack);
  const T* dp2 = reinterpret_cast<const T*>(cb.dp2);
  const T* p1g = reinterpret_cast<const T*>(cb.p1);
  // optional wall-clock stamps (profiling): [0] start, [1] setup, 3 per image for images 0..3,
  // [14] loop end, [15] slab written
  auto stamp = [&](int k) {
    if (cb.stamps && tid == 0 && blk < 512) cb.stamps[blk * 16 + k] = wall_clock64();
  };
  stamp(0);

  // ---- software pipeline: every global input of image t+1 is loaded into registers while
  //      image t computes (phases B and C), so phase A only moves registers into LDS
  // Phase-A thread roles (BwdRoles; every LDS image is written with 16-byte stores, source rows prefetched):
  //   XS : input row y = tid/4, column chunk g = tid%4 -> its chunk of the 5 shifted XS planes
  //   M1 : 16-byte chunk of the CHW16 pool1 codes -> M1
  //   P1 : pool1 channel c, row y (c*14 + y) -> its row of the 5 shifted P1T planes
  //   DS : pool2 un-pooling scatter into DYS (/ DY2T)
  constexpr int PV = 16 * (int)sizeof(T) / 16;  // uint4 per CHW16 pool1 row (2 bf16 / 4 f32)
  // Prefetch registers, one slot range per role: input pixels (4 dwords, image columns [8g-4, 8g+12) of row
  // y-2), pool1 codes (one uint4), pool1 row (PV uint4), and the un-pooling items (codes c[2], raw grads g[2]).
  // Where no thread has two of the XS / M1 / P1 roles (bf16, 8 waves) those share ONE slot range (a
  // register union: 12 dwords instead of 20, so the 8-wave kernel fits 128 VGPRs).
  constexpr bool UNION = NW == 8 && sizeof(T) == 2;
  constexpr int O_PX = 0, O_M1 = UNION ? 0 : 4, O_P1 = UNION ? 0 : 8, O_DS = O_P1 + 4 * PV, NREG = O_DS + 4;
  struct Pre {
    uint32_t r[NREG];
    DEV uint4 q(int o) const { return make_uint4(r[o], r[o + 1], r[o + 2], r[o + 3]); }
    DEV void setq(int o, const uint4& v) { r[o] = v.x; r[o + 1] = v.y; r[o + 2] = v.z; r[o + 3] = v.w; }
    DEV uint32_t code(int k) const { return r[O_DS + k]; }
    DEV T grad(int k) const {
      if constexpr (sizeof(T) == 2) return __builtin_bit_cast(T, (unsigned short)r[O_DS + 2 + k]);
      else return __builtin_bit_cast(T, r[O_DS + 2 + k]);
    }
  };
  // Branch-free inside a wave: every lane of a loading wave issues the same loads (addresses clamped into
  // range, values of lanes without the role / of images past the batch zeroed at use), so vmcnt
  // accounting stays exact; waves without a role (wave-uniform test) issue none of its loads.
  auto fetch = [&](int t) -> Pre {
    Pre f;
#pragma unroll
    for (int k = 0; k < NREG; ++k) f.r[k] = 0u;
    const bool live = t < ipb && unit * ipb + t < br.B;  // wave-uniform
    const int bb = min(unit * ipb + t, br.B - 1);
    if (R::loads_px(w)) {
      const int xt = min(tid - R::XS_T0, R::XS_N - 1);
      const uint8_t* rowp = (xb ? xb + (size_t)min(unit * ipb + (live ? t : 0), br.B - 1) * 784
                                : br.images + (size_t)bidx[live ? t : 0] * 784) + ((xt >> 2) % 28) * 28;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int col = 8 * (xt & 3) - 4 + 4 * k;
        f.r[O_PX + k] = *reinterpret_cast<const uint32_t*>(rowp + min(max(col, 0), 24));
      }
    }
    if (R::loads_m1(w))
      f.setq(O_M1, reinterpret_cast<const uint4*>(cb.m1 + (size_t)bb * M1IMG)[min(max(tid - R::M1_T0, 0), R::M1_N - 1)]);
    if (R::loads_p1(w)) {
      const int i = min(max(tid - R::P1_T0, 0), R::P1_N - 1), c = i / 14, y = i - 14 * c;
      const uint4* ps = reinterpret_cast<const uint4*>(p1g + (size_t)bb * P1IMG + c * P1CP + y * 16);
#pragma unroll
      for (int k = 0; k < PV; ++k) f.setq(O_P1 + 4 * k, ps[k]);
    }
    if (R::loads_p2(w)) {
#pragma unroll
      for (int r = 0; r < 2; ++r) {
        int n, p;
        if constexpr (sizeof(T) == 2) {  // bf16: thread j < 200 owns channels (2(j%8), 2(j%8)+1) at position j/8
          const int j = min(max(tid - R::DS_T0, 0), R::DS_N - 1);
          n = 2 * (j & 7) + r;
          p = j >> 3;
        } else {                          // f32: items (channel fastest, position)
          const int e = min(max(tid - R::F_T0 + NT * r, 0), 399);
          n = e & 15;
          p = e >> 4;
        }
        if (r < (sizeof(T) == 2 ? 2 : R::F_ITEMS)) {
          f.r[O_DS + r] = cb.m2[(size_t)bb * 400 + n * 25 + p];
          const T gv = dp2[(size_t)bb * K0P + n * 25 + p];
          if constexpr (sizeof(T) == 2) f.r[O_DS + 2 + r] = __builtin_bit_cast(unsigned short, gv);
          else f.r[O_DS + 2 + r] = __builtin_bit_cast(uint32_t, gv);
        }
      }
    }
    return f;
  };
  Pre nxt = fetch(0);  // issued before the setup below, so its latency overlaps it

  constexpr int W2CH = (10 * S::PW + KC - 1) / KC;  // conv2 wgrad: 10 rows x PW positions
  constexpr int D2CH = 480 / KC;              // conv2 dgrad K = 30 taps (kh' = -1..4) x 16 ch (15 bf16 / 30 f32)
  // (measured: a register-resident dgrad B operand pushed the kernel to 245 VGPRs and made hipcc
  //  shuttle accumulators VGPR<->AGPR around every MFMA -- the B operand is read from LDS)

  // ---- once per workgroup: zero every padded image, stage C2d
  zero_lds<T>(xs, S::ONES);
  for (int e = tid; e < S::ONES_N; e += NT) xs[S::ONES + e] = to_t<T>(1.f);
  zero_lds<T>(dy1t - S::D1PRE, S::D1PRE + 8 * S::D1P);
  zero_lds<T>(dys, 18 * 18 * 16);
  zero_lds<T>(p1t, 31 * S::P1P);
  for (int e = tid; e < S::P1P; e += NT) p1t[31 * S::P1P + e] = to_t<T>(1.f);
  if constexpr (S::DY2) zero_lds<T>(dy2t, 16 * S::D2P);
  // conv2 dgrad, two output rows per tile: out (Y = y + r, x, c) = sum over kh' in [-1, 4], kw, n of
  // dY2[y - kh'][x - kw][n] * W2[n][c][kh' + r][kw]  ->  B[(kh'+1)*5 + kw, n][(r, c)], zero where
  // kh' + r is outside 0..4.  N = (r, c) holds 12 live columns of 16 (was 6 with one row per tile).
  // Row (r, c) is C2D row c shifted by 5 taps: r = 0 -> [80 zeros | C2D[c][0..400)], r = 1 ->
  // [C2D[c][0..400) | 80 zeros]; copied as 16-byte vectors (rows c >= 6 are all zero).
  // Every thread's loads are issued (branch-free, clamped addresses) before its first LDS store: one memory
  // round trip for the whole image instead of one per loop trip.
  {
    constexpr int VE = 16 / (int)sizeof(T), RV = 480 / VE, SH = 80 / VE, NV = 16 * RV, IT = (NV + NT - 1) / NT;
    u32x4 wv[IT];
#pragma unroll
    for (int i = 0; i < IT; ++i) {
      const int e = min(tid + i * NT, NV - 1), nr = e / RV, v = e % RV, r = nr >> 3, c = nr & 7;
      const int src = r == 0 ? v - SH : v;  // source vector within C2D row c
      wv[i] = *reinterpret_cast<const u32x4*>(pack + L::C2D + min(c, 5) * 416 + min(max(src, 0), 400 / VE - 1) * VE);
    }
#pragma unroll
    for (int i = 0; i < IT; ++i) {
      const int e = tid + i * NT, nr = e / RV, v = e % RV, r = nr >> 3, c = nr & 7;
      const int src = r == 0 ? v - SH : v;
      const bool ok = c < 6 && src >= 0 && src < 400 / VE;
      if (e < NV) *reinterpret_cast<u32x4*>(w2 + nr * S::W2P + v * VE) = ok ? wv[i] : u32x4{0u, 0u, 0u, 0u};
    }
  }
  // ---- static work split of phase B (dgrad row-pair tile = 15 K-chunks, wgrad tile = 5): BwdRoles
  const int np = R::dg_np(w), q0 = R::dg_q0(w);  // dgrad row pairs [q0, q0 + np)
  const int nw = R::wg_nw(w), n0w = R::wg_n0(w);  // wgrad tiles [n0w, n0w + nw)
  constexpr int NWT = R::NWT;  // wgrad accumulators per wave
  // ---- per-lane operand offsets (loop invariant)
  // conv2 wgrad B: DENSE columns kcol = tap*6 + c (150 weights) + 1 bias column = 10 tiles of 16
  // (was tap*8 + c: 13 tiles, a quarter of them zero channels 6, 7)
  int w2off[NWT];
#pragma unroll
  for (int i = 0; i < NWT; ++i) {
    const int kcol = (n0w + i) * 16 + row, tap = kcol / 6, c = kcol - 6 * tap;
    w2off[i] = kcol < 150 ? ((tap % 5) * 6 + c) * S::P1P + (tap / 5) * S::PW : (kcol == 150 ? 31 : 30) * S::P1P;
    if (i >= nw) w2off[i] = 30 * S::P1P;  // no such tile on this wave: zero plane
  }
  // conv1 wgrad (phase C) as ONE 16x16 tile per image: M row m = (r, n) reads channel n of DY1T shifted
  // back r image rows, N column j = (kernel-row base khb in {0, 2, 4}, kw) reads XS plane kw at row khb,
  // so C[(r, n)][(khb, kw)] = dW1[n][khb + r][kw] (khb + r = 5: discarded) and column 15 (ones plane) is
  // the bias gradient.  Was two tiles (M = 6 of 16 channels, N = 26 of 32 taps): 56 -> 29 MFMAs and
  // 84 -> 58 fragment reads per image (bf16).  The row -> (r, n) and column -> (khb, kw) assignments
  // are lane permutations chosen by the bank model (scripts/lds_model.py, C2).
  constexpr uint8_t C_AMAP[16] = {8, 11, 0, 10, 4, 12, 5, 13, 15, 3, 2, 14, 9, 7, 6, 1};  // r * 8 + n
  constexpr uint8_t C_BMAP[16] = {8, 9, 12, 4, 5, 15, 10, 13, 2, 14, 6, 11, 1, 7, 3, 0};  // (khb / 2) * 5 + kw | 15
  const int c_aoff = (C_AMAP[row] & 7) * S::D1P - 32 * (C_AMAP[row] >> 3);
  const int c_boff = C_BMAP[row] < 15 ? (C_BMAP[row] % 5) * S::XP + 2 * (C_BMAP[row] / 5) * 32 : S::ONES;
  // conv2 dgrad A: the lane's K-chunk kc covers tap = 2kc + (grp >> 1) (bf16; f32: tap = kc), channels n0..; its
  // fragment sits at -(tap row kh', col kw) positions from the tile's base in the padded DYS.  The
  // lane-dependent part is folded into two base offsets -- the second tap of a bf16 chunk is one column
  // left of the first (-16 elements) unless the first ends a kernel row (tap % 5 == 4: next row, kw = 0:
  // -224) -- so every chunk's offset is a compile-time constant on one of them (no per-chunk VGPRs).
  const int dl_n = (KV == 8 ? (grp & 1) * 8 - 16 * (grp >> 1) : grp * 4);
  const int dl_s = (KV == 8 ? (grp & 1) * 8 - 224 * (grp >> 1) : grp * 4);
  auto doff = [&](int kc) {
    const int tap0 = KV == 8 ? 2 * kc : kc, khp = tap0 / 5 - 1, kw = tap0 % 5;  // pair base y <= 12: rows <= 17
    return (-khp * 18 - kw) * 16 + ((KV == 8 && kw == 4) ? dl_s : dl_n);
  };

  f32x4 accW2[NWT], accW1 = zero4();
#pragma unroll
  for (int i = 0; i < NWT; ++i) accW2[i] = zero4();
  wait_vm_all();  // loop-invariant loads done here (image 0's inputs, also in flight, are consumed next)
  __syncthreads();
  stamp(1);

  for (int t = 0; t < ipb; ++t) {
    const int b = unit * ipb + t;
    const bool valid = b < br.B;
    const Pre cur = nxt;
    // ---- phase A: stage input (5 shifted copies), pool1 (5 shifted channel-major copies),
    //      pool1 codes, and the pool2 un-pooling scatter into DYS / DY2T
    if (tid >= R::XS_T0 && tid < R::XS_T0 + R::XS_N && !ABLATED(cb.ablate, 8)) {
      // XS: planes kw = 0..4 of row y, columns [8g, 8g+8): xs[kw][y][x] = xpad[y][x + kw] = w[kw + 2 + j]
      // with w[i] = normalised pixel at image column 8g - 4 + i (0 outside the image)
      const int xt = tid - R::XS_T0, y = 2 + (xt >> 2), g = xt & 3;
      auto pixel = [&](int i) { return mnist_norm((cur.r[O_PX + (i >> 2)] >> (8 * (i & 3))) & 255u); };
      T* dst = xs + y * 32 + 8 * g;
      if constexpr (sizeof(T) == 2) {
        // pixel pairs by one v_cvt_pk_bf16_f32 each; the window leaves the image only as whole pairs -- pairs 0, 1
        // when g = 0 (columns -4..-1), pairs 4..7 when g = 3 (columns 28..35, also the clamped duplicate words)
        typedef __attribute__((ext_vector_type(2))) float f32x2;
        const uint32_t vm = valid ? 0xFFFFFFFFu : 0u;
        const uint32_t m0 = g == 0 ? 0u : vm, m3 = g == 3 ? 0u : vm;
        uint32_t D[8];
#pragma unroll
        for (int k = 1; k < 8; ++k)  // (D[0] is not read)
          D[k] = __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2{pixel(2 * k), pixel(2 * k + 1)}), bf16x2)) &
                 (k < 2 ? m0 : (k >= 4 ? m3 : vm));
        D[0] = 0u;
#pragma unroll
        for (int kw = 0; kw < 5; ++kw) {
          const int m = (kw + 2) >> 1;
          uint4 o;
          uint32_t* ov = reinterpret_cast<uint32_t*>(&o);
#pragma unroll
          for (int j = 0; j < 4; ++j)
            ov[j] = (kw & 1) ? __builtin_amdgcn_alignbyte(D[m + j + 1], D[m + j], 2) : D[m + j];
          *reinterpret_cast<uint4*>(dst + kw * S::XP) = o;
        }
      } else {
        float wv[16];
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const bool in = valid && (unsigned)(8 * g - 4 + i) < 28u;  // also masks the clamped (duplicate) words
          wv[i] = in ? pixel(i) : 0.f;
        }
#pragma unroll
        for (int kw = 0; kw < 5; ++kw) {
          float* d = reinterpret_cast<float*>(dst + kw * S::XP);
          *reinterpret_cast<f32x4*>(d) = f32x4{wv[kw + 2], wv[kw + 3], wv[kw + 4], wv[kw + 5]};
          *reinterpret_cast<f32x4*>(d + 4) = f32x4{wv[kw + 6], wv[kw + 7], wv[kw + 8], wv[kw + 9]};
        }
      }
    }
    if (tid >= R::M1_T0 && tid < R::M1_T0 + R::M1_N && !ABLATED(cb.ablate, 8))
      reinterpret_cast<uint4*>(m1s)[tid - R::M1_T0] = valid ? cur.q(O_M1) : make_uint4(0, 0, 0, 0);
    if (tid >= R::P1_T0 && tid < R::P1_T0 + R::P1_N && !ABLATED(cb.ablate, 8)) {
      // P1T: row y of planes (kw, c), kw = 0..4: p1t[kw*6+c][y][x] = pool1[y][x + kw][c] (x < PW), 0 for x + kw >= 14
      const int i = tid - R::P1_T0, c = i / 14, y = i - 14 * c;
      T pv[16];
#pragma unroll
      for (int k = 0; k < PV; ++k)
        *reinterpret_cast<uint4*>(pv + k * (16 / (int)sizeof(T))) = valid ? cur.q(O_P1 + 4 * k) : make_uint4(0, 0, 0, 0);
      T* dst = p1t + c * S::P1P + y * S::PW;
      if constexpr (sizeof(T) == 2) {
        uint32_t D[10];
#pragma unroll
        for (int k = 0; k < 7; ++k) D[k] = reinterpret_cast<const uint32_t*>(pv)[k];
        D[7] = D[8] = D[9] = 0u;  // x = 14, 15 of the CHW16 row are padding
#pragma unroll
        for (int kw = 0; kw < 5; ++kw) {
          const int m = kw >> 1;
          uint32_t o[8];
#pragma unroll
          for (int j = 0; j < 8; ++j) o[j] = (kw & 1) ? __builtin_amdgcn_alignbyte(D[m + j + 1], D[m + j], 2) : D[m + j];
          static_assert(S::PW == 16, "bf16 P1T rows: 16 wide");
          T* d = dst + kw * 6 * S::P1P;
          *reinterpret_cast<uint4*>(d) = make_uint4(o[0], o[1], o[2], o[3]);
          *reinterpret_cast<uint4*>(d + 8) = make_uint4(o[4], o[5], o[6], o[7]);
        }
      } else {
#pragma unroll
        for (int kw = 0; kw < 5; ++kw) {
          float* d = reinterpret_cast<float*>(dst + kw * 6 * S::P1P);
#pragma unroll
          for (int q = 0; q < S::PW / 4; ++q) {
            f32x4 o;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              const int xx = 4 * q + j + kw;
              o[j] = xx < 14 ? to_f(pv[xx]) : 0.f;
            }
            *reinterpret_cast<f32x4*>(d + 4 * q) = o;
          }
        }
      }
    }
    if constexpr (sizeof(T) == 2) {
      // pool2 un-pooling, two channels per thread: every DYS write is one 32-bit (channel pair) store
      if (tid >= R::DS_T0 && tid < R::DS_T0 + R::DS_N && !ABLATED(cb.ablate, 32)) {
        const int j = tid - R::DS_T0;
        const int n0 = 2 * (j & 7), p = j >> 3, py = p / 5, px = p % 5;
        // the gradient's raw bf16 bits go to the window its pool2 code names (code & 7 == 4 + window: ReLU passed,
        // argmax = window), 0 elsewhere -- selects on 16-bit values, no float round trip
        const uint32_t c0 = valid ? (cur.code(0) & 7u) : 0u, c1 = valid ? (cur.code(1) & 7u) : 0u;  // 0: all windows 0
        const uint32_t g0 = cur.r[O_DS + 2] & 0xFFFFu, g1 = cur.r[O_DS + 3] << 16;
#pragma unroll
        for (int win = 0; win < 4; ++win) {
          const int oh = 2 * py + (win >> 1), ow = 2 * px + (win & 1);
          *reinterpret_cast<uint32_t*>(dys + ((oh + 4) * 18 + ow + 4) * 16 + n0) =
              (c0 == 4u + win ? g0 : 0u) | (c1 == 4u + win ? g1 : 0u);
        }
      }
    } else {
#pragma unroll
      for (int r = 0; r < R::F_ITEMS; ++r) {
        const int e = tid - R::F_T0 + NT * r;
        if (e < 0 || e >= 400 || ABLATED(cb.ablate, 32)) break;
        const int n = e & 15, p = e >> 4, py = p / 5, px = p % 5;  // channel fastest: conflict-free DYS writes
        const uint32_t code = valid ? cur.code(r) : 0u;  // code 0: ReLU blocked, every window gets 0
        const float g = to_f(cur.grad(r));
#pragma unroll
        for (int win = 0; win < 4; ++win) {
          const int oh = 2 * py + (win >> 1), ow = 2 * px + (win & 1);
          const T v = to_t<T>(((code & 4) && (code & 3) == win) ? g : 0.f);
          dys[((oh + 4) * 18 + ow + 4) * 16 + n] = v;
          dy2t[n * S::D2P + oh * S::PW + ow] = v;
        }
      }
    }
    __syncthreads();
    if (t < 4) stamp(2 + 3 * t);
    // next image's inputs are issued here, a whole phase B + C before phase A consumes them; the loop
    // has no other global operation, so that phase's vmcnt wait is for these loads only
    nxt = fetch(t + 1);

    // ---- phase B1: conv2 wgrad  dW2[n][(tap, c)] += sum_pos dY2[pos][n] * pool1[pos + tap][c]
    //      Straight-line (constant trip counts) with the next chunk's fragments loaded before this chunk's
    //      MFMAs: a runtime trip count kept the loop rolled and every chunk waited for its own LDS reads.
    if (nw > 0 && !ABLATED(cb.ablate, 64)) {
      auto ld_a = [&](int kc) -> Frag {
        if constexpr (S::TRA) {
          // positions p0 .. p0 + 7 (row y = p0 / 16, columns x0 .. x0 + 7; x >= 10 reads DYS's zero padding) of
          // channel `row`: two 4-position x 16-channel blocks, transposed by the read.  Lane 4q + p of each
          // 16-lane group addresses position x0 + q (+ 4), channels 4p .. 4p + 3; lane i receives channel i.
          static_assert(S::PW == 16, "bf16 conv2 wgrad positions: 16 per row");
          typedef short v4s __attribute__((ext_vector_type(4)));
          const int p0 = kc * KC + grp * KV, y = p0 >> 4, x0 = p0 & 15;
          const T* a = dys + ((y + 4) * 18 + x0 + ((lane & 15) >> 2) + 4) * 16 + 4 * (lane & 3);
          const v4s lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
              (__attribute__((address_space(3))) v4s*)(const_cast<T*>(a)));
          const v4s hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
              (__attribute__((address_space(3))) v4s*)(const_cast<T*>(a + 4 * 16)));
          Frag f;
          f.v = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
          return f;
        } else {
          return M::load(dy2t + row * S::D2P + kc * KC + grp * KV);
        }
      };
      auto ld_b = [&](int kc, int i) {
        return M::load(p1t + w2off[i] + kc * KC + grp * KV);  // positions p = y * PW + x (16-byte aligned)
      };
      // NT real tiles on this wave: no zero-plane filler tile
      // fragments of chunk kc + PD are issued before chunk kc's MFMAs (constant indices: registers)
      auto wgrad2 = [&](auto ntc) {
        constexpr int NTL = decltype(ntc)::value;
        Frag fa[W2CH], fb[W2CH][NTL];
        auto issue = [&](int kc) {
          fa[kc] = ld_a(kc);
#pragma unroll
          for (int i = 0; i < NTL; ++i) fb[kc][i] = ld_b(kc, i);
        };
#pragma unroll
        for (int kc = 0; kc < BWD_PD && kc < W2CH; ++kc) issue(kc);
#pragma unroll
        for (int kc = 0; kc < W2CH; ++kc) {
          if (kc + BWD_PD < W2CH) issue(kc + BWD_PD);
#pragma unroll
          for (int i = 0; i < NTL; ++i) M::mma(accW2[i], fa[kc], fb[kc][i]);
        }
      };
      if (nw == 2) wgrad2(std::integral_constant<int, 2>{});
      else wgrad2(std::integral_constant<int, NWT>{});
    }

    // ---- phase B2: conv2 dgrad, one tile = image rows (y, y+1) x 16 columns x (r, c):
    //      dP1[y+r][x][c] = sum_{kh',kw,n} dY2[y-kh'][x-kw][n] * W2R[kh',kw,n][(r,c)]
    //      Lane group g owns x = 4g..4g+3; the pool1 un-pooling epilogue (argmax + ReLU) writes the
    //      conv1 pre-activation grad rows 2Y and 2Y+1 (Y = y + r) as ONE 16-byte store each.
    //      A wave's (up to 2) tiles share every B fragment.
    if (np > 0) {
      auto dgrad_tile_epi = [&](int y, const f32x4& acc) {
        const int c = row & 7, Y = y + (row >> 3);
        if (c < 6) {
          const uint32_t codes = *reinterpret_cast<const uint32_t*>(m1s + c * M1CP + Y * 16 + grp * 4);
          T* d = dy1t + c * S::D1P + (2 * Y) * 32 + grp * 8;
          if constexpr (sizeof(T) == 2) {
            // the gradient's bf16 bits routed by the pool1 code (bit 2: ReLU passed, bits 0-1: window) into the 16-bit
            // halves of the two output rows' dwords -- bit-field extracts and selects, one conversion per value.
            // Pooled columns x >= 14 have code 0 (conv_fwd never writes their padding bytes), so no range check.
            typedef __attribute__((ext_vector_type(2))) float f32x2;
            uint32_t w0[4], w1[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
              const uint32_t vb = __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2{acc[i], 0.f}), bf16x2));
              const uint32_t keep = (uint32_t)(((int32_t)(codes << (29 - 8 * i))) >> 31);  // bit 8i + 2 -> 0 / ~0
              const uint32_t val = (vb & keep) << (((codes >> (8 * i)) & 1u) << 4);
              const bool row1 = (codes >> (8 * i + 1)) & 1u;
              w0[i] = row1 ? 0u : val;
              w1[i] = row1 ? val : 0u;
            }
            *reinterpret_cast<uint4*>(d) = make_uint4(w0[0], w0[1], w0[2], w0[3]);
            *reinterpret_cast<uint4*>(d + 32) = make_uint4(w1[0], w1[1], w1[2], w1[3]);
            return;
          }
          T r0[8], r1[8];
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const uint32_t code = (codes >> (8 * i)) & 255u;
            const bool ok = (grp * 4 + i) < 14 && (code & 4);
            const float v = ok ? acc[i] : 0.f;
            const uint32_t am = code & 3;
            r0[2 * i] = to_t<T>(am == 0 ? v : 0.f);
            r0[2 * i + 1] = to_t<T>(am == 1 ? v : 0.f);
            r1[2 * i] = to_t<T>(am == 2 ? v : 0.f);
            r1[2 * i + 1] = to_t<T>(am == 3 ? v : 0.f);
          }
          reinterpret_cast<uint4*>(d)[0] = reinterpret_cast<const uint4*>(r0)[0];
          reinterpret_cast<uint4*>(d)[1] = reinterpret_cast<const uint4*>(r0)[1];
          reinterpret_cast<uint4*>(d + 32)[0] = reinterpret_cast<const uint4*>(r1)[0];
          reinterpret_cast<uint4*>(d + 32)[1] = reinterpret_cast<const uint4*>(r1)[1];
        }
      };
      const int x = min(row, 13);
      const T* bq = w2 + row * S::W2P + grp * KV;
      // The wave's NP row-pair tiles q0 .. q0 + NP - 1 (rows y0 + 2j) share every B fragment, and tile j sees tile
      // j - 1's dY2 window two kernel rows (SH chunks) later: A_j(kc) = A_{j-1}(kc - SH).  So only tile 0 reads
      // all D2CH = 3 SH chunks of A; tiles j >= 1 read their first SH.  The chunks are visited diagonally --
      // c, c + SH, c + 2 SH for c = 0 .. SH - 1 -- so the fragments one c needs (3 of tile 0, 1 per other tile, 3
      // B) are all the registers held: A_j(c + m SH) = L_{j-m}(c) for j >= m, else L_0(c + (m - j) SH).
      auto dgrad_tiles = [&](auto npc) {
        constexpr int NP = decltype(npc)::value;
        constexpr int SH = 160 / KC;  // chunks per two kernel rows (10 taps x 16 channels)
        static_assert(D2CH == 3 * SH, "conv2 dgrad K = 3 x two kernel rows");
        const int y0 = 2 * q0;
        const T* a0 = dys + ((y0 + 4) * 18 + x + 4) * 16;
        f32x4 acc[NP];
#pragma unroll
        for (int j = 0; j < NP; ++j) acc[j] = zero4();
        struct Set { Frag l0[3], lt[NP > 1 ? NP - 1 : 1], fb[3]; };
        auto ld = [&](int c) {
          Set r;
#pragma unroll
          for (int m = 0; m < 3; ++m) {
            r.fb[m] = M::load(bq + (c + m * SH) * KC);
            r.l0[m] = M::load(a0 + doff(c + m * SH));
          }
#pragma unroll
          for (int j = 1; j < NP; ++j) r.lt[j - 1] = M::load(a0 + 2 * j * 18 * 16 + doff(c));
          return r;
        };
        Set cur = ld(0);
#pragma unroll
        for (int c = 0; c < SH; ++c) {
          Set nxt = cur;
          if (c + 1 < SH) nxt = ld(c + 1);
#pragma unroll
          for (int m = 0; m < 3; ++m)
#pragma unroll
            for (int j = 0; j < NP; ++j)
              M::mma(acc[j], j >= m ? (j == m ? cur.l0[0] : cur.lt[j - m - 1]) : cur.l0[m - j], cur.fb[m]);
          cur = nxt;
        }
#pragma unroll
        for (int j = 0; j < NP; ++j) dgrad_tile_epi(y0 + 2 * j, acc[j]);
      };
      if (!ABLATED(cb.ablate, 128)) {
        static_assert(R::NPMAX == 2, "dgrad row pairs per wave: 1 or 2");
        if (np == 1) dgrad_tiles(std::integral_constant<int, 1>{});
        else if (np == 2) dgrad_tiles(std::integral_constant<int, 2>{});
      }
    }
    __syncthreads();
    if (t < 4) stamp(3 + 3 * t);

    // ---- phase C: conv1 wgrad  dW1[n][kh][kw] += sum_pos dY1[pos][n] * xpad[pos + kh * 32 + kw]
    //      K = positions 0..927 (28 image rows + the zero row 28 that row-shifted A rows need), chunks split
    //      round-robin over the NW waves (own accumulator each, summed in a fixed order after the loop)
    {
      constexpr int CCH = 928 / KC, CPW = CCH / NW;  // chunks per wave: CPW, + 1 on waves < CCH % NW
      if (!ABLATED(cb.ablate, 512)) {
        auto ld_a = [&](int kc) { return M::load(dy1t + c_aoff + kc * KC + grp * KV); };
        auto ld_b = [&](int kc) { return M::load(xs + c_boff + kc * KC + grp * KV); };
        Frag a = ld_a(w), bx = ld_b(w);
#pragma unroll
        for (int j = 0; j < CPW; ++j) {
          Frag an = a, bn = bx;
          if (j + 1 < CPW || w < CCH % NW) {
            const int kn = w + NW * (j + 1);
            an = ld_a(kn);
            bn = ld_b(kn);
          }
          M::mma(accW1, a, bx);
          a = an; bx = bn;
        }
        if (w < CCH % NW) M::mma(accW1, a, bx);
      }
      __syncthreads();
      if (t < 4) stamp(4 + 3 * t);
    }
  }
  stamp(14);

  // ---- write this workgroup's partial gradients (slab row = unit): assembled in LDS (the P1T region, dead after
  //      the image loop), then written as whole 16-byte vectors -- 643 coalesced stores instead of 2572 scattered
  //      4-byte ones
  static_assert(L::CONV_PARAMS % 4 == 0 && L::CONV_PARAMS * 4 <= 32 * S::P1P * (int)sizeof(T), "slab row staging");
  float* srow = reinterpret_cast<float*>(smem + S::OFF_P1T);
  float* out = srow;
#pragma unroll
  for (int i = 0; i < NWT; ++i) {
    if (i >= nw) break;
    const int kcol = (n0w + i) * 16 + row, tap = kcol / 6, c = kcol - 6 * tap;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int n = grp * 4 + r;
      if (kcol < 150) out[L::CW2 + n * 150 + c * 25 + tap] = accW2[i][r];
      else if (kcol == 150) out[L::CB2 + n] = accW2[i][r];
    }
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) red[w * 256 + (grp * 4 + i) * 16 + row] = accW1[i];
  __syncthreads();
  if (tid < 256) {
    const int m = tid >> 4, j = tid & 15;  // C row m = (r, n), column j = (khb, kw) | bias
    float v;
    if constexpr (NW == 8)
      v = ((red[0 * 256 + tid] + red[1 * 256 + tid]) + (red[2 * 256 + tid] + red[3 * 256 + tid])) +
          ((red[4 * 256 + tid] + red[5 * 256 + tid]) + (red[6 * 256 + tid] + red[7 * 256 + tid]));
    else
      v = (red[0 * 256 + tid] + red[1 * 256 + tid]) + (red[2 * 256 + tid] + red[3 * 256 + tid]);
    const int r = C_AMAP[m] >> 3, n = C_AMAP[m] & 7, bj = C_BMAP[j];
    if (n < 6) {
      if (bj == 15) {
        if (r == 0) out[L::CB1 + n] = v;
      } else {
        const int kh = 2 * (bj / 5) + r, kw = bj % 5;
        if (kh <= 4) out[L::CW1 + n * 25 + kh * 5 + kw] = v;
      }
    }
  }
  __syncthreads();
  {
    uint4* dst = reinterpret_cast<uint4*>(cb.slab + (size_t)unit * L::CONV_PARAMS);
    const uint4* src = reinterpret_cast<const uint4*>(srow);
    for (int e = tid; e < L::CONV_PARAMS / 4; e += NT) dst[e] = src[e];
  }
  stamp(15);
  // this block's hardware location, in its own row range (cb.stamps starts at STAMP_CONV_BWD)
  if (cb.stamps && tid == 0 && blk < 512)
    cb.stamps[(STAMP_BWD_HWLOC - STAMP_CONV_BWD + blk) * 16] = hw_location();
}

template <typename T, int NW>
__global__ __launch_bounds__(NW * 64) __attribute__((amdgpu_waves_per_eu(NW == 8 ? 4 : 1)))
void conv_bwd_kernel(BatchRef br, LenetConvBuffers cb, int ipb) {
  conv_bwd_block<T, NW>(br, cb, ipb, blockIdx.x, gridDim.x);
}

// Small batches, one GPU, one FC batch split: conv_bwd and the FC weight gradient + SGD update (wg::
// wgrad_sgd_tile, the wgrad_sgd_kernel body) in ONE launch -- workgroups [0, nconv) are conv_bwd's, the rest
// one 32x32 FC output tile each (waves 4.. of a wider workgroup idle).  The two touch disjoint data (FC
// operands and FC parameters / images vs the conv ones), as in the concurrent two-stream schedule, so this is
// that schedule without the fork / join: the serial small-batch chain loses a kernel boundary and the FC
// update runs in conv_bwd's shadow.  The step counters are bumped by the conv update that follows.
template <typename T, int NW>
__global__ __launch_bounds__(NW * 64) __attribute__((amdgpu_waves_per_eu(NW == 8 ? 4 : 1)))
void conv_bwd_fc_kernel(BatchRef br, LenetConvBuffers cb, int ipb, int nconv, wg::WgArgs<T> fa) {
  if ((int)blockIdx.x < nconv) {
    conv_bwd_block<T, NW>(br, cb, ipb, blockIdx.x, nconv);
  } else if (threadIdx.x < 256) {
    wg::wgrad_sgd_tile<T, LenetModel>(fa, (int)blockIdx.x - nconv);
  }
}

}  // namespace

static int fwd_ipb(int B) { return std::min(MAX_IPB, std::max(1, (B + 1023) / 1024)); }
// default conv_bwd workgroup target: 512 = one full round of 2 blocks/CU (1024 / 768 measured slower)
static int default_bwd_target() { return 512; }

static int bwd_ipb(int B, int target) {
  const int div = target > 0 ? target : default_bwd_target();
  return std::min(MAX_IPB, std::max(1, (B + div - 1) / div));
}

int lenet_conv_bwd_blocks(int B, int target) {
  const int ipb = bwd_ipb(B, target);
  return (B + ipb - 1) / ipb;
}

// Upper bound of lenet_conv_bwd_blocks(b, target) over every b <= B (partial last batches included):
// ceil(b / ceil(b / t)) <= min(b, t).  Size the conv slab with this, not with the full-batch grid.
int lenet_conv_bwd_max_blocks(int B, int target) {
  // MAX_IPB caps the images per workgroup, so huge batches use more than `target` workgroups
  return std::max({1, std::min(B, target > 0 ? target : default_bwd_target()), (B + MAX_IPB - 1) / MAX_IPB});
}

void launch_lenet_conv_fwd(DType t, bool train, const BatchRef& br, const LenetConvBuffers& cb, hipStream_t s) {
  if (br.B <= 0) return;
  const int ipb = fwd_ipb(br.B), grid = (br.B + ipb - 1) / ipb;
  // fp32 training conv_fwd on 8 waves: LeNet fp32 B=8192 0.4331-0.4339 vs 0.4380-0.4392 ms with 4, B=128 47.0 vs
  // 47.9 us, bitwise-equal parameters (profiles/r4_session2/ab_conv_fwd_f32_8waves.txt)
  constexpr int FNW = 8;
  if (t == DType::F32) {
    if (train) hipLaunchKernelGGL((conv_fwd_kernel<float, true, FNW>), dim3(grid), dim3(FNW * 64), 0, s, br, cb, ipb);
    else hipLaunchKernelGGL((conv_fwd_kernel<float, false>), dim3(grid), dim3(256), 0, s, br, cb, ipb);
  } else {
    if (train) hipLaunchKernelGGL((conv_fwd_kernel<bf16, true>), dim3(grid), dim3(256), 0, s, br, cb, ipb);
    else hipLaunchKernelGGL((conv_fwd_kernel<bf16, false>), dim3(grid), dim3(256), 0, s, br, cb, ipb);
  }
}

bool lenet_fwd_head_applies(DType t, int B) {
  // (the start-up calibration also times the separate conv_fwd + head kernels: Trainer::set_fwd_head)
  return t == DType::BF16 && B >= FH_MIN_B && (B & 15) == 0;
}

int launch_lenet_fwd_head(DType t, const BatchRef& br, const LenetConvBuffers& cb, const HeadBuffers& hb, hipStream_t s) {
  if (!lenet_fwd_head_applies(t, br.B)) return 0;
  const int grid = br.B / 16;
  hipLaunchKernelGGL(fwd_head_kernel<bf16>, dim3(grid), dim3(512), 0, s, br, cb, hb);
  return 32;
}

int launch_lenet_head16(DType t, const BatchRef& br, const HeadBuffers& hb, hipStream_t s) {
  constexpr int maxb = 2048;  // largest batch for head16_kernel (the LDS-staged head_kernel above it)
  if (t != DType::BF16 || br.B <= 0 || br.B > maxb) return 0;
  const int grid = (br.B + 15) / 16;
  hipLaunchKernelGGL(head16_kernel<bf16>, dim3(grid), dim3(512), 0, s, br, hb);
  return (grid % 8 == 0 && br.B % 32 == 0) ? 32 : 16;  // wgrad XCD mapping: as launch_lenet_fwd_head
}

void launch_lenet_conv_bwd(DType t, const BatchRef& br, const LenetConvBuffers& cb, int* nslab_out, hipStream_t s,
                           int target_blocks) {
  const int ipb = bwd_ipb(br.B, target_blocks), grid = (br.B + ipb - 1) / ipb;
  if (nslab_out) *nslab_out = grid;
  if (br.B <= 0) return;
  // Waves per workgroup (BwdRoles): fp32 -- 150 KB of LDS, one workgroup per CU -- runs 8 waves (0.440 vs
  // 0.478 ms per LeNet fp32 B=8192 step, same box); bf16 keeps 4 (two workgroups per CU: 8 waves would take
  // every VGPR of the SIMDs and starve the FC weight gradient that runs beside conv_bwd, 0.119-0.127 vs 0.103 ms;
  // round 6 timed 8 waves in every single-GPU schedule, serial included, same box: concurrent 0.1135 / serial 0.1147
  // / separate 0.1067 vs 4 waves 0.1068 / 0.1091 / 0.1009 ms, profiles/r6_session1/NOTES.md)
  if (t == DType::F32) hipLaunchKernelGGL((conv_bwd_kernel<float, 8>), dim3(grid), dim3(512), 0, s, br, cb, ipb);
  else hipLaunchKernelGGL((conv_bwd_kernel<bf16, 4>), dim3(grid), dim3(256), 0, s, br, cb, ipb);
}

int launch_lenet_conv_bwd_fc(DType t, const BatchRef& br, const LenetConvBuffers& cb, const HeadBuffers& hb,
                             const SgdFuse& fuse, hipStream_t s, int target_blocks) {
  const int ipb = bwd_ipb(br.B, target_blocks), nconv = (br.B + ipb - 1) / ipb;
  if (br.B <= 0) return nconv;
  int splits = 1, nfc = 0;
  if (t == DType::F32) {
    const auto fa = wg::make_args<float, LenetModel::Head, LenetModel>(hb, br.B, splits, nullptr, 0, &fuse, 7, &nfc);
    hipLaunchKernelGGL((conv_bwd_fc_kernel<float, 8>), dim3(nconv + nfc), dim3(512), 0, s, br, cb, ipb, nconv, fa);
  } else {
    const auto fa = wg::make_args<bf16, LenetModel::Head, LenetModel>(hb, br.B, splits, nullptr, 0, &fuse, 7, &nfc);
    hipLaunchKernelGGL((conv_bwd_fc_kernel<bf16, 4>), dim3(nconv + nfc), dim3(256), 0, s, br, cb, ipb, nconv, fa);
  }
  return nconv;
}
