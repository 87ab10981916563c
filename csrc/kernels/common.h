// Shared CDNA4 (gfx950) primitives for the MNIST training kernels.
//
// Every GEMM-shaped product in this framework is issued on the matrix cores with
// the 16x16 MFMA family, one 64-lane wave per 16x16 output tile:
//   fp32 path : v_mfma_f32_16x16x4_f32   (exact f32 products, K = 4 per instruction)
//   bf16 path : v_mfma_f32_16x16x32_bf16 (K = 32 per instruction), f32 accumulate
// To write the kernels once for both, a "K-chunk" abstraction is used: in a chunk
// every lane supplies KV *contiguous* k-elements of its A row / B column
//   lane l : row/col = l & 15, k in [ (l>>4)*KV , (l>>4)*KV + KV )
// bf16: KV = 8 -> one 16x16x32 MFMA.  fp32: KV = 4 -> four 16x16x4 MFMAs where
// instruction i consumes element i of every lane (k-slot g of lane group g is
// k = 4g+i); A and B use the same permutation, so the chunk sum is exact.
// Contiguous-k fragments mean every operand fetch is one vector load
// (16 B for bf16, 16 B for fp32) from LDS or global memory.
// C/D layout (dtype independent on gfx950): col = lane & 15, row = (lane>>4)*4 + i.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2;
typedef __attribute__((ext_vector_type(4))) unsigned u32x4;
typedef __attribute__((ext_vector_type(2))) unsigned u32x2;
typedef __bf16 bf16;

#define DEV __device__ __forceinline__

constexpr int WAVE = 64;

template <typename T> struct Mma;

template <> struct Mma<float> {
  static constexpr int KV = 4;    // contiguous k per lane per chunk
  static constexpr int KC = 16;   // k per chunk
  struct Frag { f32x4 v; };
  // EXACT cut of an fp32 fragment into three bf16 parts by truncation: hi = the top 8 significant bits, mid = the top 8
  // of the exact remainder, lo = the rest (at most 8 significant bits, so a bf16 value): x == hi + mid + lo.  Packed
  // as u32x2 (4 bf16, element 2j in bits [15:0]).
  static DEV void split3(const f32x4 x, u32x2& h, u32x2& m, u32x2& l) {
    const u32x4 xb = __builtin_bit_cast(u32x4, x);
    const u32x4 hb = xb & 0xFFFF0000u;
    const f32x4 r1 = x - __builtin_bit_cast(f32x4, hb);  // exact
    const u32x4 r1b = __builtin_bit_cast(u32x4, r1);
    const u32x4 mb = r1b & 0xFFFF0000u;
    const f32x4 r2 = r1 - __builtin_bit_cast(f32x4, mb);  // exact, low 16 bits zero
    const u32x4 lb = __builtin_bit_cast(u32x4, r2);
    h = u32x2{__builtin_amdgcn_perm(xb[1], xb[0], 0x07060302u), __builtin_amdgcn_perm(xb[3], xb[2], 0x07060302u)};
    m = u32x2{__builtin_amdgcn_perm(r1b[1], r1b[0], 0x07060302u), __builtin_amdgcn_perm(r1b[3], r1b[2], 0x07060302u)};
    l = u32x2{__builtin_amdgcn_perm(lb[1], lb[0], 0x07060302u), __builtin_amdgcn_perm(lb[3], lb[2], 0x07060302u)};
  }
  static DEV bf16x8 cat(const u32x2 p, const u32x2 q) { return __builtin_bit_cast(bf16x8, u32x4{p[0], p[1], q[0], q[1]}); }
  // a (cut here) times b given as its three bf16 parts: the six products of weight >= 2^-16 of (hi + mid + lo)^2
  // on THREE v_mfma_f32_16x16x32_bf16 -- the 32-slot MFMA sums all 8 k-slots of a lane, so a lane's slots carry two
  // parts of its 4 k-elements: [ah | al] . [bl | bh], [ah | am] . [bm | bm], [ah | am] . [bh | bh] (smallest first).
  // ~2^-24 relative error, 3 x 16 = 48 cycles per 16-k chunk against 4 x 32 = 128 for v_mfma_f32_16x16x4_f32
  // (MI355X_MICROARCH.md cycle table; scripts/diag/mfma_rate.hip).
  static DEV void mma_psb(f32x4& acc, const Frag& a, const u32x2 bh, const u32x2 bm, const u32x2 bl) {
    u32x2 ah, am, al;
    split3(a.v, ah, am, al);
    mma_pp(acc, ah, am, al, bh, bm, bl);
  }
  // both operands given as their three parts (pre-split operand images: no cut at use)
  static DEV void mma_pp(f32x4& acc, const u32x2 ah, const u32x2 am, const u32x2 al, const u32x2 bh, const u32x2 bm,
                         const u32x2 bl) {
    const bf16x8 ahm = cat(ah, am);
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(cat(ah, al), cat(bl, bh), acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ahm, cat(bm, bm), acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ahm, cat(bh, bh), acc, 0, 0, 0);
  }
  // the three parts of one fp32 value as bf16 bit patterns (the scalar split3, for pre-split operand images)
  static DEV void split3_1(const float x, uint16_t& h, uint16_t& m, uint16_t& l) {
    const uint32_t xb = __float_as_uint(x);
    const float r1 = x - __uint_as_float(xb & 0xFFFF0000u);  // exact
    const uint32_t r1b = __float_as_uint(r1);
    const float r2 = r1 - __uint_as_float(r1b & 0xFFFF0000u);  // exact, low 16 bits zero
    h = (uint16_t)(xb >> 16);
    m = (uint16_t)(r1b >> 16);
    l = (uint16_t)(__float_as_uint(r2) >> 16);
  }
  // both operands cut here (the compiler hoists the cut of a loop-invariant b)
  static DEV void mma_s(f32x4& acc, const Frag& a, const Frag& b) {
    u32x2 bh, bm, bl;
    split3(b.v, bh, bm, bl);
    mma_psb(acc, a, bh, bm, bl);
  }
#ifndef MNIST_AMD_F32_SPLIT
  static DEV void mma(f32x4& acc, const Frag& a, const Frag& b) {
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.v[0], b.v[0], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.v[1], b.v[1], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.v[2], b.v[2], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.v[3], b.v[3], acc, 0, 0, 0);
  }
#else
  // Opt-in build (-DMNIST_AMD_F32_SPLIT): each fp32 operand EXACTLY as hi + mid + lo, three bf16 parts cut by
  // truncation (hi = the top 8 significant bits, mid = the top 8 of the exact remainder, lo = the rest, which has
  // at most 8 significant bits and so is a bf16 value), and the six products of weight >= 2^-16 of
  // (hi + mid + lo)^2 -- ~2^-24 relative error, fp32-like -- on THREE v_mfma_f32_16x16x32_bf16 per K-chunk:
  // the 32-slot MFMA sums all 8 k-slots of a lane, so a lane's slots carry two parts of its 4 k-elements
  // ([ah | am] . [bh | bh], [ah | am] . [bm | bm], [ah | al] . [bl | bh]).  3 x 16 = 48 cycles per chunk against
  // 4 x 32 = 128 for the exact v_mfma_f32_16x16x4_f32 (MI355X_MICROARCH.md cycle table); the split is VALU work
  // (and / sub / perm, ~18 instructions per 4-element fragment) paid per fragment use, hoisted by the compiler
  // for loop-invariant operands.  (Round 4's rounded 3-part split on six 16x16x16 MFMAs: 40 % slower than exact;
  // profiles/r4_session2/NOTES.md.)  Measured (profiles/r5_session1/f32split): passes every fp32 tolerance test;
  // conv_fwd -7 %, but conv_bwd +13 % (its streamed operands are re-split every chunk: the VALU cost equals the
  // MFMA saving) -> LeNet fp32 4-14 % slower, MLP fp32 B=8192 9 % faster.  Not the default.
  static DEV void mma(f32x4& acc, const Frag& a, const Frag& b) { mma_s(acc, a, b); }
#endif
  static DEV Frag load(const float* p) { Frag f; f.v = *reinterpret_cast<const f32x4*>(p); return f; }
  static DEV Frag zero() { Frag f; f.v = f32x4{0.f, 0.f, 0.f, 0.f}; return f; }
  static DEV void set(Frag& f, int j, float x) { f.v[j] = x; }
  static DEV float get(const Frag& f, int j) { return f.v[j]; }
};

template <> struct Mma<bf16> {
  static constexpr int KV = 8;
  static constexpr int KC = 32;
  struct Frag { bf16x8 v; };
  static DEV void mma(f32x4& acc, const Frag& a, const Frag& b) {
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.v, b.v, acc, 0, 0, 0);
  }
  static DEV Frag load(const bf16* p) { Frag f; f.v = *reinterpret_cast<const bf16x8*>(p); return f; }
  // a fragment at an 8-byte (not 16-byte) aligned address: two 8-byte reads (a 16-byte read would be under-aligned)
  static DEV Frag load8(const bf16* p) {
    const u32x2 lo = *reinterpret_cast<const u32x2*>(p), hi = *reinterpret_cast<const u32x2*>(p + 4);
    Frag f;
    f.v = __builtin_bit_cast(bf16x8, u32x4{lo[0], lo[1], hi[0], hi[1]});
    return f;
  }
  static DEV Frag zero() {
    Frag f;
    for (int j = 0; j < 8; ++j) f.v[j] = (bf16)0.f;
    return f;
  }
  static DEV void set(Frag& f, int j, float x) { f.v[j] = (bf16)x; }
  static DEV float get(const Frag& f, int j) { return (float)f.v[j]; }
};

// Streaming (non-temporal) global stores for kernel outputs that only a LATER kernel reads: they are not
// kept dirty in this XCD's L2, so the end-of-kernel L2 write-back (cross-XCD coherence at the kernel
// boundary) has less to flush before the next kernel may start.
#ifndef MNIST_NT_STORES
#define MNIST_NT_STORES 1
#endif
template <typename V>
DEV void st_stream(V* p, const V& v) {
#if MNIST_NT_STORES
  __builtin_nontemporal_store(v, p);
#else
  *p = v;
#endif
}
DEV void st_stream16(void* p, const uint4& v) { st_stream(reinterpret_cast<u32x4*>(p), u32x4{v.x, v.y, v.z, v.w}); }

template <typename T> DEV T to_t(float x) { return (T)x; }
template <typename T> DEV float to_f(T x) { return (float)x; }

// s_waitcnt vmcnt(0) (expcnt / lgkmcnt left at their maxima; gfx9 encoding).  Placed after loads of
// loop-invariant operands and before the loop: the wait-insertion pass cannot prove across the loop's
// back edge that such registers have arrived, so without it every use inside the loop gets a
// vmcnt(N) that -- in-order counting -- also waits for the loop's own prefetch loads.
DEV void wait_vm_all() { __builtin_amdgcn_s_waitcnt(0x0F70); }

// Where this wave runs (profiling stamps): XCC id << 32 | HW_ID (cu [11:8], sh [12], se [15:13], simd [5:4]).
// s_getreg reads of HW_REG_HW_ID (4) and HW_REG_XCC_ID (20), full width.
DEV unsigned long long hw_location() {
  const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);
  const unsigned xcc = __builtin_amdgcn_s_getreg((15 << 11) | 20);
  return ((unsigned long long)(xcc & 15u) << 32) | hw;
}

// Workgroups are dispatched round-robin over the 8 XCDs (workgroup g runs on XCD g % 8, each XCD with its
// own L2).  xcd_unit maps g to the logical work unit (g % 8) * (grid / 8) + g / 8, so XCD x owns the
// contiguous units [x * grid / 8, (x + 1) * grid / 8): with the same mapping in consecutive kernels, the
// rows one kernel writes on an XCD are read by the next kernel on that XCD (L2 hits instead of MALL /
// HBM after the kernel-boundary write-back).  A bijection of [0, grid); identity when grid % 8 != 0.
DEV int xcd_unit(int g, int grid, int on) { return (on && (grid & 7) == 0) ? (g & 7) * (grid >> 3) + (g >> 3) : g; }

// 16-bit halves of two dwords packed into one (v_perm_b32): lo16 = a[15:0] | b[15:0] << 16, hi16 = a[31:16] | b[31:16] << 16
DEV uint32_t pack_lo16(uint32_t a, uint32_t b) { return __builtin_amdgcn_perm(b, a, 0x05040100u); }
DEV uint32_t pack_hi16(uint32_t a, uint32_t b) { return __builtin_amdgcn_perm(b, a, 0x07060302u); }
DEV uint32_t pack_half16(uint32_t a, uint32_t b, int hi) { return hi ? pack_hi16(a, b) : pack_lo16(a, b); }

DEV int lane_id() { return threadIdx.x & 63; }
DEV int wave_id() { return __builtin_amdgcn_readfirstlane(threadIdx.x >> 6); }

DEV f32x4 zero4() { return f32x4{0.f, 0.f, 0.f, 0.f}; }

// Counter-based hash RNG (dropout): a stateless 32-bit mix of (seed, stream, a, b).
DEV uint32_t hash4(uint32_t seed, uint32_t s, uint32_t a, uint32_t b) {
  uint32_t h = seed ^ 0x9E3779B9u;
  h ^= s * 0x85EBCA6Bu; h = (h << 13) | (h >> 19); h = h * 5u + 0xE6546B64u;
  h ^= a * 0xC2B2AE35u; h = (h << 13) | (h >> 19); h = h * 5u + 0xE6546B64u;
  h ^= b * 0x27D4EB2Fu; h = (h << 13) | (h >> 19); h = h * 5u + 0xE6546B64u;
  h ^= h >> 16; h *= 0x85EBCA6Bu; h ^= h >> 13; h *= 0xC2B2AE35u; h ^= h >> 16;
  return h;
}

// MNIST normalisation of ToTensor()+Normalize((0.1307,),(0.3081,)) (ddp_tutorial_cpu.py:13-16), folded into ONE fma
// (x / 255 - 0.1307) / 0.3081 = x * A + B (A, B rounded once from double): v_cvt_f32_ubyte + v_fma per pixel instead of
// cvt + mul + sub + mul -- the per-pixel staging is on the VALU-issue-bound image loops of conv_fwd / conv_bwd / the MLP
// head (within 1 ulp of the three-step form; the reference's own ToTensor + Normalize is not bit-reproduced either way)
constexpr float MNIST_NORM_A = (float)(1.0 / (255.0 * 0.3081));
constexpr float MNIST_NORM_B = (float)(-0.1307 / 0.3081);
DEV float mnist_norm(uint32_t u8) { return __builtin_fmaf(float(u8), MNIST_NORM_A, MNIST_NORM_B); }

DEV int round_up(int x, int m) { return (x + m - 1) / m * m; }

// wave-level reductions (64 lanes)
// DPP lane exchanges inside a 16-lane row (a few cycles each; __shfl_xor is a ds_bpermute through the
// LDS crossbar, ~100 cycles).  Butterfly for row reductions: quad xor 1, quad xor 2, half-row mirror,
// row mirror -- every lane of the row ends with the same (commutatively combined) value.
template <int CTRL>
DEV int dpp_i(int v) { return __builtin_amdgcn_update_dpp(0, v, CTRL, 0xF, 0xF, false); }
template <int CTRL>
DEV float dpp_f(float v) { return __builtin_bit_cast(float, dpp_i<CTRL>(__builtin_bit_cast(int, v))); }
constexpr int DPP_QXOR1 = 0xB1, DPP_QXOR2 = 0x4E, DPP_HMIRROR = 0x141, DPP_MIRROR = 0x140;

DEV float row16_max(float v) {
  v = fmaxf(v, dpp_f<DPP_QXOR1>(v));
  v = fmaxf(v, dpp_f<DPP_QXOR2>(v));
  v = fmaxf(v, dpp_f<DPP_HMIRROR>(v));
  return fmaxf(v, dpp_f<DPP_MIRROR>(v));
}
DEV float row16_sum(float v) {
  v += dpp_f<DPP_QXOR1>(v);
  v += dpp_f<DPP_QXOR2>(v);
  v += dpp_f<DPP_HMIRROR>(v);
  return v + dpp_f<DPP_MIRROR>(v);
}
DEV int row16_min(int v) {
  v = min(v, dpp_i<DPP_QXOR1>(v));
  v = min(v, dpp_i<DPP_QXOR2>(v));
  v = min(v, dpp_i<DPP_HMIRROR>(v));
  return min(v, dpp_i<DPP_MIRROR>(v));
}

DEV float lane_f(float v, int l) {
  return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), l));
}

// sum over the 64 lanes (every lane active); the result is wave-uniform
DEV float wave_sum(float v) {
  v = row16_sum(v);
  return (lane_f(v, 0) + lane_f(v, 16)) + (lane_f(v, 32) + lane_f(v, 48));
}
