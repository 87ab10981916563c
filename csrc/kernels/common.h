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
#ifndef MNIST_AMD_F32_SPLIT
  static DEV void mma(f32x4& acc, const Frag& a, const Frag& b) {
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.v[0], b.v[0], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.v[1], b.v[1], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.v[2], b.v[2], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.v[3], b.v[3], acc, 0, 0, 0);
  }
#else
  // Opt-in build (-DMNIST_AMD_F32_SPLIT): fp32 operands as 3 bf16 parts (hi = x rounded to bf16, then each exact
  // remainder rounded to bf16), the six products of weight >= 2^-16 of (hi + mid + lo)^2 on
  // v_mfma_f32_16x16x16_bf16, whose lane layout (4 contiguous k per lane, K = 16) is this chunk's: ~2^-24 relative
  // error (fp32-like; passes the fp32 tolerances) but 40 % SLOWER than the exact fp32 MFMAs, because the split is
  // VALU work paid per fragment use (profiles/r4_session2/NOTES.md).  Pre-split LDS operand images would remove that
  // cost but need 1.5x the fp32 images' LDS (conv_bwd fp32 already uses 150 KB of the 160 KB); not built.  (The
  // 2-part / truncated 3-term forms failed the tolerances and were removed in round 5.)
  typedef __attribute__((ext_vector_type(4))) short s16x4;
  // (whole vectors are bit-cast: hipcc (ROCm 7.2) lowered __builtin_bit_cast of an ext-vector ELEMENT --
  // x.y, x[j] -- to a read of element 0)
  static DEV s16x4 part(const f32x4 x, f32x4& rem) {  // x rounded to bf16; rem = x - that (exact)
    typedef __attribute__((ext_vector_type(4))) unsigned u4;
    typedef __attribute__((ext_vector_type(4))) unsigned short us4;
    bf16x4 h;
    h.x = (bf16)x.x;
    h.y = (bf16)x.y;
    h.z = (bf16)x.z;
    h.w = (bf16)x.w;
    const u4 hw = __builtin_convertvector(__builtin_bit_cast(us4, h), u4) << 16;  // h as fp32 bits
    rem = x - __builtin_bit_cast(f32x4, hw);
    return __builtin_bit_cast(s16x4, h);
  }
  static DEV f32x4 mf(const s16x4 a, const s16x4 b, f32x4 acc) {
    return __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a, b, acc, 0, 0, 0);
  }
  static DEV void mma(f32x4& acc, const Frag& a, const Frag& b) {
    f32x4 ra, rb, ra2, rb2;
    const s16x4 ah = part(a.v, ra), bh = part(b.v, rb);
    const s16x4 am = part(ra, ra2), bm = part(rb, rb2);
    const s16x4 al = part(ra2, ra), bl = part(rb2, rb);
    acc = mf(al, bh, acc);
    acc = mf(ah, bl, acc);
    acc = mf(am, bm, acc);
    acc = mf(am, bh, acc);
    acc = mf(ah, bm, acc);
    acc = mf(ah, bh, acc);
  }
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

// MNIST normalisation of ToTensor()+Normalize((0.1307,),(0.3081,)) (ddp_tutorial_cpu.py:13-16).
DEV float mnist_norm(uint32_t u8) { return (float(u8) * (1.0f / 255.0f) - 0.1307f) * (1.0f / 0.3081f); }

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
