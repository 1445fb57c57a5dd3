// Device-side helpers shared by the gfx950 kernels: 64-lane wave MFMA
// fragments, bf16 <-> f32, 16-byte vector moves.
//
// Operand maps (cdna_hip_programming.md §3), lane l, g = l >> 4, r = l & 15:
//   v_mfma_f32_16x16x32_bf16 : A[r][8g+j], B[8g+j][r], j = 0..7
//   C/D                      : C[4g+i][r], i = 0..3
// The f32 path runs the same 32-deep K chunk as eight v_mfma_f32_16x16x4_f32
// with element j of every lane fragment in instruction j; that permutes K
// identically for A and B, so the sum is the same and both dtypes share one
// fragment layout (8 consecutive K per lane).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace mcc {
namespace gpu {

typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x8 __attribute__((ext_vector_type(8)));

template <typename T> struct Vec8;
template <> struct Vec8<bf16> { typedef bf16x8 type; };
template <> struct Vec8<float> { typedef f32x8 type; };

__device__ __forceinline__ float to_f(float x) { return x; }
__device__ __forceinline__ float to_f(bf16 x) { return (float)x; }
template <typename T> __device__ __forceinline__ T from_f(float x) { return (T)x; }

// 8 consecutive elements, 16-byte aligned for bf16, 32-byte for f32.
__device__ __forceinline__ bf16x8 load8(const bf16* p) { return *reinterpret_cast<const bf16x8*>(p); }
__device__ __forceinline__ void store8(bf16* p, const bf16x8& v) { *reinterpret_cast<bf16x8*>(p) = v; }
// f32: two 16-byte moves (only 16-byte alignment is guaranteed).
__device__ __forceinline__ f32x8 load8(const float* p) {
  const f32x4 a = *reinterpret_cast<const f32x4*>(p);
  const f32x4 b = *reinterpret_cast<const f32x4*>(p + 4);
  return __builtin_shufflevector(a, b, 0, 1, 2, 3, 4, 5, 6, 7);
}
__device__ __forceinline__ void store8(float* p, const f32x8& v) {
  *reinterpret_cast<f32x4*>(p) = __builtin_shufflevector(v, v, 0, 1, 2, 3);
  *reinterpret_cast<f32x4*>(p + 4) = __builtin_shufflevector(v, v, 4, 5, 6, 7);
}

__device__ __forceinline__ f32x4 mma(f32x4 acc, const bf16x8& a, const bf16x8& b) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc, 0, 0, 0);
}
__device__ __forceinline__ f32x4 mma(f32x4 acc, const f32x8& a, const f32x8& b) {
#pragma unroll
  for (int j = 0; j < 8; ++j) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[j], b[j], acc, 0, 0, 0);
  return acc;
}

__device__ __forceinline__ float act_apply(int act, float v) {
  if (act == 1) return v > 0.f ? v : 0.f;
  if (act == 2) return tanhf(v);
  return v;
}
// compile-time activation: with_act(p.act, [&](auto a) { ... act_c<a.v>(x) ... })
// branches once on the uniform kind instead of once per element (an unrolled
// 128-value epilogue otherwise carries a tanh path and two scalar branches per
// value)
template <int A> struct ActK { static constexpr int v = A; };
template <int A> __device__ __forceinline__ float act_c(float v) {
  if constexpr (A == 1) return __builtin_bit_cast(float, max(__builtin_bit_cast(int, v), 0));  // ReLU (-0 -> +0)
  else if constexpr (A == 2) return tanhf(v);
  else return v;
}
template <class F> __device__ __forceinline__ void with_act(int act, F&& f) {
  if (act == 1) f(ActK<1>{});
  else if (act == 2) f(ActK<2>{});
  else f(ActK<0>{});
}
__device__ __forceinline__ bf16x4 cvt4(float a, float b, float c, float d) {
  using f2 = float __attribute__((ext_vector_type(2)));
  using h2 = bf16 __attribute__((ext_vector_type(2)));
  const h2 lo = __builtin_convertvector(f2{a, b}, h2), hi = __builtin_convertvector(f2{c, d}, h2);
  return bf16x4{lo[0], lo[1], hi[0], hi[1]};
}
// derivative expressed in the activation output y
__device__ __forceinline__ float act_grad_y(int act, float y) {
  if (act == 1) return y > 0.f ? 1.f : 0.f;
  if (act == 2) return 1.f - y * y;
  return 1.f;
}

__host__ __device__ __forceinline__ int cdiv(int a, int b) { return (a + b - 1) / b; }

__host__ __device__ __forceinline__ int align16(int bytes) { return (bytes + 15) & ~15; }

// Exact n / d for n < 2^24, d <= 2^16 via a multiply-high:
// m = ceil(2^40 / d); the error term n*(m - 2^40/d)/2^40 < 2^-16 <= 1/d.
// m = mh*2^32 + ml (mh <= 256), so n*m >> 40 = (n*mh + umulhi(n, ml)) >> 8
// with every partial in 32 bits (3 VALU).  The constructor avoids a 64-bit
// integer division (a ~100-instruction software routine): a double
// reciprocal estimate, then an exact integer fix-up.  Construct divisors
// once per kernel, outside stage loops.
struct Div {
  uint32_t mh, ml;
  Div() = default;
  // host-side magic (exact 64-bit arithmetic); pass through kernel params
  static __host__ Div host(int d) {
    Div r;
    const uint64_t dd = (uint64_t)(d > 0 ? d : 1);
    const uint64_t q = ((1ull << 40) + dd - 1) / dd;
    r.mh = (uint32_t)(q >> 32);
    r.ml = (uint32_t)q;
    return r;
  }
  __device__ __forceinline__ explicit Div(int d) {
    constexpr uint64_t P = 1ull << 40;
    const uint64_t dd = (uint64_t)(d > 0 ? d : 1);
    uint64_t q = (uint64_t)(1099511627776.0 / (double)dd);
    while (q * dd < P) ++q;
    while ((q - 1) * dd >= P) --q;
    mh = (uint32_t)(q >> 32);
    ml = (uint32_t)q;
  }
  __device__ __forceinline__ int div(int n) const {
    const uint32_t u = (uint32_t)n;
    return (int)((u * mh + __umulhi(u, ml)) >> 8);
  }
};

typedef short v4s __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) v4s lds_v4s;

// ds_read_b64_tr_b16 (cdna_hip_programming.md §5.5 T10): each 16-lane group
// reads a 4-row x 16-column block of 16-bit elements; lane 4q+p supplies the
// address of row q, columns 4p..4p+3 (rows may be anywhere in LDS), lane i
// receives column i of the 4 rows.  One call = half an MFMA K-fragment.
__device__ __forceinline__ bf16x4 tr4(const bf16* p) {
  return __builtin_bit_cast(bf16x4, __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)(const_cast<bf16*>(p))));
}

// The same read as inline asm, for loops that keep LDS-DMA (global_load_lds)
// prefetches in flight: the compiler cannot disambiguate the builtin's LDS
// access from pending DMAs and puts an `s_waitcnt vmcnt(0)` in front of it,
// which drains the whole lookahead every step.  The asm result is NOT
// tracked: issue the reads, then lds_wait(...) before using them.
__device__ __forceinline__ bf16x4 tr4_async(const bf16* p) {
  v4s r;
  const uint32_t a = (uint32_t)(uintptr_t)((const __attribute__((address_space(3))) bf16*)(p));
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(r) : "v"(a));
  return __builtin_bit_cast(bf16x4, r);
}
// ... with a constant byte offset in the instruction (no v_add per read)
template <int OFF>
__device__ __forceinline__ bf16x4 tr4_async_at(const bf16* p) {
  static_assert(OFF >= 0 && OFF < 65536, "ds offset field");
  v4s r;
  const uint32_t a = (uint32_t)(uintptr_t)((const __attribute__((address_space(3))) bf16*)(p));
  asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(r) : "v"(a), "n"(OFF));
  return __builtin_bit_cast(bf16x4, r);
}
// wait for every outstanding LDS read and pin the given fragments after it
template <typename F>
__device__ __forceinline__ void lds_pin(F& f) { asm volatile("" : "+v"(f)); }
__device__ __forceinline__ void lds_wait() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }
template <typename F0, typename... F>
__device__ __forceinline__ void lds_wait(F0& f0, F&... f) {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  lds_pin(f0);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  (lds_pin(f), ...);
}

// Reductions over the four lanes r, r + 16, r + 32, r + 48 (one column of
// an MFMA C tile C[4g + i][r]: lenet_fc P3, the MFMA classifier head) on
// v_permlane16/32_swap (VALU) instead of __shfl_xor's ds_bpermute (an LDS
// round trip per step on the softmax's critical path).
// With both operands = x, the swap leaves {x of this lane's 16-row pair
// partner, own x} in the two results (in a lane-dependent order), so a
// commutative combine gives both lanes the same value, bit for bit what the
// xor-16 / xor-32 shuffle pair gave.
__device__ __forceinline__ float ubits(uint32_t u) { return __builtin_bit_cast(float, u); }
__device__ __forceinline__ uint32_t fbits(float f) { return __builtin_bit_cast(uint32_t, f); }
__device__ __forceinline__ float sum4lanes(float x) {
  const auto a = __builtin_amdgcn_permlane16_swap(fbits(x), fbits(x), false, false);
  x = ubits(a[0]) + ubits(a[1]);
  const auto b = __builtin_amdgcn_permlane32_swap(fbits(x), fbits(x), false, false);
  return ubits(b[0]) + ubits(b[1]);
}
// first max wins (cnn.c:508-513): the larger value, on ties the lower class
__device__ __forceinline__ void argmax4lanes(float& mx, int& am) {
#pragma unroll
  for (int step = 0; step < 2; ++step) {
    const auto v = step ? __builtin_amdgcn_permlane32_swap(fbits(mx), fbits(mx), false, false)
                        : __builtin_amdgcn_permlane16_swap(fbits(mx), fbits(mx), false, false);
    const auto i = step ? __builtin_amdgcn_permlane32_swap((uint32_t)am, (uint32_t)am, false, false)
                        : __builtin_amdgcn_permlane16_swap((uint32_t)am, (uint32_t)am, false, false);
    const float va = ubits(v[0]), vb = ubits(v[1]);
    const int ia = (int)i[0], ib = (int)i[1];
    const bool b_wins = vb > va || (vb == va && ib < ia);
    mx = b_wins ? vb : va;
    am = b_wins ? ib : ia;
  }
}

}  // namespace gpu
}  // namespace mcc
