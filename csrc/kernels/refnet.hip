// Conv block of the reference model (cnn.c:416-428) on gfx950:
//   conv1 1->16, 3x3, stride 2, pad 1, ReLU   (28x28 -> 14x14)
//   conv2 16->32, 3x3, stride 2, pad 1, ReLU  (14x14 -> 7x7)
// as one forward kernel and one fused backward kernel per image, replacing
// five generic launches (two pipelined convs forward; conv2 dW, a zero-
// inserted stride-2 conv2 dX and conv1 dW backward) whose 14x14x16 bf16
// intermediate (6.3 KB per image) crossed HBM four times per step.
//
// Reference semantics: Layer_feedForw_conv / Layer_feedBack_conv
// (/root/reference/cnn.c:175-247, with the D1 index bug fixed as in
// CUDAcnn.cu:167-195).
//
// One 64-lane wave per image, wave-private LDS, persistent grids; every
// GEMM is a 16x16x32 bf16 MFMA in the TRANSPOSED orientation (rows = output
// channels, columns = pixels), so an output lane holds 4 consecutive
// channels of one pixel and stores them as one 8-byte HWC write:
//  * forward: conv1 Y1^T = W1 . patches^T (9 taps in K, K padded to 32; raw
//    integer pixels, bias * 255 in the accumulator, / 255 at the end),
//    Y1 HWC in LDS; conv2 Y2^T = W2 . patches^T (K = 2 taps x 16 channels
//    per 32-chunk); Y2 stored NHWC straight from the accumulators.
//  * backward, per image: conv1 is RECOMPUTED (cheaper than storing and
//    re-reading Y1 through HBM), in the sub-pixel phase order of the conv2
//    data gradient so its ReLU mask sits in the same lanes;
//      conv2 dW = dZ2^T . patches(Y1)   (transposed LDS reads, bias as a
//        ones column),
//      conv2 dX by sub-pixel decomposition: output phase (y & 1, x & 1)
//        gets 1, 2, 2 or 4 taps, so 36 MFMAs instead of the 81 of a
//        zero-inserted (up-sampled) dZ2,
//      conv1 dW = dZ1^T . patches(X) over the column-parity planes of X.
//    dW / db accumulate in registers across the wave's images; one slab
//    per wave, reduced in a fixed order (deterministic).
#include "kernels.h"
#include "mfma.h"
#include "mcc/ab.h"

#include <algorithm>

// ref_bwd2 phase ablations (timing studies only; tools/build_variant.sh):
// 1 = wave 0 skips conv1 + dW2, 2 = wave 1 skips everything, 4 = wave 0 skips
// dW2, 8 = wave 1 skips conv1 dW
#ifndef MCC_REF_ABL
#define MCC_REF_ABL 0
#endif

namespace mcc {
namespace gpu {
namespace {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

constexpr int kImgPix = 784;
constexpr int kY2Elems = 49 * 32;

// ---- LDS (bytes) ----
// X as exact-integer bf16, two copies so every 4-pixel window read is 8-B
// aligned: copy 0 holds column c at element c + 1, copy 2 at c + 3; 30 rows
// (r = -1 .. 28) of 32 elements.
constexpr int kXPitch = 64;
constexpr int kXCopy = 30 * kXPitch;  // 1920
// forward
constexpr int kFX0 = 0, kFX2 = kXCopy;
// Y1 of the padded 15 x 15 grid (pad row / column 0) as 4 parity planes
// (yy & 1, xx & 1) x 2 channel halves x 8 x 8 pixels x 16 B: conv2 (stride 2)
// reads one plane per tap, so the 16 lanes of a b128 read take consecutive
// 16-byte slots (2-way only where a 7-pixel output row wraps) instead of 4
// slots of a 32-byte-pitch HWC image (4-way: 57 % of the kernel's LDS cycles
// were bank conflicts, profiles/lenet5_ref_pmc_r5.txt)
constexpr int kFY1 = 2 * kXCopy;        // 3840
constexpr int kFLds = kFY1 + 8 * 1024;  // 12032
__host__ __device__ constexpr int y1p_off(int yy, int xx, int half) {
  return (((((yy & 1) * 2 + (xx & 1)) * 2 + half) * 64 + (yy >> 1) * 8 + (xx >> 1)) * 16);
}
// backward
constexpr int kBX0 = 0, kBX2 = kXCopy;
constexpr int kBXc = 2 * kXCopy;          // 3840: X column-parity planes E / O / Os, 30 rows x 32 B
constexpr int kXcPlane = 30 * 32;         // 960
constexpr int kBDz2 = kBXc + 3 * kXcPlane;  // 6720: dZ2 HWC, 9 x 9 pixels (pads 7, 8) x 64 B
constexpr int kBY1 = kBDz2 + 81 * 64;     // 11904: Y1 HWC 15 x 15 x 32 B
constexpr int kBDz1 = kBY1 + 225 * 32;    // 19104: dZ1 HWC, 16 x 16 pixels x 32 B (rows / columns 14, 15 pads)
constexpr int kBOnes = kBDz1 + 256 * 32;  // 27296: 32 B of bf16 ones
constexpr int kBLds = kBOnes + 32;        // 27328

// per-wave slab: conv2 dW accumulators [2][10][4][64], conv1 dW [4][64]
constexpr int kSlabW2 = 2 * 10 * 4 * 64;  // 5120
constexpr int kSlab = kSlabW2 + 4 * 64;   // 5376
constexpr int kBwdGrid = 256 * 4;         // one wave per SIMD (~320 registers)

__device__ __forceinline__ void u8x4_ints(uint32_t w, uint32_t& lo, uint32_t& hi) {
  const uint32_t f0 = __builtin_bit_cast(uint32_t, (float)(w & 0xffu));
  const uint32_t f1 = __builtin_bit_cast(uint32_t, (float)((w >> 8) & 0xffu));
  const uint32_t f2 = __builtin_bit_cast(uint32_t, (float)((w >> 16) & 0xffu));
  const uint32_t f3 = __builtin_bit_cast(uint32_t, (float)(w >> 24));
  lo = __builtin_amdgcn_perm(f1, f0, 0x07060302u);
  hi = __builtin_amdgcn_perm(f3, f2, 0x07060302u);
}
__device__ __forceinline__ uint32_t from_left(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, true);
}
__device__ __forceinline__ uint32_t mid16(uint32_t a, uint32_t b) { return __builtin_amdgcn_alignbit(b, a, 16); }
#ifndef MCC_REF_FENCE
#define MCC_REF_FENCE 0
#endif
#if MCC_REF_FENCE
__device__ __forceinline__ void wave_lds_sync() { asm volatile("" ::: "memory"); }
#else
__device__ __forceinline__ void wave_lds_sync() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }
#endif
__device__ __forceinline__ bf16x8 tr8(const char* p0, const char* p1) {
  const bf16x4 a = tr4(reinterpret_cast<const bf16*>(p0));
  const bf16x4 b = tr4(reinterpret_cast<const bf16*>(p1));
  return __builtin_shufflevector(a, b, 0, 1, 2, 3, 4, 5, 6, 7);
}
__device__ __forceinline__ bf16x8 join(const bf16x4& a, const bf16x4& b) {
  return __builtin_shufflevector(a, b, 0, 1, 2, 3, 4, 5, 6, 7);
}
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
// two floats -> two bf16 (RNE) in one v_cvt_pk_bf16_f32
__device__ __forceinline__ uint32_t cvt2(float a, float b) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2{a, b}), bf16x2));
}
__device__ __forceinline__ u32x2 pack4(float a, float b, float c, float d) { return u32x2{cvt2(a, b), cvt2(c, d)}; }
// ReLU on the bit pattern (one v_max_i32, no NaN canonicalisation): negative
// values and -0 become +0, so a stored zero is always +0
__device__ __forceinline__ float relu(float v) { return __builtin_bit_cast(float, max(__builtin_bit_cast(int, v), 0)); }
// nonzero bits of four non-negative bf16 (two packed words): h + 0x7fff
// carries into bit 15 of its half iff h != 0, never across halves (h <= 0x7fc0)
__device__ __forceinline__ uint32_t nz4(u32x2 v) {
  const uint32_t t0 = v.x + 0x7fff7fffu, t1 = v.y + 0x7fff7fffu;
  return ((t0 >> 15) & 1u) | ((t0 >> 30) & 2u) | ((t1 >> 13) & 4u) | ((t1 >> 28) & 8u);
}

struct WaveIdx {
  int v = 0;
  __device__ __forceinline__ void load(const int32_t* idx, int first, int stride, int B, int k0) {
    const int i = first + (k0 + (int)(threadIdx.x & 63)) * stride;
    v = idx ? idx[min(i, B - 1)] : min(i, B - 1);
  }
  __device__ __forceinline__ int get(int k) const { return __builtin_amdgcn_readlane(v, k & 63); }
};

// conv1 A operand (W1 rows = output channels): K slot k = 8 kg + e holds
// tap (kh, kw) = (kg == 0 ? e >> 2 : 2, e & 3) for kg <= 1 (kw = 3 and the
// other slots zero) -- matching the patch fragments below.
__device__ __forceinline__ bf16x8 conv1_weights(const float* w1, int lane) {
  const int ci = lane & 15, kg = lane >> 4;
  bf16x8 w;
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const int kh = kg == 0 ? (e >> 2) : 2, kw = e & 3;
    const bool ok = kg <= 1 && kw < 3 && !(kg == 1 && e >= 4);
    w[e] = (bf16)(ok ? w1[ci * 9 + kh * 3 + kw] : 0.f);
  }
  return w;
}
// conv1 patch (B operand) of output pixel (y, x) for k-group kg: two
// 4-element row windows of the padded integer copy.
__device__ __forceinline__ int xwin(int x0, int x2, int y, int x, int kh) {
  return (x & 1 ? x2 + ((2 * y + kh) * 32 + 2 * x + 2) * 2 : x0 + ((2 * y + kh) * 32 + 2 * x) * 2);
}
__device__ __forceinline__ bf16x8 conv1_patch(const char* smem, int x0, int x2, int y, int x, int kg) {
  const bf16x4 a = *reinterpret_cast<const bf16x4*>(smem + xwin(x0, x2, y, x, kg == 0 ? 0 : 2));
  const bf16x4 b = *reinterpret_cast<const bf16x4*>(smem + xwin(x0, x2, y, x, 1));
  const bf16x4 z = {(bf16)0.f, (bf16)0.f, (bf16)0.f, (bf16)0.f};
  return kg == 0 ? join(a, b) : kg == 1 ? join(a, z) : join(z, z);
}

// Stage one u8 image (the words of lane (row r = 8 it + (lane >> 3), quad
// sk = lane & 7)) into the two integer copies; also the column-parity planes
// when xc >= 0.
__device__ __forceinline__ void stage_x(char* smem, int x0, int x2, int xc, const uint32_t (&xw)[4], int lane) {
  const int sk = lane & 7, srow = lane >> 3;
#pragma unroll
  for (int it = 0; it < 4; ++it) {
    const int r = it * 8 + srow;
    uint32_t lo, hi;
    u8x4_ints(xw[it], lo, hi);
    const uint32_t plo = from_left(lo), phi = from_left(hi);
    if (r < 28) {
      // copy 0: elements 4sk .. 4sk+3 = columns 4sk-1 .. 4sk+2
      *reinterpret_cast<u32x2*>(smem + x0 + (r + 1) * kXPitch + 8 * sk) = u32x2{mid16(phi, lo), mid16(lo, hi)};
      // copy 2: elements 4sk .. 4sk+3 = columns 4sk-3 .. 4sk
      *reinterpret_cast<u32x2*>(smem + x2 + (r + 1) * kXPitch + 8 * sk) = u32x2{mid16(plo, phi), mid16(phi, lo)};
      if (xc >= 0 && sk < 7) {
        char* row = smem + xc + (r + 1) * 32 + 4 * sk;
        *reinterpret_cast<uint32_t*>(row) = __builtin_amdgcn_perm(hi, lo, 0x05040100u);                 // E: cols 4sk, 4sk+2
        *reinterpret_cast<uint32_t*>(row + kXcPlane) = __builtin_amdgcn_perm(hi, lo, 0x07060302u);      // O: 4sk+1, 4sk+3
        *reinterpret_cast<uint32_t*>(row + 2 * kXcPlane) = __builtin_amdgcn_perm(lo, phi, 0x07060302u);  // Os: 4sk-1, 4sk+1
      }
    }
  }
}
__device__ __forceinline__ void load_x(uint32_t (&xw)[4], const uint8_t* xin, int lane) {
  const int sk = lane & 7, srow = lane >> 3;
#pragma unroll
  for (int it = 0; it < 4; ++it) {
    const int yy = it * 8 + srow;
    xw[it] = (yy < 28 && sk < 7) ? *reinterpret_cast<const uint32_t*>(xin + yy * 28 + sk * 4) : 0u;
  }
}
__device__ __forceinline__ void zero_lds(char* p, int bytes, int lane) {
  const u32x4 z = {0u, 0u, 0u, 0u};
  for (int i = lane * 16; i < bytes; i += 64 * 16) *reinterpret_cast<u32x4*>(p + i) = z;
}

// conv2 A operand (W2 rows = output channels co = 16 mt + m), chunk c:
// K slot 8 kg + e = tap 2c + (kg >> 1), input channel 8 (kg & 1) + e.
__device__ __forceinline__ bf16x8 conv2_weights(const float* w2, int lane, int mt, int c) {
  const int co = 16 * mt + (lane & 15), kg = lane >> 4;
  const int t = 2 * c + (kg >> 1);
  bf16x8 w;
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const int ci = 8 * (kg & 1) + e;
    w[e] = (bf16)(t < 9 ? w2[(co * 16 + ci) * 9 + t] : 0.f);
  }
  return w;
}
__host__ __device__ constexpr int y1tap(int t) { return ((t / 3) * 15 + t % 3) * 32; }

// ============================================================================
// Forward
// ============================================================================
#ifndef MCC_REF_FWD_W4
#define MCC_REF_FWD_W4 0  // 1: cap at 128 VGPRs (4 waves per SIMD; spills 3 registers)
#endif
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(MCC_REF_FWD_W4 ? 4 : 1, MCC_REF_FWD_W4 ? 4 : 8)))
ref_fwd_kernel(RefFwdParams p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = threadIdx.x;
  const int n16 = lane & 15, g = lane >> 4;

  const bf16x8 w1 = conv1_weights(p.w1, lane);
  float b1v[4], b2v[2][4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    b1v[i] = 255.f * p.b1[4 * g + i];
    b2v[0][i] = p.b2[4 * g + i];
    b2v[1][i] = p.b2[16 + 4 * g + i];
  }
  bf16x8 w2[2][5];
#pragma unroll
  for (int mt = 0; mt < 2; ++mt)
#pragma unroll
    for (int c = 0; c < 5; ++c) w2[mt][c] = conv2_weights(p.w2, lane, mt, c);
  // conv2 B operand: this lane's tap offset per chunk (taps >= 9: zero weights)
  int koff[5];
#pragma unroll
  for (int c = 0; c < 5; ++c) {
    const int t = 2 * c + (g >> 1);  // taps >= 9: tap 0 (zero weights)
    koff[c] = t < 9 ? y1p_off(t / 3, t % 3, g & 1) : y1p_off(0, 0, g & 1);
  }

  zero_lds(smem, kFLds, lane);
  wave_lds_sync();

  uint32_t xw[4];
  WaveIdx widx;
  widx.load(p.idx, blockIdx.x, (int)gridDim.x, p.B, 0);
  auto load_img = [&](int k) {
    if ((k & 63) == 0 && k > 0) widx.load(p.idx, blockIdx.x, (int)gridDim.x, p.B, k);
    load_x(xw, p.x + (size_t)widx.get(k) * kImgPix, lane);
  };
  if ((int)blockIdx.x < p.B) load_img(0);

  for (int img = blockIdx.x, kimg = 0; img < p.B; img += (int)gridDim.x, ++kimg) {
    wave_lds_sync();
    stage_x(smem, kFX0, kFX2, -1, xw, lane);
    wave_lds_sync();
    if (img + (int)gridDim.x < p.B) load_img(kimg + 1);

    // ---- conv1: 13 tiles of 16 output pixels (natural order) ----
#pragma unroll 2
    for (int T = 0; T < 13; ++T) {
      const int px = min(16 * T + n16, 195);
      const int y = (px * 2341) >> 15, x = px - 14 * y;  // px / 14 for px < 196
      const bf16x8 pb = conv1_patch(smem, kFX0, kFX2, y, x, g);
      f32x4 acc = {b1v[0], b1v[1], b1v[2], b1v[3]};
      acc = mma(acc, w1, pb);
      // lane (pixel, g): channels 4g .. 4g+3
      const u32x2 v = pack4(relu(acc[0]) * (1.f / 255.f), relu(acc[1]) * (1.f / 255.f),
                            relu(acc[2]) * (1.f / 255.f), relu(acc[3]) * (1.f / 255.f));
      if (16 * T + n16 < 196) *reinterpret_cast<u32x2*>(smem + kFY1 + y1p_off(y + 1, x + 1, g >> 1) + 8 * (g & 1)) = v;
    }
    wave_lds_sync();

    // ---- conv2: 4 tiles of 16 output pixels x 2 channel tiles ----
    bf16* y2g = static_cast<bf16*>(p.y2) + (size_t)img * kY2Elems;
#pragma unroll 1
    for (int T = 0; T < 4; ++T) {
      const int q = min(16 * T + n16, 48);
      const int oy = (q * 37) >> 8, ox = q - 7 * oy;  // q / 7 for q < 49
      const char* pb = smem + kFY1 + (oy * 8 + ox) * 16;  // + the tap's plane / offset (koff)
      bf16x8 bf[5];
#pragma unroll
      for (int c = 0; c < 5; ++c) bf[c] = *reinterpret_cast<const bf16x8*>(pb + koff[c]);
      f32x4 acc[2];
#pragma unroll
      for (int mt = 0; mt < 2; ++mt) {
        acc[mt] = f32x4{b2v[mt][0], b2v[mt][1], b2v[mt][2], b2v[mt][3]};
#pragma unroll
        for (int c = 0; c < 5; ++c) acc[mt] = mma(acc[mt], w2[mt][c], bf[c]);
      }
      if (16 * T + n16 < 49) {
#pragma unroll
        for (int mt = 0; mt < 2; ++mt)
          *reinterpret_cast<u32x2*>(y2g + q * 32 + 16 * mt + 4 * g) =
              pack4(relu(acc[mt][0]), relu(acc[mt][1]), relu(acc[mt][2]), relu(acc[mt][3]));
      }
    }
  }
}

// ============================================================================
// Backward
// ============================================================================
//
// Sub-pixel phases of conv2's data gradient: output pixel (y, x) = (2i + py,
// 2j + px) receives dZ2 at (i + di, j + dj) through tap (kh, kw):
//   py = 0: (kh 1, di 0);  py = 1: (kh 0, di 1), (kh 2, di 0)   (same in x).
// Phase-major pixel order m = 8i + j (i, j in 0..7; 7 = padding) -> 4 tiles
// of 16 per phase; lane (pixel, g) of tile T holds i = 2T + (n >> 3), j = n & 7.
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(1, 1))) ref_bwd_kernel(RefBwdParams p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = threadIdx.x;
  const int n16 = lane & 15, g = lane >> 4;
  const int tq = (lane >> 2) & 3, tp = lane & 3;

  const bf16x8 w1 = conv1_weights(p.w1, lane);
  float b1v[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) b1v[i] = 255.f * p.b1[4 * g + i];
  // conv2 dX A operand per tap: rows = input channel ci = n16, K slot 8g + e = output channel
  bf16x8 wdx[9];
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int e = 0; e < 8; ++e) wdx[t][e] = (bf16)p.w2[((8 * g + e) * 16 + n16) * 9 + t];

  zero_lds(smem, kBLds, lane);
  wave_lds_sync();
  if (lane < 8) *reinterpret_cast<uint32_t*>(smem + kBOnes + 4 * lane) = 0x3f803f80u;

  f32x4 acc2[2][10];
#pragma unroll
  for (int mt = 0; mt < 2; ++mt)
#pragma unroll
    for (int t = 0; t < 10; ++t) acc2[mt][t] = f32x4{0.f, 0.f, 0.f, 0.f};
  f32x4 acc1 = {0.f, 0.f, 0.f, 0.f};

  // ---- per-lane LDS bases (image independent) ----
  // conv2 dW: q = 32c + 8g + 4h + tq (q >= 49: a zero dZ2 pad pixel / any Y1 pixel)
  int adz[2][2], ay1[2][2];
#pragma unroll
  for (int c = 0; c < 2; ++c)
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int q = 32 * c + 8 * g + 4 * h + tq;
      const int oy = q < 49 ? q / 7 : 8, ox = q < 49 ? q % 7 : 8;
      adz[c][h] = kBDz2 + (oy * 9 + ox) * 64 + 8 * tp;
      ay1[c][h] = q < 49 ? kBY1 + (2 * oy * 15 + 2 * ox) * 32 + 8 * tp : kBY1 + 8 * tp;
    }
  // conv1 dW: A = dZ1 rows (y = 2c + (g >> 1), x0 = 8 (g & 1)), B = X planes
  const int adz1 = kBDz1 + ((g >> 1) * 16 + 8 * (g & 1) + tq) * 32 + 8 * tp;
  int bx1;
  {
    const int t = n16, kh = t / 3, kw = t % 3;
    const int plane = kw == 1 ? 0 : kw == 2 ? 1 : 2;  // E / O / Os
    bx1 = t < 9 ? kBXc + plane * kXcPlane + ((g >> 1) * 2 + kh) * 32 + 16 * (g & 1) : kBOnes;
  }

  // ---- staged per image: X words, dY2 and Y2 (16 B pieces) ----
  uint32_t xw[4];
  u32x4 dyv[4], y2v[4];
  WaveIdx widx;
  widx.load(p.idx, blockIdx.x, (int)gridDim.x, p.B, 0);
  auto load_img = [&](int k) {
    const int img = blockIdx.x + k * (int)gridDim.x;
    if ((k & 63) == 0 && k > 0) widx.load(p.idx, blockIdx.x, (int)gridDim.x, p.B, k);
    load_x(xw, p.x + (size_t)widx.get(k) * kImgPix, lane);
    const u32x4* dyg = reinterpret_cast<const u32x4*>(static_cast<const bf16*>(p.dy2) + (size_t)img * kY2Elems);
    const u32x4* y2g = reinterpret_cast<const u32x4*>(static_cast<const bf16*>(p.y2) + (size_t)img * kY2Elems);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int w = min(lane + 64 * r, 195);
      dyv[r] = dyg[w];
      y2v[r] = y2g[w];
    }
  };
  if ((int)blockIdx.x < p.B) load_img(0);

  for (int img = blockIdx.x, kimg = 0; img < p.B; img += (int)gridDim.x, ++kimg) {
    wave_lds_sync();
    stage_x(smem, kBX0, kBX2, kBXc, xw, lane);
    // dZ2 = dY2 * (Y2 > 0), HWC into the padded 9 x 9 grid
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int w = lane + 64 * r;
      if (w < 196) {
        u32x4 z;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const uint32_t yv = y2v[r][k], dv = dyv[r][k];
          const uint32_t lo = (int)(short)(yv & 0xffffu) > 0 ? (dv & 0xffffu) : 0u;
          const uint32_t hi = (int)yv > 0x0000ffff ? (dv & 0xffff0000u) : 0u;  // upper bf16 > 0
          z[k] = lo | hi;
        }
        const int q = w >> 2, oy = (q * 37) >> 8, ox = q - 7 * oy;
        *reinterpret_cast<u32x4*>(smem + kBDz2 + (oy * 9 + ox) * 64 + 16 * (w & 3)) = z;
      }
    }
    wave_lds_sync();
    if (img + (int)gridDim.x < p.B) load_img(kimg + 1);

    // ---- recompute conv1 in phase order: Y1 HWC for conv2 dW, ReLU mask bits ----
    uint32_t mask[2] = {0u, 0u};
#pragma unroll
    for (int ph = 0; ph < 4; ++ph)
#pragma unroll
      for (int T = 0; T < 4; ++T) {
        const int i = 2 * T + (n16 >> 3), j = n16 & 7;
        const int y = 2 * i + (ph >> 1), x = 2 * j + (ph & 1);
        const bool ok = i < 7 && j < 7;
        const bf16x8 pb = conv1_patch(smem, kBX0, kBX2, ok ? y : 0, ok ? x : 0, g);
        f32x4 acc = {b1v[0], b1v[1], b1v[2], b1v[3]};
        acc = mma(acc, w1, pb);
        const float v0 = relu(acc[0]) * (1.f / 255.f), v1 = relu(acc[1]) * (1.f / 255.f);
        const float v2 = relu(acc[2]) * (1.f / 255.f), v3 = relu(acc[3]) * (1.f / 255.f);
        const u32x2 v = pack4(v0, v1, v2, v3);
        // mask on the stored (bf16) value, as the forward's consumer saw it
        const uint32_t bits = ((v.x & 0xffffu) ? 1u : 0u) | ((v.x >> 16) ? 2u : 0u) | ((v.y & 0xffffu) ? 4u : 0u) |
                              ((v.y >> 16) ? 8u : 0u);
        const int sh = 4 * ((ph * 4 + T) & 7);
        mask[(ph * 4 + T) >> 3] |= (ok ? bits : 0u) << sh;
        if (ok) *reinterpret_cast<u32x2*>(smem + kBY1 + ((y + 1) * 15 + x + 1) * 32 + 8 * g) = v;
      }
    wave_lds_sync();

    // ---- conv2 dW: acc2[mt][t] += dZ2^T (co tile mt) . patches (tap t; t = 9: ones) ----
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      bf16x8 a[2];
#pragma unroll
      for (int mt = 0; mt < 2; ++mt) a[mt] = tr8(smem + adz[c][0] + 32 * mt, smem + adz[c][1] + 32 * mt);
      bf16x8 b[10];
#pragma unroll
      for (int t = 0; t < 9; ++t) b[t] = tr8(smem + ay1[c][0] + y1tap(t), smem + ay1[c][1] + y1tap(t));
      b[9] = tr8(smem + kBOnes + 8 * (tp & 1), smem + kBOnes + 8 * (tp & 1));
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int mt = 0; mt < 2; ++mt)
#pragma unroll
        for (int t = 0; t < 10; ++t) acc2[mt][t] = mma(acc2[mt][t], a[mt], b[t]);
    }

    // ---- conv2 dX by phase: dY1^T = W2 . dZ2 patches; dZ1 = dY1 * mask -> LDS HWC ----
#pragma unroll
    for (int ph = 0; ph < 4; ++ph) {
      const int py = ph >> 1, pxx = ph & 1;
#pragma unroll
      for (int T = 0; T < 4; ++T) {
        const int i = 2 * T + (n16 >> 3), j = n16 & 7;
        const char* zb = smem + kBDz2 + (i * 9 + j) * 64 + 16 * g;
        f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int a = 0; a < 2; ++a) {
          if (py == 0 && a == 1) continue;
          const int kh = py == 0 ? 1 : (a == 0 ? 0 : 2), di = py == 1 && a == 0 ? 1 : 0;
#pragma unroll
          for (int b = 0; b < 2; ++b) {
            if (pxx == 0 && b == 1) continue;
            const int kw = pxx == 0 ? 1 : (b == 0 ? 0 : 2), dj = pxx == 1 && b == 0 ? 1 : 0;
            const bf16x8 zf = *reinterpret_cast<const bf16x8*>(zb + (di * 9 + dj) * 64);
            acc = mma(acc, wdx[kh * 3 + kw], zf);
          }
        }
        const uint32_t mb = (mask[(ph * 4 + T) >> 3] >> (4 * ((ph * 4 + T) & 7))) & 15u;
        const u32x2 v = pack4((mb & 1u) ? acc[0] : 0.f, (mb & 2u) ? acc[1] : 0.f, (mb & 4u) ? acc[2] : 0.f,
                              (mb & 8u) ? acc[3] : 0.f);
        const int y = 2 * i + py, x = 2 * j + pxx;
        *reinterpret_cast<u32x2*>(smem + kBDz1 + (y * 16 + x) * 32 + 8 * g) = v;
      }
    }
    wave_lds_sync();

    // ---- conv1 dW: acc1 += dZ1^T (rows ci) . X patches (columns taps; 9 = ones) ----
#pragma unroll
    for (int c = 0; c < 7; ++c) {
      const bf16x8 a = tr8(smem + adz1 + c * 1024, smem + adz1 + c * 1024 + 128);
      const bf16x8 b = *reinterpret_cast<const bf16x8*>(smem + bx1 + (n16 < 9 ? c * 128 : 0));
      acc1 = mma(acc1, a, b);
    }
  }

  // ---- per-wave slab (accumulator order) ----
  float* slab = p.slab + (size_t)blockIdx.x * kSlab;
#pragma unroll
  for (int mt = 0; mt < 2; ++mt)
#pragma unroll
    for (int t = 0; t < 10; ++t)
#pragma unroll
      for (int i = 0; i < 4; ++i) slab[((mt * 10 + t) * 4 + i) * 64 + lane] = acc2[mt][t][i];
#pragma unroll
  for (int i = 0; i < 4; ++i) slab[kSlabW2 + i * 64 + lane] = acc1[i];
}

// ---- two-wave backward ----
// ref_bwd_kernel runs one wave per SIMD (its 80 dW2 accumulators plus the 36
// dX weight registers do not fit two waves), so every LDS / MFMA latency of
// the image's serial chain is exposed. Here a workgroup of two waves shares
// one image at a time, the roles split by register set:
//   wave 0: accumulates conv2 dW / db of image k (40 MFMAs), then stages
//           image k+1 (global loads issued before image k's compute, LDS
//           writes after it) and recomputes ITS conv1 (16 MFMAs) -> Y1
//           (wave-private) and the ReLU mask bits, which it hands to wave 1
//           through LDS (the mask lanes are wave 1's dX output lanes);
//   wave 1: conv2 dX -> dZ1 (wave-private), conv1 dW / db (36 + 7 MFMAs).
// (Recomputing conv1 in both waves cost wave 1 -- the critical one -- ~90 us
// per step.) The column-parity planes, dZ2 and the mask are double-buffered,
// so the waves meet at ONE barrier per image. 2 waves per SIMD.
constexpr int kB2X0 = 0, kB2X2 = kXCopy;      // integer X copies (wave 0 only)
constexpr int kB2Buf = 2 * kXCopy;             // 3840: two buffers of [Xc | dZ2 | mask]
constexpr int kB2Xc = 0;                       // + buffer: column-parity planes E / O / Os
constexpr int kB2Dz2 = 3 * kXcPlane;           // + buffer: dZ2 HWC 9 x 9 x 64 B (2880), see dz2_chunk
constexpr int kB2Mask = kB2Dz2 + 81 * 64;      // + buffer: ReLU mask, 64 lanes x 8 B (8064)
constexpr int kB2BufBytes = kB2Mask + 64 * 8;  // 8576
// Y1 / dZ1: 40-B pixels (8-B channel quads, one 8-B pad), rows of 624 / 640 B,
// quad q of row r stored at quad q ^ ((r >> 1) & 1); dZ2: the 16-B channel
// chunk c of row i at chunk c ^ 2 (i & 1). With these, the phase-order Y1 /
// dZ1 writes (16 lanes of one quad at pixels 2 apart: 8-way conflicts on
// 32-B HWC pixels), the conv2 dX reads and the transposed dW reads are
// (nearly) conflict-free: 1,459 -> 510 LDS cycles per image, 1,039 -> 90 of
// them conflicts (python tools/lds_banks.py refbwd).
constexpr int kY1Px = 40, kY1Row = 624, kZ1Px = 40, kZ1Row = 640;
constexpr int kB2Y1 = kB2Buf + 2 * kB2BufBytes;  // 20992: Y1, 15 x 15 pixels (pad row / column 0) (wave 0)
constexpr int kB2Dz1 = kB2Y1 + 15 * kY1Row;      // 30352: dZ1, 14 x 16 pixels (columns 14, 15 pads) (wave 1)
constexpr int kB2Ones = kB2Dz1 + 14 * kZ1Row;    // 39312
constexpr int kB2Lds = kB2Ones + 32;             // 39344
__host__ __device__ constexpr int y1_at(int yy, int xx, int quad) {
  return yy * kY1Row + xx * kY1Px + 8 * (quad ^ ((yy >> 1) & 1));
}
__host__ __device__ constexpr int z1_at(int y, int x, int quad) {
  return y * kZ1Row + x * kZ1Px + 8 * (quad ^ ((y >> 1) & 1));
}
__host__ __device__ constexpr int dz2_at(int i, int j, int chunk) { return (i * 9 + j) * 64 + 16 * (chunk ^ (2 * (i & 1))); }
static_assert(4 * kB2Lds <= 163840, "ref_bwd2: four workgroups per CU");
static_assert(kB2BufBytes % 16 == 0 && kB2Dz2 % 16 == 0, "16-B aligned buffers");
constexpr int kBwd2Grid = 256 * 4;
static_assert(kBwd2Grid == kBwdGrid, "ref_slab_bytes covers both backward kernels");

__device__ __forceinline__ void wg_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }
// a wave's own LDS operations execute in issue order: a compiler fence suffices
__device__ __forceinline__ void lds_fence() { asm volatile("" ::: "memory"); }

// Wave 0's conv1 recompute in the data gradient's phase order (see
// ref_bwd_kernel): Y1 stores and the ReLU mask bits of the stored bf16 values.
// Every address is a per-lane base + an immediate: output pixel (y, x) =
// (4T + 2a + p, 2j + q) for tile T of phase (p, q), lane n16 = 8a + j. The
// K-padding lanes (g >= 2, and g = 1's second window) read real X rows
// against zero weights -- finite, so their products are exact zeros -- and
// the invalid pixels (i = 7 or j = 7) only feed their own, unstored columns.
__device__ __forceinline__ void ref_conv1_y1_mask(char* smem, const bf16x8& w1, const float (&b1v)[4], int n16, int g,
                                                  uint32_t (&mask)[2]) {
  const int a = n16 >> 3, j = n16 & 7;
  const int xa = 4 * a * kXPitch + 8 * j + (g == 0 ? 0 : 2 * kXPitch);  // window row kh = 0 (g = 0) / 2
  const int xb = 4 * a * kXPitch + 8 * j + kXPitch;                     // window row kh = 1
  // Y1 (yy, xx) = (y + 1, x + 1): quad swizzle ((yy >> 1) & 1) = (a + p) & 1
  const int yl[2] = {kB2Y1 + 2 * a * kY1Row + 2 * j * kY1Px + 8 * (g ^ (a & 1)),
                     kB2Y1 + 2 * a * kY1Row + 2 * j * kY1Px + 8 * (g ^ ((a + 1) & 1))};
  const bool jok = j < 7, aok = a == 0;
  mask[0] = mask[1] = 0u;
#pragma unroll
  for (int ph = 0; ph < 4; ++ph)
#pragma unroll
    for (int T = 0; T < 4; ++T) {
      const int p = ph >> 1, q = ph & 1;
      const int cb = (q ? kB2X2 + 8 : kB2X0) + (8 * T + 2 * p) * kXPitch;
      const bf16x4 va = *reinterpret_cast<const bf16x4*>(smem + xa + cb);
      const bf16x4 vb = *reinterpret_cast<const bf16x4*>(smem + xb + cb);
      f32x4 acc = {b1v[0], b1v[1], b1v[2], b1v[3]};
      acc = mma(acc, w1, join(va, vb));
      const u32x2 v = pack4(relu(acc[0]) * (1.f / 255.f), relu(acc[1]) * (1.f / 255.f), relu(acc[2]) * (1.f / 255.f),
                            relu(acc[3]) * (1.f / 255.f));
      const bool ok = jok && (T < 3 || aok);
      const uint32_t bits = nz4(v);
      mask[(ph * 4 + T) >> 3] |= (ok ? bits : 0u) << (4 * ((ph * 4 + T) & 7));
      if (ok) *reinterpret_cast<u32x2*>(smem + yl[p] + (4 * T + p + 1) * kY1Row + (q + 1) * kY1Px) = v;
    }
}

__global__ void __launch_bounds__(128) __attribute__((amdgpu_waves_per_eu(2, 2))) ref_bwd2_kernel(RefBwdParams p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int n16 = lane & 15, g = lane >> 4;
  const int tq = (lane >> 2) & 3, tp = lane & 3;
  const int grid = (int)gridDim.x;

  {
    const u32x4 z = {0u, 0u, 0u, 0u};
    for (int i = (int)threadIdx.x * 16; i < kB2Lds; i += 128 * 16) *reinterpret_cast<u32x4*>(smem + i) = z;
  }
  wg_barrier();
  if (threadIdx.x < 8) *reinterpret_cast<uint32_t*>(smem + kB2Ones + 4 * threadIdx.x) = 0x3f803f80u;
  float* slab = p.slab + (size_t)blockIdx.x * kSlab;
  auto buf = [](int k) { return kB2Buf + (k & 1) * kB2BufBytes; };

  if (wv == 0) {
    const bf16x8 w1 = conv1_weights(p.w1, lane);
    float b1v[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) b1v[i] = 255.f * p.b1[4 * g + i];
    f32x4 acc2[2][10];
#pragma unroll
    for (int mt = 0; mt < 2; ++mt)
#pragma unroll
      for (int t = 0; t < 10; ++t) acc2[mt][t] = f32x4{0.f, 0.f, 0.f, 0.f};
    // conv2 dW operands: q = 32c + 8g + 4h + tq (q >= 49: a zero dZ2 pad pixel / any Y1 pixel)
    int adz[2][2], ay1[2][2][2];  // ay1[.][.][kh >> 1]
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int q = 32 * c + 8 * g + 4 * h + tq;
        const int oy = q < 49 ? q / 7 : 8, ox = q < 49 ? q % 7 : 8;
        adz[c][h] = dz2_at(oy, ox, tp >> 1) + 8 * (tp & 1);  // + buffer + kB2Dz2; ^ 32: channels 16..31
        const int yy = q < 49 ? 2 * oy : 0, xx = q < 49 ? 2 * ox : 0;
        ay1[c][h][0] = kB2Y1 + y1_at(yy, xx, tp);          // taps kh = 0, 1 (+ kh * row + kw * pixel)
        ay1[c][h][1] = kB2Y1 + y1_at(yy + 2, xx, tp) - 2 * kY1Row;  // kh = 2
      }

    uint32_t xw[4];
    u32x4 dyv[4], y2v[4];
    WaveIdx widx;
    widx.load(p.idx, blockIdx.x, grid, p.B, 0);
    auto load = [&](int k) {
      const int img = (int)blockIdx.x + k * grid;
      if ((k & 63) == 0 && k > 0) widx.load(p.idx, blockIdx.x, grid, p.B, k);
      load_x(xw, p.x + (size_t)widx.get(k) * kImgPix, lane);
      const u32x4* dyg = reinterpret_cast<const u32x4*>(static_cast<const bf16*>(p.dy2) + (size_t)img * kY2Elems);
      const u32x4* y2g = reinterpret_cast<const u32x4*>(static_cast<const bf16*>(p.y2) + (size_t)img * kY2Elems);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int w = min(lane + 64 * r, 195);
        dyv[r] = dyg[w];
        y2v[r] = y2g[w];
      }
    };
    // image k: X copies + planes, dZ2 = dY2 * (Y2 > 0); then conv1 -> Y1 and the mask
    auto stage = [&](int k) {
      const int bo = buf(k);
      stage_x(smem, kB2X0, kB2X2, bo + kB2Xc, xw, lane);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int w = lane + 64 * r;
        if (w < 196) {
          u32x4 z;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const uint32_t yv = y2v[r][e], dv = dyv[r][e];
            const uint32_t lo = (int)(short)(yv & 0xffffu) > 0 ? (dv & 0xffffu) : 0u;
            const uint32_t hi = (int)yv > 0x0000ffff ? (dv & 0xffff0000u) : 0u;  // upper bf16 > 0
            z[e] = lo | hi;
          }
          const int q = w >> 2, oy = (q * 37) >> 8, ox = q - 7 * oy;
          *reinterpret_cast<u32x4*>(smem + bo + kB2Dz2 + dz2_at(oy, ox, w & 3)) = z;
        }
      }
      lds_fence();
      if (MCC_REF_ABL & 1) return;
      uint32_t mask[2];
      ref_conv1_y1_mask(smem, w1, b1v, n16, g, mask);
      *reinterpret_cast<u32x2*>(smem + bo + kB2Mask + 8 * lane) = u32x2{mask[0], mask[1]};
    };
    if ((int)blockIdx.x < p.B) {
      load(0);
      stage(0);
    }
    for (int img = blockIdx.x, k = 0; img < p.B; img += grid, ++k) {
      wg_barrier();  // image k staged; wave 1 done with the other buffer (image k-1)
      const bool more = img + grid < p.B;
      if (more) load(k + 1);
      const int bo = buf(k);
      if (!(MCC_REF_ABL & 5)) {
#pragma unroll
        for (int c = 0; c < 2; ++c) {
          bf16x8 a[2];
#pragma unroll
          for (int mt = 0; mt < 2; ++mt)
            a[mt] = tr8(smem + bo + kB2Dz2 + (adz[c][0] ^ (32 * mt)), smem + bo + kB2Dz2 + (adz[c][1] ^ (32 * mt)));
          // taps in two halves of 5 (t = 9: the ones column): 20 fewer live registers
#pragma unroll
          for (int t0 = 0; t0 < 10; t0 += 5) {
            bf16x8 b[5];
#pragma unroll
            for (int u = 0; u < 5; ++u) {
              const int t = t0 + u;
              const int kh = t / 3, kw = t % 3, to = kh * kY1Row + kw * kY1Px;
              b[u] = t < 9 ? tr8(smem + ay1[c][0][kh >> 1] + to, smem + ay1[c][1][kh >> 1] + to)
                           : tr8(smem + kB2Ones + 8 * (tp & 1), smem + kB2Ones + 8 * (tp & 1));
            }
#pragma unroll
            for (int mt = 0; mt < 2; ++mt)
#pragma unroll
              for (int u = 0; u < 5; ++u) acc2[mt][t0 + u] = mma(acc2[mt][t0 + u], a[mt], b[u]);
          }
        }
      }
      lds_fence();
      if (more) stage(k + 1);  // Y1 rewritten after this wave's dW2 reads (issue order)
    }
#pragma unroll
    for (int mt = 0; mt < 2; ++mt)
#pragma unroll
      for (int t = 0; t < 10; ++t)
#pragma unroll
        for (int i = 0; i < 4; ++i) slab[((mt * 10 + t) * 4 + i) * 64 + lane] = acc2[mt][t][i];
  } else {
    // conv2 dX A operand per tap: rows = input channel ci = n16, K slot 8g + e = output channel
    bf16x8 wdx[9];
#pragma unroll
    for (int t = 0; t < 9; ++t)
#pragma unroll
      for (int e = 0; e < 8; ++e) wdx[t][e] = (bf16)p.w2[((8 * g + e) * 16 + n16) * 9 + t];
    f32x4 acc1 = {0.f, 0.f, 0.f, 0.f};
    // conv1 dW: A = dZ1 rows (y = 2c + (g >> 1), x0 = 8 (g & 1)), B = X planes (tap n16; 9: ones)
    // (row 2c + (g >> 1): quad swizzle c & 1)
    const int adz1[2] = {kB2Dz1 + z1_at(g >> 1, 8 * (g & 1) + tq, tp), kB2Dz1 + z1_at(g >> 1, 8 * (g & 1) + tq, tp ^ 1)};
    // conv2 dX: dZ2 row i + di has parity ((n16 >> 3) ^ di) & 1
    const int zc[2] = {16 * (g ^ (2 * ((n16 >> 3) & 1))), 16 * (g ^ (2 * (((n16 >> 3) & 1) ^ 1)))};
    int bx1 = -1;
    if (n16 < 9) {
      const int kh = n16 / 3, kw = n16 % 3;
      const int plane = kw == 1 ? 0 : kw == 2 ? 1 : 2;  // E / O / Os
      bx1 = kB2Xc + plane * kXcPlane + ((g >> 1) * 2 + kh) * 32 + 16 * (g & 1);  // + buffer
    }
    for (int img = blockIdx.x, k = 0; img < p.B; img += grid, ++k) {
      wg_barrier();
      if (MCC_REF_ABL & 2) continue;
      const int bo = buf(k);
      const u32x2 mk = *reinterpret_cast<const u32x2*>(smem + bo + kB2Mask + 8 * lane);
      const uint32_t mask[2] = {mk.x, mk.y};
#pragma unroll
      for (int ph = 0; ph < 4; ++ph) {
        const int py = ph >> 1, pxx = ph & 1;
#pragma unroll
        for (int T = 0; T < 4; ++T) {
          const int i = 2 * T + (n16 >> 3), j = n16 & 7;
          const char* zb = smem + bo + kB2Dz2 + (i * 9 + j) * 64;
          f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int a = 0; a < 2; ++a) {
            if (py == 0 && a == 1) continue;
            const int kh = py == 0 ? 1 : (a == 0 ? 0 : 2), di = py == 1 && a == 0 ? 1 : 0;
#pragma unroll
            for (int b = 0; b < 2; ++b) {
              if (pxx == 0 && b == 1) continue;
              const int kw = pxx == 0 ? 1 : (b == 0 ? 0 : 2), dj = pxx == 1 && b == 0 ? 1 : 0;
              const bf16x8 zf = *reinterpret_cast<const bf16x8*>(zb + (di * 9 + dj) * 64 + zc[di]);
              acc = mma(acc, wdx[kh * 3 + kw], zf);
            }
          }
          const uint32_t mb = (mask[(ph * 4 + T) >> 3] >> (4 * ((ph * 4 + T) & 7))) & 15u;
          const u32x2 v = pack4((mb & 1u) ? acc[0] : 0.f, (mb & 2u) ? acc[1] : 0.f, (mb & 4u) ? acc[2] : 0.f,
                                (mb & 8u) ? acc[3] : 0.f);
          const int y = 2 * i + py, x = 2 * j + pxx;
          if (i < 7) *reinterpret_cast<u32x2*>(smem + kB2Dz1 + z1_at(y, x, g)) = v;  // (no rows 14, 15)
        }
      }
      lds_fence();
      if (MCC_REF_ABL & 8) continue;
      const char* xb = smem + (bx1 >= 0 ? bo + bx1 : kB2Ones);
      const int xstep = bx1 >= 0 ? 128 : 0;
#pragma unroll
      for (int c = 0; c < 7; ++c) {
        const int za = adz1[c & 1] + c * 2 * kZ1Row;
        const bf16x8 a = tr8(smem + za, smem + za + 4 * kZ1Px);
        const bf16x8 b = *reinterpret_cast<const bf16x8*>(xb + c * xstep);
        acc1 = mma(acc1, a, b);
      }
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) slab[kSlabW2 + i * 64 + lane] = acc1[i];
  }
}

// Fixed-order sum of the per-wave slabs -> canonical gradients.
constexpr int kRedWaves = 16;
__global__ void __launch_bounds__(64 * kRedWaves) ref_bwd_reduce_kernel(RefBwdParams p, int nslabs) {
  __shared__ float part[kRedWaves][64];
  const int l = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int pos = blockIdx.x * 64 + l;
  float s = 0.f;
#pragma unroll 8
  for (int k = w; k < nslabs; k += kRedWaves) s += p.slab[(size_t)k * kSlab + pos];
  part[w][l] = s;
  __syncthreads();
  if (w != 0) return;
  float v = part[0][l];
#pragma unroll
  for (int i = 1; i < kRedWaves; ++i) v += part[i][l];
  if (pos < kSlabW2) {
    const int mt = pos / 2560, t = (pos / 256) % 10, i = (pos / 64) & 3, ln = pos & 63;
    // dW2 tile: rows = output channels (MFMA rows 4 (ln >> 4) + i), columns = input channels
    const int co = 16 * mt + 4 * (ln >> 4) + i, ci = ln & 15;
    if (t < 9) p.gw2[(co * 16 + ci) * 9 + t] = v;
    else if (ci == 0) p.gb2[co] = v;
  } else {
    const int q = pos - kSlabW2, i = q >> 6, ln = q & 63;
    const int ci = 4 * (ln >> 4) + i, t = ln & 15;
    if (t < 9) p.gw1[ci * 9 + t] = v * (1.f / 255.f);
    else if (t == 9) p.gb1[ci] = v;
  }
}

}  // namespace

size_t ref_slab_bytes(bool f32) { return f32 ? ref32_slab_bytes() : (size_t)kBwdGrid * kSlab * 4; }

void ref_forward(const RefFwdParams& p, hipStream_t s) {
  if (p.f32) return ref32_forward(p, s);
  if (p.B <= 0) return;
  // persistent grid = what the device holds at once (132 VGPRs: 3 waves per
  // SIMD, 12 per CU): a grid past residency (it was 14 per CU) runs its
  // last workgroups as a second, mostly idle round
  static int resident = 0;
  if (resident == 0) {
    int per_cu = 0, dev = 0, cus = 0;
    MCC_CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, ref_fwd_kernel, 64, kFLds) == hipSuccess &&
                  hipGetDevice(&dev) == hipSuccess &&
                  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess,
              "ref_forward: occupancy query failed");
    resident = std::max(1, per_cu) * std::max(1, cus);
  }
  const int grid = std::min(p.B, resident);
  hipLaunchKernelGGL(ref_fwd_kernel, dim3(grid), dim3(64), kFLds, s, p);
}

void ref_backward(const RefBwdParams& p, hipStream_t s) {
  if (p.f32) return ref32_backward(p, s);
  if (p.B <= 0) return;
  if (ab_flag("ref_bwd1")) hipLaunchKernelGGL(ref_bwd_kernel, dim3(kBwdGrid), dim3(64), kBLds, s, p);
  else hipLaunchKernelGGL(ref_bwd2_kernel, dim3(kBwd2Grid), dim3(128), kB2Lds, s, p);
  hipLaunchKernelGGL(ref_bwd_reduce_kernel, dim3(kSlab / 64), dim3(64 * kRedWaves), 0, s, p, kBwdGrid);
}

}  // namespace gpu
}  // namespace mcc
