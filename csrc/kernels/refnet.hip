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

#include <algorithm>

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
constexpr int kFY1 = 2 * kXCopy;       // 3840: Y1 HWC, 15 x 15 pixels (pad row / column 0) x 32 B
constexpr int kFLds = kFY1 + 225 * 32;  // 11040
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

__device__ __forceinline__ uint32_t bf16_bits(float v) {
  return (uint32_t)__builtin_bit_cast(unsigned short, (bf16)v);
}
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
__device__ __forceinline__ void wave_lds_sync() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }
__device__ __forceinline__ bf16x8 tr8(const char* p0, const char* p1) {
  const bf16x4 a = tr4(reinterpret_cast<const bf16*>(p0));
  const bf16x4 b = tr4(reinterpret_cast<const bf16*>(p1));
  return __builtin_shufflevector(a, b, 0, 1, 2, 3, 4, 5, 6, 7);
}
__device__ __forceinline__ bf16x8 join(const bf16x4& a, const bf16x4& b) {
  return __builtin_shufflevector(a, b, 0, 1, 2, 3, 4, 5, 6, 7);
}
__device__ __forceinline__ u32x2 pack4(float a, float b, float c, float d) {
  return u32x2{bf16_bits(a) | (bf16_bits(b) << 16), bf16_bits(c) | (bf16_bits(d) << 16)};
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
__global__ void __launch_bounds__(64) ref_fwd_kernel(RefFwdParams p) {
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
    const int t = 2 * c + (g >> 1);
    koff[c] = (t < 9 ? y1tap(t) : 0) + 16 * (g & 1);
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
      const u32x2 v = pack4(fmaxf(acc[0], 0.f) * (1.f / 255.f), fmaxf(acc[1], 0.f) * (1.f / 255.f),
                            fmaxf(acc[2], 0.f) * (1.f / 255.f), fmaxf(acc[3], 0.f) * (1.f / 255.f));
      if (16 * T + n16 < 196) *reinterpret_cast<u32x2*>(smem + kFY1 + ((y + 1) * 15 + x + 1) * 32 + 8 * g) = v;
    }
    wave_lds_sync();

    // ---- conv2: 4 tiles of 16 output pixels x 2 channel tiles ----
    bf16* y2g = static_cast<bf16*>(p.y2) + (size_t)img * kY2Elems;
#pragma unroll 1
    for (int T = 0; T < 4; ++T) {
      const int q = min(16 * T + n16, 48);
      const int oy = (q * 37) >> 8, ox = q - 7 * oy;  // q / 7 for q < 49
      const char* pb = smem + kFY1 + (2 * oy * 15 + 2 * ox) * 32;
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
              pack4(fmaxf(acc[mt][0], 0.f), fmaxf(acc[mt][1], 0.f), fmaxf(acc[mt][2], 0.f), fmaxf(acc[mt][3], 0.f));
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
        const float v0 = fmaxf(acc[0], 0.f) * (1.f / 255.f), v1 = fmaxf(acc[1], 0.f) * (1.f / 255.f);
        const float v2 = fmaxf(acc[2], 0.f) * (1.f / 255.f), v3 = fmaxf(acc[3], 0.f) * (1.f / 255.f);
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
  const int grid = std::min(p.B, 256 * 14);
  hipLaunchKernelGGL(ref_fwd_kernel, dim3(grid), dim3(64), kFLds, s, p);
}

void ref_backward(const RefBwdParams& p, hipStream_t s) {
  if (p.f32) return ref32_backward(p, s);
  if (p.B <= 0) return;
  hipLaunchKernelGGL(ref_bwd_kernel, dim3(kBwdGrid), dim3(64), kBLds, s, p);
  hipLaunchKernelGGL(ref_bwd_reduce_kernel, dim3(kSlab / 64), dim3(64 * kRedWaves), 0, s, p, kBwdGrid);
}

}  // namespace gpu
}  // namespace mcc
