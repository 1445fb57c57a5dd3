// fp32 conv block of the reference model (cnn.c:416-428) on gfx950:
//   conv1 1->16, 3x3, stride 2, pad 1, ReLU   (28x28 -> 14x14)
//   conv2 16->32, 3x3, stride 2, pad 1, ReLU  (14x14 -> 7x7)
// one forward and one fused backward kernel, the fp32 counterpart of
// refnet.hip (same algorithm: one wave per image, conv1 recomputed in the
// backward, sub-pixel conv2 data gradient), replacing five generic fp32
// launches (conv_fwd_kernel<float> x 3, conv_dw_kernel<float> x 2) that
// round-tripped the 14x14x16 fp32 intermediate through HBM.
//
// Reference semantics: Layer_feedForw_conv / Layer_feedBack_conv
// (/root/reference/cnn.c:175-247, the D1 index bug fixed as in
// CUDAcnn.cu:167-195); exact fp32 products and fp32 accumulation.
//
// Every GEMM runs on v_mfma_f32_16x16x4_f32 (f32 in, f32 accumulate: the
// fp32 matrix rate equals the fp32 vector rate on gfx950, and the MFMA needs
// no FMA-issue bandwidth), lane (r, g = lane >> 4) supplying A[r][g],
// B[g][r], result C[4g + i][r].  With 32 cycles per instruction the kernels
// are MFMA-bound, so operands come from LDS as plain 4- and 16-byte reads
// and the K orders are chosen to minimise padding:
//  * conv1: rows = 16 channels, columns = 16 pixels, K = 9 taps in 3
//    instructions (tap 4j + g);
//  * conv2: rows = output channels, columns = pixels, K = (tap, ci) with
//    lane g holding input channels 4g .. 4g + 3 of a tap (one 16-byte read);
//  * conv2 dW: rows = co, columns = ci, K = output pixels (13 steps of 4);
//    db2 on the VALU;
//  * conv2 dX per sub-pixel phase: rows = ci, columns = pixels, K = co with
//    lane g holding co 8g .. 8g + 7 (two 16-byte reads per tap);
//  * conv1 dW: rows = ci, columns = 9 taps + a ones column (db1), K = the
//    196 conv1 pixels.
// dW / db accumulate in registers across a wave's images; one slab per wave,
// reduced in a fixed order (deterministic).
#include "kernels.h"
#include "mfma.h"
#include "mcc/ab.h"

#include <algorithm>

namespace mcc {
namespace gpu {
namespace {

constexpr int kImgPix = 784;
constexpr int kY2 = 49 * 32;

// ---- LDS (floats) ----
// X / 255, padded: row r = input row r - 1, column c = input column c - 1
// (r, c = 0 .. 28; row / column 0 stay zero); pitch 32.
constexpr int kXP = 32;
constexpr int kXF = 29 * kXP;  // 928
// Y1 HWC, 15 x 15 pixels (row / column 0 zero padding) x 16 channels; the
// backward overwrites it in place with dZ1.
constexpr int kY1 = kXF;
constexpr int kY1F = 225 * 16;  // 3600
// dZ2 HWC on an 8 x 8 grid (row / column 7 zero) x 32 channels (backward)
constexpr int kZ2 = kY1 + kY1F;
constexpr int kZ2F = 64 * 32;  // 2048
constexpr int kFwdLds = (kXF + kY1F) * 4;         // 18,112 B: 8 waves per CU
constexpr int kBwdLds = (kXF + kY1F + kZ2F) * 4;  // 26,304 B
constexpr int kFwdGrid = 256 * 8;
constexpr int kBwdGrid = 256 * 4;  // one wave per SIMD (~340 registers: dW2 accumulators + dX weights)

// per-wave slab: conv2 dW accumulators [2][9][4][64], conv1 dW [4][64], db2 [64]
constexpr int kSlabW2 = 2 * 9 * 4 * 64;  // 4608
constexpr int kSlabW1 = kSlabW2;
constexpr int kSlabB2 = kSlabW1 + 4 * 64;  // 4864
constexpr int kSlab = kSlabB2 + 64;        // 4928

__device__ __forceinline__ f32x4 mfma4(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ void wave_lds_sync() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }
__device__ __forceinline__ f32x4 ld4(const float* p) { return *reinterpret_cast<const f32x4*>(p); }
__device__ __forceinline__ void st4(float* p, const f32x4& v) { *reinterpret_cast<f32x4*>(p) = v; }
// ReLU on the bit pattern (v_max_i32: no NaN canonicalisation, -0 -> +0)
__device__ __forceinline__ float relu(float v) { return __builtin_bit_cast(float, max(__builtin_bit_cast(int, v), 0)); }
__device__ __forceinline__ f32x4 relu4(const f32x4& v) { return f32x4{relu(v[0]), relu(v[1]), relu(v[2]), relu(v[3])}; }
__device__ __forceinline__ void wg_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }
__device__ __forceinline__ void lds_fence() { asm volatile("" ::: "memory"); }

struct WaveIdx {
  int v = 0;
  __device__ __forceinline__ void load(const int32_t* idx, int first, int stride, int B, int k0) {
    const int i = first + (k0 + (int)(threadIdx.x & 63)) * stride;
    v = idx ? idx[min(i, B - 1)] : min(i, B - 1);
  }
  __device__ __forceinline__ int get(int k) const { return __builtin_amdgcn_readlane(v, k & 63); }
};

// u8 image words: lane word w = lane + 64 it (< 196) = row w / 7, pixels 4 (w % 7) ..
__device__ __forceinline__ void load_x(uint32_t (&xw)[4], const uint8_t* xin, int lane) {
#pragma unroll
  for (int it = 0; it < 4; ++it) {
    const int w = min(lane + 64 * it, 195);
    xw[it] = *reinterpret_cast<const uint32_t*>(xin + 4 * w);
  }
}
__device__ __forceinline__ void stage_x(float* smem, const uint32_t (&xw)[4], int lane) {
#pragma unroll
  for (int it = 0; it < 4; ++it) {
    const int w = lane + 64 * it;
    if (w < 196) {
      const int row = (w * 9363) >> 16, c4 = 4 * (w - 7 * row);  // w / 7 for w < 196
      float* d = smem + (row + 1) * kXP + c4 + 1;
#pragma unroll
      for (int e = 0; e < 4; ++e) d[e] = (float)((xw[it] >> (8 * e)) & 0xffu) * (1.f / 255.f);
    }
  }
}
__device__ __forceinline__ void zero_lds(float* p, int floats, int lane) {
  for (int i = lane * 4; i < floats; i += 256) st4(p + i, f32x4{0.f, 0.f, 0.f, 0.f});
}

// conv1 operands: A = W1[channel r][tap 4j + g] (zero for taps >= 9); the
// B offset of the lane's tap relative to the pixel's (2y, 2x) padded corner.
struct Conv1 {
  float w[3];
  int off[3];
  f32x4 bias;
  __device__ __forceinline__ void init(const float* w1, const float* b1, int r, int g) {
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      const int t = 4 * j + g;
      w[j] = t < 9 ? w1[r * 9 + t] : 0.f;
      off[j] = t < 9 ? (t / 3) * kXP + t % 3 : 0;
    }
    bias = f32x4{b1[4 * g], b1[4 * g + 1], b1[4 * g + 2], b1[4 * g + 3]};
  }
  // 13 tiles of 16 pixels -> relu(Y1) into the padded HWC grid
  __device__ __forceinline__ void run(float* smem, int r, int g) const {
#pragma unroll 2
    for (int T = 0; T < 13; ++T) {
      const int px = min(16 * T + r, 195);
      const int y = (px * 2341) >> 15, x = px - 14 * y;  // px / 14 for px < 196
      const float* xb = smem + 2 * y * kXP + 2 * x;
      f32x4 acc = bias;
#pragma unroll
      for (int j = 0; j < 3; ++j) acc = mfma4(w[j], xb[off[j]], acc);
      if (16 * T + r < 196) st4(smem + kY1 + ((y + 1) * 15 + x + 1) * 16 + 4 * g, relu4(acc));
    }
  }
};

// ============================================================================
// Forward
// ============================================================================
__global__ void __launch_bounds__(64) ref32_fwd_kernel(RefFwdParams p) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int lane = threadIdx.x;
  const int r = lane & 15, g = lane >> 4;

  Conv1 c1;
  c1.init(p.w1, p.b1, r, g);
  // conv2 A operand: W2[co = 16 mt + r][ci = 4 g + c][tap t]
  float w2[2][9][4];
#pragma unroll
  for (int mt = 0; mt < 2; ++mt)
#pragma unroll
    for (int t = 0; t < 9; ++t)
#pragma unroll
      for (int c = 0; c < 4; ++c) w2[mt][t][c] = p.w2[((16 * mt + r) * 16 + 4 * g + c) * 9 + t];
  f32x4 b2v[2];
#pragma unroll
  for (int mt = 0; mt < 2; ++mt) b2v[mt] = ld4(p.b2 + 16 * mt + 4 * g);

  zero_lds(smem, kXF + kY1F, lane);
  wave_lds_sync();

  uint32_t xw[4];
  WaveIdx widx;
  widx.load(p.idx, blockIdx.x, (int)gridDim.x, p.B, 0);
  auto load_img = [&](int k) {
    if ((k & 63) == 0 && k > 0) widx.load(p.idx, blockIdx.x, (int)gridDim.x, p.B, k);
    load_x(xw, p.x + (size_t)widx.get(k) * kImgPix, lane);
  };
  if ((int)blockIdx.x < p.B) load_img(0);

  float* y2all = static_cast<float*>(p.y2);
  for (int img = blockIdx.x, kimg = 0; img < p.B; img += (int)gridDim.x, ++kimg) {
    wave_lds_sync();
    stage_x(smem, xw, lane);
    wave_lds_sync();
    if (img + (int)gridDim.x < p.B) load_img(kimg + 1);

    c1.run(smem, r, g);
    wave_lds_sync();

    // ---- conv2: 4 tiles of 16 output pixels x 2 channel tiles, K = 9 taps x 16 ci ----
    float* y2g = y2all + (size_t)img * kY2;
#pragma unroll 1
    for (int T = 0; T < 4; ++T) {
      const int q = min(16 * T + r, 48);
      const int oy = (q * 9363) >> 16, ox = q - 7 * oy;  // q / 7
      const float* yb = smem + kY1 + (2 * oy * 15 + 2 * ox) * 16 + 4 * g;
      f32x4 acc[2] = {b2v[0], b2v[1]};
#pragma unroll
      for (int t = 0; t < 9; ++t) {
        const f32x4 v = ld4(yb + ((t / 3) * 15 + t % 3) * 16);
#pragma unroll
        for (int c = 0; c < 4; ++c)
#pragma unroll
          for (int mt = 0; mt < 2; ++mt) acc[mt] = mfma4(w2[mt][t][c], v[c], acc[mt]);
      }
      if (16 * T + r < 49) {
#pragma unroll
        for (int mt = 0; mt < 2; ++mt) st4(y2g + q * 32 + 16 * mt + 4 * g, relu4(acc[mt]));
      }
    }
  }
}

// ============================================================================
// Backward
// ============================================================================
// Sub-pixel phases of conv2's data gradient: conv1 pixel (y, x) = (2i + py,
// 2j + px) receives dZ2 at (i + di, j + dj) through tap (kh, kw):
//   py = 0: (kh 1, di 0);  py = 1: (kh 0, di 1), (kh 2, di 0)   (same in x).
// Tile T of a phase: lane r -> i = 2T + (r >> 3), j = r & 7 (7 = padding).
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(1, 1))) ref32_bwd_kernel(RefBwdParams p) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int lane = threadIdx.x;
  const int r = lane & 15, g = lane >> 4;

  Conv1 c1;
  c1.init(p.w1, p.b1, r, g);
  // conv2 dX A operand per tap: W2[co = 8 g + s][ci = r][t]
  float wdx[9][8];
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int s = 0; s < 8; ++s) wdx[t][s] = p.w2[((8 * g + s) * 16 + r) * 9 + t];

  zero_lds(smem, kXF + kY1F + kZ2F, lane);
  wave_lds_sync();

  f32x4 acc2[2][9];
#pragma unroll
  for (int mt = 0; mt < 2; ++mt)
#pragma unroll
    for (int t = 0; t < 9; ++t) acc2[mt][t] = f32x4{0.f, 0.f, 0.f, 0.f};
  f32x4 acc1 = {0.f, 0.f, 0.f, 0.f};
  float db2 = 0.f;
  // conv1 dW B operand: tap r of the lane's pixel (r = 9: ones for db1)
  const int x1off = r < 9 ? (r / 3) * kXP + r % 3 : 0;
  const float x1one = r == 9 ? 1.f : 0.f;

  uint32_t xw[4];
  f32x4 dyv[7], y2v[7];
  const float* y2all = static_cast<const float*>(p.y2);
  const float* dyall = static_cast<const float*>(p.dy2);
  WaveIdx widx;
  widx.load(p.idx, blockIdx.x, (int)gridDim.x, p.B, 0);
  auto load_img = [&](int k) {
    const int img = blockIdx.x + k * (int)gridDim.x;
    if ((k & 63) == 0 && k > 0) widx.load(p.idx, blockIdx.x, (int)gridDim.x, p.B, k);
    load_x(xw, p.x + (size_t)widx.get(k) * kImgPix, lane);
#pragma unroll
    for (int it = 0; it < 7; ++it) {
      const int e4 = min(lane + 64 * it, 391);
      dyv[it] = ld4(dyall + (size_t)img * kY2 + 4 * e4);
      y2v[it] = ld4(y2all + (size_t)img * kY2 + 4 * e4);
    }
  };
  if ((int)blockIdx.x < p.B) load_img(0);

  for (int img = blockIdx.x, kimg = 0; img < p.B; img += (int)gridDim.x, ++kimg) {
    wave_lds_sync();
    stage_x(smem, xw, lane);
    // dZ2 = dY2 * (Y2 > 0) into the 8 x 8 grid
#pragma unroll
    for (int it = 0; it < 7; ++it) {
      const int e4 = lane + 64 * it;
      if (e4 < 392) {
        const int q = e4 >> 3, c4 = 4 * (e4 & 7);
        const int oy = (q * 9363) >> 16, ox = q - 7 * oy;
        f32x4 z;
#pragma unroll
        for (int k = 0; k < 4; ++k) z[k] = y2v[it][k] > 0.f ? dyv[it][k] : 0.f;
        st4(smem + kZ2 + (oy * 8 + ox) * 32 + c4, z);
      }
    }
    wave_lds_sync();
    if (img + (int)gridDim.x < p.B) load_img(kimg + 1);

    // ---- recompute conv1 -> Y1 ----
    c1.run(smem, r, g);
    wave_lds_sync();

    // ---- conv2 dW: acc2[mt][t] += dZ2^T (co) . Y1 patches (ci), K = output pixels ----
#pragma unroll 1
    for (int s = 0; s < 13; ++s) {
      const int q = 4 * s + g;
      const bool ok = q < 49;
      const int oy = (q * 9363) >> 16, ox = q - 7 * oy;
      const float* zb = smem + kZ2 + (ok ? oy * 8 + ox : 63) * 32 + r;  // (7, 7): zero
      const float* yb = smem + kY1 + (ok ? (2 * oy * 15 + 2 * ox) * 16 : 0) + r;
      const float a0 = zb[0], a1 = zb[16];
      float b[9];
#pragma unroll
      for (int t = 0; t < 9; ++t) b[t] = yb[((t / 3) * 15 + t % 3) * 16];
#pragma unroll
      for (int t = 0; t < 9; ++t) {
        acc2[0][t] = mfma4(a0, b[t], acc2[0][t]);
        acc2[1][t] = mfma4(a1, b[t], acc2[1][t]);
      }
    }
    // db2 (VALU): lane -> co = lane & 31, pixels of parity lane >> 5
#pragma unroll 5
    for (int q = lane >> 5; q < 49; q += 2) {
      const int oy = (q * 9363) >> 16, ox = q - 7 * oy;
      db2 += smem[kZ2 + (oy * 8 + ox) * 32 + (lane & 31)];
    }
    wave_lds_sync();

    // ---- conv2 dX by phase: dY1^T = W2 . dZ2 patches; dZ1 = dY1 * (Y1 > 0) over Y1 in place ----
#pragma unroll
    for (int ph = 0; ph < 4; ++ph) {
      const int py = ph >> 1, pxx = ph & 1;
#pragma unroll 1
      for (int T = 0; T < 4; ++T) {
        const int i = 2 * T + (r >> 3), j = r & 7;
        const bool ok = i < 7 && j < 7;
        const float* zb = smem + kZ2 + (min(i, 6) * 8 + min(j, 6)) * 32 + 8 * g;
        f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int a = 0; a < 2; ++a) {
          if (py == 0 && a == 1) continue;
          const int kh = py == 0 ? 1 : (a == 0 ? 0 : 2), di = py == 1 && a == 0 ? 1 : 0;
#pragma unroll
          for (int b = 0; b < 2; ++b) {
            if (pxx == 0 && b == 1) continue;
            const int kw = pxx == 0 ? 1 : (b == 0 ? 0 : 2), dj = pxx == 1 && b == 0 ? 1 : 0;
            const f32x4 z0 = ld4(zb + (di * 8 + dj) * 32), z1 = ld4(zb + (di * 8 + dj) * 32 + 4);
#pragma unroll
            for (int s = 0; s < 4; ++s) acc = mfma4(wdx[kh * 3 + kw][s], z0[s], acc);
#pragma unroll
            for (int s = 0; s < 4; ++s) acc = mfma4(wdx[kh * 3 + kw][4 + s], z1[s], acc);
          }
        }
        if (ok) {
          const int y = 2 * i + py, x = 2 * j + pxx;
          float* yp = smem + kY1 + ((y + 1) * 15 + x + 1) * 16 + 4 * g;
          const f32x4 y1 = ld4(yp);
          f32x4 dz;
#pragma unroll
          for (int k = 0; k < 4; ++k) dz[k] = y1[k] > 0.f ? acc[k] : 0.f;
          st4(yp, dz);
        }
      }
    }
    wave_lds_sync();

    // ---- conv1 dW: acc1 += dZ1^T (rows ci) . X patches (columns taps; 9 = ones), K = 196 pixels ----
#pragma unroll 7
    for (int s = 0; s < 49; ++s) {
      const int px = 4 * s + g;
      const int y = (px * 2341) >> 15, x = px - 14 * y;
      const float a = smem[kY1 + ((y + 1) * 15 + x + 1) * 16 + r];
      const float bx = smem[2 * y * kXP + 2 * x + x1off];
      acc1 = mfma4(a, r < 9 ? bx : x1one, acc1);
    }
  }

  // ---- per-wave slab (accumulator order) ----
  float* slab = p.slab + (size_t)blockIdx.x * kSlab;
#pragma unroll
  for (int mt = 0; mt < 2; ++mt)
#pragma unroll
    for (int t = 0; t < 9; ++t)
#pragma unroll
      for (int i = 0; i < 4; ++i) slab[((mt * 9 + t) * 4 + i) * 64 + lane] = acc2[mt][t][i];
#pragma unroll
  for (int i = 0; i < 4; ++i) slab[kSlabW1 + i * 64 + lane] = acc1[i];
  slab[kSlabB2 + lane] = db2;
}

// ---- two-wave backward ----
// ref32_bwd_kernel holds the dW2 accumulators and the dX weights in one wave
// (one wave per SIMD), so its 610 MFMAs per image run with every LDS and
// dependency latency exposed (2.7 ms for a 1.3 ms MFMA floor). Here a
// workgroup of two waves shares one image, the roles split by register set:
//   wave 0: stages image k's X (global loads one image ahead), recomputes
//           conv1 -> Y1, then conv2 dW / db (39 + 234 MFMAs);
//   wave 1: stages image k's dZ2 = dY2 * (Y2 > 0) (its 56 prefetch registers
//           fit beside the dX weights, not beside the dW2 accumulators), then
//           conv2 dX -> dZ1 (compact, wave-private; the ReLU mask read from
//           Y1) and conv1 dW (288 + 49 MFMAs).
// Two barriers per image (A: image staged, B: both done with it); the other
// workgroup's waves on the SIMD fill the barrier waits. 2 waves per SIMD.
constexpr int kB2Z1 = kZ2 + kZ2F;               // dZ1 [196 pixels][16 ci] (wave 1)
constexpr int kB2Floats = kB2Z1 + 196 * 16;     // 9712
constexpr int kBwd2Lds = kB2Floats * 4;         // 38,848 B
static_assert(4 * kBwd2Lds <= 163840, "ref32_bwd2: four workgroups per CU");

__global__ void __launch_bounds__(128) __attribute__((amdgpu_waves_per_eu(2, 2))) ref32_bwd2_kernel(RefBwdParams p) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int r = lane & 15, g = lane >> 4;
  const int grid = (int)gridDim.x;
  for (int i = (int)threadIdx.x * 4; i < kB2Floats; i += 128 * 4) st4(smem + i, f32x4{0.f, 0.f, 0.f, 0.f});
  wg_barrier();
  float* slab = p.slab + (size_t)blockIdx.x * kSlab;

  if (wv == 0) {
    Conv1 c1;
    c1.init(p.w1, p.b1, r, g);
    f32x4 acc2[2][9];
#pragma unroll
    for (int mt = 0; mt < 2; ++mt)
#pragma unroll
      for (int t = 0; t < 9; ++t) acc2[mt][t] = f32x4{0.f, 0.f, 0.f, 0.f};
    float db2 = 0.f;
    uint32_t xw[4];
    WaveIdx widx;
    widx.load(p.idx, blockIdx.x, grid, p.B, 0);
    auto load_img = [&](int k) {
      if ((k & 63) == 0 && k > 0) widx.load(p.idx, blockIdx.x, grid, p.B, k);
      load_x(xw, p.x + (size_t)widx.get(k) * kImgPix, lane);
    };
    if ((int)blockIdx.x < p.B) load_img(0);
    for (int img = blockIdx.x, k = 0; img < p.B; img += grid, ++k) {
      stage_x(smem, xw, lane);
      if (img + grid < p.B) load_img(k + 1);
      lds_fence();
      c1.run(smem, r, g);
      wg_barrier();  // A: X, dZ2, Y1 of image k ready
      // conv2 dW: acc2[mt][t] += dZ2^T (co) . Y1 patches (ci), K = output pixels
#pragma unroll 2
      for (int s = 0; s < 13; ++s) {  // (2 steps per iteration: the next step's reads overlap these MFMAs)
        const int q = 4 * s + g;
        const bool ok = q < 49;
        const int oy = (q * 9363) >> 16, ox = q - 7 * oy;
        const float* zb = smem + kZ2 + (ok ? oy * 8 + ox : 63) * 32 + r;  // (7, 7): zero
        const float* yb = smem + kY1 + (ok ? (2 * oy * 15 + 2 * ox) * 16 : 0) + r;
        const float a0 = zb[0], a1 = zb[16];
        float b[9];
#pragma unroll
        for (int t = 0; t < 9; ++t) b[t] = yb[((t / 3) * 15 + t % 3) * 16];
#pragma unroll
        for (int t = 0; t < 9; ++t) {
          acc2[0][t] = mfma4(a0, b[t], acc2[0][t]);
          acc2[1][t] = mfma4(a1, b[t], acc2[1][t]);
        }
      }
      // db2 (VALU): lane -> co = lane & 31, pixels of parity lane >> 5
#pragma unroll 5
      for (int q = lane >> 5; q < 49; q += 2) {
        const int oy = (q * 9363) >> 16, ox = q - 7 * oy;
        db2 += smem[kZ2 + (oy * 8 + ox) * 32 + (lane & 31)];
      }
      wg_barrier();  // B: image k consumed
    }
#pragma unroll
    for (int mt = 0; mt < 2; ++mt)
#pragma unroll
      for (int t = 0; t < 9; ++t)
#pragma unroll
        for (int i = 0; i < 4; ++i) slab[((mt * 9 + t) * 4 + i) * 64 + lane] = acc2[mt][t][i];
    slab[kSlabB2 + lane] = db2;
  } else {
    // conv2 dX A operand per tap: W2[co = 8 g + s][ci = r][t]
    float wdx[9][8];
#pragma unroll
    for (int t = 0; t < 9; ++t)
#pragma unroll
      for (int s = 0; s < 8; ++s) wdx[t][s] = p.w2[((8 * g + s) * 16 + r) * 9 + t];
    f32x4 acc1 = {0.f, 0.f, 0.f, 0.f};
    // conv1 dW B operand: tap r of the lane's pixel (r = 9: ones for db1)
    const int x1off = r < 9 ? (r / 3) * kXP + r % 3 : 0;
    const float x1one = r == 9 ? 1.f : 0.f;
    // dZ2 staging (this wave has the free registers for the one-image-ahead loads)
    f32x4 dyv[7], y2v[7];
    const float* y2all = static_cast<const float*>(p.y2);
    const float* dyall = static_cast<const float*>(p.dy2);
    auto load_img = [&](int img) {
#pragma unroll
      for (int it = 0; it < 7; ++it) {
        const int e4 = min(lane + 64 * it, 391);
        dyv[it] = ld4(dyall + (size_t)img * kY2 + 4 * e4);
        y2v[it] = ld4(y2all + (size_t)img * kY2 + 4 * e4);
      }
    };
    if ((int)blockIdx.x < p.B) load_img(blockIdx.x);
    for (int img = blockIdx.x; img < p.B; img += grid) {
      // dZ2 = dY2 * (Y2 > 0) into the 8 x 8 grid
#pragma unroll
      for (int it = 0; it < 7; ++it) {
        const int e4 = lane + 64 * it;
        if (e4 < 392) {
          const int q = e4 >> 3, c4 = 4 * (e4 & 7);
          const int oy = (q * 9363) >> 16, ox = q - 7 * oy;
          f32x4 z;
#pragma unroll
          for (int e = 0; e < 4; ++e) z[e] = y2v[it][e] > 0.f ? dyv[it][e] : 0.f;
          st4(smem + kZ2 + (oy * 8 + ox) * 32 + c4, z);
        }
      }
      if (img + grid < p.B) load_img(img + grid);
      wg_barrier();  // A
      // conv2 dX by phase: dY1^T = W2 . dZ2 patches; dZ1 = dY1 * (Y1 > 0). The
      // phase's 4 tiles run together: 4 independent accumulator chains, and a
      // tap's 8 fragment reads are issued a tap ahead of its MFMAs.
#pragma unroll
      for (int ph = 0; ph < 4; ++ph) {
        const int py = ph >> 1, pxx = ph & 1;
        constexpr int kTaps[4] = {1, 2, 2, 4};
        f32x4 acc[4];
#pragma unroll
        for (int T = 0; T < 4; ++T) acc[T] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int u = 0; u < kTaps[ph]; ++u) {
          // tap u of the phase: (a, b) = (u >> 1, u & 1) for phase 3, else the single varying index
          const int a = py == 0 ? 0 : (pxx == 0 ? u : u >> 1);
          const int b = pxx == 0 ? 0 : (py == 0 ? u : u & 1);
          const int kh = py == 0 ? 1 : (a == 0 ? 0 : 2), di = py == 1 && a == 0 ? 1 : 0;
          const int kw = pxx == 0 ? 1 : (b == 0 ? 0 : 2), dj = pxx == 1 && b == 0 ? 1 : 0;
          f32x4 z[4][2];
#pragma unroll
          for (int T = 0; T < 4; ++T) {
            const int i = 2 * T + (r >> 3), j = r & 7;
            const float* zb = smem + kZ2 + (min(i, 6) * 8 + min(j, 6)) * 32 + 8 * g + (di * 8 + dj) * 32;
            z[T][0] = ld4(zb);
            z[T][1] = ld4(zb + 4);
          }
#pragma unroll
          for (int s2 = 0; s2 < 8; ++s2)
#pragma unroll
            for (int T = 0; T < 4; ++T) acc[T] = mfma4(wdx[kh * 3 + kw][s2], z[T][s2 >> 2][s2 & 3], acc[T]);
        }
#pragma unroll
        for (int T = 0; T < 4; ++T) {
          const int i = 2 * T + (r >> 3), j = r & 7;
          if (i < 7 && j < 7) {
            const int y = 2 * i + py, x = 2 * j + pxx;
            const f32x4 y1 = ld4(smem + kY1 + ((y + 1) * 15 + x + 1) * 16 + 4 * g);
            f32x4 dz;
#pragma unroll
            for (int e = 0; e < 4; ++e) dz[e] = y1[e] > 0.f ? acc[T][e] : 0.f;
            st4(smem + kB2Z1 + (y * 14 + x) * 16 + 4 * g, dz);
          }
        }
      }
      lds_fence();
      // conv1 dW: acc1 += dZ1^T (rows ci) . X patches (columns taps; 9 = ones), K = 196 pixels
#pragma unroll 7
      for (int s = 0; s < 49; ++s) {
        const int px = 4 * s + g;
        const int y = (px * 2341) >> 15, x = px - 14 * y;
        const float a = smem[kB2Z1 + px * 16 + r];
        const float bx = smem[2 * y * kXP + 2 * x + x1off];
        acc1 = mfma4(a, r < 9 ? bx : x1one, acc1);
      }
      wg_barrier();  // B
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) slab[kSlabW1 + i * 64 + lane] = acc1[i];
  }
}

// Fixed-order sum of the per-wave slabs -> canonical gradients.
constexpr int kRedWaves = 16;
__global__ void __launch_bounds__(64 * kRedWaves) ref32_bwd_reduce_kernel(RefBwdParams p, int nslabs) {
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
    const int slot = pos >> 6, ln = pos & 63;
    const int mt = slot / 36, t = (slot >> 2) % 9, i = slot & 3;
    const int co = 16 * mt + 4 * (ln >> 4) + i, ci = ln & 15;
    p.gw2[(co * 16 + ci) * 9 + t] = v;
  } else if (pos < kSlabB2) {
    const int q = pos - kSlabW1, i = q >> 6, ln = q & 63;
    const int ci = 4 * (ln >> 4) + i, t = ln & 15;
    if (t < 9) p.gw1[ci * 9 + t] = v;
    else if (t == 9) p.gb1[ci] = v;
  } else {
    const float both = v + __shfl_down(v, 32);  // the two pixel parities of co = l
    if (l < 32) p.gb2[l] = both;
  }
}

}  // namespace

size_t ref32_slab_bytes() { return (size_t)kBwdGrid * kSlab * 4; }

void ref32_forward(const RefFwdParams& p, hipStream_t s) {
  if (p.B <= 0) return;
  const int grid = std::min(p.B, kFwdGrid);
  hipLaunchKernelGGL(ref32_fwd_kernel, dim3(grid), dim3(64), kFwdLds, s, p);
}

void ref32_backward(const RefBwdParams& p, hipStream_t s) {
  if (p.B <= 0) return;
  if (ab_flag("ref_bwd1")) hipLaunchKernelGGL(ref32_bwd_kernel, dim3(kBwdGrid), dim3(64), kBwdLds, s, p);
  else hipLaunchKernelGGL(ref32_bwd2_kernel, dim3(kBwdGrid), dim3(128), kBwd2Lds, s, p);
  hipLaunchKernelGGL(ref32_bwd_reduce_kernel, dim3(kSlab / 64), dim3(64 * kRedWaves), 0, s, p, kBwdGrid);
}

}  // namespace gpu
}  // namespace mcc
