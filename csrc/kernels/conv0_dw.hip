// Weight gradient of the large-image FIRST conv layer (u8 input with few
// channels, 3x3, stride 1, pad 1, fused ReLU + 2x2/2 max-pool): VGG-11's
// conv1, bf16.
//
//   dW[co][c][ky][kx] = sum_px dZ[px][co] X(px, (ky,kx,c)),  db[co] = sum_px dZ[px][co]
//   (reference math: Layer_feedBack_conv, cnn.c:212-247; OIHW as CUDAcnn.cu)
//
// The generic path for this layer materialised dZ = unpool(dY) at full
// resolution (grad_xform: 1.6 GB written + read at B=256, 224^2, 64 channels)
// and an im2col copy of the u8 input (0.8 GB), then ran the implicit-GEMM dW
// over both: ~2 ms/step for a 46 GFLOP GEMM whose inputs are 0.6 GB.  Here the
// GEMM operands are built in LDS straight from the pooled dY / argmax and the
// u8 images, so the kernel reads each pooled gradient once:
//
//   * K = pixels, walked in pooled-window order: a K-step is 16 windows = 64
//     pixels; the dZ^T tile [co][px] takes the window's dY at its argmax
//     position and zeros at the other three (argmax 4 = ReLU-inactive: all
//     zero), one 8-byte LDS store per (channel, window);
//   * the X^T tile [k][px], k = (ky*3 + kx)*C + c plus a ones column (bias),
//     is gathered from the u8 image (bf16 of x/255, as the forward stages it);
//   * MFMA 16x16x32 bf16, each wave owns 16 output channels x 32 columns;
//     the next K-step's loads are issued before the current MFMAs (register
//     prefetch), LDS double-buffered, one barrier per step;
//   * per-workgroup fp32 slabs, reduced over workgroups in a fixed order.
#include "kernels.h"
#include "mcc/ab.h"
#include "mfma.h"

#include <algorithm>

namespace mcc {
namespace gpu {

namespace {

typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));

constexpr int kC0T = 256;      // threads: 4 waves x 16 output channels
constexpr int kC0W = 16;       // pooled windows per K-step (64 pixels)
constexpr int kC0K = 32;       // GEMM columns: KS*KS*C taps + ones column, padded
constexpr int kC0Ld = 64 + 8;  // LDS row stride (bf16) of the [row][px] tiles

__global__ void __launch_bounds__(kC0T) conv0_dw_kernel(Conv0DwParams p) {
  __shared__ __attribute__((aligned(16))) bf16 Dt[2][64 * kC0Ld];     // dZ^T [co][px]
  __shared__ __attribute__((aligned(16))) bf16 Xt[2][kC0K * kC0Ld];   // X^T [k][px]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r16 = lane & 15, g = lane >> 4;
  const int PHW = p.PH * p.PW;
  const int64_t nwin = (int64_t)p.B * PHW;  // < 2^24 (conv0_dw_supported): exact magic division
  const Div d_phw(PHW), d_pw(p.PW);
  const int64_t nsteps = (nwin + kC0W - 1) / kC0W;
  const int64_t per = (nsteps + gridDim.x - 1) / gridDim.x;
  const int64_t s0 = (int64_t)blockIdx.x * per, s1 = nsteps < s0 + per ? nsteps : s0 + per;
  const int kf = 9 * p.C;

  // D staging: window w (0..15), four channels co4..co4+3
  const int dw_ = tid >> 4, co4 = (tid & 15) * 4;
  // X staging: pixel xp (0..63) of the step, columns 8*xq .. 8*xq+7
  const int xp = tid >> 2, xq = tid & 3;
  int kky[8], kkx[8], kc[8], kkind[8];  // kind 0 tap, 1 ones, 2 zero
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const int k = 8 * xq + e;
    const int tap = k / p.C;
    kc[e] = k - tap * p.C;
    kky[e] = tap / 3;
    kkx[e] = tap - kky[e] * 3;
    kkind[e] = k < kf ? 0 : (k == kf ? 1 : 2);
  }

  uint2 dv = make_uint2(0, 0);  // 4 bf16 of dY
  uint32_t da = 0x04040404u;    // 4 argmax bytes
  uint32_t xv[4];               // 8 bf16 of X
  auto load = [&](int64_t step) {
    {
      const int64_t w = step * kC0W + dw_;
      const bool ok = w < nwin && co4 < p.Cout;
      const int64_t o = ok ? w * p.Cout + co4 : 0;
      dv = ok ? *reinterpret_cast<const uint2*>(p.dy + o) : make_uint2(0, 0);
      da = ok ? *reinterpret_cast<const uint32_t*>(p.arg + o) : 0x04040404u;
    }
    {
      const int64_t w = step * kC0W + (xp >> 2);
      const int pos = xp & 3;
      const bool wok = w < nwin;
      const int wi = wok ? (int)w : 0;  // 64-bit divisions here were ~200 VALU per K-step
      const int b = d_phw.div(wi);
      const int rem = wi - b * PHW;
      const int wy = d_pw.div(rem), wx = rem - wy * p.PW;
      const int y = 2 * wy + (pos >> 1), x = 2 * wx + (pos & 1);
      const int img = p.idx ? p.idx[b] : b;
      const uint8_t* src = p.x + (size_t)img * p.H * p.W * p.C;
      float f[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int iy = y + kky[e] - 1, ix = x + kkx[e] - 1;
        const bool in = wok && kkind[e] == 0 && (unsigned)iy < (unsigned)p.H && (unsigned)ix < (unsigned)p.W;
        const int off = in ? (iy * p.W + ix) * p.C + kc[e] : 0;
        const float v = (float)src[off] * (1.0f / 255.0f);
        f[e] = in ? v : ((wok && kkind[e] == 1) ? 1.f : 0.f);
      }
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const bf16x2 h = {(bf16)f[2 * e], (bf16)f[2 * e + 1]};
        xv[e] = __builtin_bit_cast(uint32_t, h);
      }
    }
  };
  auto store = [&](int buf) {
    bf16* D = Dt[buf];
    const uint16_t v[4] = {(uint16_t)(dv.x & 0xffffu), (uint16_t)(dv.x >> 16), (uint16_t)(dv.y & 0xffffu),
                           (uint16_t)(dv.y >> 16)};
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const uint32_t a = (da >> (8 * c)) & 0xffu;
      const uint32_t lo = (a == 0 ? (uint32_t)v[c] : 0u) | (a == 1 ? (uint32_t)v[c] << 16 : 0u);
      const uint32_t hi = (a == 2 ? (uint32_t)v[c] : 0u) | (a == 3 ? (uint32_t)v[c] << 16 : 0u);
      *reinterpret_cast<uint2*>(D + (co4 + c) * kC0Ld + 4 * dw_) = make_uint2(lo, hi);
    }
    bf16* X = Xt[buf];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const uint32_t w2 = xv[e];
      X[(8 * xq + 2 * e) * kC0Ld + xp] = __builtin_bit_cast(bf16, (uint16_t)(w2 & 0xffffu));
      X[(8 * xq + 2 * e + 1) * kC0Ld + xp] = __builtin_bit_cast(bf16, (uint16_t)(w2 >> 16));
    }
  };

  f32x4 acc[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
  const int corow = wave * 16 + r16;  // A row (output channel) of this lane
  if (s0 < s1) load(s0);
  for (int64_t s = s0; s < s1; ++s) {
    const int buf = (int)((s - s0) & 1);
    store(buf);
    __syncthreads();
    if (s + 1 < s1) load(s + 1);
    const bf16* D = Dt[buf];
    const bf16* X = Xt[buf];
#pragma unroll
    for (int h = 0; h < 2; ++h) {  // 32 pixels each
      const bf16x8 a = load8(D + corow * kC0Ld + 32 * h + 8 * g);
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const bf16x8 b = load8(X + (16 * j + r16) * kC0Ld + 32 * h + 8 * g);
        acc[j] = mma(acc[j], a, b);
      }
    }
  }
  // slab[wg][co][k]: lane holds rows (co) 4g..4g+3 of column r16 of tile j
  float* slab = p.slab + (size_t)blockIdx.x * 64 * kC0K;
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int i = 0; i < 4; ++i) slab[(wave * 16 + 4 * g + i) * kC0K + 16 * j + r16] = acc[j][i];
}

// dW[co][c][ky][kx] (k = (ky*3 + kx)*C + c) and db[co] (k = 9C): a fixed-order
// sum over the workgroup slabs, one workgroup per output column
__global__ void __launch_bounds__(256) conv0_dw_reduce_kernel(Conv0DwParams p, int nslab, float* gw, float* gb) {
  __shared__ float part[256];
  const int col = blockIdx.x;  // co * kC0K + k
  const int co = col / kC0K, k = col - co * kC0K;
  const int kf = 9 * p.C;
  float v = 0.f;
  for (int s = threadIdx.x; s < nslab; s += 256) v += p.slab[(size_t)s * 64 * kC0K + col];
  part[threadIdx.x] = v;
  __syncthreads();
  for (int hh = 128; hh > 0; hh >>= 1) {
    if ((int)threadIdx.x < hh) part[threadIdx.x] += part[threadIdx.x + hh];
    __syncthreads();
  }
  if (threadIdx.x != 0 || co >= p.Cout || k > kf) return;
  if (k == kf) {
    gb[co] = part[0];
  } else {
    const int tap = k / p.C, c = k - tap * p.C;
    gw[((size_t)co * p.C + c) * 9 + tap] = part[0];
  }
}

// ---------------------------------------------------------------------------
// Row-staged variant for C = 3, Cout = 32 / 64, W % 32 == 0 (CIFAR-3conv
// conv1 at 32x32, VGG-11 conv1 at 224x224).  The kernel above gathers the X^T
// tile byte by byte from global memory (8 scattered loads per thread per
// K-step plus a pixel decode); here the operands come from LDS-staged rows:
//   * unit = (image, pooled row, 16-window segment) = 2 x 32 pixels; one wave
//     owns a unit, staging into its own LDS region (no workgroup barriers) the
//     4 u8 input rows it touches (26 dwords each, zero outside the image) and
//     the segment's pooled dY / argmax transposed to [co][window]; the next
//     unit's dwords are in flight in registers meanwhile;
//   * K-step = one pixel row of the segment (32 pixels), lane group g owns
//     pixels 8g..8g+7 = windows 4g..4g+3: the A fragment (dZ^T) is one
//     ds_read_b64 of dY + one ds_read_b32 of argmax, the value routed to its
//     argmax pixel with selects;
//   * the B fragment (X^T, column = tap (ky, kx, c) or the ones column) is 8
//     bytes at stride 3 of one staged row: two ds_read_b128, six v_alignbyte
//     by the lane-constant (1 + 3kx + c) & 3 (after which every byte sits at a
//     fixed position), eight v_cvt_f32_ubyteN; u8 integers are exact in bf16
//     and 1/255 is applied to the fp32 tap columns at the end;
//   * waves accumulate privately, reduce through LDS once, and write the same
//     [wg][64][32] slab as the kernel above (same fixed-order reduce).
constexpr int kRT = 256;          // 4 waves
constexpr int kRRow = 112;        // staged row pitch (bytes): 26 dwords + b128 over-read
constexpr int kRDp = 20;          // dY^T pitch (bf16) / argmax^T pitch (bytes)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <int NT>  // NT = Cout / 16
__global__ void __launch_bounds__(kRT) conv0_dw_rows_kernel(Conv0DwParams p) {
  constexpr int COUT = 16 * NT;
  constexpr int PER_WAVE = 4 * kRRow + COUT * kRDp * 2 + COUT * kRDp;  // bytes
  constexpr int RDY = COUT / 8, RAR = COUT / 16;                      // dY / argmax dwords per lane
  __shared__ __attribute__((aligned(16))) uint8_t lds[4 * PER_WAVE];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r = lane & 15, g = lane >> 4;
  uint8_t* rows = lds + wave * PER_WAVE;
  uint16_t* Dt = reinterpret_cast<uint16_t*>(rows + 4 * kRRow);
  uint8_t* At = rows + 4 * kRRow + COUT * kRDp * 2;
  for (int i = lane; i < kRRow; i += 64) reinterpret_cast<uint32_t*>(rows)[i] = 0u;  // 4 rows

  // B column of this lane per tile j: k = 16j + r: tap (ky, kx, c) = (k/9, k%9/3, k%3), 27 = ones
  int boff[2], bsh[2], bky[2];
  bool btap[2], bone[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int k = 16 * j + r;
    const int kk = k < 27 ? k : 0;
    const int ky = kk / 9, kx = (kk % 9) / 3, c = kk % 3;
    const int o0 = 1 + 3 * (8 * g + kx) + c;  // byte of pixel 8g - 1 + kx, channel c, in the staged row
    boff[j] = o0 & ~3;
    bsh[j] = o0 & 3;
    bky[j] = ky;
    btap[j] = k < 27;
    bone[j] = k == 27;
  }

  const int PH = p.PH, nseg = p.PW / 16;
  const int64_t nunits = (int64_t)p.B * PH * nseg;
  const int64_t wid = (int64_t)blockIdx.x * 4 + wave, nw = (int64_t)gridDim.x * 4;
  const int RW = 3 * p.W / 4;  // dwords per image row

  uint32_t prow[2], pdy[RDY], par[RAR];
  auto fetch = [&](int64_t u) {
    const int seg = (int)(u % nseg);
    const int64_t bw = u / nseg;
    const int b = (int)(bw / PH), wy = (int)(bw - (int64_t)b * PH);
    const int img = p.idx ? p.idx[b] : b;
    const uint8_t* src = p.x + (size_t)img * p.H * p.W * 3;
#pragma unroll
    for (int q = 0; q < 2; ++q) {  // 4 rows x 26 dwords: dword 24*seg - 1 + d of row 2wy - 1 + rr
      const int i = lane + 64 * q;
      const int rr = i / 26, d = i - rr * 26;
      const int y = 2 * wy - 1 + rr, dw = 24 * seg - 1 + d;
      const bool ok = i < 104 && (unsigned)y < (unsigned)p.H && (unsigned)dw < (unsigned)RW;
      prow[q] = ok ? reinterpret_cast<const uint32_t*>(src + (size_t)y * p.W * 3)[dw] : 0u;
    }
    const size_t w0 = ((size_t)b * PH + wy) * p.PW + 16 * seg;  // first window of the segment
    const uint32_t* gdy = reinterpret_cast<const uint32_t*>(p.dy + w0 * COUT);
    const uint32_t* gar = reinterpret_cast<const uint32_t*>(p.arg + w0 * COUT);
#pragma unroll
    for (int q = 0; q < RDY; ++q) pdy[q] = gdy[lane + 64 * q];
#pragma unroll
    for (int q = 0; q < RAR; ++q) par[q] = gar[lane + 64 * q];
  };
  auto stash = [&]() {
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int i = lane + 64 * q;
      const int rr = i / 26, d = i - rr * 26;
      if (i < 104) reinterpret_cast<uint32_t*>(rows + rr * kRRow)[d] = prow[q];
    }
#pragma unroll
    for (int q = 0; q < RDY; ++q) {  // dword = channels (co, co+1) of window wx
      const int e = 2 * (lane + 64 * q);
      const int wx = e / COUT, co = e % COUT;
      Dt[co * kRDp + wx] = (uint16_t)(pdy[q] & 0xffffu);
      Dt[(co + 1) * kRDp + wx] = (uint16_t)(pdy[q] >> 16);
    }
#pragma unroll
    for (int q = 0; q < RAR; ++q) {  // dword = channels co..co+3 of window wx
      const int e = 4 * (lane + 64 * q);
      const int wx = e / COUT, co = e % COUT;
#pragma unroll
      for (int t = 0; t < 4; ++t) At[(co + t) * kRDp + wx] = (uint8_t)(par[q] >> (8 * t));
    }
  };

  f32x4 acc[NT][2];
#pragma unroll
  for (int i = 0; i < NT; ++i) acc[i][0] = acc[i][1] = f32x4{0.f, 0.f, 0.f, 0.f};
  int64_t u = wid;
  if (u < nunits) fetch(u);
  for (; u < nunits; u += nw) {
    stash();  // wave-private: in-order after this wave's reads of the previous unit
    if (u + nw < nunits) fetch(u + nw);
#pragma unroll
    for (int dy = 0; dy < 2; ++dy) {
      bf16x8 bf[2];
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const uint8_t* rp = rows + (dy + bky[j]) * kRRow + boff[j];
        const u32x4 d0 = *reinterpret_cast<const u32x4*>(rp);
        const u32x4 d1 = *reinterpret_cast<const u32x4*>(rp + 16);
        const int sh = bsh[j];
        const uint32_t e0 = __builtin_amdgcn_alignbyte(d0.y, d0.x, sh);
        const uint32_t e1 = __builtin_amdgcn_alignbyte(d0.z, d0.y, sh);
        const uint32_t e2 = __builtin_amdgcn_alignbyte(d0.w, d0.z, sh);
        const uint32_t e3 = __builtin_amdgcn_alignbyte(d1.x, d0.w, sh);
        const uint32_t e4 = __builtin_amdgcn_alignbyte(d1.y, d1.x, sh);
        const uint32_t e5 = __builtin_amdgcn_alignbyte(d1.z, d1.y, sh);
        // pixel j' at byte 3j' of e0..e5
        float f[8] = {(float)(e0 & 0xffu), (float)(e0 >> 24), (float)((e1 >> 16) & 0xffu), (float)((e2 >> 8) & 0xffu),
                      (float)(e3 & 0xffu), (float)(e3 >> 24), (float)((e4 >> 16) & 0xffu), (float)((e5 >> 8) & 0xffu)};
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          const float v = btap[j] ? f[q] : (bone[j] ? 1.f : 0.f);
          bf[j][q] = (bf16)v;
        }
      }
#pragma unroll
      for (int i = 0; i < NT; ++i) {
        const int co = 16 * i + r;
        const uint2 dv = *reinterpret_cast<const uint2*>(Dt + co * kRDp + 4 * g);
        const uint32_t av = *reinterpret_cast<const uint32_t*>(At + co * kRDp + 4 * g);
        uint32_t w[4];
#pragma unroll
        for (int ww = 0; ww < 4; ++ww) {
          const uint32_t v = ((ww < 2 ? dv.x : dv.y) >> (16 * (ww & 1))) & 0xffffu;
          const uint32_t a = (av >> (8 * ww)) & 0xffu;
          w[ww] = (a == (uint32_t)(2 * dy) ? v : 0u) | (a == (uint32_t)(2 * dy + 1) ? v << 16 : 0u);
        }
        const bf16x8 af = __builtin_bit_cast(bf16x8, u32x4{w[0], w[1], w[2], w[3]});
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = mma(acc[i][j], af, bf[j]);
      }
    }
  }
  // waves in order through LDS, then the slab [64][kC0K] (tap columns scaled by 1/255)
  __syncthreads();
  float* red = reinterpret_cast<float*>(lds);  // COUT x 32 floats (<= 8 KB < 4 * PER_WAVE)
  for (int w = 0; w < 4; ++w) {
    if (wave == w) {
#pragma unroll
      for (int i = 0; i < NT; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            float& d = red[(16 * i + 4 * g + q) * kC0K + 16 * j + r];
            d = w == 0 ? acc[i][j][q] : d + acc[i][j][q];
          }
    }
    __syncthreads();
  }
  float* slab = p.slab + (size_t)blockIdx.x * 64 * kC0K;
  for (int i = threadIdx.x; i < 64 * kC0K; i += kRT) {
    const int co = i / kC0K, k = i - co * kC0K;
    slab[i] = co < COUT ? red[i] * (k < 27 ? 1.0f / 255.0f : 1.0f) : 0.f;
  }
}

bool conv0_dw_rows_ok(const Conv0DwParams& p) {
  return p.C == 3 && (p.Cout == 32 || p.Cout == 64) && p.W % 32 == 0 && p.H % 2 == 0 && p.PH == p.H / 2 &&
         p.PW == p.W / 2 && (int64_t)p.B * p.PH * (p.PW / 16) < (1ll << 40);
}
int conv0_dw_rows_grid(const Conv0DwParams& p) {
  const int64_t nunits = (int64_t)p.B * p.PH * (p.PW / 16);
  // (4 workgroups per CU; 2, 8 and 16 measured within 1.5% on CIFAR-3conv)
  return (int)std::max<int64_t>(1, std::min<int64_t>((nunits + 3) / 4, 256 * 4));
}

int conv0_dw_grid(const Conv0DwParams& p) {
  const int64_t nsteps = ((int64_t)p.B * p.PH * p.PW + kC0W - 1) / kC0W;
  return (int)std::max<int64_t>(1, std::min<int64_t>(nsteps, 256 * 8));
}

}  // namespace

bool conv0_dw_supported(const Conv0DwParams& p) {
  return p.C >= 1 && 9 * p.C + 1 <= kC0K && p.Cout >= 1 && p.Cout <= 64 && p.Cout % 4 == 0 && p.H % 2 == 0 &&
         p.W % 2 == 0 && p.PH == p.H / 2 && p.PW == p.W / 2 && (int64_t)p.H * p.W * p.C < (1 << 30) &&
         (int64_t)p.B * p.PH * p.PW < (1 << 24);
}

size_t conv0_dw_slab_bytes(const Conv0DwParams& p) {
  return (size_t)std::max(conv0_dw_grid(p), conv0_dw_rows_ok(p) ? conv0_dw_rows_grid(p) : 0) * 64 * kC0K * 4;
}

void conv0_dw(const Conv0DwParams& p, float* gw, float* gb, hipStream_t s) {
  MCC_CHECK(conv0_dw_supported(p) && p.x && p.dy && p.arg && p.slab, "conv0_dw: bad params");
  int grid;
  if (conv0_dw_rows_ok(p)) {
    grid = conv0_dw_rows_grid(p);
    if (p.Cout == 32) hipLaunchKernelGGL((conv0_dw_rows_kernel<2>), dim3((unsigned)grid), dim3(kRT), 0, s, p);
    else hipLaunchKernelGGL((conv0_dw_rows_kernel<4>), dim3((unsigned)grid), dim3(kRT), 0, s, p);
  } else {
    grid = conv0_dw_grid(p);
    hipLaunchKernelGGL(conv0_dw_kernel, dim3((unsigned)grid), dim3(kC0T), 0, s, p);
  }
  hipLaunchKernelGGL(conv0_dw_reduce_kernel, dim3((unsigned)(p.Cout * kC0K)), dim3(256), 0, s, p, grid, gw, gb);
}

}  // namespace gpu
}  // namespace mcc
