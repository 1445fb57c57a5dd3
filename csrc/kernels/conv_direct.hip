// Direct (VALU) fp32 convolution with a fused ReLU + 2x2/2 max-pool for the
// small LeNet-class layers: forward (the instantiated (KS, Cin, Cout) shapes,
// u8 dataset or fp32 NHWC input) and the single-channel first layer's weight
// gradient.
//
// Reference math: Layer_feedForw_conv / Layer_feedBack_conv (cnn.c:175-247,
// correct OIHW indexing as CUDAcnn.cu:167-195).  Why not MFMA here: in fp32
// the matrix cores give no more FLOP/s than the vector ALUs on MI355X (both
// ~157 TFLOP/s dense), while these layers' GEMM shapes (K = 25 taps x Cin,
// N = Cout = 6 or 16) fill 16x16x4 f32 MFMA tiles poorly and pad K; the
// direct form does only useful FMAs.  (bf16 keeps the tap-packed MFMA kernels
// conv_pipe_fwd / conv_rows, where the matrix rate is 16x the vector rate.)
//
// Work item = (image, 2x2 pooling window): per input channel the window's
// (KS+1)^2 input patch is loaded from the channel-planar LDS tile into
// registers and the four conv outputs of every output channel take 4*KS*KS
// FMAs against wave-uniform weights (scalar loads, no LDS traffic for them);
// then max / first-max argmax (PyTorch order), bias, ReLU; argmax byte 4
// marks a ReLU-inactive window (nothing is routed back), as in every other
// pooled kernel.
//
// Weight gradient (Cin = 1): the same items; only the argmax position of a
// window receives dY, so each channel contributes g*[arg == pos] x patch(pos)
// for the four positions into per-thread accumulators [C][KS*KS] (+ bias).
// dY and the argmax bytes of a group are staged in LDS with the images
// (coalesced loads, no per-item global latency).  The accumulators are
// reduced over the wave (shuffles), the workgroup (LDS) and the workgroups
// (a parallel fixed-order slab sum): deterministic.
#include "kernels.h"
#include "mfma.h"

#include <algorithm>

namespace mcc {
namespace gpu {

namespace {

constexpr int kDT = 256;   // threads per workgroup
constexpr int kDImgs = 8;  // images per group
constexpr int kDMaxC = 8;  // weight-gradient channel bound

struct Tile {  // LDS image tile: NHWC with a zero halo (TW pixels per row)
  int TH, TW, IMG;
};
__host__ __device__ inline Tile d_tile(const Conv1DirectParams& p) {
  Tile t;
  t.TH = p.OH + p.KS - 1;
  t.TW = ((p.OW + p.KS - 1) + 1) & ~1;  // even: 8-byte aligned single-channel patch rows
  t.IMG = t.TH * t.TW * p.Cin;
  return t;
}

// Per-thread staging geometry, fixed for the launch (the group's items are the
// same every time):
//  * fp32 NHWC input without padding: the LDS tile IS the global layout
//    (TW == W), a straight 16-byte copy of the group's images;
//  * u8 single-channel dataset images: items of four pixels (one 32-bit load,
//    two 8-byte LDS stores at the padded position), the image's dataset index
//    from a per-group LDS table.
constexpr int kDU8Items = 8;  // u8 items per thread: kDImgs * H * W / 4 <= 8 * kDT
struct Stager {
  int src[kDU8Items], dst[kDU8Items], img[kDU8Items];
  __device__ __forceinline__ void init(const Conv1DirectParams& p, const Tile& t) {
    const int wq = p.W >> 2, per = p.H * wq;
#pragma unroll
    for (int i = 0; i < kDU8Items; ++i) {
      const int e = threadIdx.x + i * kDT;
      const int m = e / per, r = e - m * per;
      const int y = r / wq, xq = r - y * wq;
      img[i] = m < kDImgs ? m : -1;
      src[i] = y * p.W + 4 * xq;
      dst[i] = m * t.IMG + (y + p.pad) * t.TW + 4 * xq + p.pad;
    }
  }
  __device__ __forceinline__ void stage(const Conv1DirectParams& p, const Tile& t, float* xs, const int* sidx,
                                        int img0, int nimg) {
    if (p.xf) {
      const int n4 = nimg * t.IMG / 4;
      const float4* g = reinterpret_cast<const float4*>(p.xf + (size_t)img0 * t.IMG);
      for (int i = threadIdx.x; i < n4; i += kDT) reinterpret_cast<float4*>(xs)[i] = g[i];
      return;
    }
    const float sc = 1.0f / 255.0f;
#pragma unroll
    for (int i = 0; i < kDU8Items; ++i) {
      if (img[i] < 0 || img[i] >= nimg) continue;
      const uint32_t v = *reinterpret_cast<const uint32_t*>(p.x + (size_t)sidx[img[i]] * p.H * p.W + src[i]);
      float* d = xs + dst[i];  // 8-byte aligned (pad even)
      *reinterpret_cast<float2*>(d) = make_float2((float)(v & 0xffu) * sc, (float)((v >> 8) & 0xffu) * sc);
      *reinterpret_cast<float2*>(d + 2) = make_float2((float)((v >> 16) & 0xffu) * sc, (float)(v >> 24) * sc);
    }
  }
};

// dataset indices of the group's images (read by Stager::stage after the barrier)
__device__ __forceinline__ void d_index(const Conv1DirectParams& p, int* sidx, int img0, int nimg) {
  if ((int)threadIdx.x < nimg) sidx[threadIdx.x] = p.idx ? p.idx[img0 + threadIdx.x] : img0 + threadIdx.x;
}

// (KS+1)^2 patch of input channel ci at the 2x2 window (py, px)
template <int KS, int CIN>
__device__ __forceinline__ void d_patch(const float* img, int TW, int py, int px, int ci, float (&P)[KS + 1][KS + 1]) {
  const float* b = img + ((2 * py) * TW + 2 * px) * CIN + ci;
#pragma unroll
  for (int i = 0; i <= KS; ++i) {
    if constexpr (CIN == 1) {  // 8-byte aligned rows (TW, pad even)
#pragma unroll
      for (int j = 0; j + 1 <= KS; j += 2) {
        const float2 v = *reinterpret_cast<const float2*>(b + i * TW + j);
        P[i][j] = v.x;
        P[i][j + 1] = v.y;
      }
      if ((KS + 1) & 1) P[i][KS] = b[i * TW + KS];
    } else {
#pragma unroll
      for (int j = 0; j <= KS; ++j) P[i][j] = b[(i * TW + j) * CIN];
    }
  }
}

// (weights and outputs are separate __restrict__ arguments: the weight loads
// are then provably unclobbered by the output stores and become scalar loads)
template <int KS, int CIN, int COUT>
__global__ void __launch_bounds__(kDT) conv_direct_fwd_kernel(Conv1DirectParams p, const float* __restrict__ wgt,
                                                            const float* __restrict__ bias, float* __restrict__ out,
                                                            uint8_t* __restrict__ out_arg) {
  extern __shared__ __attribute__((aligned(16))) float xs[];
  __shared__ int sidx[kDImgs];
  const Tile t = d_tile(p);
  for (int i = threadIdx.x; i < kDImgs * t.IMG; i += kDT) xs[i] = 0.f;
  Stager sg;
  sg.init(p, t);
  const int PHW = p.PH * p.PW;
  const int ngroups = (p.N + kDImgs - 1) / kDImgs;
  for (int grp = blockIdx.x; grp < ngroups; grp += gridDim.x) {
    const int img0 = grp * kDImgs, nimg = min(kDImgs, p.N - img0);
    d_index(p, sidx, img0, nimg);
    __syncthreads();  // previous group's reads done (and the zero fill, first time)
    sg.stage(p, t, xs, sidx, img0, nimg);
    __syncthreads();
    for (int it = threadIdx.x; it < nimg * PHW; it += kDT) {
      const int m = it / PHW, w = it - m * PHW;
      const int py = w / p.PW, px = w - py * p.PW;
      float acc[COUT][4];  // TL, TR, BL, BR
#pragma unroll
      for (int c = 0; c < COUT; ++c) acc[c][0] = acc[c][1] = acc[c][2] = acc[c][3] = 0.f;
      for (int ci = 0; ci < CIN; ++ci) {
        float P[KS + 1][KS + 1];
        d_patch<KS, CIN>(xs + m * t.IMG, t.TW, py, px, ci, P);
#pragma unroll
        for (int c = 0; c < COUT; ++c) {
          const float* wc = wgt + (c * CIN + ci) * KS * KS;  // wave-uniform: scalar loads
#pragma unroll
          for (int kh = 0; kh < KS; ++kh) {
#pragma unroll
            for (int kw = 0; kw < KS; ++kw) {
              const float wv = wc[kh * KS + kw];
              acc[c][0] = fmaf(wv, P[kh][kw], acc[c][0]);
              acc[c][1] = fmaf(wv, P[kh][kw + 1], acc[c][1]);
              acc[c][2] = fmaf(wv, P[kh + 1][kw], acc[c][2]);
              acc[c][3] = fmaf(wv, P[kh + 1][kw + 1], acc[c][3]);
            }
          }
        }
      }
      float y[COUT];
      uint32_t arg[(COUT + 3) / 4];
#pragma unroll
      for (int q = 0; q < (COUT + 3) / 4; ++q) arg[q] = 0;
#pragma unroll
      for (int c = 0; c < COUT; ++c) {
        float best = acc[c][0];
        int a = 0;
        if (acc[c][1] > best) { best = acc[c][1]; a = 1; }
        if (acc[c][2] > best) { best = acc[c][2]; a = 2; }
        if (acc[c][3] > best) { best = acc[c][3]; a = 3; }
        y[c] = fmaxf(best + bias[c], 0.f);
        arg[c >> 2] |= (uint32_t)(y[c] > 0.f ? a : 4) << (8 * (c & 3));
      }
      const size_t o = ((size_t)(img0 + m) * PHW + w) * COUT;
      if constexpr (COUT % 4 == 0) {
#pragma unroll
        for (int c = 0; c < COUT; c += 4)
          *reinterpret_cast<float4*>(out + o + c) = make_float4(y[c], y[c + 1], y[c + 2], y[c + 3]);
#pragma unroll
        for (int q = 0; q < COUT / 4; ++q) *reinterpret_cast<uint32_t*>(out_arg + o + 4 * q) = arg[q];
      } else {
        static_assert(COUT % 2 == 0, "even channel count");
#pragma unroll
        for (int c = 0; c < COUT; c += 2) *reinterpret_cast<float2*>(out + o + c) = make_float2(y[c], y[c + 1]);
#pragma unroll
        for (int c = 0; c < COUT; c += 2)
          *reinterpret_cast<unsigned short*>(out_arg + o + c) =
              (unsigned short)((arg[c >> 2] >> (8 * (c & 3))) & 0xffffu);
      }
    }
  }
}

template <int KS, int CM>  // CM: channel bound of the accumulator array (registers)
__global__ void __launch_bounds__(kDT) conv1_direct_dw_kernel(Conv1DirectParams p) {
  constexpr int KK = KS * KS;
  extern __shared__ __attribute__((aligned(16))) float xs[];
  __shared__ float red[kDT / 64][CM * (KK + 1)];
  __shared__ int sidx[kDImgs];
  const Tile t = d_tile(p);
  const int PHW = p.PH * p.PW;
  const int gsz = kDImgs * PHW * p.C;  // dY floats (and argmax bytes) per group
  float* dys = xs + kDImgs * t.IMG;
  uint8_t* args = reinterpret_cast<uint8_t*>(dys + gsz);
  for (int i = threadIdx.x; i < kDImgs * t.IMG; i += kDT) xs[i] = 0.f;
  Stager sg;
  sg.init(p, t);
  const int ngroups = (p.N + kDImgs - 1) / kDImgs;
  float acc[CM][KK + 1];
#pragma unroll
  for (int c = 0; c < CM; ++c)
#pragma unroll
    for (int k = 0; k <= KK; ++k) acc[c][k] = 0.f;
  for (int grp = blockIdx.x; grp < ngroups; grp += gridDim.x) {
    const int img0 = grp * kDImgs, nimg = min(kDImgs, p.N - img0);
    d_index(p, sidx, img0, nimg);
    __syncthreads();
    sg.stage(p, t, xs, sidx, img0, nimg);
    {  // the group's dY and argmax bytes: contiguous runs (PHW * C a multiple of 4: host check)
      const int n4 = nimg * PHW * p.C / 4;
      const float4* gdy = reinterpret_cast<const float4*>(p.dy + (size_t)img0 * PHW * p.C);
      const uint32_t* garg = reinterpret_cast<const uint32_t*>(p.arg + (size_t)img0 * PHW * p.C);
      for (int i = threadIdx.x; i < n4; i += kDT) {
        reinterpret_cast<float4*>(dys)[i] = gdy[i];
        reinterpret_cast<uint32_t*>(args)[i] = garg[i];
      }
    }
    __syncthreads();
    for (int it = threadIdx.x; it < nimg * PHW; it += kDT) {
      const int m = it / PHW, w = it - m * PHW;
      const int py = w / p.PW, px = w - py * p.PW;
      float P[KS + 1][KS + 1];
      d_patch<KS, 1>(xs + m * t.IMG, t.TW, py, px, 0, P);
      const int o = it * p.C;
#pragma unroll
      for (int c = 0; c < CM; ++c) {
        if (c >= p.C) break;
        const float gy = dys[o + c];
        const int a = args[o + c];  // 4: ReLU-inactive window, nothing routed
        const float g0 = a == 0 ? gy : 0.f, g1 = a == 1 ? gy : 0.f;
        const float g2 = a == 2 ? gy : 0.f, g3 = a == 3 ? gy : 0.f;
#pragma unroll
        for (int kh = 0; kh < KS; ++kh) {
#pragma unroll
          for (int kw = 0; kw < KS; ++kw) {
            float v = acc[c][kh * KS + kw];
            v = fmaf(g0, P[kh][kw], v);
            v = fmaf(g1, P[kh][kw + 1], v);
            v = fmaf(g2, P[kh + 1][kw], v);
            v = fmaf(g3, P[kh + 1][kw + 1], v);
            acc[c][kh * KS + kw] = v;
          }
        }
        acc[c][KK] += (a < 4) ? gy : 0.f;
      }
    }
  }
  // wave sums (fixed butterfly), then the workgroup's waves in order
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int c = 0; c < CM; ++c) {
    if (c >= p.C) break;
#pragma unroll
    for (int k = 0; k <= KK; ++k) {
      float v = acc[c][k];
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
      if (lane == 0) red[wave][c * (KK + 1) + k] = v;
    }
  }
  __syncthreads();
  const int ncol = p.C * (KK + 1);
  for (int i = threadIdx.x; i < ncol; i += kDT) {
    float v = 0.f;
#pragma unroll
    for (int w = 0; w < kDT / 64; ++w) v += red[w][i];
    p.slab[(size_t)blockIdx.x * ncol + i] = v;
  }
}

// Data gradient of a pooled 5x5 conv (stride 1, no padding): dX = full
// correlation of dZ = unpool(dY, argmax) with the flipped weights.  Item =
// (image, 2x2 block of dX pixels); its 6x6 dZ patch is exactly 3x3 pooling
// windows (the block is 2-aligned and the halo KS-1 = 4 is even), so the
// patch is decoded from the group's pooled dY / argmax in LDS (value at the
// argmax position, zeros elsewhere; argmax 4 routes nothing) instead of
// staging the 4x larger unpooled tensor.  Then 4*KS*KS FMAs per (input,
// output channel) pair with scalar-loaded flipped weights, as the forward.
constexpr int kDxImgs = 16;
template <int KS, int CI, int CO>  // CI: dZ channels (forward Cout), CO: dX channels (forward Cin)
__global__ void __launch_bounds__(kDT) conv_direct_dx_kernel(Conv1DirectParams p, const float* __restrict__ wgt,
                                                           float* __restrict__ out) {
  static_assert(KS == 5, "the 3x3-window patch decode assumes KS - 1 == 4");
  extern __shared__ __attribute__((aligned(16))) float dys[];
  const int PHW = p.PH * p.PW;  // pooled grid of dY
  const int BH = p.H / 2, BW = p.W / 2, nb = BH * BW;  // 2x2 blocks of the dX grid (H x W)
  uint8_t* args = reinterpret_cast<uint8_t*>(dys + kDxImgs * PHW * CI);
  const int ngroups = (p.N + kDxImgs - 1) / kDxImgs;
  for (int grp = blockIdx.x; grp < ngroups; grp += gridDim.x) {
    const int img0 = grp * kDxImgs, nimg = min(kDxImgs, p.N - img0);
    __syncthreads();
    {
      const int n4 = nimg * PHW * CI / 4;
      const float4* g = reinterpret_cast<const float4*>(p.dy + (size_t)img0 * PHW * CI);
      const uint32_t* ga = reinterpret_cast<const uint32_t*>(p.arg + (size_t)img0 * PHW * CI);
      for (int i = threadIdx.x; i < n4; i += kDT) {
        reinterpret_cast<float4*>(dys)[i] = g[i];
        reinterpret_cast<uint32_t*>(args)[i] = ga[i];
      }
    }
    __syncthreads();
    for (int it = threadIdx.x; it < nimg * nb; it += kDT) {
      const int m = it / nb, b = it - m * nb;
      const int by = b / BW, bx = b - by * BW;
      float acc[CO][4];
#pragma unroll
      for (int c = 0; c < CO; ++c) acc[c][0] = acc[c][1] = acc[c][2] = acc[c][3] = 0.f;
      const float* dimg = dys + m * PHW * CI;
      const uint8_t* aimg = args + m * PHW * CI;
      for (int i = 0; i < CI; ++i) {
        float P[KS + 1][KS + 1];
#pragma unroll
        for (int wr = 0; wr < 3; ++wr) {
#pragma unroll
          for (int wc = 0; wc < 3; ++wc) {
            const int wy = by - 2 + wr, wx = bx - 2 + wc;
            const bool ok = (unsigned)wy < (unsigned)p.PH && (unsigned)wx < (unsigned)p.PW;
            const int o = ok ? (wy * p.PW + wx) * CI + i : 0;
            const float g = ok ? dimg[o] : 0.f;
            const int a = ok ? aimg[o] : 4;
            P[2 * wr][2 * wc] = a == 0 ? g : 0.f;
            P[2 * wr][2 * wc + 1] = a == 1 ? g : 0.f;
            P[2 * wr + 1][2 * wc] = a == 2 ? g : 0.f;
            P[2 * wr + 1][2 * wc + 1] = a == 3 ? g : 0.f;
          }
        }
#pragma unroll
        for (int c = 0; c < CO; ++c) {
          // flipped weight of (dX channel c, dZ channel i, tap kh, kw) = w[i][c][KS-1-kh][KS-1-kw]
          const float* wc = wgt + (i * CO + c) * KS * KS;
#pragma unroll
          for (int kh = 0; kh < KS; ++kh) {
#pragma unroll
            for (int kw = 0; kw < KS; ++kw) {
              const float wv = wc[(KS - 1 - kh) * KS + (KS - 1 - kw)];
              acc[c][0] = fmaf(wv, P[kh][kw], acc[c][0]);
              acc[c][1] = fmaf(wv, P[kh][kw + 1], acc[c][1]);
              acc[c][2] = fmaf(wv, P[kh + 1][kw], acc[c][2]);
              acc[c][3] = fmaf(wv, P[kh + 1][kw + 1], acc[c][3]);
            }
          }
        }
      }
      // dX pixels (2by + r, 2bx + q), CO channels each: two rows of 2*CO contiguous floats
#pragma unroll
      for (int r = 0; r < 2; ++r) {
        float* d = out + (((size_t)(img0 + m) * p.H + 2 * by + r) * p.W + 2 * bx) * CO;
#pragma unroll
        for (int c = 0; c < CO; c += 2) {
          *reinterpret_cast<float2*>(d + c) = make_float2(acc[c][2 * r], acc[c + 1][2 * r]);
          *reinterpret_cast<float2*>(d + CO + c) = make_float2(acc[c][2 * r + 1], acc[c + 1][2 * r + 1]);
        }
      }
    }
  }
}

// One workgroup per column (c, k): 256 strided partial sums over the slabs,
// then a fixed LDS tree.  k < KK: weight, k == KK: bias.
__global__ void __launch_bounds__(256) conv1_direct_dw_reduce_kernel(Conv1DirectParams p, int nslab, float* gw,
                                                                     float* gb) {
  __shared__ float part[256];
  const int KK = p.KS * p.KS, ncol = p.C * (KK + 1);
  const int i = blockIdx.x;
  float v = 0.f;
  for (int s = threadIdx.x; s < nslab; s += 256) v += p.slab[(size_t)s * ncol + i];
  part[threadIdx.x] = v;
  __syncthreads();
  for (int h = 128; h > 0; h >>= 1) {
    if ((int)threadIdx.x < h) part[threadIdx.x] += part[threadIdx.x + h];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    const int c = i / (KK + 1), k = i - c * (KK + 1);
    if (k < KK) gw[c * KK + k] = part[0];
    else gb[c] = part[0];
  }
}

size_t fwd_lds(const Conv1DirectParams& p) { return (size_t)kDImgs * d_tile(p).IMG * 4; }
size_t dw_lds(const Conv1DirectParams& p) {
  return fwd_lds(p) + (size_t)kDImgs * p.PH * p.PW * p.C * 5;  // + dY floats + argmax bytes
}

}  // namespace

bool conv_direct_fwd_supported(const Conv1DirectParams& p) {
  const bool shape = p.KS == 5 && ((p.Cin == 1 && p.C == 6) || (p.Cin == 6 && p.C == 16));
  const Tile t = d_tile(p);
  const bool stage_ok = p.Cin == 1 ? (p.W % 4 == 0 && p.pad % 2 == 0 && kDImgs * p.H * (p.W / 4) <= kDU8Items * kDT)
                                   : (p.pad == 0 && t.TW == p.W && t.IMG % 4 == 0);
  return shape && stage_ok && p.OH % 2 == 0 && p.OW % 2 == 0 && p.OH == p.H + 2 * p.pad - p.KS + 1 &&
         p.OW == p.W + 2 * p.pad - p.KS + 1 && p.PH == p.OH / 2 && p.PW == p.OW / 2 && fwd_lds(p) <= 64 * 1024;
}

// dX geometry: p.H x p.W = the forward input (dX) grid, p.PH x p.PW = pooled dY
bool conv_direct_dx_supported(const Conv1DirectParams& p) {
  return p.KS == 5 && p.pad == 0 && p.Cin == 6 && p.C == 16 && p.OH == p.H - 4 && p.OW == p.W - 4 &&
         p.H % 2 == 0 && p.W % 2 == 0 && p.PH == p.OH / 2 && p.PW == p.OW / 2 && (p.PH * p.PW * p.C) % 4 == 0 &&
         (size_t)kDxImgs * p.PH * p.PW * p.C * 5 <= 64 * 1024;
}

void conv_direct_dx(const Conv1DirectParams& p, float* dx, hipStream_t s) {
  MCC_CHECK(conv_direct_dx_supported(p) && p.w && p.dy && p.arg && dx, "conv_direct_dx: bad params");
  const int ngroups = (p.N + kDxImgs - 1) / kDxImgs;
  const dim3 grid((unsigned)std::max(1, std::min(ngroups, 256 * 4))), block(kDT);
  const size_t lds = (size_t)kDxImgs * p.PH * p.PW * p.C * 5;
  hipLaunchKernelGGL((conv_direct_dx_kernel<5, 16, 6>), grid, block, lds, s, p, p.w, dx);
}

bool conv1_direct_dw_supported(const Conv1DirectParams& p) {
  return p.Cin == 1 && p.C >= 1 && p.C <= kDMaxC && (p.KS == 3 || p.KS == 5) && p.OH % 2 == 0 && p.OW % 2 == 0 &&
         p.W % 4 == 0 && p.pad % 2 == 0 && kDImgs * p.H * (p.W / 4) <= kDU8Items * kDT &&
         (p.PH * p.PW * p.C) % 4 == 0 &&
         p.OH == p.H + 2 * p.pad - p.KS + 1 && p.OW == p.W + 2 * p.pad - p.KS + 1 && p.PH == p.OH / 2 &&
         p.PW == p.OW / 2 && dw_lds(p) <= 96 * 1024;
}

static int direct_grid(const Conv1DirectParams& p) {
  const int ngroups = (p.N + kDImgs - 1) / kDImgs;
  return std::max(1, std::min(ngroups, 256 * 4));
}

size_t conv1_direct_slab_bytes(const Conv1DirectParams& p) {
  return (size_t)direct_grid(p) * p.C * (p.KS * p.KS + 1) * 4;
}

void conv_direct_forward(const Conv1DirectParams& p, hipStream_t s) {
  MCC_CHECK(conv_direct_fwd_supported(p) && (p.x || p.xf) && p.w && p.bias && p.out && p.out_arg,
            "conv_direct_forward: bad params");
  const dim3 grid((unsigned)direct_grid(p)), block(kDT);
  if (p.Cin == 1)
    hipLaunchKernelGGL((conv_direct_fwd_kernel<5, 1, 6>), grid, block, fwd_lds(p), s, p, p.w, p.bias, p.out, p.out_arg);
  else
    hipLaunchKernelGGL((conv_direct_fwd_kernel<5, 6, 16>), grid, block, fwd_lds(p), s, p, p.w, p.bias, p.out,
                       p.out_arg);
}

void conv1_direct_dw(const Conv1DirectParams& p, float* gw, float* gb, hipStream_t s) {
  MCC_CHECK(conv1_direct_dw_supported(p) && p.x && p.dy && p.arg && p.slab, "conv1_direct_dw: bad params");
  const int grid = direct_grid(p);
  const dim3 g((unsigned)grid), b(kDT);
  if (p.KS == 5 && p.C <= 6) hipLaunchKernelGGL((conv1_direct_dw_kernel<5, 6>), g, b, dw_lds(p), s, p);
  else if (p.KS == 5) hipLaunchKernelGGL((conv1_direct_dw_kernel<5, kDMaxC>), g, b, dw_lds(p), s, p);
  else hipLaunchKernelGGL((conv1_direct_dw_kernel<3, kDMaxC>), g, b, dw_lds(p), s, p);
  const int ncol = p.C * (p.KS * p.KS + 1);
  hipLaunchKernelGGL(conv1_direct_dw_reduce_kernel, dim3((unsigned)ncol), dim3(256), 0, s, p, grid, gw, gb);
}

}  // namespace gpu
}  // namespace mcc
