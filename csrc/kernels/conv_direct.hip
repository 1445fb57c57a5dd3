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
#include "mcc/ab.h"
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
// (each item packed in one register -- source offset (10 bits), LDS offset
// (14 bits), image + 1 (4 bits, 0: no item) -- to keep the per-thread table
// at 8 registers in the register-hungry accumulator kernels)
template <int NT, int NIMG>  // threads, images per group
struct StagerT {
  uint32_t it[kDU8Items];
  __device__ __forceinline__ void init(const Conv1DirectParams& p, const Tile& t) {
    const int wq = p.W >> 2, per = p.H * wq;
#pragma unroll
    for (int i = 0; i < kDU8Items; ++i) {
      const int e = threadIdx.x + i * NT;
      const int m = e / per, r = e - m * per;
      const int y = r / wq, xq = r - y * wq;
      const uint32_t src = y * p.W + 4 * xq, dst = m * t.IMG + (y + p.pad) * t.TW + 4 * xq + p.pad;
      it[i] = m < NIMG ? src | dst << 10 | (uint32_t)(m + 1) << 24 : 0u;
    }
  }
  __device__ __forceinline__ void stage(const Conv1DirectParams& p, const Tile& t, float* xs, const int* sidx,
                                        int img0, int nimg) {
    if (p.xf) {
      const int n4 = nimg * t.IMG / 4;
      const float4* g = reinterpret_cast<const float4*>(p.xf + (size_t)img0 * t.IMG);
      for (int i = threadIdx.x; i < n4; i += NT) reinterpret_cast<float4*>(xs)[i] = g[i];
      return;
    }
    const float sc = 1.0f / 255.0f;
    uint32_t v[kDU8Items];  // all loads in flight first (invalid items read image 0's first word)
#pragma unroll
    for (int i = 0; i < kDU8Items; ++i) {
      const int m = (int)(it[i] >> 24) - 1;
      const bool ok = m >= 0 && m < nimg;
      v[i] = *reinterpret_cast<const uint32_t*>(p.x + (ok ? (size_t)sidx[m] * p.H * p.W + (it[i] & 1023u) : 0));
    }
#pragma unroll
    for (int i = 0; i < kDU8Items; ++i) {
      const int m = (int)(it[i] >> 24) - 1;
      if (m < 0 || m >= nimg) continue;
      float* d = xs + ((it[i] >> 10) & 16383u);  // 8-byte aligned (pad even)
      *reinterpret_cast<float2*>(d) = make_float2((float)(v[i] & 0xffu) * sc, (float)((v[i] >> 8) & 0xffu) * sc);
      *reinterpret_cast<float2*>(d + 2) = make_float2((float)((v[i] >> 16) & 0xffu) * sc, (float)(v[i] >> 24) * sc);
    }
  }
};
using Stager = StagerT<kDT, kDImgs>;
// the packed fields' ranges (host check)
__host__ __device__ inline bool stager_fits(const Conv1DirectParams& p, const Tile& t) {
  return p.H * p.W <= 1024 && kDImgs * t.IMG <= 16384 && p.W % 4 == 0 && p.pad % 2 == 0 &&
         kDImgs * p.H * (p.W / 4) <= kDU8Items * kDT;
}

// dataset indices of the group's images (read by Stager::stage after the barrier)
__device__ __forceinline__ void d_index(const Conv1DirectParams& p, int* sidx, int img0, int nimg) {
  if ((int)threadIdx.x < nimg) sidx[threadIdx.x] = p.idx ? p.idx[img0 + threadIdx.x] : img0 + threadIdx.x;
}

// fp32 pairs: one v_pk_fma_f32 does two FMAs (the VALU's full fp32 rate).
// Accumulators pair adjacent channels; the other operand is one input value
// splatted to both halves.  Input values are kept as register PAIRS (f2) and
// splatted with a shuffle that folds into the instruction's op_sel: a lone
// float used as a splat source would occupy a whole aligned register pair.
typedef float f2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f2 splat(f2 v, int hi) {  // hi: a constant once the loops are unrolled
  return hi ? __builtin_shufflevector(v, v, 1, 1) : __builtin_shufflevector(v, v, 0, 0);
}
#define MCC_PS(row, j) splat((row)[(j) >> 1], (j) & 1)
__device__ __forceinline__ f2 pfma(f2 a, f2 b, f2 c) { return __builtin_elementwise_fma(a, b, c); }

// (KS+1)^2 patch of input channel ci at the 2x2 window (py, px), rows as
// (KS+1)/2 register pairs (KS odd)
template <int KS, int CIN>
__device__ __forceinline__ void d_patch(const float* img, int TW, int py, int px, int ci,
                                        f2 (&P)[KS + 1][(KS + 1) / 2]) {
  static_assert(KS & 1, "odd kernel: even patch rows");
  const float* b = img + ((2 * py) * TW + 2 * px) * CIN + ci;
#pragma unroll
  for (int i = 0; i <= KS; ++i) {
#pragma unroll
    for (int j = 0; j < (KS + 1) / 2; ++j) {
      if constexpr (CIN == 1)  // 8-byte aligned rows (TW, pad even)
        P[i][j] = *reinterpret_cast<const f2*>(b + i * TW + 2 * j);
      else
        P[i][j] = f2{b[(i * TW + 2 * j) * CIN], b[(i * TW + 2 * j + 1) * CIN]};
    }
  }
}

// (weights and outputs are separate __restrict__ arguments: the weight loads
// are then provably unclobbered by the output stores and become scalar loads;
// waves_per_eu(4): four waves per SIMD)
// wt: tap-major weights [Cin][KS*KS][COUT] (the engine's packed copy)
// NIMG: images per staged group, chosen so the group's (image, window) items
// fill the 256 threads' last round: conv2 (25 windows per image) 10 -> 250
// items (at 8: 200, 22 % of the lanes idle; 3 instead of 4 workgroups per CU
// for the LDS); conv1 (196 per image) 9 -> 1,764 = 6.9 rounds (at 8: 6.1).
template <int KS, int CIN, int COUT, int NIMG = kDImgs>
__global__ void __launch_bounds__(kDT) __attribute__((amdgpu_waves_per_eu(4))) conv_direct_fwd_kernel(Conv1DirectParams p, const float* __restrict__ wt,
                                                            const float* __restrict__ bias, float* __restrict__ out,
                                                            uint8_t* __restrict__ out_arg) {
  static_assert(COUT % 2 == 0, "channel pairs");
  constexpr int CP = COUT / 2;
  extern __shared__ __attribute__((aligned(16))) float xs[];
  __shared__ int sidx[NIMG];
  const Tile t = d_tile(p);
  for (int i = threadIdx.x; i < NIMG * t.IMG; i += kDT) xs[i] = 0.f;
  StagerT<kDT, NIMG> sg;
  if constexpr (CIN == 1) sg.init(p, t);
  const int PHW = p.PH * p.PW;
  const int ngroups = (p.N + NIMG - 1) / NIMG;
  for (int grp = blockIdx.x; grp < ngroups; grp += gridDim.x) {
    const int img0 = grp * NIMG, nimg = min(NIMG, p.N - img0);
    d_index(p, sidx, img0, nimg);
    __syncthreads();  // previous group's reads done (and the zero fill, first time)
    if constexpr (CIN == 1) {
      sg.stage(p, t, xs, sidx, img0, nimg);
    } else {  // fp32 NHWC input without padding: the tile is the global layout
      const int n4 = nimg * t.IMG / 4;
      const float4* g = reinterpret_cast<const float4*>(p.xf + (size_t)img0 * t.IMG);
      for (int i = threadIdx.x; i < n4; i += kDT) reinterpret_cast<float4*>(xs)[i] = g[i];
    }
    __syncthreads();
    for (int it = threadIdx.x; it < nimg * PHW; it += kDT) {
      const int m = it / PHW, w = it - m * PHW;
      const int py = w / p.PW, px = w - py * p.PW;
      f2 acc[CP][4];  // TL, TR, BL, BR
#pragma unroll
      for (int c = 0; c < CP; ++c) acc[c][0] = acc[c][1] = acc[c][2] = acc[c][3] = f2{0.f, 0.f};
      // The weights are loop-invariant, and left alone the compiler hoists all
      // of conv1's (150 floats) out of the item loop -- more than the SGPR
      // file -- and spills them to VGPR lanes: 712 v_readlane per 300 packed
      // FMAs (924 us at B = 131072).  An opaque copy of the pointer per item
      // keeps them as scalar loads next to their use (549 us).  conv2's
      // weights live inside the channel loop and are not hoisted.
      // The copy is a constant-address-space pointer: laundered as a generic
      // one it lost the __restrict__ no-clobber proof and the 150 weights
      // became 38 flat_load_dwordx4 per item (vector memory, counted on both
      // vmcnt and lgkmcnt) instead of scalar loads.
      typedef __attribute__((address_space(4))) const float cfloat;
      cfloat* wtv = (cfloat*)wt;
      if constexpr (CIN == 1) asm volatile("" : "+s"(wtv));  // (conv2: measured 793 -> 1511 us with it)
      for (int ci = 0; ci < CIN; ++ci) {
        f2 P[KS + 1][(KS + 1) / 2];
        d_patch<KS, CIN>(xs + m * t.IMG, t.TW, py, px, ci, P);
        cfloat* wc = wtv + ci * KS * KS * COUT;  // wave-uniform: scalar loads
#pragma unroll
        for (int kh = 0; kh < KS; ++kh) {
#pragma unroll
          for (int kw = 0; kw < KS; ++kw) {
#pragma unroll
            for (int c = 0; c < CP; ++c) {
              const f2 wv = *reinterpret_cast<__attribute__((address_space(4))) const f2*>(wc + (kh * KS + kw) * COUT + 2 * c);
              acc[c][0] = pfma(wv, MCC_PS(P[kh], kw), acc[c][0]);
              acc[c][1] = pfma(wv, MCC_PS(P[kh], kw + 1), acc[c][1]);
              acc[c][2] = pfma(wv, MCC_PS(P[kh + 1], kw), acc[c][2]);
              acc[c][3] = pfma(wv, MCC_PS(P[kh + 1], kw + 1), acc[c][3]);
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
        float v[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) v[q] = (c & 1) ? acc[c >> 1][q].y : acc[c >> 1][q].x;
        float best = v[0];
        int a = 0;
        if (v[1] > best) { best = v[1]; a = 1; }
        if (v[2] > best) { best = v[2]; a = 2; }
        if (v[3] > best) { best = v[3]; a = 3; }
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

template <int KS, int CM, bool EXACT>  // CM: channel bound of the accumulator array (registers), even; EXACT: p.C == CM
__global__ void __launch_bounds__(kDT) __attribute__((amdgpu_waves_per_eu(2))) conv1_direct_dw_kernel(Conv1DirectParams p) {
  static_assert(CM % 2 == 0, "channel pairs");
  constexpr int KK = KS * KS, CP = CM / 2;
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
  f2 acc[CP][KK + 1];  // channel pairs (2c, 2c+1); [KK]: bias
#pragma unroll
  for (int c = 0; c < CP; ++c)
#pragma unroll
    for (int k = 0; k <= KK; ++k) acc[c][k] = f2{0.f, 0.f};
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
      f2 P[KS + 1][(KS + 1) / 2];
      d_patch<KS, 1>(xs + m * t.IMG, t.TW, py, px, 0, P);
      const int o = it * p.C;
#pragma unroll
      for (int c = 0; c < CP; ++c) {
        if (!EXACT && 2 * c >= p.C) break;  // (p.C even: host check)
        const float2 gy = *reinterpret_cast<const float2*>(dys + o + 2 * c);
        const int a0 = args[o + 2 * c], a1 = args[o + 2 * c + 1];  // 4: ReLU-inactive window
        const f2 g0 = {a0 == 0 ? gy.x : 0.f, a1 == 0 ? gy.y : 0.f};
        const f2 g1 = {a0 == 1 ? gy.x : 0.f, a1 == 1 ? gy.y : 0.f};
        const f2 g2 = {a0 == 2 ? gy.x : 0.f, a1 == 2 ? gy.y : 0.f};
        const f2 g3 = {a0 == 3 ? gy.x : 0.f, a1 == 3 ? gy.y : 0.f};
#pragma unroll
        for (int kh = 0; kh < KS; ++kh) {
#pragma unroll
          for (int kw = 0; kw < KS; ++kw) {
            f2 v = acc[c][kh * KS + kw];
            v = pfma(g0, MCC_PS(P[kh], kw), v);
            v = pfma(g1, MCC_PS(P[kh], kw + 1), v);
            v = pfma(g2, MCC_PS(P[kh + 1], kw), v);
            v = pfma(g3, MCC_PS(P[kh + 1], kw + 1), v);
            acc[c][kh * KS + kw] = v;
          }
        }
        acc[c][KK] += f2{a0 < 4 ? gy.x : 0.f, a1 < 4 ? gy.y : 0.f};
      }
    }
  }
  // wave sums (fixed butterfly), then the workgroup's waves in order
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int c = 0; c < CM; ++c) {
    if (!EXACT && c >= p.C) break;
#pragma unroll
    for (int k = 0; k <= KK; ++k) {
      float v = (c & 1) ? acc[c >> 1][k].y : acc[c >> 1][k].x;
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

// Single-channel first-layer weight gradient, C = 6, one WAVE per channel
// pair (192 threads; 26 packed accumulators per thread instead of 78: no
// spills, 3 waves per SIMD) and 4 images per group: 39.5 KB of LDS, so 4
// workgroups share a CU and one workgroup's staging barriers are covered by
// the other three.  Measured at B = 163840: 944 us; the all-pairs kernel
// below 1,237 us at 131072; a 384-thread pair split with 8-image groups (79
// KB, 2 workgroups per CU) 1,145 us.  The patch is re-read per pair (18
// ds_read_b64 per 100 packed FMAs, still VALU-bound).
constexpr int kDW3T = 192, kDW3Imgs = 4;
template <int KS>
__global__ void __launch_bounds__(kDW3T) __attribute__((amdgpu_waves_per_eu(3))) conv1_direct_dw_w3_kernel(Conv1DirectParams p) {
  constexpr int KK = KS * KS, C = 6;
  extern __shared__ __attribute__((aligned(16))) float xs[];
  __shared__ float red[3][2 * (KK + 1)];
  __shared__ int sidx[kDW3Imgs];
  const Tile t = d_tile(p);
  const int PHW = p.PH * p.PW;
  float* dys = xs + kDW3Imgs * t.IMG;
  uint8_t* args = reinterpret_cast<uint8_t*>(dys + kDW3Imgs * PHW * C);
  for (int i = threadIdx.x; i < kDW3Imgs * t.IMG; i += kDW3T) xs[i] = 0.f;
  StagerT<kDW3T, kDW3Imgs> sg;
  sg.init(p, t);
  const int cp = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int ngroups = (p.N + kDW3Imgs - 1) / kDW3Imgs;
  f2 acc[KK + 1];
#pragma unroll
  for (int k = 0; k <= KK; ++k) acc[k] = f2{0.f, 0.f};
  for (int grp = blockIdx.x; grp < ngroups; grp += gridDim.x) {
    const int img0 = grp * kDW3Imgs, nimg = min(kDW3Imgs, p.N - img0);
    if ((int)threadIdx.x < nimg) sidx[threadIdx.x] = p.idx ? p.idx[img0 + threadIdx.x] : img0 + threadIdx.x;
    __syncthreads();
    sg.stage(p, t, xs, sidx, img0, nimg);
    {
      const int n4 = nimg * PHW * C / 4;
      const float4* gdy = reinterpret_cast<const float4*>(p.dy + (size_t)img0 * PHW * C);
      const uint32_t* garg = reinterpret_cast<const uint32_t*>(p.arg + (size_t)img0 * PHW * C);
      for (int i = threadIdx.x; i < n4; i += kDW3T) {
        reinterpret_cast<float4*>(dys)[i] = gdy[i];
        reinterpret_cast<uint32_t*>(args)[i] = garg[i];
      }
    }
    __syncthreads();
    for (int it = lane; it < nimg * PHW; it += 64) {
      const int m = it / PHW, w = it - m * PHW;
      const int py = w / p.PW, px = w - py * p.PW;
      f2 P[KS + 1][(KS + 1) / 2];
      d_patch<KS, 1>(xs + m * t.IMG, t.TW, py, px, 0, P);
      const int o = it * C + 2 * cp;
      const float2 gy = *reinterpret_cast<const float2*>(dys + o);
      const int a0 = args[o], a1 = args[o + 1];
      const f2 g0 = {a0 == 0 ? gy.x : 0.f, a1 == 0 ? gy.y : 0.f};
      const f2 g1 = {a0 == 1 ? gy.x : 0.f, a1 == 1 ? gy.y : 0.f};
      const f2 g2 = {a0 == 2 ? gy.x : 0.f, a1 == 2 ? gy.y : 0.f};
      const f2 g3 = {a0 == 3 ? gy.x : 0.f, a1 == 3 ? gy.y : 0.f};
#pragma unroll
      for (int kh = 0; kh < KS; ++kh) {
#pragma unroll
        for (int kw = 0; kw < KS; ++kw) {
          f2 v = acc[kh * KS + kw];
          v = pfma(g0, MCC_PS(P[kh], kw), v);
          v = pfma(g1, MCC_PS(P[kh], kw + 1), v);
          v = pfma(g2, MCC_PS(P[kh + 1], kw), v);
          v = pfma(g3, MCC_PS(P[kh + 1], kw + 1), v);
          acc[kh * KS + kw] = v;
        }
      }
      acc[KK] += f2{a0 < 4 ? gy.x : 0.f, a1 < 4 ? gy.y : 0.f};
    }
  }
#pragma unroll
  for (int k = 0; k <= KK; ++k) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      float v = h ? acc[k].y : acc[k].x;
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
      if (lane == 0) red[cp][h * (KK + 1) + k] = v;
    }
  }
  __syncthreads();
  const int ncol = C * (KK + 1);
  for (int i = threadIdx.x; i < ncol; i += kDW3T) {
    const int c = i / (KK + 1), k = i - c * (KK + 1);
    p.slab[(size_t)blockIdx.x * ncol + i] = red[c >> 1][(c & 1) * (KK + 1) + k];
  }
}

// Data gradient of LeNet-5's pooled conv2 (6 -> 16, 5x5, stride 1, no
// padding: 14x14x6 -> 10x10x16 -> pool -> 5x5x16) in SCATTER form:
// dZ = unpool(dY, argmax) is nonzero only at each pooling window's argmax, so
// dX = sum over (channel co, window) of dY x W[co][ci] placed at the argmax
// position.  A lane owns one (image, ci) pair and one half of its 14x14 dX
// plane (7 rows x 14 = 98 accumulators in registers); the placement depends
// on the argmax class (ay, ax) of the window, so every class is applied with
// a mask (dY where the argmax is that class, else 0) -- static register
// indices, no branches, only the taps that land in the lane's half.  240 K
// FMAs per image instead of the 470 K of the full correlation over the
// unpooled grid (the zeros of three unpooled positions and the border taps);
// an LDS-atomic scatter of only the nonzero terms (60 K) measured 15x slower
// (ds_add_f32 retires about one lane per clock), and a v_pk_fma_f32 variant
// over input-channel pairs (thirds of the plane, one kernel row of weights
// at a time) 1.8x slower (2,020 vs 1,099 us).  Round 6, two more packed
// forms, both slower than this one (1,037 us in the same run): column pairs
// with even / odd weight layouts (196 registers, 2 waves per SIMD) 1,286 us,
// and image PAIRS per lane over a quarter plane (every product a splat-weight
// v_pk_fma_f32: half the FMA issues) 1,104 us at 2 waves per SIMD, 1,234 at 3
// (spilling); this form spills too (168 registers + 628 in scratch) and is
// still the fastest: the issue count is not what bounds it.
// Workgroup = 4 waves = 2 image groups x 2 halves: waves 2k, 2k+1 share group
// k's staged dY / argmax codes (10 images, lanes 0..59 = image x ci); the
// weights are staged once per workgroup as [co][ci][28] (16-byte rows).
constexpr int kDxImgW = 10;                    // images per group
constexpr int kDxWRow = 28;                    // floats per (co, ci) weight row
constexpr int kDxWFloats = 16 * 6 * kDxWRow;   // 2688
constexpr int kDxImgF = 25 * 16;               // dY floats per image (5 x 5 windows x 16 channels)
constexpr int kDxGrpF = kDxImgW * kDxImgF + kDxImgW * kDxImgF / 4;   // dY + argmax bytes: 5,000 floats
constexpr int kDxLds = (kDxWFloats + 2 * kDxGrpF) * 4;               // 50,752 B: three workgroups per CU
template <int HALF>
__device__ __forceinline__ void dx_half(const float* __restrict__ ws, const float* dimg, const uint8_t* aimg, int ci,
                                        float (&acc)[7][14]) {
#pragma unroll
  for (int y = 0; y < 7; ++y)
#pragma unroll
    for (int x = 0; x < 14; ++x) acc[y][x] = 0.f;
#pragma unroll 1
  for (int co = 0; co < 16; ++co) {
    float w[28];
    const float4* wr = reinterpret_cast<const float4*>(ws + (co * 6 + ci) * kDxWRow);
#pragma unroll
    for (int q = 0; q < 7; ++q) {
      const float4 v = wr[q];
      w[4 * q] = v.x; w[4 * q + 1] = v.y; w[4 * q + 2] = v.z; w[4 * q + 3] = v.w;
    }
#pragma unroll
    for (int py = 0; py < 5; ++py) {
      // rows 2py + ay + kh (ay <= 1, kh <= 4) must meet this half's rows
      if (2 * py + 5 < 7 * HALF || 2 * py > 7 * HALF + 6) continue;
#pragma unroll
      for (int px = 0; px < 5; ++px) {
        const int o = (py * 5 + px) * 16 + co;
        const float gv = dimg[o];
        const int a = aimg[o];
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          const float m = a == c ? gv : 0.f;  // argmax 4 (ReLU-inactive): nothing
          const int y0 = 2 * py + (c >> 1) - 7 * HALF, x0 = 2 * px + (c & 1);
#pragma unroll
          for (int kh = 0; kh < 5; ++kh) {
            if (y0 + kh < 0 || y0 + kh >= 7) continue;
#pragma unroll
            for (int kw = 0; kw < 5; ++kw)
              acc[y0 + kh][x0 + kw] = __builtin_fmaf(w[kh * 5 + kw], m, acc[y0 + kh][x0 + kw]);
          }
        }
        __builtin_amdgcn_sched_barrier(0);  // one window at a time (register budget)
      }
    }
  }
}
__global__ void __launch_bounds__(256, 3) conv_direct_dx_kernel(Conv1DirectParams p, const float* __restrict__ wd,
                                                               float* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) float dxs[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int grp = wave >> 1, half = wave & 1;
  float* ws = dxs;                                  // [co][ci][28]
  float* dys = dxs + kDxWFloats + grp * kDxGrpF;    // [img][window][co]
  const uint8_t* ags = reinterpret_cast<const uint8_t*>(dys + kDxImgW * kDxImgF);
  for (int i = tid; i < 16 * 6 * 25; i += 256) {
    const int co = i / 150, r = i - co * 150, ci = r / 25, t = r - ci * 25;
    ws[(co * 6 + ci) * kDxWRow + t] = wd[(co * 25 + 24 - t) * 6 + ci];  // W[co][ci][t] (wd is flipped tap-major)
  }
  const int im = lane / 6, ci = lane - 6 * im;  // lane -> (image of the group, input channel)
  const int ngroups = (p.N + kDxImgW - 1) / kDxImgW;
  const int npairs = (ngroups + 1) / 2;
  for (int pi = blockIdx.x; pi < npairs; pi += gridDim.x) {
    const int gi = 2 * pi + grp;
    const int img0 = gi * kDxImgW, nimg = max(0, min(kDxImgW, p.N - img0));
    __syncthreads();  // the previous groups' reads are done (and, first time, the weights are staged)
    if (half == 0) {
      const float4* g = reinterpret_cast<const float4*>(p.dy + (size_t)img0 * kDxImgF);
      const uint32_t* ga = reinterpret_cast<const uint32_t*>(p.arg + (size_t)img0 * kDxImgF);
      const int n4 = nimg * kDxImgF / 4;
      for (int i = lane; i < n4; i += 64) {
        reinterpret_cast<float4*>(dys)[i] = g[i];
        reinterpret_cast<uint32_t*>(dys + kDxImgW * kDxImgF)[i] = ga[i];
      }
    }
    __syncthreads();
    const bool live = lane < 6 * kDxImgW && im < nimg;
    const float* dimg = dys + (live ? im : 0) * kDxImgF;
    const uint8_t* aimg = ags + (live ? im : 0) * kDxImgF;
    float acc[7][14];
    if (half == 0) dx_half<0>(ws, dimg, aimg, ci, acc);
    else dx_half<1>(ws, dimg, aimg, ci, acc);
    if (live) {
      float* d = out + ((size_t)(img0 + im) * 196 + 98 * half) * 6 + ci;
#pragma unroll
      for (int y = 0; y < 7; ++y)
#pragma unroll
        for (int x = 0; x < 14; ++x) d[(y * 14 + x) * 6] = acc[y][x];
    }
  }
}

// Weight gradient of the pooled 6 -> 16 5x5 conv (fp32, stride 1, no
// padding): dW[c][ci][t] = sum over images and pooling windows of
// dY[c] * X[ci][argmax pixel + t].  Item = (image, pooling window); a thread
// owns one (4-channel group, input channel) combination for the whole launch
// -- 2 channel pairs x 25 taps of packed accumulators -- and walks the
// group's items with the other threads of its combination (kWSlots of them).
// Per item it decodes the four window positions' gradients from the pooled
// dY / argmax (zeros except at the argmax), streams the 6x6 input patch of
// its channel row by row from LDS and does 2 x 25 x 4 packed FMAs.  Partial
// sums: slots in a fixed order through LDS, then one slab per workgroup,
// reduced by conv1_direct_dw_reduce_kernel (deterministic).
// (4-image groups in 192-thread workgroups: 27 KB of LDS, 5 workgroups per
// CU cover each other's staging barriers: 1,427 us at B = 163840 vs 1,562
// with 8-image groups in 384-thread workgroups)
constexpr int kWImgs = 4;                  // images per group
constexpr int kWThreads = 192;
template <int CIN, int COUT, int NP>       // NP channel pairs per combination
struct DwGeom {
  static constexpr int cg = 2 * NP;        // channels per combination
  static constexpr int combos = (COUT / cg) * CIN;
  static constexpr int slots = kWThreads / combos;
  static constexpr int threads = combos * slots;
  static constexpr int ncol = COUT * (CIN * 25 + 1);
};
template <int KS, int CIN, int COUT, int NP>
__global__ void __launch_bounds__((DwGeom<CIN, COUT, NP>::threads)) __attribute__((amdgpu_waves_per_eu(NP == 1 ? 4 : 3)))
conv_direct_dw_kernel(Conv1DirectParams p) {
  using G = DwGeom<CIN, COUT, NP>;
  constexpr int kWCG = G::cg;
  static_assert(KS == 5 && COUT % kWCG == 0 && (NP == 1 || NP == 2), "shape");
  constexpr int KK = KS * KS;
  extern __shared__ __attribute__((aligned(16))) float xs[];
  const int TW = p.W, IMG = p.H * p.W * CIN;  // NHWC input, no padding
  const int PHW = p.PH * p.PW;
  float* dys = xs + kWImgs * IMG;
  uint8_t* args = reinterpret_cast<uint8_t*>(dys + kWImgs * PHW * COUT);
  const int combo = threadIdx.x % G::combos, slot = threadIdx.x / G::combos;
  const int cg = combo / CIN, ci = combo - cg * CIN;
  f2 acc[NP][KK];
  f2 accb[NP];
#pragma unroll
  for (int q = 0; q < NP; ++q) accb[q] = f2{0.f, 0.f};
#pragma unroll
  for (int q = 0; q < NP; ++q)
#pragma unroll
    for (int k = 0; k < KK; ++k) acc[q][k] = f2{0.f, 0.f};
  const int ngroups = (p.N + kWImgs - 1) / kWImgs;
  for (int grp = blockIdx.x; grp < ngroups; grp += gridDim.x) {
    const int img0 = grp * kWImgs, nimg = min(kWImgs, p.N - img0);
    __syncthreads();
    {  // contiguous runs: images (IMG % 4 == 0), pooled dY and argmax (PHW * COUT % 4 == 0)
      const int nx = nimg * IMG / 4;
      const float4* gx = reinterpret_cast<const float4*>(p.xf + (size_t)img0 * IMG);
      for (int i = threadIdx.x; i < nx; i += G::threads) reinterpret_cast<float4*>(xs)[i] = gx[i];
      const int n4 = nimg * PHW * COUT / 4;
      const float4* gdy = reinterpret_cast<const float4*>(p.dy + (size_t)img0 * PHW * COUT);
      const uint32_t* garg = reinterpret_cast<const uint32_t*>(p.arg + (size_t)img0 * PHW * COUT);
      for (int i = threadIdx.x; i < n4; i += G::threads) {
        reinterpret_cast<float4*>(dys)[i] = gdy[i];
        reinterpret_cast<uint32_t*>(args)[i] = garg[i];
      }
    }
    __syncthreads();
    for (int it = slot; it < nimg * PHW; it += G::slots) {
      const int m = it / PHW, w = it - m * PHW;
      const int py = w / p.PW, px = w - py * p.PW;
      const int o = it * COUT + cg * kWCG;
      f2 g[NP][4];  // [pair][window position]
#pragma unroll
      for (int q = 0; q < NP; ++q) {
        const float2 gy = *reinterpret_cast<const float2*>(dys + o + 2 * q);
        const int a0 = args[o + 2 * q], a1 = args[o + 2 * q + 1];
#pragma unroll
        for (int e = 0; e < 4; ++e) g[q][e] = f2{a0 == e ? gy.x : 0.f, a1 == e ? gy.y : 0.f};
        if (ci == 0) accb[q] += f2{a0 < 4 ? gy.x : 0.f, a1 < 4 ? gy.y : 0.f};
      }
      const float* x = xs + m * IMG + ((2 * py) * TW + 2 * px) * CIN + ci;
#pragma unroll
      for (int r = 0; r <= KS; ++r) {  // patch row r feeds tap rows r (top positions) and r - 1 (bottom)
        f2 R[(KS + 1) / 2];
#pragma unroll
        for (int j = 0; j < (KS + 1) / 2; ++j) R[j] = f2{x[(r * TW + 2 * j) * CIN], x[(r * TW + 2 * j + 1) * CIN]};
#pragma unroll
        for (int q = 0; q < NP; ++q) {
#pragma unroll
          for (int kw = 0; kw < KS; ++kw) {
            if (r < KS) {
              acc[q][r * KS + kw] = pfma(g[q][0], MCC_PS(R, kw), acc[q][r * KS + kw]);
              acc[q][r * KS + kw] = pfma(g[q][1], MCC_PS(R, kw + 1), acc[q][r * KS + kw]);
            }
            if (r > 0) {
              acc[q][(r - 1) * KS + kw] = pfma(g[q][2], MCC_PS(R, kw), acc[q][(r - 1) * KS + kw]);
              acc[q][(r - 1) * KS + kw] = pfma(g[q][3], MCC_PS(R, kw + 1), acc[q][(r - 1) * KS + kw]);
            }
          }
        }
      }
    }
  }
  // slots in order into LDS [combo][4 channels][KK + 1], then the slab
  __syncthreads();
  constexpr int per = kWCG * (KK + 1);
  float* red = xs;
  for (int s = 0; s < G::slots; ++s) {
    if (slot == s) {
#pragma unroll
      for (int c = 0; c < kWCG; ++c) {
#pragma unroll
        for (int k = 0; k < KK; ++k) {
          const float v = (c & 1) ? acc[c >> 1][k].y : acc[c >> 1][k].x;
          float& d = red[combo * per + c * (KK + 1) + k];
          d = s == 0 ? v : d + v;
        }
        const float vb = (c & 1) ? accb[c >> 1].y : accb[c >> 1].x;
        float& d = red[combo * per + c * (KK + 1) + KK];
        d = s == 0 ? vb : d + vb;
      }
    }
    __syncthreads();
  }
  // slab column (c, k): k < CIN*KK weight (ci, tap), k == CIN*KK bias (from the ci == 0 combos)
  for (int i = threadIdx.x; i < G::ncol; i += G::threads) {
    const int c = i / (CIN * KK + 1), k = i - c * (CIN * KK + 1);
    const int g4 = c / kWCG, cc = c - g4 * kWCG;
    const int kci = k < CIN * KK ? k / KK : 0, t = k < CIN * KK ? k - kci * KK : KK;
    p.slab[(size_t)blockIdx.x * G::ncol + i] = red[(g4 * CIN + kci) * per + cc * (KK + 1) + t];
  }
}

// One workgroup per column (c, k): 256 strided partial sums over the slabs,
// then a fixed LDS tree.  k < Cin*KS*KS: weight, k == Cin*KS*KS: bias.
__global__ void __launch_bounds__(256) conv1_direct_dw_reduce_kernel(Conv1DirectParams p, int nslab, float* gw,
                                                                     float* gb) {
  __shared__ float part[256];
  const int KK = p.Cin * p.KS * p.KS, ncol = p.C * (KK + 1);  // KK: weights per output channel
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

constexpr int kDImgs2 = 10;  // conv2 forward (Cin > 1): images per group
constexpr int kDImgs1 = 9;   // conv1 forward (Cin == 1)
int fwd_imgs(const Conv1DirectParams& p) { return p.Cin == 1 ? kDImgs1 : kDImgs2; }
size_t fwd_lds(const Conv1DirectParams& p) { return (size_t)kDImgs * d_tile(p).IMG * 4; }
size_t fwd_lds_n(const Conv1DirectParams& p) { return (size_t)fwd_imgs(p) * d_tile(p).IMG * 4; }
size_t dw_lds(const Conv1DirectParams& p) {
  return fwd_lds(p) + (size_t)kDImgs * p.PH * p.PW * p.C * 5;  // + dY floats + argmax bytes
}

}  // namespace

bool conv_direct_fwd_supported(const Conv1DirectParams& p) {
  const bool shape = p.KS == 5 && ((p.Cin == 1 && p.C == 6) || (p.Cin == 6 && p.C == 16));
  const Tile t = d_tile(p);
  const bool stage_ok = p.Cin == 1 ? stager_fits(p, t) : (p.pad == 0 && t.TW == p.W && t.IMG % 4 == 0);
  return shape && stage_ok && p.OH % 2 == 0 && p.OW % 2 == 0 && p.OH == p.H + 2 * p.pad - p.KS + 1 &&
         p.OW == p.W + 2 * p.pad - p.KS + 1 && p.PH == p.OH / 2 && p.PW == p.OW / 2 && fwd_lds_n(p) <= 64 * 1024;
}

// dX geometry: p.H x p.W = the forward input (dX) grid, p.PH x p.PW = pooled dY
bool conv_direct_dx_supported(const Conv1DirectParams& p) {
  // the scatter kernel is specialised to LeNet-5's conv2 (14x14x6 -> 10x10x16 -> 5x5x16)
  return p.KS == 5 && p.pad == 0 && p.Cin == 6 && p.C == 16 && p.H == 14 && p.W == 14 && p.OH == 10 && p.OW == 10 &&
         p.PH == 5 && p.PW == 5;
}

void conv_direct_dx(const Conv1DirectParams& p, float* dx, hipStream_t s) {
  MCC_CHECK(conv_direct_dx_supported(p) && p.wd && p.dy && p.arg && dx, "conv_direct_dx: bad params");
  MCC_CHECK(reinterpret_cast<uintptr_t>(p.dy) % 16 == 0 && reinterpret_cast<uintptr_t>(p.arg) % 4 == 0,
            "conv_direct_dx: dY / argmax alignment");
  const int npairs = ((p.N + kDxImgW - 1) / kDxImgW + 1) / 2;
  const dim3 grid((unsigned)std::max(1, std::min(npairs, 256 * 3))), block(256);
  hipLaunchKernelGGL(conv_direct_dx_kernel, grid, block, kDxLds, s, p, p.wd, dx);
}

bool conv1_direct_dw_supported(const Conv1DirectParams& p) {
  return p.Cin == 1 && p.C >= 2 && p.C <= kDMaxC && p.C % 2 == 0 && (p.KS == 3 || p.KS == 5) && p.OH % 2 == 0 &&
         p.OW % 2 == 0 && stager_fits(p, d_tile(p)) && (p.PH * p.PW * p.C) % 4 == 0 &&
         p.OH == p.H + 2 * p.pad - p.KS + 1 && p.OW == p.W + 2 * p.pad - p.KS + 1 && p.PH == p.OH / 2 &&
         p.PW == p.OW / 2 && dw_lds(p) <= 96 * 1024;
}

static int direct_grid(const Conv1DirectParams& p) {
  const int ngroups = (p.N + kDImgs - 1) / kDImgs;
  return std::max(1, std::min(ngroups, 256 * 4));
}

static int dw3_grid(const Conv1DirectParams& p) {
  return std::max(1, std::min((p.N + kDW3Imgs - 1) / kDW3Imgs, 256 * 4));
}
// LeNet-5's conv1 (28x28 u8, pad 2, 6 channels): the sparse kernel of lenet_f32.hip
static bool lenet32_dw1_shape(const Conv1DirectParams& p) {
  return p.Cin == 1 && p.C == 6 && p.KS == 5 && p.pad == 2 && p.H == 28 && p.W == 28 && p.PH == 14 && p.PW == 14;
}
size_t conv1_direct_slab_bytes(const Conv1DirectParams& p) {
  const int g = std::max(std::max(direct_grid(p), dw3_grid(p)), lenet32_dw1_shape(p) ? lenet32_dw1_grid(p.N) : 0);
  return (size_t)g * p.C * (p.KS * p.KS + 1) * 4;
}

void conv_direct_forward(const Conv1DirectParams& p, hipStream_t s) {
  MCC_CHECK(conv_direct_fwd_supported(p) && (p.x || p.xf) && p.wt && p.bias && p.out && p.out_arg,
            "conv_direct_forward: bad params");
  const dim3 grid((unsigned)direct_grid(p)), block(kDT);
  if (p.Cin == 1 && ab_flag("f32_fwd1_g8"))
    hipLaunchKernelGGL((conv_direct_fwd_kernel<5, 1, 6>), grid, block, fwd_lds(p), s, p, p.wt, p.bias, p.out,
                       p.out_arg);
  else if (p.Cin == 1) {
    const Tile t = d_tile(p);  // the stager's packed item fields with 9 images
    MCC_CHECK(kDImgs1 * t.IMG <= 16384 && kDImgs1 * p.H * (p.W / 4) <= kDU8Items * kDT, "conv_direct_forward: tile");
    const int ng = (p.N + kDImgs1 - 1) / kDImgs1;
    hipLaunchKernelGGL((conv_direct_fwd_kernel<5, 1, 6, kDImgs1>), dim3((unsigned)std::max(1, std::min(ng, 256 * 4))),
                       block, fwd_lds_n(p), s, p, p.wt, p.bias, p.out, p.out_arg);
  }
  else if (p.H == 14 && p.W == 14 && p.pad == 0 && ab_flag("f32_mfma_fwd2"))
    lenet32_conv2_fwd(p, s);  // f32 MFMA (lenet_f32.hip; measured slower, opt-in)
  else if (ab_flag("f32_fwd2_g8"))
    hipLaunchKernelGGL((conv_direct_fwd_kernel<5, 6, 16>), grid, block, fwd_lds(p), s, p, p.wt, p.bias, p.out,
                       p.out_arg);
  else {
    const int ng = (p.N + kDImgs2 - 1) / kDImgs2;
    hipLaunchKernelGGL((conv_direct_fwd_kernel<5, 6, 16, kDImgs2>), dim3((unsigned)std::max(1, std::min(ng, 256 * 3))),
                       block, fwd_lds_n(p), s, p, p.wt, p.bias, p.out, p.out_arg);
  }
}

static void dw_reduce(const Conv1DirectParams& p, int grid, float* gw, float* gb, hipStream_t s) {
  const int ncol = p.C * (p.Cin * p.KS * p.KS + 1);
  hipLaunchKernelGGL(conv1_direct_dw_reduce_kernel, dim3((unsigned)ncol), dim3(256), 0, s, p, grid, gw, gb);
}

void conv1_direct_dw(const Conv1DirectParams& p, float* gw, float* gb, hipStream_t s) {
  MCC_CHECK(conv1_direct_dw_supported(p) && p.x && p.dy && p.arg && p.slab, "conv1_direct_dw: bad params");
  const int grid = direct_grid(p);
  const dim3 g((unsigned)grid), b(kDT);
  if (lenet32_dw1_shape(p) && !ab_flag("f32_dense_dw")) {
    lenet32_dw1(p, s);
    dw_reduce(p, lenet32_dw1_grid(p.N), gw, gb, s);
    return;
  }
  if (p.KS == 5 && p.C == 6) {
    const int g3 = dw3_grid(p);
    const size_t lds = (size_t)kDW3Imgs * d_tile(p).IMG * 4 + (size_t)kDW3Imgs * p.PH * p.PW * p.C * 5;
    hipLaunchKernelGGL((conv1_direct_dw_w3_kernel<5>), dim3((unsigned)g3), dim3(kDW3T), lds, s, p);
    dw_reduce(p, g3, gw, gb, s);
    return;
  }
  else if (p.KS == 5) hipLaunchKernelGGL((conv1_direct_dw_kernel<5, kDMaxC, false>), g, b, dw_lds(p), s, p);
  else hipLaunchKernelGGL((conv1_direct_dw_kernel<3, kDMaxC, false>), g, b, dw_lds(p), s, p);
  dw_reduce(p, grid, gw, gb, s);
}

// conv2-shaped (6 -> 16, 5x5, unpadded, pooled) weight gradient
static size_t dw2_lds(const Conv1DirectParams& p) {
  return (size_t)kWImgs * (p.H * p.W * p.Cin * 4 + p.PH * p.PW * p.C * 5);
}
static int dw2_grid(const Conv1DirectParams& p) {
  return std::max(1, std::min((p.N + kWImgs - 1) / kWImgs, 256 * 5));
}
bool conv_direct_dw_supported(const Conv1DirectParams& p) {
  return p.KS == 5 && p.pad == 0 && p.Cin == 6 && p.C == 16 && p.OH == p.H - 4 && p.OW == p.W - 4 &&
         p.OH % 2 == 0 && p.OW % 2 == 0 && p.PH == p.OH / 2 && p.PW == p.OW / 2 && (p.H * p.W * p.Cin) % 4 == 0 &&
         (p.PH * p.PW * p.C) % 4 == 0 && dw2_lds(p) <= 64 * 1024;
}
size_t conv_direct_dw_slab_bytes(const Conv1DirectParams& p) {
  return (size_t)std::max(dw2_grid(p), lenet32_dw2_grid(p.N)) * p.C * (p.Cin * p.KS * p.KS + 1) * 4;
}
void conv_direct_dw(const Conv1DirectParams& p, float* gw, float* gb, hipStream_t s) {
  MCC_CHECK(conv_direct_dw_supported(p) && p.xf && p.dy && p.arg && p.slab, "conv_direct_dw: bad params");
  if (p.H == 14 && p.W == 14 && !ab_flag("f32_dense_dw")) {  // LeNet-5's conv2: sparse kernel (lenet_f32.hip)
    lenet32_dw2(p, s);
    dw_reduce(p, lenet32_dw2_grid(p.N), gw, gb, s);
    return;
  }
  const int grid = dw2_grid(p);
  // one channel pair per thread (NP = 1): 1,274 us at B = 131072 vs 1,409 us
  // with two pairs (fewer patch reads, but 158 registers and 3 waves per SIMD)
  hipLaunchKernelGGL((conv_direct_dw_kernel<5, 6, 16, 1>), dim3((unsigned)grid), dim3(DwGeom<6, 16, 1>::threads),
                     dw2_lds(p), s, p);
  dw_reduce(p, grid, gw, gb, s);
}

}  // namespace gpu
}  // namespace mcc
