// CIFAR-3conv conv2 on gfx950: conv 32 -> 64 channels, 3x3, pad 1, on 16x16
// images, ReLU + 2x2 max-pool.  Reference semantics: Layer_feedForw_conv /
// Layer_feedBack_conv (/root/reference/cnn.c:175-247, with the correct OIHW
// indexing of CUDAcnn.cu:167-195); the pool is a BASELINE.json addition.
//
// This layer was the weakest of the CIFAR-3conv step on the generic
// small-image kernels (conv_pipe: forward 1.27 ms ~ 480 TFLOP/s, data
// gradient 1.98 ms, weight gradient 2.10 ms at B = 65,024, with 44-67 % of
// their LDS cycles bank conflicts), while conv3 -- the same 4.7 M MACs per
// image -- ran ~1 ms per pass on the implicit GEMM.  Per image the forward is
// a 256 x 64 x 288 GEMM (rows = output pixels, K = 9 taps x 32 channels):
//
//  * one 256-thread workgroup per image at a time, persistent over the batch,
//    two per CU (two waves per SIMD); wave (wm, wn) owns 128 output pixels x
//    32 channels = 16 accumulator tiles, and holds the B fragments of its 32
//    channels for all 9 taps in registers for the whole launch (72 VGPRs), so
//    the K loop reads only the A operand from LDS: 8 ds_read_b128 per 16
//    MFMAs (0.5 KB per MFMA; the LDS delivers 1 KB per MFMA issue slot);
//  * the zero-padded input image (18 x 18 pixels x 64 B) is staged once per
//    image, double buffered (register prefetch of the next image during the
//    MFMAs, one barrier per image); the 16-byte channel chunk c of padded
//    pixel (Y, X) sits at chunk c ^ 2 (Y & 1): with the 18-pixel pitch every
//    16-lane group of every A-fragment read hits 16 distinct 16-byte bank
//    slots (bank model: conflict-free for all 9 taps and 8 row tiles, vs
//    2-way without the swizzle);
//  * GEMM rows are ordered (pool window, position) so a lane's four
//    accumulator values are the four positions of one 2x2 window of one
//    channel: the max-pool and its first-max-wins argmax are three in-lane
//    compares, then bias + ReLU once (both monotone), as the generic path;
//  * every A-fragment address is a per-lane base (two: the tap row parity
//    flips the swizzle) plus a compile-time immediate.
#include "kernels.h"
#include "mfma.h"

#include <algorithm>

namespace mcc {
namespace gpu {
namespace {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

constexpr int kP = 18;                 // padded tile pitch (pixels)
constexpr int kPix = 64;               // bytes per staged pixel (32 bf16 channels)
constexpr int kTile = kP * kP * kPix;  // 20,736 B
constexpr int kImgIn = 16 * 16 * 32;   // input elements per image
constexpr int kImgOut = 8 * 8 * 64;    // pooled output elements per image

// LDS byte offset of 16-byte chunk c (channels 8c .. 8c+7) of padded pixel (Y, X)
__device__ __forceinline__ int tile_off(int Y, int X, int c) { return (Y * kP + X) * kPix + 16 * (c ^ (2 * (Y & 1))); }

__global__ void __launch_bounds__(256, 2) cifar_c2_fwd_kernel(CifarC2Params p) {
  __shared__ __attribute__((aligned(16))) char smem[2 * kTile];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wv >> 1, wn = wv & 1;
  const int r16 = lane & 15, g = lane >> 4;
  const int grid = (int)gridDim.x;

  for (int i = tid * 16; i < 2 * kTile; i += 256 * 16) *reinterpret_cast<u32x4*>(smem + i) = u32x4{0u, 0u, 0u, 0u};

  // B fragments: channels 32 wn + 16 nt + r16, tap t, input channels 8g .. 8g+7
  const bf16* w = static_cast<const bf16*>(p.w);
  bf16x8 wb[2][9];
#pragma unroll
  for (int nt = 0; nt < 2; ++nt)
#pragma unroll
    for (int t = 0; t < 9; ++t) wb[nt][t] = load8(w + (size_t)(32 * wn + 16 * nt + r16) * p.ldw + 32 * t + 8 * g);
  const float bv0 = p.bias[32 * wn + r16], bv1 = p.bias[32 * wn + 16 + r16];

  // A fragments: row m = 128 wm + 16 T + r16 of the image GEMM is position
  // pos = r16 & 3 = (dy, dx) of window 32 wm + 4 T + (r16 >> 2), i.e. output
  // pixel (8 wm + 2 (T >> 1) + dy, 8 (T & 1) + 2 (r16 >> 2) + dx); tap (ky, kx)
  // reads padded pixel (y + ky, x + kx), whose row parity is dy ^ (ky & 1)
  const int dy = (r16 >> 1) & 1, dx = r16 & 1;
  const int y0 = 8 * wm + dy, x0 = 2 * (r16 >> 2) + dx;
  const int la0 = (y0 * kP + x0) * kPix + 16 * (g ^ (2 * dy));
  const int la1 = ((y0 + 1) * kP + x0) * kPix + 16 * (g ^ (2 * (dy ^ 1)));

  // staging: 16-byte chunk j = tid + 256 i of an image = pixel j >> 2, chunk j & 3
  int soff[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int j = tid + 256 * i, pp = j >> 2;
    soff[i] = tile_off((pp >> 4) + 1, (pp & 15) + 1, j & 3);
  }
  const char* xg = static_cast<const char*>(p.x);
  u32x4 st[4];
  auto load = [&](int img) {
    const u32x4* src = reinterpret_cast<const u32x4*>(xg + (size_t)img * (kImgIn * 2));
#pragma unroll
    for (int i = 0; i < 4; ++i) st[i] = src[tid + 256 * i];
  };
  __syncthreads();  // zero fill before the first interior write
  int img = blockIdx.x;
  if (img < p.B) load(img);
  for (int k = 0; img < p.B; img += grid, ++k) {
    char* tb = smem + (k & 1) * kTile;
#pragma unroll
    for (int i = 0; i < 4; ++i) *reinterpret_cast<u32x4*>(tb + soff[i]) = st[i];
    __syncthreads();  // image k staged; every wave is past its reads of image k - 1's buffer ... of k - 2's
    if (img + grid < p.B) load(img + grid);

    f32x4 acc[8][2];
#pragma unroll
    for (int t = 0; t < 8; ++t) acc[t][0] = acc[t][1] = f32x4{0.f, 0.f, 0.f, 0.f};
    // one tap of look-ahead: tap + 1's eight A fragments are read while tap's
    // sixteen MFMAs issue (a full unroll would hoist all 72 reads)
    auto read_a = [&](int tap, bf16x8 (&a)[8]) {
      const int ky = tap / 3, kx = tap % 3;
      const char* base = tb + (ky == 1 ? la1 : la0) + ((ky == 2 ? 2 * kP : 0) + kx) * kPix;
#pragma unroll
      for (int t = 0; t < 8; ++t)
        a[t] = *reinterpret_cast<const bf16x8*>(base + ((t >> 1) * 2 * kP + (t & 1) * 8) * kPix);
    };
    bf16x8 a[2][8];
    read_a(0, a[0]);
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) {
      if (tap + 1 < 9) read_a(tap + 1, a[(tap + 1) & 1]);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int t = 0; t < 8; ++t) {
        acc[t][0] = mma(acc[t][0], a[tap & 1][t], wb[0][tap]);
        acc[t][1] = mma(acc[t][1], a[tap & 1][t], wb[1][tap]);
      }
      __builtin_amdgcn_sched_barrier(0);
    }

    // pool + bias + ReLU: lane (channel r16 of tile nt, window g of row tile T)
    bf16* yo = static_cast<bf16*>(p.y) + (size_t)img * kImgOut;
    uint8_t* ao = p.arg + (size_t)img * kImgOut;
#pragma unroll
    for (int t = 0; t < 8; ++t) {
      const int win = 32 * wm + 4 * t + g;
#pragma unroll
      for (int nt = 0; nt < 2; ++nt) {
        const f32x4 v = acc[t][nt];
        float best = v[0];
        int arg = 0;
#pragma unroll
        for (int i = 1; i < 4; ++i) {  // first max wins: TL, TR, BL, BR
          const bool gt = v[i] > best;
          best = gt ? v[i] : best;
          arg = gt ? i : arg;
        }
        const bf16 yb = (bf16)fmaxf(best + (nt ? bv1 : bv0), 0.f);
        const int o = win * 64 + 32 * wn + 16 * nt + r16;
        yo[o] = yb;
        ao[o] = (uint8_t)((float)yb > 0.f ? arg : 4);  // 4: ReLU-inactive window
      }
    }
  }
}

// ---------------------------------------------------------------- backward
// Both backward kernels rebuild the unpooled pre-activation gradient dZ of an
// image in LDS from the pooled dY and the argmax codes (dZ = dY at the
// window's argmax position, 0 elsewhere and in ReLU-inactive windows), then
// run the image's GEMM on MFMA.  One 512-thread workgroup per CU (8 waves,
// two per SIMD), persistent over the batch, double-buffered LDS images with
// a register prefetch of the next image's loads and one barrier per image.

// d[k] (channels 2k, 2k+1) kept where the channel's argmax byte equals pos
__device__ __forceinline__ u32x4 unpool_pos(const u32x4& d, uint32_t a0, uint32_t a1, uint32_t pos) {
  u32x4 o;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const uint32_t a = (k < 2 ? a0 : a1) >> (16 * (k & 1));
    const uint32_t lo = (a & 0xffu) == pos ? 0x0000ffffu : 0u;
    const uint32_t hi = ((a >> 8) & 0xffu) == pos ? 0xffff0000u : 0u;
    o[k] = d[k] & (lo | hi);
  }
  return o;
}

// ---- data gradient: dX = conv(dZ padded by 1, flipped W), per image the
// swapped GEMM dX^T [32 ci][256 px] = Wd [32][576] x dZ-patches [576][256 px],
// so a lane's four accumulators are four consecutive channels of one pixel
// (8-byte stores).  The flipped weights (A operand) of both 16-channel tiles
// stay in registers for the whole launch (144 VGPRs); the K loop reads only
// the dZ patches (B operand): 2 ds_read_b128 per 4 MFMAs.
//
// dZ image in LDS: four planes of 16 channels, each [18 x 18 padded px][32 B];
// B-fragment lane (pixel x = r16 of image row y, chunk 4 kc + g) reads plane
// 2 kc + (g >> 1), half g & 1: within a ds_read_b128 lane group the 16 lanes
// hit 8 consecutive pixels x 2 halves = 256 distinct bytes for every tap
// (conflict-free, tools/lds_banks.py), and every read is a per-lane base
// plus a compile-time offset.  The plane stride is 32 mod 128 B so the
// unpool stores (8 lanes = 8 chunks of one pixel) hit 8 distinct bank groups.
constexpr int kDxPS = 324 * 32 + 32;  // 10,400 B
constexpr int kDxBuf = 4 * kDxPS;     // 41,600 B

__global__ void __launch_bounds__(512, 1) cifar_c2_dx_kernel(CifarC2BwdParams p) {
  __shared__ __attribute__((aligned(16))) char smem[2 * kDxBuf];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);  // image rows 2 wv, 2 wv + 1
  const int r16 = lane & 15, g = lane >> 4;
  const int grid = (int)gridDim.x;

  for (int i = tid * 16; i < 2 * kDxBuf; i += 512 * 16) *reinterpret_cast<u32x4*>(smem + i) = u32x4{0u, 0u, 0u, 0u};

  // A fragments: input channel 16 ct + r16, k = 32 ks + 8 g (tap ks >> 1, output channels 32 (ks & 1) + 8 g ..)
  const bf16* wd = static_cast<const bf16*>(p.wd);
  bf16x8 wa[2][18];
#pragma unroll
  for (int ct = 0; ct < 2; ++ct)
#pragma unroll
    for (int ks = 0; ks < 18; ++ks) wa[ct][ks] = load8(wd + (size_t)(16 * ct + r16) * p.ldw + 32 * ks + 8 * g);

  const int lb = (g >> 1) * kDxPS + ((2 * wv) * kP + r16) * 32 + 16 * (g & 1);

  // staging: thread (window w, channel chunk c): 16 B of dY + 8 B of argmax,
  // four 16-byte stores (the window's positions) into plane c >> 1
  const int w = tid >> 3, c = tid & 7;
  const int sbase = (c >> 1) * kDxPS + ((2 * (w >> 3) + 1) * kP + 2 * (w & 7) + 1) * 32 + 16 * (c & 1);
  const char* dyg = static_cast<const char*>(p.dy);
  u32x4 sd;
  uint32_t sa0, sa1;
  auto load = [&](int img) {
    const size_t e = (size_t)img * kImgOut + w * 64 + 8 * c;
    sd = *reinterpret_cast<const u32x4*>(dyg + 2 * e);
    const uint2 a = *reinterpret_cast<const uint2*>(p.arg + e);
    sa0 = a.x; sa1 = a.y;
  };
  bf16* dxo = static_cast<bf16*>(p.dx);
  __syncthreads();  // zero fill before the first interior write
  int img = blockIdx.x;
  if (img < p.B) load(img);
  for (int k = 0; img < p.B; img += grid, ++k) {
    char* tb = smem + (k & 1) * kDxBuf;
#pragma unroll
    for (int pos = 0; pos < 4; ++pos)
      *reinterpret_cast<u32x4*>(tb + sbase + ((pos >> 1) * kP + (pos & 1)) * 32) = unpool_pos(sd, sa0, sa1, pos);
    __syncthreads();  // image k staged; every wave is past image k - 1's reads of this buffer (k - 2)
    if (img + grid < p.B) load(img + grid);

    f32x4 acc[2][2];
#pragma unroll
    for (int ct = 0; ct < 2; ++ct) acc[ct][0] = acc[ct][1] = f32x4{0.f, 0.f, 0.f, 0.f};
    const char* rb = tb + lb;
    auto read_b = [&](int ks, bf16x8 (&b)[2]) {
      const int tap = ks >> 1, off = (ks & 1) * 2 * kDxPS + ((tap / 3) * kP + tap % 3) * 32;
#pragma unroll
      for (int pt = 0; pt < 2; ++pt) b[pt] = *reinterpret_cast<const bf16x8*>(rb + off + pt * kP * 32);
    };
    bf16x8 b[2][2];
    read_b(0, b[0]);
#pragma unroll
    for (int ks = 0; ks < 18; ++ks) {
      if (ks + 1 < 18) read_b(ks + 1, b[(ks + 1) & 1]);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int ct = 0; ct < 2; ++ct)
#pragma unroll
        for (int pt = 0; pt < 2; ++pt) acc[ct][pt] = mma(acc[ct][pt], wa[ct][ks], b[ks & 1][pt]);
      __builtin_amdgcn_sched_barrier(0);
    }

    // lane: channels 16 ct + 4 g .. + 3 of pixel (2 wv + pt, r16)
    bf16* o = dxo + (size_t)img * kImgIn;
#pragma unroll
    for (int pt = 0; pt < 2; ++pt)
#pragma unroll
      for (int ct = 0; ct < 2; ++ct) {
        const f32x4 v = acc[ct][pt];
        *reinterpret_cast<bf16x4*>(o + ((2 * wv + pt) * 16 + r16) * 32 + 16 * ct + 4 * g) = cvt4(v[0], v[1], v[2], v[3]);
      }
  }
}

// ---- weight gradient: per image dW [64 co][288 = (tap, ci)] += dZ^T [64][256 px]
// x X-patches [256 px][288], K = the image's pixels in (pool window, position)
// order.  Wave (kq, nh) owns all 64 output channels x the 9 taps of input
// channels 16 nh .. 16 nh + 15 (36 accumulator tiles) over the image's
// K-quarter kq (64 pixels = 16 windows); the four K-quarter partials are summed
// through LDS once at the end and each workgroup writes one slab row.
//
//  * dZ^T image [64 co][256 k], 512-byte rows, 16-byte chunk q of row co at
//    q ^ (co & 15): the A-fragment ds_read_b128 and the unpool ds_write_b64
//    (lane = window) are conflict-free;
//  * X image: two planes of 16 channels, [18 x 18 padded px][32 B], read by
//    ds_read_b64_tr_b16 (row q of a 4 x 16 block = window position q, so a
//    half-wave's 8 rows are two 2 x 2 pixel blocks 4 pixels apart: 8 distinct
//    32-byte slots mod 256 B, conflict-free at every tap), all reads a per-lane
//    base + compile-time offset; plane stride 64 mod 128 B for the staging stores;
//  * the bias gradient (sum of dZ = sum of dY over active windows) is summed in
//    the staging threads, fp32.
constexpr int kXPS = 324 * 32 + 64;     // 10,432 B
constexpr int kZT = 64 * 512;           // 32,768 B
constexpr int kDwBuf = kZT + 2 * kXPS;  // 53,632 B
constexpr int kDwCols = 304;            // slab columns: 288 weights, bias at 288
constexpr int kDwRed = 2 * 4 * 9 * 4 * 64;  // floats of one K-quarter partial
constexpr int kDwLds = 2 * kDwRed * 4 > 2 * kDwBuf ? 2 * kDwRed * 4 : 2 * kDwBuf;  // 147,456 B
constexpr int kDwGrid = 256;

__device__ __forceinline__ int zt_off(int co, int k) { return co * 512 + 16 * ((k >> 3) ^ (co & 15)) + 2 * (k & 7); }

__global__ void __launch_bounds__(512, 1) cifar_c2_dw_kernel(CifarC2BwdParams p) {
  __shared__ __attribute__((aligned(16))) char smem[kDwLds];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int kq = wv >> 1, nh = wv & 1;
  const int r16 = lane & 15, g = lane >> 4;
  const int grid = (int)gridDim.x;

  for (int i = tid * 16; i < 2 * kDwBuf; i += 512 * 16) *reinterpret_cast<u32x4*>(smem + i) = u32x4{0u, 0u, 0u, 0u};

  // A fragments (dZ^T rows co = 16 ct + r16, k = 32 ks + 8 g), ks = 2 kq + ksl
  int za[2][4];
#pragma unroll
  for (int ksl = 0; ksl < 2; ++ksl)
#pragma unroll
    for (int ct = 0; ct < 4; ++ct) za[ksl][ct] = zt_off(16 * ct + r16, 32 * (2 * kq + ksl) + 8 * g);
  // B fragments: lane 4 q + p of group g supplies window 8 ks + 2 g + s, position q, channels 16 nh + 4 p ..
  const int q4 = r16 >> 2, p4 = r16 & 3;
  const int xb = kZT + nh * kXPS + ((4 * kq + (q4 >> 1)) * kP + 4 * g + (q4 & 1)) * 32 + 8 * p4;

  // staging: dZ -- thread (window w, chunk c = wave): 8 channels x 4 positions;
  // X -- two 16-byte chunks per thread
  const int w = tid & 63, c = tid >> 6;
  int zo[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) zo[j] = zt_off(8 * c + j, 4 * w);
  int xo[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int j = tid + 512 * i, pp = j >> 2, cc = j & 3;
    xo[i] = kZT + (cc >> 1) * kXPS + (((pp >> 4) + 1) * kP + (pp & 15) + 1) * 32 + 16 * (cc & 1);
  }
  const char* dyg = static_cast<const char*>(p.dy);
  const char* xg = static_cast<const char*>(p.x);
  u32x4 sd, sx[2];
  uint32_t sa0, sa1;
  auto load = [&](int img) {
    const size_t e = (size_t)img * kImgOut + w * 64 + 8 * c;
    sd = *reinterpret_cast<const u32x4*>(dyg + 2 * e);
    const uint2 a = *reinterpret_cast<const uint2*>(p.arg + e);
    sa0 = a.x; sa1 = a.y;
    const u32x4* src = reinterpret_cast<const u32x4*>(xg + (size_t)img * (kImgIn * 2));
#pragma unroll
    for (int i = 0; i < 2; ++i) sx[i] = src[tid + 512 * i];
  };
  float bsum[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) bsum[j] = 0.f;

  f32x4 acc[4][9];
#pragma unroll
  for (int ct = 0; ct < 4; ++ct)
#pragma unroll
    for (int t = 0; t < 9; ++t) acc[ct][t] = f32x4{0.f, 0.f, 0.f, 0.f};

  __syncthreads();  // zero fill before the first interior write
  int img = blockIdx.x;
  if (img < p.B) load(img);
  for (int k = 0; img < p.B; img += grid, ++k) {
    char* tb = smem + (k & 1) * kDwBuf;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const uint32_t v = (sd[j >> 1] >> (16 * (j & 1))) & 0xffffu;
      const uint32_t a = ((j < 4 ? sa0 : sa1) >> (8 * (j & 3))) & 0xffu;
      uint2 o;
      o.x = a == 0 ? v : (a == 1 ? v << 16 : 0u);
      o.y = a == 2 ? v : (a == 3 ? v << 16 : 0u);
      *reinterpret_cast<uint2*>(tb + zo[j]) = o;
      bsum[j] += a < 4 ? __uint_as_float(v << 16) : 0.f;
    }
#pragma unroll
    for (int i = 0; i < 2; ++i) *reinterpret_cast<u32x4*>(tb + xo[i]) = sx[i];
    __syncthreads();  // image k staged; buffer k & 1's previous readers (image k - 2) are done
    if (img + grid < p.B) load(img + grid);

#pragma unroll
    for (int ksl = 0; ksl < 2; ++ksl) {
      bf16x8 a[4];
#pragma unroll
      for (int ct = 0; ct < 4; ++ct) a[ct] = *reinterpret_cast<const bf16x8*>(tb + za[ksl][ct]);
      const bf16* xr = reinterpret_cast<const bf16*>(tb + xb);
#pragma unroll
      for (int t = 0; t < 9; ++t) {
        const int off = ((2 * ksl + t / 3) * kP + t % 3) * 16;  // in bf16 elements (32 B per pixel)
        const bf16x4 lo = tr4(xr + off), hi = tr4(xr + off + 2 * 16);  // s = 0, 1: windows 2 apart in x = +2 px
        const bf16x8 bfr = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
#pragma unroll
        for (int ct = 0; ct < 4; ++ct) acc[ct][t] = mma(acc[ct][t], a[ct], bfr);
      }
    }
  }

  // sum the K-quarter partials: (1 -> 0, 3 -> 2), then 2 -> 0
  __syncthreads();
  float* red = reinterpret_cast<float*>(smem);
#define MCC_C2_RED(STMT)                  \
  _Pragma("unroll") for (int ct = 0; ct < 4; ++ct) \
  _Pragma("unroll") for (int t = 0; t < 9; ++t)    \
  _Pragma("unroll") for (int i = 0; i < 4; ++i) { const int ri = (((nh * 4 + ct) * 9 + t) * 4 + i) * 64 + lane; STMT; }
  if (kq & 1) { float* r = red + (kq >> 1) * kDwRed; MCC_C2_RED(r[ri] = acc[ct][t][i]) }
  __syncthreads();
  if (!(kq & 1)) { const float* r = red + (kq >> 1) * kDwRed; MCC_C2_RED(acc[ct][t][i] += r[ri]) }
  __syncthreads();
  if (kq == 2) { MCC_C2_RED(red[ri] = acc[ct][t][i]) }
  __syncthreads();
  float* slab = p.slab + (size_t)blockIdx.x * 64 * kDwCols;
  if (kq == 0) {
    MCC_C2_RED(acc[ct][t][i] += red[ri])
#undef MCC_C2_RED
#pragma unroll
    for (int ct = 0; ct < 4; ++ct)
#pragma unroll
      for (int t = 0; t < 9; ++t)
#pragma unroll
        for (int i = 0; i < 4; ++i) slab[(16 * ct + 4 * g + i) * kDwCols + 32 * t + 16 * nh + r16] = acc[ct][t][i];
  }
  // bias: wave c holds channels 8 c .. 8 c + 7 over its 64 windows
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    float v = bsum[j];
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) v += __shfl_xor(v, m, 64);
    bsum[j] = v;
  }
  if (lane == 0) {
#pragma unroll
    for (int j = 0; j < 8; ++j) slab[(8 * c + j) * kDwCols + 288] = bsum[j];
  }
}

}  // namespace

bool cifar_c2_supported(int inC, int H, int W, int C, int KS, int stride, int pad, int act_relu, int pooled) {
  return inC == 32 && H == 16 && W == 16 && C == 64 && KS == 3 && stride == 1 && pad == 1 && act_relu && pooled;
}

void cifar_c2_forward(const CifarC2Params& p, hipStream_t s) {
  if (p.B <= 0) return;
  MCC_CHECK(p.x && p.w && p.bias && p.y && p.arg && p.ldw >= 288 && p.ldw % 8 == 0, "cifar_c2_forward: bad params");
  MCC_CHECK((int64_t)p.B * kImgIn < (1ll << 31), "cifar_c2_forward: batch exceeds 32-bit offsets");
  const int grid = std::min(p.B, 2 * 256);
  hipLaunchKernelGGL(cifar_c2_fwd_kernel, dim3(grid), dim3(256), 0, s, p);
}

void cifar_c2_dx(const CifarC2BwdParams& p, hipStream_t s) {
  if (p.B <= 0) return;
  MCC_CHECK(p.dy && p.arg && p.wd && p.dx && p.ldw >= 576 && p.ldw % 8 == 0, "cifar_c2_dx: bad params");
  MCC_CHECK((int64_t)p.B * kImgIn < (1ll << 31), "cifar_c2_dx: batch exceeds 32-bit offsets");
  hipLaunchKernelGGL(cifar_c2_dx_kernel, dim3(std::min(p.B, 256)), dim3(512), 0, s, p);
}

size_t cifar_c2_dw_scratch_bytes() {
  const size_t nv = 64 * kDwCols;
  return (kDwGrid + (kDwGrid + 63) / 64) * nv * 4;  // slabs, then dw_slab_reduce's chunk partials
}

void cifar_c2_dw(const CifarC2BwdParams& p, float* gw, float* gb, hipStream_t s) {
  if (p.B <= 0) return;
  MCC_CHECK(p.dy && p.arg && p.x && p.slab && gw && gb, "cifar_c2_dw: bad params");
  MCC_CHECK((int64_t)p.B * kImgIn < (1ll << 31), "cifar_c2_dw: batch exceeds 32-bit offsets");
  const int grid = std::min(p.B, kDwGrid);
  hipLaunchKernelGGL(cifar_c2_dw_kernel, dim3(grid), dim3(512), 0, s, p);
  dw_slab_reduce(p.slab, grid, 64, kDwCols, p.slab + (size_t)kDwGrid * 64 * kDwCols, 64, 32, 3, XL_C8, 32, 288, gw, gb,
                 s);
}

}  // namespace gpu
}  // namespace mcc
