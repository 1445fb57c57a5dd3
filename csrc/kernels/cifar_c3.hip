// CIFAR-3conv conv3 on gfx950: conv 64 -> 128 channels, 3x3, pad 1, on 8x8
// images, ReLU + 2x2 max-pool; forward, data gradient and weight gradient.
// Reference semantics: Layer_feedForw_conv / Layer_feedBack_conv
// (/root/reference/cnn.c:175-247, with the correct OIHW indexing of
// CUDAcnn.cu:167-195); the pool is a BASELINE.json addition.
//
// On the implicit GEMM this layer ran at 27-28 % MFMA busy (profiles/
// cifar3_pmc_r6.txt: forward 910 us, data gradient 950 us, weight gradient
// 1,012 us, plus a 314 us grad_xform pass unpooling dY for them, at
// B = 65,024).  Per image every pass is a 64 x 128 x 576 GEMM (4.7 M MACs);
// the kernels here follow the conv2 ones (cifar_c2.hip): one image at a time
// per persistent workgroup, its zero-padded operand images staged in LDS
// (double-buffered, register prefetch of the next image, one barrier per
// image), layouts chosen with the bank model (tools/lds_banks.py: every read
// and staging store conflict-free), and the unpooled dZ rebuilt in LDS from
// the pooled dY and the forward's argmax codes (no grad_xform pass):
//
//  * forward: rows = (pool window, position), so a lane's four accumulators
//    are one window of one channel (in-lane max-pool + first-max argmax, then
//    bias + ReLU); each wave holds the B fragments of its 32 output channels
//    for all 18 K steps in registers (144 VGPRs) and reads only the A operand
//    from LDS (4 ds_read_b128 per 8 MFMAs).  The input image is four planes
//    of 16 channels, [10 rows x 12 px][32 B]: the 12-pixel row pitch puts the
//    two pixel rows of a window row 4 slots apart, so the 16 lanes of a
//    ds_read_b128 group read 16 distinct 16-byte bank slots at every tap.
//  * data gradient: the swapped GEMM dX^T [64 ci][64 px] = Wd x dZ-patches
//    with K = 9 taps x 128 = 1,152: a wave's 32 input channels need 288 VGPRs
//    of flipped weights, so the kernel runs one wave per SIMD (two 2-wave
//    workgroups per CU) and keeps all of them in registers; dZ in eight
//    16-channel planes of the same [10 x 12 px] geometry; a B-fragment lane
//    reads pixel (row 2 pt + (r >> 3), column (r & 7) ^ 4 (r >> 3)) so each
//    ds_read_b128 group spans 8 distinct 32-byte slots per half.
//  * weight gradient: dZ^T [128 co][64 px] (K in window-position order, the
//    16-byte chunk q of row co at q ^ ((co >> 1) & 7)) and X in four
//    16-channel planes of [10 x 10 px][32 B] read by ds_read_b64_tr_b16
//    (a half-wave's 8 rows are two 2 x 2 pixel blocks 4 pixels apart: 8
//    distinct slots); wave (co half, ci quarter) owns 4 x 9 accumulator
//    tiles for the whole launch, then one slab row per workgroup and
//    dw_slab_reduce; the bias gradient is summed by the dZ staging threads.
#include "kernels.h"
#include "mfma.h"

#include <algorithm>

namespace mcc {
namespace gpu {
namespace {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));


// [10 x 12 px][32 B] planes (forward X, data-gradient dZ); stride 32 mod 128 B
// so the 8 lanes of a ds_write_b128 group (8 chunks of one pixel) hit 8
// distinct bank groups
constexpr int kPit = 12;
constexpr int kPS = 10 * kPit * 32 + 32;  // 3,872 B
__device__ __forceinline__ int poff(int Y, int X) { return (Y * kPit + X) * 32; }

// d[k] (channels 2k, 2k+1) kept where the channel's argmax byte equals pos
__device__ __forceinline__ u32x4 unpool_pos3(const u32x4& d, uint32_t a0, uint32_t a1, uint32_t pos) {
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

// ------------------------------------------------------------------ forward
constexpr int kFBuf = 4 * kPS;  // 15,488 B

// tile t of the batch -> (image, tile row, tile column); TY x TX tiles per image
struct Tile3 {
  int img, ty, tx;
};
__device__ __forceinline__ Tile3 tile_of(int t, int TY, int TX) {
  Tile3 r;
  r.img = t / (TY * TX);
  const int q = t - r.img * TY * TX;
  r.ty = q / TX;
  r.tx = q - r.ty * TX;
  return r;
}

// TILED = false: one 8 x 8 tile per image (CIFAR-3conv): the halo is the zero
// padding, written once by the initial fill; only the 64 interior pixels are staged
template <bool TILED>
__global__ void __launch_bounds__(256, 2) cifar_c3_fwd_kernel(CifarC3Params p) {
  __shared__ __attribute__((aligned(16))) char smem[2 * kFBuf];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);  // output channels 32 wv .. 32 wv + 31
  const int r16 = lane & 15, g = lane >> 4;
  const int grid = (int)gridDim.x;
  const int H = p.H, W = p.W, TY = H >> 3, TX = W >> 3, PH = H >> 1, PW = W >> 1;
  const int ntiles = p.B * TY * TX;

  for (int i = tid * 16; i < 2 * kFBuf; i += 256 * 16) *reinterpret_cast<u32x4*>(smem + i) = u32x4{0u, 0u, 0u, 0u};

  // B fragments: channel 32 wv + 16 nt + r16, k = 32 ks + 8 g (tap ks >> 1, input channels 32 (ks & 1) + 8 g ..)
  const bf16* w = static_cast<const bf16*>(p.w);
  bf16x8 wb[2][18];
#pragma unroll
  for (int nt = 0; nt < 2; ++nt)
#pragma unroll
    for (int ks = 0; ks < 18; ++ks) wb[nt][ks] = load8(w + (size_t)(32 * wv + 16 * nt + r16) * p.ldw + 32 * ks + 8 * g);
  const float bv0 = p.bias[32 * wv + r16], bv1 = p.bias[32 * wv + 16 + r16];

  // A fragments: row tile T = window row T of the 8 x 8 output tile; lane row
  // r16 = window slot r16 >> 2 (window column), position r16 & 3 = (dy, dx);
  // chunk g of the K step's 32 channels -> plane 2 (ks & 1) + (g >> 1), half g & 1
  const int la = (g >> 1) * kPS + poff((r16 >> 1) & 1, 2 * (r16 >> 2) + (r16 & 1)) + 16 * (g & 1);

  // staging: the tile's 10 x 10 input halo (zero outside the image) as 800
  // 16-byte items j = tid + 256 i: halo pixel j >> 3, channel chunk j & 7
  constexpr int NS = TILED ? 4 : 2;
  int soff[NS], goff[NS], shy[NS], shx[NS];
#pragma unroll
  for (int i = 0; i < NS; ++i) {
    const int j = tid + 256 * i, c = j & 7;
    const int px = j >> 3, hy = TILED ? px / 10 : (px >> 3) + 1, hx = TILED ? px % 10 : (px & 7) + 1;
    shy[i] = !TILED || j < 800 ? hy : -100;  // (-100: no item)
    shx[i] = hx;
    soff[i] = (c >> 1) * kPS + poff(hy, hx) + 16 * (c & 1);
    goff[i] = (hy * W + hx) * 64 + 8 * c;
  }
  const bf16* xg = static_cast<const bf16*>(p.x);
  u32x4 st[NS];
  auto load = [&](int t) {
    const Tile3 q = tile_of(t, TY, TX);
    const int y0 = q.ty * 8 - 1, x0 = q.tx * 8 - 1;
    const bf16* base = xg + ((size_t)q.img * H * W + (int64_t)y0 * W + x0) * 64;
#pragma unroll
    for (int i = 0; i < NS; ++i) {
      const int y = y0 + shy[i], x = x0 + shx[i];
      const bool in = !TILED || (shy[i] >= 0 && y >= 0 && y < H && x >= 0 && x < W);
      st[i] = in ? *reinterpret_cast<const u32x4*>(base + goff[i]) : u32x4{0u, 0u, 0u, 0u};
    }
  };
  __syncthreads();  // zero fill before the first write
  int t = blockIdx.x;
  if (t < ntiles) load(t);
  for (int k = 0; t < ntiles; t += grid, ++k) {
    char* tb = smem + (k & 1) * kFBuf;
#pragma unroll
    for (int i = 0; i < NS; ++i)
      if (shy[i] >= 0) *reinterpret_cast<u32x4*>(tb + soff[i]) = st[i];
    __syncthreads();  // tile k staged; every wave is past tile k - 1's reads of this buffer (k - 2)
    const Tile3 q = tile_of(t, TY, TX);
    if (t + grid < ntiles) load(t + grid);

    f32x4 acc[4][2];
#pragma unroll
    for (int r = 0; r < 4; ++r) acc[r][0] = acc[r][1] = f32x4{0.f, 0.f, 0.f, 0.f};
    const char* rb = tb + la;
    auto read_a = [&](int ks, bf16x8 (&a)[4]) {
      const int tap = ks >> 1, off = (ks & 1) * 2 * kPS + poff(tap / 3, tap % 3);
#pragma unroll
      for (int r = 0; r < 4; ++r) a[r] = *reinterpret_cast<const bf16x8*>(rb + off + poff(2 * r, 0));
    };
    bf16x8 a[2][4];
    read_a(0, a[0]);
#pragma unroll
    for (int ks = 0; ks < 18; ++ks) {
      if (ks + 1 < 18) read_a(ks + 1, a[(ks + 1) & 1]);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        acc[r][0] = mma(acc[r][0], a[ks & 1][r], wb[0][ks]);
        acc[r][1] = mma(acc[r][1], a[ks & 1][r], wb[1][ks]);
      }
      __builtin_amdgcn_sched_barrier(0);
    }

    // pool + bias + ReLU: lane (channel r16 of tile nt, window g of window row r)
    const size_t obase = ((size_t)q.img * PH + q.ty * 4) * PW + q.tx * 4;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const size_t o0 = (obase + (size_t)r * PW + g) * 128;
#pragma unroll
      for (int nt = 0; nt < 2; ++nt) {
        const f32x4 v = acc[r][nt];
        float best = v[0];
        int arg = 0;
#pragma unroll
        for (int i = 1; i < 4; ++i) {  // first max wins: TL, TR, BL, BR
          const bool gt = v[i] > best;
          best = gt ? v[i] : best;
          arg = gt ? i : arg;
        }
        const bf16 yb = (bf16)fmaxf(best + (nt ? bv1 : bv0), 0.f);
        const size_t o = o0 + 32 * wv + 16 * nt + r16;
        static_cast<bf16*>(p.y)[o] = yb;
        p.arg[o] = (uint8_t)((float)yb > 0.f ? arg : 4);  // 4: ReLU-inactive window
      }
    }
  }
}

// ------------------------------------------------------------ data gradient
constexpr int kXBuf = 8 * kPS;  // 30,976 B: dZ, eight 16-channel planes

template <bool TILED>
__global__ void __launch_bounds__(128) __attribute__((amdgpu_waves_per_eu(1, 1)))
cifar_c3_dx_kernel(CifarC3BwdParams p) {
  __shared__ __attribute__((aligned(16))) char smem[2 * kXBuf];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);  // input channels 32 wv .. 32 wv + 31
  const int r16 = lane & 15, g = lane >> 4;
  const int grid = (int)gridDim.x;
  const int H = p.H, W = p.W, TY = H >> 3, TX = W >> 3, PH = H >> 1, PW = W >> 1;
  const int ntiles = p.B * TY * TX;

  for (int i = tid * 16; i < 2 * kXBuf; i += 128 * 16) *reinterpret_cast<u32x4*>(smem + i) = u32x4{0u, 0u, 0u, 0u};

  // A fragments: input channel 32 wv + 16 ct + r16, k = 32 ks + 8 g (tap ks >> 2,
  // output channels 32 (ks & 3) + 8 g ..)
  const bf16* wd = static_cast<const bf16*>(p.wd);
  bf16x8 wa[2][36];
#pragma unroll
  for (int ct = 0; ct < 2; ++ct)
#pragma unroll
    for (int ks = 0; ks < 36; ++ks) wa[ct][ks] = load8(wd + (size_t)(32 * wv + 16 * ct + r16) * p.ldw + 32 * ks + 8 * g);

  // B fragments: pixel tile pt = tile rows 2 pt, 2 pt + 1; lane column r16 ->
  // pixel (2 pt + (r16 >> 3), (r16 & 7) ^ 4 (r16 >> 3)), chunk 4 (ks & 3) + g
  const int py = r16 >> 3, px = (r16 & 7) ^ (4 * py);
  const int lb = (g >> 1) * kPS + poff(py, px) + 16 * (g & 1);

  // staging: the 10 x 10 dZ halo of the tile = the positions of 6 x 6 pooled
  // windows (tile windows -1 .. 4); item (window a, b; channel chunk c) for
  // j = tid + 128 i < 576, its in-halo positions as a 4-bit mask
  const char* dyg = static_cast<const char*>(p.dy);
  // (TILED = false: the tile's 16 windows only, all four positions; the halo
  // ring is the zero padding of the initial fill)
  constexpr int NS = TILED ? 5 : 2;
  int sbase[NS], sgoff[NS], swa[NS], swb[NS];
  uint32_t smask[NS];
#pragma unroll
  for (int i = 0; i < NS; ++i) {
    const int j = tid + 128 * i, wi = j >> 4, c = j & 15;
    const int wa_ = TILED ? wi / 6 : (wi >> 2) + 1, wb_ = TILED ? wi % 6 : (wi & 3) + 1;
    uint32_t m = 0;
#pragma unroll
    for (int pos = 0; pos < 4; ++pos) {
      const int hy = 2 * wa_ + (pos >> 1) - 1, hx = 2 * wb_ + (pos & 1) - 1;
      if ((!TILED || j < 576) && hy >= 0 && hy < 10 && hx >= 0 && hx < 10) m |= 1u << pos;
    }
    smask[i] = m;
    swa[i] = wa_;
    swb[i] = wb_;
    sbase[i] = (c >> 1) * kPS + (((2 * wa_ - 1) * kPit) + 2 * wb_ - 1) * 32 + 16 * (c & 1);  // (may be < 0: masked)
    sgoff[i] = ((wa_ - 1) * PW + (wb_ - 1)) * 128 + 8 * c;
  }
  u32x4 sd[NS];
  uint32_t sa[NS][2];
  auto load = [&](int t) {
    const Tile3 q = tile_of(t, TY, TX);
    const int wy0 = q.ty * 4, wx0 = q.tx * 4;
    const size_t base = ((size_t)q.img * PH + wy0) * PW + wx0;  // pooled pixel of tile window (0, 0)
#pragma unroll
    for (int i = 0; i < NS; ++i) {
      const int wy = wy0 + swa[i] - 1, wx = wx0 + swb[i] - 1;
      const bool in = !TILED || (smask[i] && wy >= 0 && wy < PH && wx >= 0 && wx < PW);
      const int64_t e = (int64_t)base * 128 + sgoff[i];
      sd[i] = in ? *reinterpret_cast<const u32x4*>(dyg + 2 * e) : u32x4{0u, 0u, 0u, 0u};
      uint2 av = {0u, 0u};
      if (in) av = *reinterpret_cast<const uint2*>(p.arg + e);
      sa[i][0] = av.x; sa[i][1] = av.y;
    }
  };
  bf16* dxo = static_cast<bf16*>(p.dx);
  __syncthreads();  // zero fill before the first write
  int t = blockIdx.x;
  if (t < ntiles) load(t);
  for (int k = 0; t < ntiles; t += grid, ++k) {
    char* tb = smem + (k & 1) * kXBuf;
#pragma unroll
    for (int i = 0; i < NS; ++i)
#pragma unroll
      for (int pos = 0; pos < 4; ++pos)
        if (!TILED || (smask[i] & (1u << pos)))
          *reinterpret_cast<u32x4*>(tb + sbase[i] + poff(pos >> 1, pos & 1)) = unpool_pos3(sd[i], sa[i][0], sa[i][1], pos);
    __syncthreads();  // tile k staged; buffer k & 1's previous readers (tile k - 2) are done
    const Tile3 q = tile_of(t, TY, TX);
    if (t + grid < ntiles) load(t + grid);

    f32x4 acc[2][4];
#pragma unroll
    for (int ct = 0; ct < 2; ++ct)
#pragma unroll
      for (int pt = 0; pt < 4; ++pt) acc[ct][pt] = f32x4{0.f, 0.f, 0.f, 0.f};
    const char* rb = tb + lb;
    auto read_b = [&](int ks, bf16x8 (&b)[4]) {
      const int tap = ks >> 2, off = (ks & 3) * 2 * kPS + poff(tap / 3, tap % 3);
#pragma unroll
      for (int pt = 0; pt < 4; ++pt) b[pt] = *reinterpret_cast<const bf16x8*>(rb + off + poff(2 * pt, 0));
    };
    bf16x8 b[2][4];
    read_b(0, b[0]);
#pragma unroll
    for (int ks = 0; ks < 36; ++ks) {
      if (ks + 1 < 36) read_b(ks + 1, b[(ks + 1) & 1]);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int ct = 0; ct < 2; ++ct)
#pragma unroll
        for (int pt = 0; pt < 4; ++pt) acc[ct][pt] = mma(acc[ct][pt], wa[ct][ks], b[ks & 1][pt]);
      __builtin_amdgcn_sched_barrier(0);
    }

    // lane: channels 32 wv + 16 ct + 4 g .. + 3 of its pixel in tile row pair pt
    const size_t obase = ((size_t)q.img * H + q.ty * 8) * W + q.tx * 8;
#pragma unroll
    for (int pt = 0; pt < 4; ++pt)
#pragma unroll
      for (int ct = 0; ct < 2; ++ct) {
        const f32x4 v = acc[ct][pt];
        *reinterpret_cast<bf16x4*>(dxo + (obase + (size_t)(2 * pt + py) * W + px) * 64 + 32 * wv + 16 * ct + 4 * g) =
            cvt4(v[0], v[1], v[2], v[3]);
      }
  }
}

// ----------------------------------------------------------- weight gradient
constexpr int kWXPS = 10 * 10 * 32 + 32;         // 3,232 B: X plane [10 x 10 px][32 B], 32 mod 128
constexpr int kWZT = 128 * 128;                  // 16,384 B: dZ^T [128 co][64 k]
constexpr int kWBuf = kWZT + 4 * kWXPS;          // 29,312 B
constexpr int kDw3Cols = 592;                    // slab columns: 576 weights (tap * 64 + ci), bias at 576
constexpr int kDw3Grid = 256;

__device__ __forceinline__ int zt3(int co, int k) { return co * 128 + 16 * ((k >> 3) ^ ((co >> 1) & 7)) + 2 * (k & 7); }

template <bool TILED>
__global__ void __launch_bounds__(512, 1) cifar_c3_dw_kernel(CifarC3BwdParams p) {
  __shared__ __attribute__((aligned(16))) char smem[2 * kWBuf];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wc = wv & 1, wn = wv >> 1;  // output channels 64 wc .., input channels 16 wn .. (all 9 taps)
  const int r16 = lane & 15, g = lane >> 4;
  const int grid = (int)gridDim.x;
  const int H = p.H, W = p.W, TY = H >> 3, TX = W >> 3, PH = H >> 1, PW = W >> 1;
  const int ntiles = p.B * TY * TX;

  for (int i = tid * 16; i < 2 * kWBuf; i += 512 * 16) *reinterpret_cast<u32x4*>(smem + i) = u32x4{0u, 0u, 0u, 0u};

  // A fragments (dZ^T rows 64 wc + 16 ct + r16, k = 32 ks + 8 g)
  int za[2][4];
#pragma unroll
  for (int ks = 0; ks < 2; ++ks)
#pragma unroll
    for (int ct = 0; ct < 4; ++ct) za[ks][ct] = zt3(64 * wc + 16 * ct + r16, 32 * ks + 8 * g);
  // B fragments: lane 4 q + p of group g supplies window 8 ks + 2 g + s (window
  // row 2 ks + (g >> 1), column 2 (g & 1) + s), position q, channels 4 p .. of plane wn
  const int q4 = r16 >> 2, p4 = r16 & 3;
  const int xb = kWZT + wn * kWXPS + ((2 * (g >> 1) + (q4 >> 1)) * 10 + 4 * (g & 1) + (q4 & 1)) * 32 + 8 * p4;

  // staging: threads 0..255 rebuild dZ^T from the tile's 4 x 4 pooled windows
  // (window w, chunk c: 8 channels x 4 positions) and sum the bias; threads
  // 256..511 stage the 10 x 10 X halo (zero outside the image), 800 items
  const bool zthr = tid < 256;
  const int w = tid & 15, c = (tid >> 4) & 15;
  int zo[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) zo[j] = zt3(8 * c + j, 4 * w);
  constexpr int NX = TILED ? 4 : 2;  // (TILED = false: the 64 interior pixels; the halo is the zero fill)
  int xo[NX], xgo[NX], xhy[NX], xhx[NX];
#pragma unroll
  for (int i = 0; i < NX; ++i) {
    const int j = (tid & 255) + 256 * i, px = j >> 3, cc = j & 7;
    const int hy = TILED ? px / 10 : (px >> 3) + 1, hx = TILED ? px % 10 : (px & 7) + 1;
    xhy[i] = !TILED || j < 800 ? hy : -100;
    xhx[i] = hx;
    xo[i] = kWZT + (cc >> 1) * kWXPS + (hy * 10 + hx) * 32 + 16 * (cc & 1);
    xgo[i] = (hy * W + hx) * 64 + 8 * cc;
  }
  const char* dyg = static_cast<const char*>(p.dy);
  const bf16* xg = static_cast<const bf16*>(p.x);
  u32x4 sv[NX];
  uint32_t sa0 = 0u, sa1 = 0u;
  auto load = [&](int t) {
    const Tile3 q = tile_of(t, TY, TX);
    if (zthr) {
      const size_t e = (((size_t)q.img * PH + q.ty * 4 + (w >> 2)) * PW + q.tx * 4 + (w & 3)) * 128 + 8 * c;
      sv[0] = *reinterpret_cast<const u32x4*>(dyg + 2 * e);
      const uint2 a = *reinterpret_cast<const uint2*>(p.arg + e);
      sa0 = a.x; sa1 = a.y;
    } else {
      const int y0 = q.ty * 8 - 1, x0 = q.tx * 8 - 1;
      const bf16* base = xg + ((size_t)q.img * H * W + (int64_t)y0 * W + x0) * 64;
#pragma unroll
      for (int i = 0; i < NX; ++i) {
        const int y = y0 + xhy[i], x = x0 + xhx[i];
        const bool in = !TILED || (xhy[i] >= 0 && y >= 0 && y < H && x >= 0 && x < W);
        sv[i] = in ? *reinterpret_cast<const u32x4*>(base + xgo[i]) : u32x4{0u, 0u, 0u, 0u};
      }
    }
  };
  float bsum[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) bsum[j] = 0.f;

  f32x4 acc[4][9];
#pragma unroll
  for (int ct = 0; ct < 4; ++ct)
#pragma unroll
    for (int t = 0; t < 9; ++t) acc[ct][t] = f32x4{0.f, 0.f, 0.f, 0.f};

  __syncthreads();  // zero fill before the first write
  int t = blockIdx.x;
  if (t < ntiles) load(t);
  for (int k = 0; t < ntiles; t += grid, ++k) {
    char* tb = smem + (k & 1) * kWBuf;
    if (zthr) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const uint32_t v = (sv[0][j >> 1] >> (16 * (j & 1))) & 0xffffu;
        const uint32_t a = ((j < 4 ? sa0 : sa1) >> (8 * (j & 3))) & 0xffu;
        uint2 o;
        o.x = a == 0 ? v : (a == 1 ? v << 16 : 0u);
        o.y = a == 2 ? v : (a == 3 ? v << 16 : 0u);
        *reinterpret_cast<uint2*>(tb + zo[j]) = o;
        bsum[j] += a < 4 ? __uint_as_float(v << 16) : 0.f;
      }
    } else {
#pragma unroll
      for (int i = 0; i < NX; ++i)
        if (xhy[i] >= 0) *reinterpret_cast<u32x4*>(tb + xo[i]) = sv[i];
    }
    __syncthreads();  // tile k staged; buffer k & 1's previous readers (tile k - 2) are done
    if (t + grid < ntiles) load(t + grid);

#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16x8 a[4];
#pragma unroll
      for (int ct = 0; ct < 4; ++ct) a[ct] = *reinterpret_cast<const bf16x8*>(tb + za[ks][ct]);
      const bf16* xr = reinterpret_cast<const bf16*>(tb + xb);
#pragma unroll
      for (int tp = 0; tp < 9; ++tp) {
        const int off = ((4 * ks + tp / 3) * 10 + tp % 3) * 16;  // bf16 elements (32 B per pixel)
        const bf16x4 lo = tr4(xr + off), hi = tr4(xr + off + 2 * 16);  // s = 0, 1: +2 px
        const bf16x8 bfr = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
#pragma unroll
        for (int ct = 0; ct < 4; ++ct) acc[ct][tp] = mma(acc[ct][tp], a[ct], bfr);
      }
    }
  }

  float* slab = p.slab + (size_t)blockIdx.x * 128 * kDw3Cols;
#pragma unroll
  for (int ct = 0; ct < 4; ++ct)
#pragma unroll
    for (int tp = 0; tp < 9; ++tp)
#pragma unroll
      for (int i = 0; i < 4; ++i)
        slab[(64 * wc + 16 * ct + 4 * g + i) * kDw3Cols + 64 * tp + 16 * wn + r16] = acc[ct][tp][i];
  // bias: the 16 lanes (windows) of a 16-lane group share channel chunk c
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    float v = bsum[j];
#pragma unroll
    for (int m = 8; m >= 1; m >>= 1) v += __shfl_xor(v, m, 16);
    bsum[j] = v;
  }
  if (zthr && w == 0) {
#pragma unroll
    for (int j = 0; j < 8; ++j) slab[(8 * c + j) * kDw3Cols + 576] = bsum[j];
  }
}

}  // namespace

bool cifar_c3_supported(int inC, int H, int W, int C, int KS, int stride, int pad, int act_relu, int pooled) {
  return inC == 64 && H % 8 == 0 && W % 8 == 0 && H > 0 && W > 0 && C == 128 && KS == 3 && stride == 1 && pad == 1 &&
         act_relu && pooled;
}
static int c3_tiles(int B, int H, int W) {
  MCC_CHECK(H > 0 && W > 0 && H % 8 == 0 && W % 8 == 0, "cifar_c3: H, W must be multiples of 8");
  MCC_CHECK((int64_t)B * H * W * 128 < (1ll << 40) && (int64_t)B * (H / 8) * (W / 8) < (1ll << 31),
            "cifar_c3: batch too large");
  return B * (H / 8) * (W / 8);
}

void cifar_c3_forward(const CifarC3Params& p, hipStream_t s) {
  if (p.B <= 0) return;
  MCC_CHECK(p.x && p.w && p.bias && p.y && p.arg && p.ldw >= 576 && p.ldw % 8 == 0, "cifar_c3_forward: bad params");
  const int nt = c3_tiles(p.B, p.H, p.W);
  if (p.H == 8 && p.W == 8) hipLaunchKernelGGL(cifar_c3_fwd_kernel<false>, dim3(std::min(nt, 2 * 256)), dim3(256), 0, s, p);
  else hipLaunchKernelGGL(cifar_c3_fwd_kernel<true>, dim3(std::min(nt, 2 * 256)), dim3(256), 0, s, p);
}

void cifar_c3_dx(const CifarC3BwdParams& p, hipStream_t s) {
  if (p.B <= 0) return;
  MCC_CHECK(p.dy && p.arg && p.wd && p.dx && p.ldw >= 1152 && p.ldw % 8 == 0, "cifar_c3_dx: bad params");
  const int nt = c3_tiles(p.B, p.H, p.W);
  if (p.H == 8 && p.W == 8) hipLaunchKernelGGL(cifar_c3_dx_kernel<false>, dim3(std::min(nt, 2 * 256)), dim3(128), 0, s, p);
  else hipLaunchKernelGGL(cifar_c3_dx_kernel<true>, dim3(std::min(nt, 2 * 256)), dim3(128), 0, s, p);
}

size_t cifar_c3_dw_scratch_bytes() {
  const size_t nv = 128 * kDw3Cols;
  return (kDw3Grid + (kDw3Grid + 63) / 64) * nv * 4;  // slabs, then dw_slab_reduce's chunk partials
}

void cifar_c3_dw(const CifarC3BwdParams& p, float* gw, float* gb, hipStream_t s) {
  if (p.B <= 0) return;
  MCC_CHECK(p.dy && p.arg && p.x && p.slab && gw && gb, "cifar_c3_dw: bad params");
  const int grid = std::min(c3_tiles(p.B, p.H, p.W), kDw3Grid);
  if (p.H == 8 && p.W == 8) hipLaunchKernelGGL(cifar_c3_dw_kernel<false>, dim3(grid), dim3(512), 0, s, p);
  else hipLaunchKernelGGL(cifar_c3_dw_kernel<true>, dim3(grid), dim3(512), 0, s, p);
  dw_slab_reduce(p.slab, grid, 128, kDw3Cols, p.slab + (size_t)kDw3Grid * 128 * kDw3Cols, 128, 64, 3, XL_C8, 64, 576,
                 gw, gb, s);
}

}  // namespace gpu
}  // namespace mcc
