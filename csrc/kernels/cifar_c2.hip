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

}  // namespace gpu
}  // namespace mcc
