// Forward of the u8 first conv layer of the RGB models (C = 3, 3x3, stride 1,
// pad 1, bias + ReLU + 2x2/2 max-pool fused): CIFAR-3conv conv1 (32x32 -> 32
// channels) and VGG-11 conv1 (224x224 -> 64 channels), bf16 MFMA.
//
// Reference math: Layer_feedForw_conv (cnn.c:175-210), OIHW weights as
// CUDAcnn.cu:167-195; the input is pixel/255 (cnn.c:457).
//
// The layer's GEMM is tiny (K = 27) and its cost is building the A operand,
// so the kernel is organised around that:
//   * work unit = (image, pooled output row): one wave stages the 4 input rows
//     it needs (u8, 3W bytes each, zero rows above/below the image, a zero
//     pixel either side) into its own LDS region with dword loads, the next
//     unit's rows already in flight in registers (no workgroup barriers);
//   * MFMA rows = 4 pooling windows x their 4 positions, so every lane holds a
//     whole 2x2 window of one channel: max-pool + argmax are in-lane;
//   * K is laid out per kernel row: lane group g (< 3) takes the 9-byte run
//     (3 pixels x 3 channels) of input row y-1+g -- bytes 0..7 in the first
//     16x16x32 MFMA, byte 8 in the second (whose other K slots have zero
//     weights; group 3 repeats row +2 against zero weights).  A run is one
//     ds_read_b96 plus two v_alignbyte, and the bytes convert to bf16 exactly
//     (integers < 256); 1/255 is applied to the fp32 sums;
//   * the weight fragments are built once per workgroup from the canonical
//     fp32 weights (bf16 RNE, as the packed copies) and stay in registers.
#include "kernels.h"
#include "mfma.h"

#include <algorithm>

namespace mcc {
namespace gpu {

namespace {

constexpr int kU8T = 256;  // 4 waves, each an independent row worker

typedef unsigned int u32x3 __attribute__((ext_vector_type(3)));

__host__ __device__ inline int u8_row_pitch(int W) { return (3 * W + 12 + 15) & ~15; }
// dwords of the 4 staged rows per lane (register prefetch)
__host__ __device__ inline int u8_row_dwords(int W) { return 3 * W / 4; }

template <int NT, int RD>  // NT: 16-channel output tiles; RD: staged dwords per lane (ceil(4 rows / 64 lanes))
__global__ void __launch_bounds__(kU8T) u8conv_fwd_kernel(U8ConvParams p) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r = lane & 15, g = lane >> 4;
  const int RP = u8_row_pitch(p.W), RDW = u8_row_dwords(p.W);
  uint8_t* rows = lds + wave * 4 * RP;
  for (int i = lane; i < RP; i += 64) *reinterpret_cast<uint32_t*>(rows + 4 * i) = 0u;  // 4 rows x RP bytes
  const int PH = p.H / 2, PW = p.W / 2;

  // weight fragments: MFMA 0, K slot 8g+e: (ky = g, kx = e/3, c = e%3); MFMA 1: slot 8g (ky = g, kx = 2, c = 2)
  bf16x8 b0[NT], b1[NT];
#pragma unroll
  for (int j = 0; j < NT; ++j) {
    const int n = 16 * j + r;
    const float* wn = p.w + (size_t)n * 27;  // OIHW: [n][c][ky][kx]
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int kx = e / 3, c = e % 3;
      b0[j][e] = (bf16)(g < 3 ? wn[c * 9 + g * 3 + kx] : 0.f);
      b1[j][e] = (bf16)(g < 3 && e == 0 ? wn[2 * 9 + g * 3 + 2] : 0.f);
    }
  }
  float bias[NT];
#pragma unroll
  for (int j = 0; j < NT; ++j) bias[j] = p.bias[16 * j + r];

  // lane's MFMA row: window w = r/4 of a tile, position (dy, dx) = (r%4 / 2, r%2)
  const int wr = r >> 2, dy = (r >> 1) & 1, dx = r & 1;
  const int srow = dy + (g < 3 ? g : 2);  // staged row (0 = input row y0 - 1)
  const int ntiles = PW / 4;

  // units (image b, pooled row wy) advance by nwaves: (b, wy) carried, no
  // per-unit division (round 5: the 64-bit u / PH and the per-dword i / RDW
  // divisions were ~40 % of this kernel's VALU on CIFAR-3conv)
  const int nunits = p.N * PH;  // host: < 2^31
  const int wave_id = blockIdx.x * (kU8T / 64) + wave, nwaves = gridDim.x * (kU8T / 64);
  const int adv_b = nwaves / PH, adv_y = nwaves - adv_b * PH;

  // register prefetch of a unit's 4 rows: dword i of the 4 rows = lane + 64 * q;
  // per q: source offset within the first row's image position, LDS offset | staged row (2 bits)
  int qsrc[RD], qlds[RD];
#pragma unroll
  for (int q = 0; q < RD; ++q) {
    const int i = lane + 64 * q;
    const int rr = i / RDW, dw = i - rr * RDW;
    qsrc[q] = rr * p.W * 3 + 4 * dw;
    qlds[q] = i < 4 * RDW ? ((rr * RP + 4 + 4 * dw) | rr) : -1;
  }
  uint32_t pre[RD];
  auto fetch = [&](int b, int wy) {
    const int img = p.idx ? p.idx[b] : b;
    const uint8_t* src = p.x + (size_t)img * p.H * p.W * 3 + (ptrdiff_t)(2 * wy - 1) * p.W * 3;
#pragma unroll
    for (int q = 0; q < RD; ++q) {
      const int y = 2 * wy - 1 + (qlds[q] & 3);
      const bool ok = qlds[q] >= 0 && (unsigned)y < (unsigned)p.H;
      pre[q] = ok ? *reinterpret_cast<const uint32_t*>(src + qsrc[q]) : 0u;
    }
  };
  auto stash = [&]() {
#pragma unroll
    for (int q = 0; q < RD; ++q)
      if (qlds[q] >= 0) *reinterpret_cast<uint32_t*>(rows + (qlds[q] & ~3)) = pre[q];
  };

  int u = wave_id;
  int b = u / PH, wy = u - (u / PH) * PH;
  if (u < nunits) fetch(b, wy);
  for (; u < nunits; u += nwaves) {
    stash();  // (wave-private region: the wave's own earlier reads are ordered before these writes)
    const int bc = b, wyc = wy;
    wy += adv_y;
    b += adv_b;
    if (wy >= PH) { wy -= PH; ++b; }
    if (u + nwaves < nunits) fetch(b, wy);
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): the LDS writes landed (single wave: no barrier)
    __builtin_amdgcn_wave_barrier();
    for (int t = 0; t < ntiles; ++t) {
      const int x = 2 * (4 * t + wr) + dx;
      const int off = 1 + 3 * x;  // byte of pixel x-1 in the staged row (data starts at 4)
      const u32x3 d = *reinterpret_cast<const u32x3*>(rows + srow * RP + (off & ~3));
      const int sh = 8 * (off & 3);
      const uint32_t lo = __builtin_amdgcn_alignbyte(d.y, d.x, off & 3);
      const uint32_t hi = __builtin_amdgcn_alignbyte(d.z, d.y, off & 3);
      const uint32_t b8 = (uint32_t)(((uint64_t)d.z << 32 | d.y) >> (sh + 32)) & 0xffu;  // byte 8
      // bytes -> bf16: an integer < 256 is exact in fp32 with a zero low half,
      // so its bf16 is the float's high half (v_cvt_f32_ubyteN + one v_perm per pair)
      auto ip2 = [](uint32_t w, int k) {  // bytes k, k+1 of w
        const uint32_t f0 = __builtin_bit_cast(uint32_t, (float)((w >> (8 * k)) & 0xffu));
        const uint32_t f1 = __builtin_bit_cast(uint32_t, (float)((w >> (8 * k + 8)) & 0xffu));
        return __builtin_amdgcn_perm(f1, f0, 0x07060302u);
      };
      typedef uint32_t u32x4v __attribute__((ext_vector_type(4)));
      const bf16x8 a0 = __builtin_bit_cast(bf16x8, (u32x4v{ip2(lo, 0), ip2(lo, 2), ip2(hi, 0), ip2(hi, 2)}));
      const uint32_t f8 = __builtin_bit_cast(uint32_t, (float)b8) >> 16;
      const bf16x8 a1 = __builtin_bit_cast(bf16x8, (u32x4v{f8, 0u, 0u, 0u}));
      const int wx = 4 * t + g;  // the window this lane's accumulators hold
      const size_t o = (((size_t)bc * PH + wyc) * PW + wx) * p.Cout + r;
#pragma unroll
      for (int j = 0; j < NT; ++j) {
        f32x4 acc = {0.f, 0.f, 0.f, 0.f};
        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0, b0[j], acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1, b1[j], acc, 0, 0, 0);
        float best = acc[0];
        int a = 0;
        if (acc[1] > best) { best = acc[1]; a = 1; }
        if (acc[2] > best) { best = acc[2]; a = 2; }
        if (acc[3] > best) { best = acc[3]; a = 3; }
        // ReLU on the bit pattern (v_max_i32: no NaN canonicalisation)
        const float y = __builtin_bit_cast(float, max(__builtin_bit_cast(int, fmaf(best, 1.0f / 255.0f, bias[j])), 0));
        reinterpret_cast<bf16*>(p.out)[o + 16 * j] = (bf16)y;
        p.out_arg[o + 16 * j] = (uint8_t)(y > 0.f ? a : 4);
      }
    }
  }
}

}  // namespace

bool u8conv_fwd_supported(const U8ConvParams& p) {
  return p.N >= 1 && p.H % 2 == 0 && p.W % 8 == 0 && (p.Cout == 32 || p.Cout == 64) &&
         (3 * p.W) % 4 == 0 && 4 * u8_row_dwords(p.W) <= 64 * 12 && (int64_t)p.N * p.H * p.W * 3 < (1ll << 40) &&
         (int64_t)p.N * (p.H / 2) < (1ll << 31);
}

void u8conv_forward(const U8ConvParams& p, hipStream_t s) {
  MCC_CHECK(u8conv_fwd_supported(p) && p.x && p.w && p.bias && p.out && p.out_arg, "u8conv_forward: bad params");
  const int64_t nunits = (int64_t)p.N * (p.H / 2);
  // (8 workgroups per CU; 4 and 16 measured within 1.5% on CIFAR-3conv)
  const int grid = (int)std::max<int64_t>(1, std::min<int64_t>((nunits + 3) / 4, 256 * 8));
  const size_t lds = (size_t)4 * 4 * u8_row_pitch(p.W);
  const int rd = (4 * u8_row_dwords(p.W) + 63) / 64;
  const dim3 g((unsigned)grid), b(kU8T);
#define MCC_U8(NT, RD) hipLaunchKernelGGL((u8conv_fwd_kernel<NT, RD>), g, b, lds, s, p)
  if (p.Cout == 32) {
    if (rd <= 2) MCC_U8(2, 2);
    else MCC_U8(2, 12);
  } else {
    if (rd <= 2) MCC_U8(4, 2);
    else MCC_U8(4, 12);
  }
#undef MCC_U8
}

}  // namespace gpu
}  // namespace mcc
