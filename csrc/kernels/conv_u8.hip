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

  const int64_t nunits = (int64_t)p.N * PH;
  const int64_t wave_id = (int64_t)blockIdx.x * (kU8T / 64) + wave, nwaves = (int64_t)gridDim.x * (kU8T / 64);

  // register prefetch of a unit's 4 rows: dword i of the 4 rows = lane + 64 * q
  uint32_t pre[RD];
  auto fetch = [&](int64_t u) {
    const int b = (int)(u / PH), wy = (int)(u - (int64_t)b * PH);
    const int img = p.idx ? p.idx[b] : b;
    const uint8_t* src = p.x + (size_t)img * p.H * p.W * 3;
#pragma unroll
    for (int q = 0; q < RD; ++q) {
      const int i = lane + 64 * q;
      const int rr = i / RDW, dw = i - rr * RDW;
      const int y = 2 * wy - 1 + rr;
      const bool ok = i < 4 * RDW && (unsigned)y < (unsigned)p.H;
      pre[q] = ok ? *reinterpret_cast<const uint32_t*>(src + (size_t)y * p.W * 3 + 4 * dw) : 0u;
    }
  };
  auto stash = [&]() {
#pragma unroll
    for (int q = 0; q < RD; ++q) {
      const int i = lane + 64 * q;
      const int rr = i / RDW, dw = i - rr * RDW;
      if (i < 4 * RDW) *reinterpret_cast<uint32_t*>(rows + rr * RP + 4 + 4 * dw) = pre[q];
    }
  };

  int64_t u = wave_id;
  if (u < nunits) fetch(u);
  for (; u < nunits; u += nwaves) {
    stash();  // (wave-private region: the wave's own earlier reads are ordered before these writes)
    const int b = (int)(u / PH), wy = (int)(u - (int64_t)b * PH);
    if (u + nwaves < nunits) fetch(u + nwaves);
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
      bf16x8 a0, a1;
      a0[0] = (bf16)(float)(lo & 0xffu);
      a0[1] = (bf16)(float)((lo >> 8) & 0xffu);
      a0[2] = (bf16)(float)((lo >> 16) & 0xffu);
      a0[3] = (bf16)(float)(lo >> 24);
      a0[4] = (bf16)(float)(hi & 0xffu);
      a0[5] = (bf16)(float)((hi >> 8) & 0xffu);
      a0[6] = (bf16)(float)((hi >> 16) & 0xffu);
      a0[7] = (bf16)(float)(hi >> 24);
      a1 = bf16x8{(bf16)(float)b8, (bf16)0.f, (bf16)0.f, (bf16)0.f, (bf16)0.f, (bf16)0.f, (bf16)0.f, (bf16)0.f};
      const int wx = 4 * t + g;  // the window this lane's accumulators hold
      const size_t o = (((size_t)b * PH + wy) * PW + wx) * p.Cout + r;
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
        const float y = fmaxf(best * (1.0f / 255.0f) + bias[j], 0.f);
        reinterpret_cast<bf16*>(p.out)[o + 16 * j] = (bf16)y;
        p.out_arg[o + 16 * j] = (uint8_t)(y > 0.f ? a : 4);
      }
    }
  }
}

}  // namespace

bool u8conv_fwd_supported(const U8ConvParams& p) {
  return p.N >= 1 && p.H % 2 == 0 && p.W % 8 == 0 && (p.Cout == 32 || p.Cout == 64) &&
         (3 * p.W) % 4 == 0 && 4 * u8_row_dwords(p.W) <= 64 * 12 && (int64_t)p.N * p.H * p.W * 3 < (1ll << 40);
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
