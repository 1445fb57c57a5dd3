// Sparse fp32 weight gradients of LeNet-5's two pooled convs (BASELINE
// config 2, "LeNet-5 fp32 on one MI355X"):
//   conv1: 1 -> 6, 5x5, pad 2 (28x28), ReLU, 2x2 pool  (input: u8 images)
//   conv2: 6 -> 16, 5x5, valid (10x10), ReLU, 2x2 pool (input: Y1 NHWC fp32)
//
// Reference math: Layer_feedBack_conv (/root/reference/cnn.c:212-247, the D1
// index bug fixed as CUDAcnn.cu:167-195); the pool is a BASELINE.json
// addition.  A conv followed by a 2x2 max-pool receives gradient only at each
// window's argmax (the unpooled dZ is zero at the other three positions and at
// ReLU-inactive windows), so
//   dW[co][ci][kh][kw] = sum over images, windows w of
//                        dY[co][w] * X[ci][argmax(co, w) + (kh, kw)],
//   db[co]             = sum of dY[co][w] over active windows:
// a quarter of the MACs of the dense correlation over the unpooled grid,
// which conv_direct_dw / conv1_direct_dw_w3 (conv_direct.hip) evaluate with
// three zero gradients per window.  The argmax moves the patch per
// (channel, window), so the gather is not a GEMM: these run on the VALU
// (v_pk_fma_f32, the full fp32 rate -- gfx950's fp32 matrix rate is the same,
// and an MFMA form would have to do the dense 4x work).
//
//  * conv2 dW: a lane owns one output channel co (16 per wave row) and one
//    window slot; its 6 input channels x 25 taps of accumulators are 75
//    packed pairs.  Y1 is staged as 8-float pixels (channels 6, 7 zero), so a
//    tap is one ds_read_b128 + one ds_read_b64.  The 16 lanes of a row read
//    the same window: at most 4 distinct pixels (the argmax positions), on
//    disjoint banks -- conflict-free.
//  * conv1 dW: a lane owns (co, window slot); per window 5 kernel rows x 3
//    aligned 8-byte reads of the padded image (two copies shifted by one
//    element, so any argmax column is aligned) feed 15 packed FMAs over kw
//    pairs.
// Partial sums: fixed-order shuffles / LDS per workgroup, one slab per
// workgroup, summed in fixed order by conv1_direct_dw_reduce_kernel's layout
// ([grid][C][Cin*25 + 1]): deterministic.
#include "kernels.h"
#include "mfma.h"

#include <algorithm>

namespace mcc {
namespace gpu {
namespace {

typedef float f2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f2 pfma(f2 a, f2 b, f2 c) { return __builtin_elementwise_fma(a, b, c); }

// ds_read_b128 lane groups (MI355X_MICROARCH.md, LDS table): group of lane l, and l's index in it
__device__ constexpr unsigned char kB128Group[64] = {
    0, 0, 0, 0, 1, 1, 1, 1, 1, 1, 1, 1, 0, 0, 0, 0, 1, 1, 1, 1, 0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1,
    2, 2, 2, 2, 3, 3, 3, 3, 3, 3, 3, 3, 2, 2, 2, 2, 3, 3, 3, 3, 2, 2, 2, 2, 2, 2, 2, 2, 3, 3, 3, 3};
__device__ constexpr unsigned char kB128Pos[64] = {
    0, 1, 2, 3, 0, 1, 2, 3, 4, 5, 6, 7, 4, 5, 6, 7, 8, 9, 10, 11, 8, 9, 10, 11, 12, 13, 14, 15, 12, 13, 14, 15,
    0, 1, 2, 3, 0, 1, 2, 3, 4, 5, 6, 7, 4, 5, 6, 7, 8, 9, 10, 11, 8, 9, 10, 11, 12, 13, 14, 15, 12, 13, 14, 15};

// ---------------------------------------------------------------- conv2 dW
constexpr int kD2Imgs = 4;                 // images per staged group
constexpr int kD2T = 256;                  // 4 waves x (16 channels x 4 window slots)
constexpr int kD2Y1 = 196 * 8;             // floats per staged image (8-float pixels)
constexpr int kD2Dy = 25 * 16;             // pooled dY floats / codes per image
constexpr int kD2Lds = kD2Imgs * (kD2Y1 * 4 + kD2Dy * 4 + kD2Dy);  // 33,088 B
constexpr int kD2Col = 16 * 151;           // slab columns: [co][ci * 25 + tap | 150: bias]
constexpr int kD2Px = (kD2Imgs * 196 + kD2T - 1) / kD2T;        // staged pixels per thread (4)
constexpr int kD2Q = (kD2Imgs * kD2Dy / 4 + kD2T - 1) / kD2T;   // staged dY quads per thread (2)
constexpr int kD2Red = 4 * 16 * 151 * 4;   // reduction scratch [wave][co][151] (38.7 KB)

// The next group's global loads are issued into registers before the current
// group's windows are processed (a group's staging would otherwise expose the
// HBM latency once per group: 4 images).
// conv2 dW window slots: slot -> (window, second window or -1), windows
// py * 5 + px; slots 2k and 2k + 1 hold vertical neighbours (row 4: two
// columns apart)
__device__ constexpr signed char kD2Win[16][2] = {{0, 13}, {5, 18}, {1, 14}, {6, 19}, {2, 20}, {7, 22},
                                                  {3, 21}, {8, 23}, {4, 24}, {9, -1}, {10, -1}, {15, -1},
                                                  {11, -1}, {16, -1}, {12, -1}, {17, -1}};
// taps (kh, 0..4) of a window: the 8-byte halves (floats 4, 5 of each pixel)
__device__ __forceinline__ void d2_row(uint32_t a, int kh, f2 (&r)[5]) {
  const uint32_t b = a + (uint32_t)(kh * 14 * 8 * 4 + 16);
  asm volatile("ds_read_b64 %0, %1 offset:0" : "=v"(r[0]) : "v"(b));
  asm volatile("ds_read_b64 %0, %1 offset:32" : "=v"(r[1]) : "v"(b));
  asm volatile("ds_read_b64 %0, %1 offset:64" : "=v"(r[2]) : "v"(b));
  asm volatile("ds_read_b64 %0, %1 offset:96" : "=v"(r[3]) : "v"(b));
  asm volatile("ds_read_b64 %0, %1 offset:128" : "=v"(r[4]) : "v"(b));
}

__global__ void __launch_bounds__(kD2T) __attribute__((amdgpu_waves_per_eu(2, 2))) lenet32_dw2_kernel(Conv1DirectParams p) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* y1s = smem;
  float* dys = smem + kD2Imgs * kD2Y1;
  uint8_t* ars = reinterpret_cast<uint8_t*>(dys + kD2Imgs * kD2Dy);
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  // the 16 lanes of each ds_read_b128 lane group (MI355X_MICROARCH.md, LDS
  // table) take the 16 channels of ONE window slot: a group then reads at
  // most 4 distinct pixels (the argmax positions), 8 * 4 bytes apart at
  // 8-float pixels -- conflict-free
  const int gi = kB128Group[lane], co = kB128Pos[lane];
  const int slot = wv * 4 + gi;  // 16 window slots per workgroup
  // this lane's windows (kD2Win: all 25 once).  The 8-byte reads of a
  // half-wave (ds_read_b64: lanes 0-31 = slots 4wv, 4wv + 1) pair windows
  // whose corners are 32 banks apart (vertical neighbours, or two columns
  // apart in row 4), so their 2 x 4 argmax pixels never share a bank; with
  // slot = window (adjacent windows, 16 banks apart) two of the four pixel
  // sets collided (SQ_LDS_BANK_CONFLICT 30 % of 91 % LDS-active cycles)
  const int w0 = kD2Win[slot][0], w1 = kD2Win[slot][1];
  const int p0 = (2 * (w0 / 5) * 14 + 2 * (w0 % 5)) * 8;
  const int p1 = w1 >= 0 ? (2 * (w1 / 5) * 14 + 2 * (w1 % 5)) * 8 : p0;

  for (int i = t * 4; i < kD2Imgs * kD2Y1; i += kD2T * 4) *reinterpret_cast<f32x4*>(y1s + i) = f32x4{0.f, 0.f, 0.f, 0.f};

  f2 acc[25][3];
#pragma unroll
  for (int k = 0; k < 25; ++k) acc[k][0] = acc[k][1] = acc[k][2] = f2{0.f, 0.f};
  float accb = 0.f;

  f2 px[kD2Px][3];
  f32x4 dq[kD2Q];
  uint32_t aq[kD2Q];
  auto issue = [&](int grp) {
    const int img0 = grp * kD2Imgs, nimg = min(kD2Imgs, p.N - img0);
    const float* gx = p.xf + (size_t)img0 * 196 * 6;
#pragma unroll
    for (int j = 0; j < kD2Px; ++j) {
      const int i = min(t + kD2T * j, nimg * 196 - 1);
#pragma unroll
      for (int c = 0; c < 3; ++c) px[j][c] = *reinterpret_cast<const f2*>(gx + i * 6 + 2 * c);
    }
    const f32x4* gd = reinterpret_cast<const f32x4*>(p.dy + (size_t)img0 * kD2Dy);
    const uint32_t* ga = reinterpret_cast<const uint32_t*>(p.arg + (size_t)img0 * kD2Dy);
#pragma unroll
    for (int j = 0; j < kD2Q; ++j) {
      const int i = min(t + kD2T * j, nimg * kD2Dy / 4 - 1);
      dq[j] = gd[i];
      aq[j] = ga[i];
    }
  };
  auto stage = [&](int nimg) {
#pragma unroll
    for (int j = 0; j < kD2Px; ++j) {
      const int i = t + kD2T * j;
      if (i < nimg * 196) {
        *reinterpret_cast<f32x4*>(y1s + i * 8) = f32x4{px[j][0].x, px[j][0].y, px[j][1].x, px[j][1].y};
        *reinterpret_cast<f2*>(y1s + i * 8 + 4) = px[j][2];
      }
    }
#pragma unroll
    for (int j = 0; j < kD2Q; ++j) {
      const int i = t + kD2T * j;
      if (i < nimg * kD2Dy / 4) {
        reinterpret_cast<f32x4*>(dys)[i] = dq[j];
        reinterpret_cast<uint32_t*>(ars)[i] = aq[j];
      }
    }
  };

  const int ngroups = (p.N + kD2Imgs - 1) / kD2Imgs;
  if ((int)blockIdx.x < ngroups) issue(blockIdx.x);
  for (int grp = blockIdx.x; grp < ngroups; grp += gridDim.x) {
    const int nimg = min(kD2Imgs, p.N - grp * kD2Imgs);
    __syncthreads();  // the previous group's reads are done
    stage(nimg);
    __syncthreads();
    if (grp + (int)gridDim.x < ngroups) issue(grp + gridDim.x);
    // No branch on the window's activity: a wave's 64 lanes (4 windows x 16
    // channels) almost never are ALL inactive, so a branch would not skip the
    // FMAs -- an inactive (code 4) lane multiplies position 0's patch by 0.
    for (int m = 0; m < nimg; ++m) {
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int w = j ? w1 : w0;
        if (j == 1 && w1 < 0) break;
        const int it = m * 25 + w;
        const float dy0 = dys[it * 16 + co];
        const int code = ars[it * 16 + co];
        const float dy = code < 4 ? dy0 : 0.f;
        accb += dy;
        const f2 g = f2{dy, dy};
        const float* y = y1s + m * kD2Y1 + (j ? p1 : p0) + (((code >> 1) & 1) * 14 + (code & 1)) * 8;
        const uint32_t ya = (uint32_t)(uintptr_t)((const __attribute__((address_space(3))) float*)y);
#pragma unroll
        for (int kh = 0; kh < 5; ++kh) {
          // the 8-byte halves as single ds_read_b64 (asm): left to the
          // compiler they merge into ds_read2_b64, banked (a/4) mod 32 over
          // 16 contiguous lanes, which undoes the pairing above
          f2 v2[5];
          d2_row(ya, kh, v2);
          lds_wait();
#pragma unroll
          for (int kw = 0; kw < 5; ++kw) {
            asm volatile("" : "+v"(v2[kw]));
            const f32x4 v = *reinterpret_cast<const f32x4*>(y + (kh * 14 + kw) * 8);
            f2* a = acc[kh * 5 + kw];
            a[0] = pfma(g, f2{v[0], v[1]}, a[0]);
            a[1] = pfma(g, f2{v[2], v[3]}, a[1]);
            a[2] = pfma(g, v2[kw], a[2]);
          }
        }
      }
    }
  }
  // ---- workgroup reduction in a fixed order: window slots of a wave by
  // xor-shuffles (16, 32), the four waves through LDS in wave order ----
  __syncthreads();
  // the four lanes of a channel in a wave are l, l ^ 4, l ^ 32, l ^ 36
  // (kB128Pos): xor-shuffles 4, 32 in a fixed order, then the waves
  float* red = smem;  // [4 waves][16 co][151]
  auto put = [&](int k, float v) {
    v += __shfl_xor(v, 4);
    v += __shfl_xor(v, 32);
    if (gi == 0) red[(wv * 16 + co) * 151 + k] = v;
  };
#pragma unroll
  for (int k = 0; k < 25; ++k) {
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      put((2 * c) * 25 + k, acc[k][c].x);
      put((2 * c + 1) * 25 + k, acc[k][c].y);
    }
  }
  put(150, accb);
  __syncthreads();
  float* slab = p.slab + (size_t)blockIdx.x * kD2Col;
  for (int i = t; i < kD2Col; i += kD2T)
    slab[i] = ((red[i] + red[kD2Col + i]) + red[2 * kD2Col + i]) + red[3 * kD2Col + i];
}

// ---------------------------------------------------------------- conv1 dW
constexpr int kD1Imgs = 2;                  // 30.7 KB of LDS: four workgroups per CU
constexpr int kD1T = 256;                   // 4 waves x (6 channels x 10 window slots) + 4 idle lanes per wave
constexpr int kD1P = 36;                    // padded-image pitch (floats): columns 0 .. 32 read
constexpr int kD1Copy = 32 * kD1P + 32;     // 1184 floats per shifted copy (32 padded rows; +32: the
                                            // second copy on other banks than the first)
constexpr int kD1X = 2 * kD1Copy;           // floats per staged image (copies shift 0 and 1)
constexpr int kD1Lds = kD1Imgs * (kD1X * 4 + 196 * 6 * 4 + 196 * 6);  // 30,704 B
constexpr int kD1Col = 6 * 26;              // slab columns [co][tap | 25: bias]
constexpr int kD1W = (kD1Imgs * 196 + kD1T - 1) / kD1T;      // staged u8 words per thread
constexpr int kD1Q = (kD1Imgs * 294 + kD1T - 1) / kD1T;      // staged dY quads per thread
static_assert(40 * 6 * 26 * 4 <= kD1Lds, "reduction scratch fits in the staging LDS");

// the 5 x 3 patch reads of one conv1-dW window as single ds_read_b64 (byte
// offsets kh * kD1P * 4 + {0, 8, 16}); results valid after lds_wait()
template <int KH>
__device__ __forceinline__ void d1_rows(uint32_t a, f2 (&r)[5][3]) {
  if constexpr (KH < 5) {
    asm volatile("ds_read_b64 %0, %1 offset:%2" : "=v"(r[KH][0]) : "v"(a), "n"(KH * kD1P * 4));
    asm volatile("ds_read_b64 %0, %1 offset:%2" : "=v"(r[KH][1]) : "v"(a), "n"(KH * kD1P * 4 + 8));
    asm volatile("ds_read_b64 %0, %1 offset:%2" : "=v"(r[KH][2]) : "v"(a), "n"(KH * kD1P * 4 + 16));
    d1_rows<KH + 1>(a, r);
  }
}

__global__ void __launch_bounds__(kD1T) lenet32_dw1_kernel(Conv1DirectParams p) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* xs = smem;
  float* dys = smem + kD1Imgs * kD1X;
  uint8_t* ars = reinterpret_cast<uint8_t*>(dys + kD1Imgs * 196 * 6);
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const int ls = lane / 6, co = lane - 6 * ls;          // lanes 60..63: ls = 10 (idle)
  const bool live = ls < 10;
  const int slot = wv * 10 + min(ls, 9);                // 40 window slots per workgroup
  for (int i = t * 4; i < kD1Imgs * kD1X; i += kD1T * 4) *reinterpret_cast<f32x4*>(xs + i) = f32x4{0.f, 0.f, 0.f, 0.f};

  f2 acc[5][3];
#pragma unroll
  for (int k = 0; k < 5; ++k) acc[k][0] = acc[k][1] = acc[k][2] = f2{0.f, 0.f};
  float accb = 0.f;

  // staging registers of one group; the dataset indices of a group are
  // loaded one group earlier still (lane m < 4: image m), so the image loads
  // never wait on a dependent index load
  const int ngroups = (p.N + kD1Imgs - 1) / kD1Imgs;
  auto load_idx = [&](int grp) {
    const int i = min(grp * kD1Imgs + (lane & 3), p.N - 1);
    return p.idx ? p.idx[i] : i;
  };
  uint32_t xw[kD1W];
  f32x4 dq[kD1Q];
  uint32_t aq[kD1Q];
  auto issue = [&](int grp, int idxv) {
    const int img0 = grp * kD1Imgs, nimg = min(kD1Imgs, p.N - img0);
#pragma unroll
    for (int j = 0; j < kD1W; ++j) {
      const int i = min(t + kD1T * j, nimg * 196 - 1);
      const int m = i / 196, wd = i - 196 * m;
      const int src = __shfl(idxv, m);
      xw[j] = *reinterpret_cast<const uint32_t*>(p.x + (size_t)src * 784 + 4 * wd);
    }
    const f32x4* gd = reinterpret_cast<const f32x4*>(p.dy + (size_t)img0 * 196 * 6);
    const uint32_t* ga = reinterpret_cast<const uint32_t*>(p.arg + (size_t)img0 * 196 * 6);
#pragma unroll
    for (int j = 0; j < kD1Q; ++j) {
      const int i = min(t + kD1T * j, nimg * 294 - 1);
      dq[j] = gd[i];
      aq[j] = ga[i];
    }
  };
  auto stage = [&](int nimg) {
    // 4-pixel items -> Xpad[r + 2][c + 2] (copy 0) and copy 1 (position q
    // holds Xpad[.][q + 1])
#pragma unroll
    for (int j = 0; j < kD1W; ++j) {
      const int i = t + kD1T * j;
      if (i < nimg * 196) {
        const int m = i / 196, wd = i - 196 * m;
        const int r = (wd * 9363) >> 16, c4 = 4 * (wd - 7 * r);  // wd / 7
        float v[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = (float)((xw[j] >> (8 * e)) & 0xffu) * (1.f / 255.f);
        float* d0 = xs + m * kD1X + (r + 2) * kD1P + c4 + 2;
        float* d1 = d0 + kD1Copy - 1;
        *reinterpret_cast<f2*>(d0) = f2{v[0], v[1]};
        *reinterpret_cast<f2*>(d0 + 2) = f2{v[2], v[3]};
#pragma unroll
        for (int e = 0; e < 4; ++e) d1[e] = v[e];
      }
    }
#pragma unroll
    for (int j = 0; j < kD1Q; ++j) {
      const int i = t + kD1T * j;
      if (i < nimg * 294) {
        reinterpret_cast<f32x4*>(dys)[i] = dq[j];
        reinterpret_cast<uint32_t*>(ars)[i] = aq[j];
      }
    }
  };

  int idx_next = 0;
  if ((int)blockIdx.x < ngroups) {
    issue(blockIdx.x, load_idx(blockIdx.x));
    idx_next = load_idx(blockIdx.x + gridDim.x);
  }
  for (int grp = blockIdx.x; grp < ngroups; grp += gridDim.x) {
    const int nimg = min(kD1Imgs, p.N - grp * kD1Imgs);
    __syncthreads();
    stage(nimg);
    __syncthreads();
    if (grp + (int)gridDim.x < ngroups) {
      issue(grp + gridDim.x, idx_next);
      idx_next = load_idx(grp + 2 * gridDim.x);
    }
    if (live) {
      // Branch-free items (see conv2 dW).  A wave takes a block of 2 window
      // columns x 5 window rows, lane slot ls = (row ls >> 1, column ls & 1):
      // a window's four argmax positions use banks b + {0,1,4,5,32,33,36,37}
      // (b = 2 wx + 8 wy mod 64; the second copy 32 banks off), and the
      // windows a half-wave reads (slots 0..5 / 5..9: 3 block rows) then
      // have disjoint bank sets -- the consecutive windows of a row did not
      // (SQ_LDS_BANK_CONFLICT 57 % of LDS cycles).  21 blocks per image
      // (7 column pairs x 3 row blocks of 5, 5, 4 rows).
      const int nblk = nimg * 21;
      for (int bi = wv; bi < nblk; bi += 4) {
        const int m = (bi * 3121) >> 16, r = bi - 21 * m;      // bi / 21 (bi < 64)
        const int rb = (r * 37) >> 8, cb = r - 7 * rb;         // r / 7 (r < 21)
        const int wy = 5 * rb + (ls >> 1), wx = 2 * cb + (ls & 1);
        if (wy < 14) {
          const int it = m * 196 + wy * 14 + wx;
          const float dy0 = dys[it * 6 + co];
          const int code = ars[it * 6 + co];
          const float dy = code < 4 ? dy0 : 0.f;
          accb += dy;
          const f2 g = f2{dy, dy};
          const float* x = xs + m * kD1X + (code & 1) * kD1Copy + (2 * wy + ((code >> 1) & 1)) * kD1P + 2 * wx;
#ifndef MCC_D1_COMPILER_READS
          // 15 single ds_read_b64 in inline asm: left to the compiler, the
          // adjacent 8-byte reads were merged into ds_read2_b32 / ds_read2_b64,
          // whose banking is (a/4) mod 32 -- the second image copy's 32-bank
          // offset then collides (SQ_LDS_BANK_CONFLICT 47 % of 93 % LDS-active
          // cycles, 11 LDS cycles per instruction)
          const uint32_t xa = (uint32_t)(uintptr_t)((const __attribute__((address_space(3))) float*)x);
          f2 rd[5][3];
          d1_rows<0>(xa, rd);
          lds_wait();
#pragma unroll
          for (int kh = 0; kh < 5; ++kh) {
            asm volatile("" : "+v"(rd[kh][0]), "+v"(rd[kh][1]), "+v"(rd[kh][2]));
            acc[kh][0] = pfma(g, rd[kh][0], acc[kh][0]);
            acc[kh][1] = pfma(g, rd[kh][1], acc[kh][1]);
            acc[kh][2] = pfma(g, rd[kh][2], acc[kh][2]);  // .y: tap kw = 5 (unused)
          }
#else
#pragma unroll
          for (int kh = 0; kh < 5; ++kh) {
            const f2 a = *reinterpret_cast<const f2*>(x + kh * kD1P);
            const f2 b = *reinterpret_cast<const f2*>(x + kh * kD1P + 2);
            const f2 c = *reinterpret_cast<const f2*>(x + kh * kD1P + 4);
            acc[kh][0] = pfma(g, a, acc[kh][0]);
            acc[kh][1] = pfma(g, b, acc[kh][1]);
            acc[kh][2] = pfma(g, c, acc[kh][2]);  // .y: tap kw = 5 (unused)
          }
#endif
        }
      }
    }
  }
  __syncthreads();
  float* red = smem;  // [40 slots][6 co][26]
  if (live) {
    float* r = red + (slot * 6 + co) * 26;
#pragma unroll
    for (int kh = 0; kh < 5; ++kh) {
      r[kh * 5 + 0] = acc[kh][0].x;
      r[kh * 5 + 1] = acc[kh][0].y;
      r[kh * 5 + 2] = acc[kh][1].x;
      r[kh * 5 + 3] = acc[kh][1].y;
      r[kh * 5 + 4] = acc[kh][2].x;
    }
    r[25] = accb;
  }
  __syncthreads();
  float* slab = p.slab + (size_t)blockIdx.x * kD1Col;
  for (int i = t; i < kD1Col; i += kD1T) {
    float v = 0.f;
    for (int s = 0; s < 40; ++s) v += red[s * kD1Col + i];
    slab[i] = v;
  }
}

}  // namespace

// ---------------------------------------------------------------------------
// conv2 forward on exact f32 MFMA (round 5): 6 -> 16, 5x5 valid (14x14 ->
// 10x10), ReLU, 2x2 max-pool with argmax.  One wave per image; the GEMM is
// C[pixel][co] = sum_k patch[pixel][k] W[k][co], K = 25 taps x 6 channels =
// 150 (38 steps of v_mfma_f32_16x16x4_f32, 152: zero weights past 150), the
// 100 pixels window-major in 7 tiles of 16 rows (row 4w + i = position i of
// pooling window w), so lane (co, g) of tile T holds the four positions of
// window 4T + g: the pool, its first-max argmax, bias and ReLU are in-lane.
// Operands: the image's Y1 (HWC, 6 floats per pixel, as stored) in LDS, A
// read per lane at a per-lane base + a per-step offset register; weights in
// 38 registers.  MEASURED, NOT THE DEFAULT (MCC_AB=f32_mfma_fwd2 selects it):
// 1,073 us vs 1,051 us for the packed-FMA kernel conv_direct_fwd<5, 6, 16>
// at B = 163,840 (two interleaved accumulator chains: 1,155 us) -- the f32
// matrix rate equals the packed-FMA vector rate on gfx950, and the MFMA
// form's 266 instructions per image (16 / 16 useful rows, K 152 / 150) run
// as one dependent chain per tile against one LDS operand read each.
constexpr int kC2Steps = 38;
constexpr int kC2Img = 14 * 14 * 6;  // floats
__global__ void __launch_bounds__(64) lenet32_conv2_fwd_kernel(Conv1DirectParams p, const float* __restrict__ wt,
                                                               const float* __restrict__ bias, float* __restrict__ out,
                                                               uint8_t* __restrict__ out_arg) {
  __shared__ __attribute__((aligned(16))) float ys[kC2Img + 4];
  const int lane = threadIdx.x, r = lane & 15, g = lane >> 4;
  // B operand: W[k = 4s + g][co = r], k = tap * 6 + ci (tap-major packed copy: wt[ci][tap][co])
  float wb[kC2Steps];
  int koff[kC2Steps];
#pragma unroll
  for (int st = 0; st < kC2Steps; ++st) {
    const int k = 4 * st + g;
    const int tap = k / 6, ci = k - 6 * tap;
    wb[st] = k < 150 ? wt[(ci * 25 + tap) * 16 + r] : 0.f;
    koff[st] = k < 150 ? ((tap / 5) * 14 + tap % 5) * 6 + ci : 0;
  }
  const float bv = bias[r];
  const int pos = r & 3, pofs = ((pos >> 1) * 14 + (pos & 1)) * 6;
  const int grid = (int)gridDim.x;
  for (int img = blockIdx.x; img < p.N; img += grid) {
    // (no register prefetch: 16 waves per CU hide the load; 20 more VGPRs
    // would cost a wave per SIMD)
    const float4* src = reinterpret_cast<const float4*>(p.xf + (size_t)img * kC2Img);
    float4 v4[5];
#pragma unroll
    for (int i = 0; i < 5; ++i) v4[i] = src[min(lane + 64 * i, kC2Img / 4 - 1)];
    __syncthreads();  // (one wave: orders the previous image's reads before the overwrite)
#pragma unroll
    for (int i = 0; i < 5; ++i)
      if (lane + 64 * i < kC2Img / 4) reinterpret_cast<float4*>(ys)[lane + 64 * i] = v4[i];
    __syncthreads();
    float* o = out + (size_t)img * 25 * 16;
    uint8_t* oa = out_arg + (size_t)img * 25 * 16;
#pragma unroll 1
    for (int T = 0; T < 7; ++T) {
      // A operand rows: row r -> window 4T + (r >> 2) (25..27: padding), position r & 3
      const int wr = min(4 * T + (r >> 2), 24);
      const int py = (wr * 13) >> 6, px = wr - 5 * py;  // wr / 5 for wr < 25
      const float* yb = ys + (2 * py * 14 + 2 * px) * 6 + pofs;
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int st = 0; st < kC2Steps; ++st)
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(yb[koff[st]], wb[st], acc, 0, 0, 0);
      // lane: window 4T + g, positions 0..3 (first max wins), channel r
      float best = acc[0];
      uint32_t a = 0;
      if (acc[1] > best) { best = acc[1]; a = 1; }
      if (acc[2] > best) { best = acc[2]; a = 2; }
      if (acc[3] > best) { best = acc[3]; a = 3; }
      const float y = fmaxf(best + bv, 0.f);
      const int w = 4 * T + g;
      if (w < 25) {
        o[w * 16 + r] = y;
        oa[w * 16 + r] = (uint8_t)(y > 0.f ? a : 4u);
      }
    }
  }
}

int lenet32_conv2_fwd_grid(int N) { return std::max(1, std::min(N, 256 * 16)); }  // 16 waves per CU (<= 128 VGPRs)
void lenet32_conv2_fwd(const Conv1DirectParams& p, hipStream_t s) {
  MCC_CHECK(p.Cin == 6 && p.C == 16 && p.KS == 5 && p.pad == 0 && p.H == 14 && p.W == 14 && p.PH == 5 && p.PW == 5 &&
                p.xf && p.wt && p.bias && p.out && p.out_arg,
            "lenet32_conv2_fwd: LeNet-5 conv2 shape only");
  hipLaunchKernelGGL(lenet32_conv2_fwd_kernel, dim3((unsigned)lenet32_conv2_fwd_grid(p.N)), dim3(64), 0, s, p, p.wt,
                     p.bias, p.out, p.out_arg);
}

int lenet32_dw2_grid(int N) { return std::max(1, std::min((N + kD2Imgs - 1) / kD2Imgs, 256 * 2)); }  // 2 per CU (VGPRs)
int lenet32_dw1_grid(int N) { return std::max(1, std::min((N + kD1Imgs - 1) / kD1Imgs, 256 * 4)); }

void lenet32_dw2(const Conv1DirectParams& p, hipStream_t s) {
  // (dynamic LDS sized for the end-of-kernel reduction scratch)
  hipLaunchKernelGGL(lenet32_dw2_kernel, dim3((unsigned)lenet32_dw2_grid(p.N)), dim3(kD2T),
                     std::max(kD2Lds, kD2Red), s, p);
}
void lenet32_dw1(const Conv1DirectParams& p, hipStream_t s) {
  hipLaunchKernelGGL(lenet32_dw1_kernel, dim3((unsigned)lenet32_dw1_grid(p.N)), dim3(kD1T), kD1Lds, s, p);
}

}  // namespace gpu
}  // namespace mcc
