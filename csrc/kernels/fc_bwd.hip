// Fused backward of a small fully-connected layer (K <= 127 inputs, N <= 96
// outputs, bf16): one pass over the batch computes BOTH
//
//   dX[m][k]   = act'(X[m][k]) * sum_n dZ[m][n] W[n][k]         (data gradient)
//   dW[n][k]  += sum_m dZ[m][n] X[m][k],  db[n] += sum_m dZ[m][n] (weight gradient)
//
// (reference math: Layer_feedBack_full, cnn.c:145-173).  The unfused path
// streamed dZ and X twice (split-K weight-gradient GEMM + slab reduce, then
// the data-gradient FC kernel): three launches and two passes over the
// operands for LeNet-5's 120 -> 84 layer.  Here a persistent workgroup walks
// 64-row blocks: dZ and [X | 1] are staged once into LDS, the data gradient
// is an MFMA over N (W^T resident in LDS, bf16 copies of the fp32 master as
// the packed compute copy), masked by act'(X) and written back through an LDS
// tile as 16-byte rows, and the weight gradient accumulates in registers over
// all of the workgroup's rows (operands read with ds_read_b64_tr_b16, K =
// rows); one fp32 slab per workgroup, reduced in a fixed order (dw_reduce).
#include "kernels.h"
#include "mfma.h"

#include <algorithm>

namespace mcc {
namespace gpu {

namespace {

constexpr int kFbT = 256;         // 4 waves
constexpr int kFbRows = 64;       // rows per block (16 per wave in the data gradient)
constexpr int kFbNP = 96;         // N padded (3 K-chunks of the data gradient, 6 dW row fragments)
constexpr int kFbKP = 128;        // K + bias column padded (8 dX column / dW column fragments)
constexpr int kFbLdN = kFbNP + 8;  // LDS row strides (bf16): +16 bytes against bank aliasing
constexpr int kFbLdK = kFbKP + 8;
constexpr int kFbLds = (kFbKP * kFbLdN + kFbRows * kFbLdN + 2 * kFbRows * kFbLdK) * 2;

__global__ void __launch_bounds__(kFbT) fc_small_bwd_kernel(FcBwdParams p) {
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  bf16* WT = reinterpret_cast<bf16*>(smem_raw);  // [k][n] = bf16(W[n][k])
  bf16* DZ = WT + kFbKP * kFbLdN;                // [row][n]
  bf16* X = DZ + kFbRows * kFbLdN;               // [row][k], column K = 1 (bias)
  bf16* OUT = X + kFbRows * kFbLdK;              // [row][k] data-gradient tile
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r16 = lane & 15, g = lane >> 4;
  const int q = r16 >> 2, pp = r16 & 3;

  for (int i = tid; i < kFbKP * kFbNP; i += kFbT) {
    const int k = i / kFbNP, n = i - k * kFbNP;
    WT[k * kFbLdN + n] = (n < p.N && k < p.K) ? (bf16)p.w[(size_t)n * p.K + k] : (bf16)0.f;
  }

  // transposed fragment: rows kr..kr+3 (block rows = K of the dW MFMA), 16 columns from col0
  auto tr = [&](const bf16* img, int ld, int kr, int col0) {
    return tr4(img + (kr + q) * ld + col0 + 4 * pp);
  };

  f32x4 acc_w[6][2];  // dW fragments: n-frag f (16 n), k-frags 2*wave + j
#pragma unroll
  for (int f = 0; f < 6; ++f)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc_w[f][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nblk = cdiv(p.M, kFbRows);
  // staging pieces of one block, loaded one block ahead into registers
  // ("issue early / write late"): dZ 64 rows x 12 pieces, [X|1] 64 x 16,
  // 3 + 4 per thread; rows past M load a clamped row and are zeroed
  constexpr int PZ = kFbRows * (kFbNP / 8) / kFbT, PX = kFbRows * (kFbKP / 8) / kFbT;
  bf16x8 rz[PZ], rx[PX];
  auto gload = [&](int blk) {
    const int row0 = blk * kFbRows;
#pragma unroll
    for (int j = 0; j < PZ; ++j) {
      const int i = j * kFbT + tid;
      const int r = i / (kFbNP / 8), c8 = (i - r * (kFbNP / 8)) * 8;
      const int m = min(row0 + r, p.M - 1);
      const int cc = c8 < p.N ? c8 : 0;  // ldz >= round_up(N, 8): in-row
      rz[j] = load8(static_cast<const bf16*>(p.dz) + (size_t)m * p.ldz + cc);
    }
#pragma unroll
    for (int j = 0; j < PX; ++j) {
      const int i = j * kFbT + tid;
      const int r = i / (kFbKP / 8), c8 = (i - r * (kFbKP / 8)) * 8;
      const int m = min(row0 + r, p.M - 1);
      const int cc = c8 < p.K ? c8 : 0;  // K % 8 == 0 (host)
      rx[j] = load8(static_cast<const bf16*>(p.x) + (size_t)m * p.ldx + cc);
    }
  };
  auto lstore = [&](int blk) {
    const int row0 = blk * kFbRows;
#pragma unroll
    for (int j = 0; j < PZ; ++j) {
      const int i = j * kFbT + tid;
      const int r = i / (kFbNP / 8), c8 = (i - r * (kFbNP / 8)) * 8;
      const bool live = row0 + r < p.M;
      bf16x8 v = rz[j];
#pragma unroll
      for (int e = 0; e < 8; ++e)
        if (!live || c8 + e >= p.N) v[e] = (bf16)0.f;
      store8(DZ + r * kFbLdN + c8, v);
    }
#pragma unroll
    for (int j = 0; j < PX; ++j) {
      const int i = j * kFbT + tid;
      const int r = i / (kFbKP / 8), c8 = (i - r * (kFbKP / 8)) * 8;
      const bool live = row0 + r < p.M;
      bf16x8 v = rx[j];
#pragma unroll
      for (int e = 0; e < 8; ++e)
        if (!live || c8 >= p.K) v[e] = (bf16)((live && c8 + e == p.K) ? 1.f : 0.f);
      store8(X + r * kFbLdK + c8, v);
    }
  };
  if (blockIdx.x < nblk) gload(blockIdx.x);
  for (int blk = blockIdx.x; blk < nblk; blk += gridDim.x) {
    const int row0 = blk * kFbRows;
    __syncthreads();  // previous block's LDS reads done (and WT written)
    lstore(blk);
    __syncthreads();
    if (blk + (int)gridDim.x < nblk) gload(blk + gridDim.x);  // lands during this block's MFMAs

    // ---- data gradient: rows 16*wave.., all K columns ----
    {
      bf16x8 a[3];
#pragma unroll
      for (int c = 0; c < 3; ++c) a[c] = load8(DZ + (16 * wave + r16) * kFbLdN + 32 * c + 8 * g);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        if (16 * j >= p.K) break;
        f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int c = 0; c < 3; ++c) acc = mma(acc, load8(WT + (16 * j + r16) * kFbLdN + 32 * c + 8 * g), a[c]);
        // C^T: lane holds k = 16j + 4g + i of row 16*wave + r16
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int k = 16 * j + 4 * g + i;
          const float y = (float)X[(16 * wave + r16) * kFbLdK + k];
          OUT[(16 * wave + r16) * kFbLdK + k] = (bf16)(acc[i] * act_grad_y(p.act, y));
        }
      }
    }
    // ---- weight gradient: dW[n][k] += sum_rows DZ[row][n] X[row][k] ----
#pragma unroll
    for (int ks = 0; ks < kFbRows / 32; ++ks) {
      const int kr = 32 * ks + 8 * g;
      bf16x8 b[2];
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int c0 = 16 * (2 * wave + j);
        const bf16x4 lo = tr(X, kFbLdK, kr, c0), hi = tr(X, kFbLdK, kr + 4, c0);
        b[j] = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
      }
#pragma unroll
      for (int f = 0; f < 6; ++f) {
        const bf16x4 lo = tr(DZ, kFbLdN, kr, 16 * f), hi = tr(DZ, kFbLdN, kr + 4, 16 * f);
        const bf16x8 a = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
#pragma unroll
        for (int j = 0; j < 2; ++j) acc_w[f][j] = mma(acc_w[f][j], a, b[j]);
      }
    }
    __syncthreads();  // OUT complete
    // ---- data-gradient rows out (16-byte pieces) ----
    for (int i = tid; i < kFbRows * (kFbKP / 8); i += kFbT) {
      const int r = i / (kFbKP / 8), c8 = (i - r * (kFbKP / 8)) * 8;
      const int m = row0 + r;
      if (m < p.M && c8 < p.K) store8(static_cast<bf16*>(p.dx) + (size_t)m * p.lddx + c8, load8(OUT + r * kFbLdK + c8));
    }
  }
  // ---- this workgroup's slab [n][k] (k = K: bias) ----
  float* slab = p.slab + (size_t)blockIdx.x * p.N * p.ldp;
#pragma unroll
  for (int f = 0; f < 6; ++f)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int k = 16 * (2 * wave + j) + r16;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int n = 16 * f + 4 * g + i;
        if (n < p.N && k <= p.K) slab[(size_t)n * p.ldp + k] = acc_w[f][j][i];
      }
    }
}

}  // namespace

bool fc_small_bwd_supported(int N, int K) { return N >= 1 && N <= kFbNP && K >= 8 && K < kFbKP && K % 8 == 0; }

int fc_small_bwd_grid(int M) { return std::max(1, std::min(cdiv(M, kFbRows), 256)); }

void fc_small_bwd(const FcBwdParams& p, hipStream_t s) {
  MCC_CHECK(fc_small_bwd_supported(p.N, p.K) && p.M > 0, "fc_small_bwd: needs N <= 96, K < 128, K % 8 == 0");
  MCC_CHECK(p.ldz % 8 == 0 && p.ldz >= ((p.N + 7) & ~7) && p.ldx % 8 == 0 && p.ldx >= p.K && p.lddx % 8 == 0 &&
                p.lddx >= p.K && p.ldp >= p.K + 1 && p.dz && p.x && p.w && p.dx && p.slab,
            "fc_small_bwd: bad leading dims / buffers");
  hipLaunchKernelGGL(fc_small_bwd_kernel, dim3((unsigned)fc_small_bwd_grid(p.M)), dim3(kFbT), kFbLds, s, p);
}

}  // namespace gpu
}  // namespace mcc
