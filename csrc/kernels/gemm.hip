// LDS-tiled MFMA GEMM for the fully-connected layers, with fused epilogues.
//
// Replaces the reference's scalar FC loops: forward W*x + b then tanh/softmax
// (Layer_feedForw_full, cnn.c:113-152) and the fused dX/dW/db backward loop
// (Layer_feedBack_full, cnn.c:154-173).  Here, for a batch of M samples:
//   forward   Y  = act(X W^T + b)        EPI_BIAS_ACT  (EPI_LOGITS for the last layer)
//   data grad dX = (dY W) * act'(Xprev)  EPI_DACT      (W^T shadow keeps B K-contiguous)
//   weight    dW = dY^T X, db = dY^T 1   EPI_PARTIAL   (split-K over the batch; the
//             bias gradient is a ones-column appended to X — no separate reduce)
// C[M][N] = A[M][K] * B[N][K]^T; `ta`/`tb` say an operand is stored K-major, in
// which case the staging pass transposes it into the [row][k] LDS image.
#include "kernels.h"
#include "mfma.h"

namespace mcc {
namespace gpu {

namespace {

template <typename T>
__device__ __forceinline__ float ld_elem(const T* base, int ld, bool trans, int r, int k, int R, int K) {
  if (r >= R || k >= K) return 0.f;
  return to_f(trans ? base[(size_t)k * ld + r] : base[(size_t)r * ld + k]);
}

// Stage a ROWS x 32 tile (rows r0.., k k0..) of op(X) into lds[row][LDK].
template <typename T, int ROWS, int LDK>
__device__ __forceinline__ void stage_operand(T* lds, const T* X, int ld, bool trans, int r0, int k0, int R,
                                              int K, int ones_row) {
  typedef typename Vec8<T>::type V8;
  constexpr int NV = ROWS * 4;  // 8-element vectors in the tile
  for (int v = threadIdx.x; v < NV; v += blockDim.x) {
    if (!trans) {
      const int row = v >> 2, kv = (v & 3) * 8;
      const int gr = r0 + row, gk = k0 + kv;
      V8 x;
      if (gr < R && gr != ones_row && gk + 8 <= K) {
        x = load8(X + (size_t)gr * ld + gk);
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float f = gr == ones_row ? (gk + j < K ? 1.f : 0.f) : ld_elem(X, ld, false, gr, gk + j, R, K);
          x[j] = from_f<T>(f);
        }
      }
      store8(lds + row * LDK + kv, x);
    } else {
      constexpr int RV = ROWS / 8;
      const int kr = v / RV, rv = (v - kr * RV) * 8;
      const int gk = k0 + kr, gr = r0 + rv;
      V8 x;
      if (gk < K && gr + 8 <= R && (ones_row < gr || ones_row >= gr + 8)) {
        x = load8(X + (size_t)gk * ld + gr);
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float f = (gr + j) == ones_row ? (gk < K ? 1.f : 0.f) : ld_elem(X, ld, true, gr + j, gk, R, K);
          x[j] = from_f<T>(f);
        }
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) lds[(rv + j) * LDK + kr] = x[j];
    }
  }
}

template <typename T, int BM, int BN>
__global__ void __launch_bounds__(256) gemm_kernel(GemmParams p) {
  typedef typename Vec8<T>::type V8;
  constexpr int BK = 32;
  constexpr int LDK = BK + (sizeof(T) == 2 ? 8 : 4);
  __shared__ __attribute__((aligned(16))) T As[BM * LDK];
  __shared__ __attribute__((aligned(16))) T Bs[BN * LDK];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r16 = lane & 15, g = lane >> 4;
  const int wm = wave >> 1, wn = wave & 1;
  constexpr int WM = BM / 2, WN = BN / 2, FM = WM / 16, FN = WN / 16;
  const int m0 = blockIdx.y * BM, n0 = blockIdx.x * BN;
  const int kchunks = cdiv(p.K, BK);
  const int per = cdiv(kchunks, (int)gridDim.z);
  const int kc0 = blockIdx.z * per, kc1 = min(kchunks, kc0 + per);
  const T* A = static_cast<const T*>(p.A);
  const T* B = static_cast<const T*>(p.B);

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  for (int kc = kc0; kc < kc1; ++kc) {
    const int k0 = kc * BK;
    __syncthreads();
    stage_operand<T, BM, LDK>(As, A, p.lda, p.ta, m0, k0, p.M, p.K, -1);
    stage_operand<T, BN, LDK>(Bs, B, p.ldb, p.tb, n0, k0, p.N, p.K, p.ones_col);
    __syncthreads();
    V8 a[FM], b[FN];
#pragma unroll
    for (int i = 0; i < FM; ++i) a[i] = load8(As + (wm * WM + i * 16 + r16) * LDK + 8 * g);
#pragma unroll
    for (int j = 0; j < FN; ++j) b[j] = load8(Bs + (wn * WN + j * 16 + r16) * LDK + 8 * g);
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) acc[i][j] = mma(acc[i][j], a[i], b[j]);
  }

  T* C = static_cast<T*>(p.C);
  const T* aux = static_cast<const T*>(p.aux);
#pragma unroll
  for (int i = 0; i < FM; ++i) {
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int col = n0 + wn * WN + j * 16 + r16;
      if (col >= p.N) continue;
      const float bv = (p.epi == EPI_BIAS_ACT || p.epi == EPI_LOGITS) && p.bias ? p.bias[col] : 0.f;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int row = m0 + wm * WM + i * 16 + 4 * g + e;
        if (row >= p.M) continue;
        const float v = acc[i][j][e];
        switch (p.epi) {
          case EPI_BIAS_ACT:
            C[(size_t)row * p.ldc + col] = from_f<T>(act_apply(p.act, v + bv));
            break;
          case EPI_LOGITS:
            p.Cf[(size_t)row * p.ldc + col] = v + bv;
            break;
          case EPI_DACT: {
            float d = 1.f;
            if (p.act != ACT_NONE) d = act_grad_y(p.act, to_f(aux[(size_t)row * p.ldaux + col]));
            C[(size_t)row * p.ldc + col] = from_f<T>(v * d);
            break;
          }
          default:
            p.Cf[(size_t)blockIdx.z * p.partial_stride + (size_t)row * p.ldc + col] = v;
        }
      }
    }
  }
}

__global__ void dw_reduce_kernel(DwReduceParams p) {
  const int kc = p.kfeat + 1;
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= (int64_t)p.Nout * kc) return;
  const int n = (int)(j / kc), k = (int)(j - (int64_t)n * kc);
  const float* src = p.part + (size_t)n * p.ldp + k;
  float acc = 0.f;
  for (int s = 0; s < p.S; ++s) acc += src[(size_t)s * p.partial_stride];
  float* dst;
  if (k < p.kfeat) {
    int kk = k;
    if (p.permC > 0) {
      const int hw = k / p.permC, c = k - hw * p.permC;
      kk = c * p.permHW + hw;
    }
    dst = p.gw + (size_t)n * p.kfeat + kk;
  } else {
    dst = p.gb + n;
  }
  *dst = p.beta != 0.f ? p.beta * *dst + acc : acc;
}

template <typename T>
void launch_gemm(const GemmParams& p, hipStream_t s) {
  const dim3 block(256);
  // Tile choice: wide-N tiles for the skinny forward/backward-data GEMMs
  // (N <= 128 is one tile, A is streamed once), 64x64 otherwise.
  if (p.N > 64 && p.N <= 128 && p.M >= 1024) {
    const dim3 grid((unsigned)cdiv(p.N, 128), (unsigned)cdiv(p.M, 64), (unsigned)p.splitk);
    hipLaunchKernelGGL((gemm_kernel<T, 64, 128>), grid, block, 0, s, p);
  } else if (p.M >= 4096 && p.N >= 128) {
    const dim3 grid((unsigned)cdiv(p.N, 128), (unsigned)cdiv(p.M, 128), (unsigned)p.splitk);
    hipLaunchKernelGGL((gemm_kernel<T, 128, 128>), grid, block, 0, s, p);
  } else {
    const dim3 grid((unsigned)cdiv(p.N, 64), (unsigned)cdiv(p.M, 64), (unsigned)p.splitk);
    hipLaunchKernelGGL((gemm_kernel<T, 64, 64>), grid, block, 0, s, p);
  }
}

}  // namespace

void gemm(DType t, const GemmParams& p, hipStream_t s) {
  MCC_CHECK(p.M > 0 && p.N > 0 && p.K > 0, "gemm: empty problem");
  MCC_CHECK(p.lda % 8 == 0 && p.ldb % 8 == 0, "gemm: leading dims must be multiples of 8");
  MCC_CHECK(p.splitk >= 1, "gemm: splitk >= 1");
  MCC_CHECK(p.splitk == 1 || p.epi == EPI_PARTIAL, "gemm: split-K needs the partial epilogue");
  if (t == DType::BF16) launch_gemm<bf16>(p, s);
  else launch_gemm<float>(p, s);
}

void dw_reduce(const DwReduceParams& p, hipStream_t s) {
  const int64_t n = (int64_t)p.Nout * (p.kfeat + 1);
  hipLaunchKernelGGL(dw_reduce_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, p);
}

}  // namespace gpu
}  // namespace mcc
