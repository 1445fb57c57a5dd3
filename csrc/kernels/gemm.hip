// LDS-tiled MFMA GEMM for the fully-connected layers and the im2col conv
// path, with fused epilogues.
//
// Replaces the reference's scalar FC loops: forward W*x + b then tanh/softmax
// (Layer_feedForw_full, cnn.c:113-152) and the fused dX/dW/db backward loop
// (Layer_feedBack_full, cnn.c:154-173).  Here, for a batch of M samples:
//   forward   Y  = act(X W^T + b)        EPI_BIAS_ACT  (EPI_LOGITS for the last layer)
//   data grad dX = (dY W) * act'(Xprev)  EPI_DACT      (W^T shadow keeps B K-contiguous)
//   weight    dW = dY^T X, db = dY^T 1   EPI_PARTIAL   (split-K over the batch; the
//             bias gradient is a ones-column appended to X — no separate reduce)
// C[M][N] = A[M][K] * B[N][K]^T; `ta`/`tb`: the operand is stored K-major.
//
// gfx950 structure: 256 threads = 4 waves, BK = 32 (one 16x16x32 bf16 MFMA
// K-step), LDS double buffer + register prefetch (the global loads of tile
// k+1 are in flight while tile k is multiplied; one barrier per K-step).
// K-major (transposed) bf16 operands are staged exactly as they sit in memory
// (16-byte row copies) and read with ds_read_b64_tr_b16, the CDNA4 hardware
// transpose read, instead of being transposed element by element.
#include "kernels.h"
#include "mcc/ab.h"
#include "mfma.h"

#include <algorithm>

namespace mcc {
namespace gpu {

namespace {

typedef short v4s __attribute__((ext_vector_type(4)));

typedef __attribute__((address_space(3))) v4s lds_v4s;

// ds_read_b64_tr_b16 (cdna_hip_programming.md §5.5 T10); `p` points into LDS.
__device__ __forceinline__ v4s ds_tr16(const bf16* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)(const_cast<bf16*>(p)));
}

template <typename T>
__device__ __forceinline__ float ld_elem(const T* base, int ld, bool trans, int r, int k, int R, int K) {
  if (r >= R || k >= K) return 0.f;
  return to_f(trans ? base[(size_t)k * ld + r] : base[(size_t)r * ld + k]);
}

// One operand tile (ROWS x 32) moving global -> registers -> LDS.
// Layout in LDS: !TRANS:        [ROWS][LDK] (k contiguous);
//                TRANS && TR:   [32][ROWS + 8] (rows of k, read by ds_read_b64_tr_b16);
//                TRANS && !TR (fp32): [32][ROWS + 4] (rows of k as they sit in
//                  memory, 16-byte stores; a fragment is 8 ds_read_b32 down a
//                  column -- the f32 MFMA takes one k per lane per instruction,
//                  so nothing needs transposing.  Until round 4 these tiles
//                  were transposed by 8 scalar LDS stores per vector, 4-way
//                  bank-conflicted: ref fp32 FC1 weight gradient 2.1 ms.)
template <typename T, int ROWS, bool TRANS, bool TR>
struct Operand {
  typedef typename Vec8<T>::type V8;
  static constexpr int LDK = 32 + (sizeof(T) == 2 ? 8 : 4);
  static constexpr int LDM = ROWS + (TR ? 8 : 4);
  static constexpr int ELEMS = TRANS ? 32 * LDM : ROWS * LDK;
  static constexpr int NVEC = ROWS * 4;  // 8-element vectors per tile
  static constexpr int PER = (NVEC + 255) / 256;
  V8 r[PER];

  __device__ __forceinline__ void load(const T* X, int ld, int r0, int k0, int R, int K, int ones_row) {
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      const int v = threadIdx.x + j * 256;
      if (v >= NVEC) break;
      if (!TRANS) {
        const int row = v >> 2, kv = (v & 3) * 8;
        const int gr = r0 + row, gk = k0 + kv;
        if (gr < R && gr != ones_row && gk + 8 <= K) {
          r[j] = load8(X + (size_t)gr * ld + gk);
        } else {
#pragma unroll
          for (int e = 0; e < 8; ++e)
            r[j][e] = from_f<T>(gr == ones_row ? (gk + e < K ? 1.f : 0.f) : ld_elem(X, ld, false, gr, gk + e, R, K));
        }
      } else {
        constexpr int RV = ROWS / 8;
        const int kr = v / RV, rv = (v - kr * RV) * 8;
        const int gk = k0 + kr, gr = r0 + rv;
        if (gk < K && gr + 8 <= R && (ones_row < gr || ones_row >= gr + 8)) {
          r[j] = load8(X + (size_t)gk * ld + gr);
        } else {
#pragma unroll
          for (int e = 0; e < 8; ++e)
            r[j][e] = from_f<T>((gr + e) == ones_row ? (gk < K ? 1.f : 0.f) : ld_elem(X, ld, true, gr + e, gk, R, K));
        }
      }
    }
  }

  __device__ __forceinline__ void store(T* lds) const {
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      const int v = threadIdx.x + j * 256;
      if (v >= NVEC) break;
      if (!TRANS) {
        store8(lds + (v >> 2) * LDK + (v & 3) * 8, r[j]);
      } else {
        constexpr int RV = ROWS / 8;
        const int kr = v / RV, rv = (v - kr * RV) * 8;
        store8(lds + kr * LDM + rv, r[j]);
      }
    }
  }

  // MFMA fragment of the 16-row block starting at `row0`: lane (r16, g) gets
  // rows row0 + r16, k = 8g .. 8g+7.
  __device__ __forceinline__ static V8 frag(const T* lds, int row0, int r16, int g) {
    if constexpr (TRANS && TR) {
      // lane 4q+p of each 16-lane group addresses row (k) q, columns 4p..4p+3
      const int q = r16 >> 2, pp = r16 & 3;
      const bf16* b = reinterpret_cast<const bf16*>(lds);
      const bf16x4 lo = __builtin_bit_cast(bf16x4, ds_tr16(b + (8 * g + q) * LDM + row0 + 4 * pp));
      const bf16x4 hi = __builtin_bit_cast(bf16x4, ds_tr16(b + (8 * g + 4 + q) * LDM + row0 + 4 * pp));
      return __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
    } else if constexpr (TRANS) {
      V8 v;
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = lds[(8 * g + e) * LDM + row0 + r16];
      return v;
    } else {
      return load8(lds + (row0 + r16) * LDK + 8 * g);
    }
  }
};

template <typename T, int BM, int BN, int WAVES_M, bool TA, bool TB>
__global__ void __launch_bounds__(256) gemm_kernel(GemmParams p) {
  typedef typename Vec8<T>::type V8;
  constexpr bool TR = sizeof(T) == 2;
  typedef Operand<T, BM, TA, TR> OpA;
  typedef Operand<T, BN, TB, TR> OpB;
  constexpr int WAVES_N = 4 / WAVES_M;
  constexpr int WTM = BM / WAVES_M, WTN = BN / WAVES_N;
  constexpr int FM = WTM / 16, FN = WTN / 16;
  __shared__ __attribute__((aligned(16))) T As[2][OpA::ELEMS];
  __shared__ __attribute__((aligned(16))) T Bs[2][OpB::ELEMS];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r16 = lane & 15, g = lane >> 4;
  const int wm = wave / WAVES_N, wn = wave % WAVES_N;
  const int m0 = blockIdx.y * BM, n0 = blockIdx.x * BN;
  const int kchunks = cdiv(p.K, 32);
  const int per = cdiv(kchunks, (int)gridDim.z);
  const int kc0 = blockIdx.z * per, kc1 = min(kchunks, kc0 + per);
  const T* A = static_cast<const T*>(p.A);
  const T* B = static_cast<const T*>(p.B);

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // EPI_DACT: the act' operand (4 outputs per fragment per lane) is requested
  // before the K loop, so its latency hides behind the GEMM instead of
  // stalling the epilogue (short-K data gradients: K = 10..120 is 1-4 chunks)
  constexpr bool kPreAux = FM * FN <= 4;
  float auxv[kPreAux ? FM : 1][kPreAux ? FN : 1][4];
  if constexpr (kPreAux) {
    if (p.epi == EPI_DACT && p.act != ACT_NONE) {
      const T* aux = static_cast<const T*>(p.aux);
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) {
          const int col = n0 + wn * WTN + j * 16 + r16;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int row = m0 + wm * WTM + i * 16 + 4 * g + e;
            auxv[i][j][e] = (col < p.N && row < p.M) ? to_f(aux[(size_t)row * p.ldaux + col]) : 0.f;
          }
        }
    }
  }

  OpA la;
  OpB lb;
  if (kc0 < kc1) {
    la.load(A, p.lda, m0, kc0 * 32, p.M, p.K, -1);
    lb.load(B, p.ldb, n0, kc0 * 32, p.N, p.K, p.ones_col);
    la.store(As[0]);
    lb.store(Bs[0]);
  }
  __syncthreads();
  int buf = 0;
  for (int kc = kc0; kc < kc1; ++kc) {
    const bool more = kc + 1 < kc1;
    if (more) {  // prefetch tile k+1 (in flight during the MFMAs below)
      la.load(A, p.lda, m0, (kc + 1) * 32, p.M, p.K, -1);
      lb.load(B, p.ldb, n0, (kc + 1) * 32, p.N, p.K, p.ones_col);
    }
    V8 a[FM], b[FN];
#pragma unroll
    for (int i = 0; i < FM; ++i) a[i] = OpA::frag(As[buf], wm * WTM + i * 16, r16, g);
#pragma unroll
    for (int j = 0; j < FN; ++j) b[j] = OpB::frag(Bs[buf], wn * WTN + j * 16, r16, g);
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) acc[i][j] = mma(acc[i][j], a[i], b[j]);
    if (more) {
      la.store(As[buf ^ 1]);
      lb.store(Bs[buf ^ 1]);
    }
    __syncthreads();
    buf ^= 1;
  }

  T* C = static_cast<T*>(p.C);
  const T* aux = static_cast<const T*>(p.aux);
#pragma unroll
  for (int i = 0; i < FM; ++i) {
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int col = n0 + wn * WTN + j * 16 + r16;
      if (col >= p.N) continue;
      const float bv = (p.epi == EPI_BIAS_ACT || p.epi == EPI_LOGITS) && p.bias ? p.bias[col] : 0.f;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int row = m0 + wm * WTM + i * 16 + 4 * g + e;
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
            if (p.act != ACT_NONE) {
              float y;
              if constexpr (kPreAux) y = auxv[i][j][e];
              else y = to_f(aux[(size_t)row * p.ldaux + col]);
              d = act_grad_y(p.act, y);
            }
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

// Sum split-K partials.  L lanes per output (L = 4, 16 or 64 by the number
// of partials S), each summing every L-th partial with two accumulators (the
// loads of ~S/L partials are in flight together), then a fixed-order
// shuffle reduction: deterministic, and the dependency chain is S/(2L) loads
// instead of S (a 512-slab head reduce was 22 us on one lane per output).
template <int L>
__global__ void __launch_bounds__(256) dw_reduce_kernel(DwReduceParams p) {
  const int kc = p.kfeat + 1;
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t j = t / L;
  const int sl = (int)(t & (L - 1));
  const bool ok = j < (int64_t)p.Nout * kc;
  const int n = ok ? (int)(j / kc) : 0, k = ok ? (int)(j - (int64_t)n * kc) : 0;
  const float* src = p.part + (size_t)n * p.ldp + k;
  const size_t st = (size_t)p.partial_stride;
  float a0 = 0.f, a1 = 0.f;
  if (ok) {
    int s = sl;
    for (; s + L < p.S; s += 2 * L) {
      a0 += src[(size_t)s * st];
      a1 += src[(size_t)(s + L) * st];
    }
    for (; s < p.S; s += L) a0 += src[(size_t)s * st];
  }
  float acc = a0 + a1;
#pragma unroll
  for (int o = 1; o < L; o <<= 1) acc += __shfl_xor(acc, o);
  if (!ok || sl != 0) return;
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

// The same sum for many outputs (FC weight gradients: the reference model's
// FC2 has 40,200 over 896 slabs): a wave takes 64 CONSECUTIVE outputs, so
// every load is one contiguous 256-byte run of one slab (the L-lane form
// reads 64 slabs per instruction, one 4-byte word of each); the WV waves of a
// workgroup split the slabs and meet in LDS in a fixed order.
template <int WV>
__global__ void __launch_bounds__(64 * WV) dw_reduce_cols_kernel(DwReduceParams p) {
  __shared__ float part[WV][64];
  const int kc = p.kfeat + 1;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t j = (int64_t)blockIdx.x * 64 + lane;
  const bool ok = j < (int64_t)p.Nout * kc;
  const int n = ok ? (int)(j / kc) : 0, k = ok ? (int)(j - (int64_t)n * kc) : 0;
  const float* src = p.part + (size_t)n * p.ldp + k;
  const size_t st = (size_t)p.partial_stride;
  float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
  int s = w;
  for (; s + 3 * WV < p.S; s += 4 * WV) {
    a0 += src[(size_t)s * st];
    a1 += src[(size_t)(s + WV) * st];
    a2 += src[(size_t)(s + 2 * WV) * st];
    a3 += src[(size_t)(s + 3 * WV) * st];
  }
  for (; s < p.S; s += WV) a0 += src[(size_t)s * st];
  part[w][lane] = (a0 + a1) + (a2 + a3);
  __syncthreads();
  if (w != 0 || !ok) return;
  float acc = part[0][lane];
#pragma unroll
  for (int v = 1; v < WV; ++v) acc += part[v][lane];
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

// Finishing pass of a split-K forward GEMM: out = epi(sum_s part[s] + bias).
template <typename T>
__global__ void __launch_bounds__(256) splitk_finish_kernel(GemmParams p, const float* __restrict__ part, int S) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (int64_t)p.M * p.N) return;
  const int m = (int)(t / p.N), n = (int)(t - (int64_t)m * p.N);
  const size_t stride = (size_t)p.M * p.ldc;
  const float* src = part + (size_t)m * p.ldc + n;
  float a0 = 0.f, a1 = 0.f;
  int z = 0;
  for (; z + 1 < S; z += 2) {
    a0 += src[z * stride];
    a1 += src[(z + 1) * stride];
  }
  if (z < S) a0 += src[z * stride];
  float v = a0 + a1 + (p.bias ? p.bias[n] : 0.f);
  if (p.epi == EPI_LOGITS) p.Cf[(size_t)m * p.ldc + n] = v;
  else static_cast<T*>(p.C)[(size_t)m * p.ldc + n] = from_f<T>(act_apply(p.act, v));
}

template <typename T, int BM, int BN, int WAVES_M>
void launch_cfg(const GemmParams& p, hipStream_t s) {
  const dim3 grid((unsigned)cdiv(p.N, BN), (unsigned)cdiv(p.M, BM), (unsigned)p.splitk), block(256);
  if (!p.ta && !p.tb) hipLaunchKernelGGL((gemm_kernel<T, BM, BN, WAVES_M, false, false>), grid, block, 0, s, p);
  else if (!p.ta && p.tb) hipLaunchKernelGGL((gemm_kernel<T, BM, BN, WAVES_M, false, true>), grid, block, 0, s, p);
  else if (p.ta && !p.tb) hipLaunchKernelGGL((gemm_kernel<T, BM, BN, WAVES_M, true, false>), grid, block, 0, s, p);
  else hipLaunchKernelGGL((gemm_kernel<T, BM, BN, WAVES_M, true, true>), grid, block, 0, s, p);
}

template <typename T>
void launch_gemm(const GemmParams& p, hipStream_t s) {
  // Tile choice: the largest tile that still gives >= 2 workgroups per CU
  // (latency of the staging pipeline is hidden across co-resident groups);
  // skinny-N problems (FC layers, N <= 128) use a full-width N tile so A is
  // streamed once.
  auto wgs = [&](int bm, int bn) { return (int64_t)cdiv(p.M, bm) * cdiv(p.N, bn) * p.splitk; };
  const int64_t want = 512;
  // fp32: 64x64 tiles throughout (the f32 operands double the LDS and
  // register footprint of a tile; measured on LeNet-5 fp32, B = 131072, all
  // FC GEMMs on one shape: 64x64 21.53 M img/s, 32x64 21.46 M, the bf16
  // choice below 20.83 M, 64x128 19.90 M, 32x128 19.91 M, 128x128 19.26 M)
  if (sizeof(T) == 4) {
    if (wgs(64, 64) >= 256 || p.M > 32) launch_cfg<T, 64, 64, 2>(p, s);
    else launch_cfg<T, 32, 64, 2>(p, s);
    return;
  }
  if (p.N > 64 && p.N <= 128) {
    if (wgs(64, 128) >= want) launch_cfg<T, 64, 128, 2>(p, s);
    else launch_cfg<T, 32, 128, 1>(p, s);
  } else if (p.N <= 64) {
    if (wgs(64, 64) >= want) launch_cfg<T, 64, 64, 2>(p, s);
    else launch_cfg<T, 32, 64, 2>(p, s);
  } else {
    if (wgs(128, 128) >= want) launch_cfg<T, 128, 128, 2>(p, s);
    else if (wgs(64, 128) >= want) launch_cfg<T, 64, 128, 2>(p, s);
    else if (wgs(64, 64) >= want || p.M > 32) launch_cfg<T, 64, 64, 2>(p, s);
    else launch_cfg<T, 32, 64, 2>(p, s);
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

int gemm_fwd_splitk(int M, int N, int K) {
  // long-K bf16 layers with M, N >= 256 (VGG-11 FC1: 640 x 4096 x 25088):
  // split K so that 128x128 tiles fill the chip (launch_gemm then picks them)
  // -- 64x64 tiles over the whole K ran at ~310 TFLOP/s
  if (M >= 256 && N >= 256 && K >= 8192) {
    const int64_t t128 = (int64_t)cdiv(M, 128) * cdiv(N, 128);
    int sk = (int)std::min<int64_t>(8, std::max<int64_t>(1, (1024 + t128 - 1) / t128));
    return std::max(1, std::min(sk, K / 1024));
  }
  const int64_t tiles = (int64_t)cdiv(M, 64) * cdiv(N, 64);
  if (tiles >= 512 || K < 1024) return 1;
  int sk = (int)std::min<int64_t>(16, 1024 / std::max<int64_t>(1, tiles));
  sk = std::min(sk, K / 256);
  return std::max(1, sk);
}

void gemm_splitk_fwd(DType t, const GemmParams& p0, float* scratch, int splitk, hipStream_t s) {
  MCC_CHECK(p0.epi == EPI_BIAS_ACT || p0.epi == EPI_LOGITS, "gemm_splitk_fwd: forward epilogues only");
  if (splitk <= 1) { gemm(t, p0, s); return; }
  GemmParams p = p0;
  p.epi = EPI_PARTIAL;
  p.Cf = scratch;
  p.splitk = splitk;
  p.partial_stride = (int64_t)p.M * p.ldc;
  gemm(t, p, s);
  const int64_t n = (int64_t)p0.M * p0.N;
  const dim3 grid((unsigned)((n + 255) / 256));
  if (t == DType::BF16) hipLaunchKernelGGL(splitk_finish_kernel<bf16>, grid, dim3(256), 0, s, p0, scratch, splitk);
  else hipLaunchKernelGGL(splitk_finish_kernel<float>, grid, dim3(256), 0, s, p0, scratch, splitk);
}

void dw_reduce(const DwReduceParams& p, hipStream_t s) {
  const int64_t n = (int64_t)p.Nout * (p.kfeat + 1);
  if (n >= 8192 && !ab_flag("dw_reduce_lanes")) {  // enough outputs to fill the chip 64 at a time
    hipLaunchKernelGGL(dw_reduce_cols_kernel<4>, dim3((unsigned)((n + 63) / 64)), dim3(256), 0, s, p);
    return;
  }
  if (p.S >= 256) hipLaunchKernelGGL(dw_reduce_kernel<64>, dim3((unsigned)((64 * n + 255) / 256)), dim3(256), 0, s, p);
  else if (p.S >= 64) hipLaunchKernelGGL(dw_reduce_kernel<16>, dim3((unsigned)((16 * n + 255) / 256)), dim3(256), 0, s, p);
  else hipLaunchKernelGGL(dw_reduce_kernel<4>, dim3((unsigned)((4 * n + 255) / 256)), dim3(256), 0, s, p);
}

}  // namespace gpu
}  // namespace mcc
