// Fully-connected layers as "weights-resident" MFMA GEMMs (bf16).
//
// Reference: Layer_feedForw_full (cnn.c:113-152) and the dX part of
// Layer_feedBack_full (cnn.c:154-173), per sample in fp64.  Here, for a
// minibatch of M samples: Y = act(X W^T + b) (forward), logits (last layer,
// fp32), or dX = (dY W) * act'(Xprev) (data gradient, with the W^T shadow as
// the weight operand).
//
// Shape regime: M (batch) is large, N and K are a few hundred at most, so
// the whole weight matrix (<= ~110 KB bf16) fits in one CU's LDS.  A
// workgroup stages W once (16-byte copies, rows skewed by 16 B so a
// fragment read is bank-conflict free), then each of its 4 waves owns 16
// rows of the batch: the wave's A fragments for ALL K chunks are loaded
// straight from HBM into registers (no LDS round trip, read exactly once)
// and reused against every column tile of W.  Results go through a small
// wave-private LDS tile and leave as 16-byte row stores.  No K loop barriers.
#include <algorithm>

#include "kernels.h"
#include "mfma.h"

namespace mcc {
namespace gpu {

namespace {

constexpr int kFcThreads = 256;
constexpr int kFcRows = 64;       // rows per workgroup (16 per wave)
constexpr int kFcMaxChunks = 16;  // K <= 512
constexpr int kFcGroupTiles = 8;  // column tiles per staged output group (128 columns)
constexpr int kFcStageLd = kFcGroupTiles * 16 + 8;

__host__ __device__ inline int fc_ldk(int K) { return ((K + 31) & ~31) + 8; }
__host__ __device__ inline int fc_npad(int N) { return (N + 15) & ~15; }
__host__ __device__ inline size_t fc_lds(int N, int K) {
  return (size_t)fc_npad(N) * fc_ldk(K) * 2 + (size_t)4 * 16 * kFcStageLd * 2;
}

template <int EPI, int ACT>
__global__ void __launch_bounds__(kFcThreads) fc_kernel(FcParams p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int ldk = fc_ldk(p.K);
  const int npad = fc_npad(p.N);
  const int nch = (p.K + 31) >> 5;
  bf16* ws = reinterpret_cast<bf16*>(smem);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r16 = lane & 15, g = lane >> 4;
  bf16* stg = reinterpret_cast<bf16*>(smem + (size_t)npad * ldk * 2) + wave * 16 * kFcStageLd;
  long long* dbg = p.dbg ? p.dbg + ((size_t)blockIdx.x * 4 + wave) * 4 : nullptr;
  if (dbg && lane == 0) dbg[0] = (long long)__builtin_amdgcn_s_memrealtime();

  // ---- W -> LDS (zero padding rows/columns: they meet the K / N tails) ----
  {
    // U independent 16-byte loads in flight per thread before their LDS
    // stores (a load->store loop would pay the L2 latency per vector)
    constexpr int U = 16;
    const bf16* W = static_cast<const bf16*>(p.W);
    const int vpr = ldk >> 3;  // 16-byte vectors per LDS row
    const int nv = npad * vpr;
    for (int v0 = tid; v0 < nv; v0 += U * kFcThreads) {
      bf16x8 x[U];
      int off[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int v = v0 + u * kFcThreads;
        const int r = v / vpr, c = (v - r * vpr) * 8;
        off[u] = v < nv ? r * ldk + c : -1;
        if (v < nv && r < p.N && c < p.K) {  // packed weights: zero columns up to ldw
          x[u] = load8(W + (size_t)r * p.ldw + c);
        } else {
#pragma unroll
          for (int j = 0; j < 8; ++j) x[u][j] = (bf16)0.f;
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u)
        if (off[u] >= 0) store8(ws + off[u], x[u]);
    }
  }

  // ---- this wave's A fragments, straight from global.  K need not be a
  // multiple of 8: the producers leave the leading-dim padding columns 0 ----
  const int row0 = blockIdx.x * kFcRows + wave * 16;
  const int arow = row0 + r16;
  const bf16* A = static_cast<const bf16*>(p.A);
  bf16x8 a[kFcMaxChunks];
#pragma unroll
  for (int q = 0; q < kFcMaxChunks; ++q) {
    const int k = q * 32 + 8 * g;
    if (q < nch && arow < p.M && k < p.K) {
      a[q] = load8(A + (size_t)arow * p.lda + k);
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) a[q][j] = (bf16)0.f;
    }
  }
  if (dbg && lane == 0) dbg[1] = (long long)__builtin_amdgcn_s_memrealtime();
  __syncthreads();
  if (dbg && lane == 0) dbg[2] = (long long)__builtin_amdgcn_s_memrealtime();

  const int ntiles = npad >> 4;
  for (int t0 = 0; t0 < ntiles; t0 += kFcGroupTiles) {
    const int tn = min(kFcGroupTiles, ntiles - t0);
    for (int tt = 0; tt < tn; ++tt) {
      const int col = (t0 + tt) * 16 + r16;
      const bf16* wrow = ws + col * ldk + 8 * g;
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int q = 0; q < kFcMaxChunks; ++q)
        if (q < nch) acc = mma(acc, a[q], load8(wrow + q * 32));
      const bool cv = col < p.N;
      float bv = 0.f;
      if (EPI != EPI_DACT && cv && p.bias) bv = p.bias[col];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int row = row0 + 4 * g + i;
        float v = acc[i] + bv;
        if (EPI == EPI_BIAS_ACT) {
          v = ACT == ACT_RELU ? fmaxf(v, 0.f) : (ACT == ACT_TANH ? tanhf(v) : v);
        } else if (EPI == EPI_DACT) {
          if (ACT != ACT_NONE && cv && row < p.M) {
            const float y = (float)static_cast<const bf16*>(p.aux)[(size_t)row * p.ldaux + col];
            v *= ACT == ACT_RELU ? (y > 0.f ? 1.f : 0.f) : (1.f - y * y);
          }
        } else if (EPI == EPI_LOGITS) {
          if (cv && row < p.M) p.Cf[(size_t)row * p.ldc + col] = v;
          continue;
        }
        stg[(4 * g + i) * kFcStageLd + tt * 16 + r16] = (bf16)v;
      }
    }
    if (EPI == EPI_LOGITS) continue;
    // wave-private tile -> 16 rows x (tn*16) columns, 16-byte stores (ldc % 8 == 0)
    __builtin_amdgcn_wave_barrier();
    const int c0 = t0 * 16;
    const int ncols = min(tn * 16, p.ldc - c0);  // write up to the leading dim (pad columns too)
    const int vpr = ncols >> 3;
    bf16* C = static_cast<bf16*>(p.C);
    for (int v = lane; v < 16 * vpr; v += 64) {
      const int r = v / vpr, c = (v - r * vpr) * 8;
      const int row = row0 + r;
      if (row < p.M) store8(C + (size_t)row * p.ldc + c0 + c, load8(stg + r * kFcStageLd + c));
    }
    __builtin_amdgcn_wave_barrier();
  }
  if (dbg && lane == 0) dbg[3] = (long long)__builtin_amdgcn_s_memrealtime();
}

}  // namespace

bool fc_supported(int N, int K) {
  return N > 0 && K > 0 && K <= kFcMaxChunks * 32 && fc_lds(N, K) <= 160 * 1024;
}

void fc_forward(const FcParams& p, hipStream_t s) {
  MCC_CHECK(fc_supported(p.N, p.K), "fc_forward: shape outside the weights-resident regime");
  MCC_CHECK(p.lda % 8 == 0 && p.ldw % 8 == 0 && p.lda >= ((p.K + 7) & ~7) && p.ldw >= ((p.K + 7) & ~7) &&
                (p.epi == EPI_LOGITS || p.ldc % 8 == 0),
            "fc_forward: leading dims must be multiples of 8 covering K");
  if (p.M <= 0) return;
  const dim3 grid((unsigned)cdiv(p.M, kFcRows)), block(kFcThreads);
  const size_t lds = fc_lds(p.N, p.K);
  auto go = [&](auto kern) { hipLaunchKernelGGL(kern, grid, block, lds, s, p); };
  switch (p.epi) {
    case EPI_BIAS_ACT:
      if (p.act == ACT_RELU) go(fc_kernel<EPI_BIAS_ACT, ACT_RELU>);
      else if (p.act == ACT_TANH) go(fc_kernel<EPI_BIAS_ACT, ACT_TANH>);
      else go(fc_kernel<EPI_BIAS_ACT, ACT_NONE>);
      break;
    case EPI_LOGITS:
      go(fc_kernel<EPI_LOGITS, ACT_NONE>);
      break;
    case EPI_DACT:
      if (p.act == ACT_RELU) go(fc_kernel<EPI_DACT, ACT_RELU>);
      else if (p.act == ACT_TANH) go(fc_kernel<EPI_DACT, ACT_TANH>);
      else go(fc_kernel<EPI_DACT, ACT_NONE>);
      break;
    default:
      MCC_CHECK(false, "fc_forward: unsupported epilogue");
  }
}

}  // namespace gpu
}  // namespace mcc
