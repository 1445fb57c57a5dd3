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

constexpr int kFcThreads = 512;  // 8 waves: 256 measured 7.8 us/step slower over LeNet-5's five FC kernels (profiles/fc_waves_ab_r2.txt)
constexpr int kFcWaves = kFcThreads / 64;
constexpr int kFcRows = 16 * kFcWaves;  // rows per workgroup (16 per wave)
constexpr int kFcMaxChunks = 16;  // K <= 512
constexpr int kFcGroupTiles = 8;  // column tiles per staged output group (128 columns)
constexpr int kFcStageLd = kFcGroupTiles * 16 + 8;

typedef __attribute__((address_space(1))) void gvoid;
typedef __attribute__((address_space(3))) void lvoid;

// K chunks (of 32) the kernel is unrolled for: a power of two >= the real count
__host__ __device__ inline int fc_nchb(int K) {
  const int n = (K + 31) >> 5;
  return n <= 1 ? 1 : n <= 2 ? 2 : n <= 4 ? 4 : n <= 8 ? 8 : 16;
}
__host__ __device__ inline int fc_npad(int N) { return (N + 15) & ~15; }
// W is staged densely, exactly as packed in memory ([N][ldw]); reads run up
// to NCH*32 columns past a row start, so the region is padded with zeros
__host__ __device__ inline int fc_welems(int N, int ldw, int K) {
  return ((fc_npad(N) * ldw + fc_nchb(K) * 32 + 7) & ~7);
}
__host__ __device__ inline size_t fc_lds(int N, int ldw, int K) {
  return (size_t)fc_welems(N, ldw, K) * 2 + (size_t)fc_npad(N) * 4 + (size_t)kFcWaves * 16 * kFcStageLd * 2;
}

// P (persistent): large W (one or two workgroups per CU) is staged once per
// workgroup and reused over several row blocks; small W keeps one row block
// per workgroup (enough workgroups per CU to hide the A-fragment latency).
template <int EPI, int ACT, int NCH, bool P>
__global__ void __launch_bounds__(kFcThreads) fc_kernel(FcParams p0) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const FcParams& p = p0;
  const int cols = p.ldc;  // stored columns (up to the leading dim: its padding is written as 0)
  const int ldk = p.ldw;
  const int npad = fc_npad(p.N);
  const int wel = fc_welems(p.N, p.ldw, p.K);
  bf16* ws = reinterpret_cast<bf16*>(smem);
  float* bias_s = reinterpret_cast<float*>(smem + (size_t)wel * 2);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r16 = lane & 15, g = lane >> 4;
  bf16* stg = reinterpret_cast<bf16*>(smem + (size_t)wel * 2 + (size_t)npad * 4) + wave * 16 * kFcStageLd;
  long long* dbg = p.dbg ? p.dbg + ((size_t)blockIdx.x * kFcWaves + wave) * 4 : nullptr;
  if (dbg && lane == 0) dbg[0] = (long long)__builtin_amdgcn_s_memrealtime();

  // ---- W -> LDS: the packed [N][ldw] block is contiguous, so it moves as
  // 1 KB async global->LDS DMA pieces (64 lanes x 16 B, no registers, no
  // index math), piece i by wave i % 4; the tail is zeroed by plain stores ----
  {
    const bf16* W = static_cast<const bf16*>(p.W);
    const int wv = p.N * p.ldw;  // elements of real weights (multiple of 8)
    const int npieces = (wv + 511) >> 9;
    for (int i = wave; i < npieces; i += kFcThreads / 64) {
      const int e = i * 512 + lane * 8;
      if (e < wv) __builtin_amdgcn_global_load_lds((gvoid*)(W + e), (lvoid*)(ws + i * 512), 16, 0, 0);
    }
    const bf16x8 z = {};
    for (int e = wv + tid * 8; e < wel; e += kFcThreads * 8) store8(ws + e, z);
    for (int n = tid; n < npad; n += kFcThreads) bias_s[n] = (EPI != EPI_DACT && n < p.N && p.bias) ? p.bias[n] : 0.f;
  }

  // ---- this wave's A fragments, straight from HBM into registers.  K need
  // not be a multiple of 8: producers leave the leading-dim padding at 0.
  // Persistent: the workgroup keeps W and walks row blocks blockIdx.x,
  // +gridDim.x, ... (W is staged once per CU instead of once per 64 rows) ----
  const bf16* A = static_cast<const bf16*>(p.A);
  const int nrb = (p.M + kFcRows - 1) / kFcRows;
  bf16x8 a[NCH];
  auto load_a = [&](int rb) {
    const int arow = rb * kFcRows + wave * 16 + r16;
#pragma unroll
    for (int q = 0; q < NCH; ++q) {
      const int k = q * 32 + 8 * g;
      if (arow < p.M && k < p.K) a[q] = load8(A + (size_t)arow * p.lda + k);
      else a[q] = bf16x8{};
    }
  };
  load_a(blockIdx.x);
  if (dbg && lane == 0) dbg[1] = (long long)__builtin_amdgcn_s_memrealtime();
  __syncthreads();  // also drains the DMA (vmcnt)
  if (dbg && lane == 0) dbg[2] = (long long)__builtin_amdgcn_s_memrealtime();
  for (int rb = blockIdx.x; rb < (P ? nrb : (int)blockIdx.x + 1); rb += gridDim.x) {
  const int row0 = rb * kFcRows + wave * 16;
  // 16-byte act' operand loads (rows 16-byte aligned, the leading dim's
  // padding readable; otherwise per-element loads in the epilogue)
  const bool vaux = EPI == EPI_DACT && ACT != ACT_NONE && (p.ldaux & 7) == 0 && p.ldaux >= p0.ldc &&
                    (reinterpret_cast<uintptr_t>(p.aux) & 15) == 0;

  auto epilogue = [&](const f32x4& acc, int tile, int slot) {
    const int col = tile * 16 + r16;
    const bool cv = col < p.N;
    const float bv = bias_s[col];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = row0 + 4 * g + i;
      float v = acc[i] + bv;
      if (EPI == EPI_BIAS_ACT) {
        v = ACT == ACT_RELU ? fmaxf(v, 0.f) : (ACT == ACT_TANH ? tanhf(v) : v);
      } else if (EPI == EPI_DACT) {
        if (ACT != ACT_NONE && cv && row < p.M) {
          // the forward activation: pre-staged in this lane's own stage slot
          // (overwritten below with the result), or a 2-byte load
          const float y = vaux ? (float)stg[(4 * g + i) * kFcStageLd + slot * 16 + r16]
                               : (float)static_cast<const bf16*>(p.aux)[(size_t)row * p.ldaux + col];
          v *= ACT == ACT_RELU ? (y > 0.f ? 1.f : 0.f) : (1.f - y * y);
        }
      }
      if (EPI == EPI_LOGITS) {
        if (cv && row < p.M) p.Cf[(size_t)row * p.ldc + col] = v;
      } else {
        stg[(4 * g + i) * kFcStageLd + slot * 16 + r16] = (bf16)v;
      }
    }
  };

  const int ntiles = npad >> 4;
  for (int t0 = 0; t0 < ntiles; t0 += kFcGroupTiles) {
    const int tn = min(kFcGroupTiles, ntiles - t0);
    if (EPI == EPI_DACT && ACT != ACT_NONE && vaux) {
      // act' operand of the group: 16 rows x (tn*16) columns of the forward
      // activation as coalesced 16-byte loads into the wave's stage tile,
      // issued before the MFMAs (one 2-byte load per output element exposed
      // its latency in every epilogue)
      const int ncols = min(tn * 16, cols - t0 * 16);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int v = lane + 64 * j;
        const int r = v >> 4, c = (v & 15) * 8;
        const int row = row0 + r;
        bf16x8 y = {};
        if (c < ncols && row < p.M) y = load8(static_cast<const bf16*>(p.aux) + (size_t)row * p.ldaux + t0 * 16 + c);
        store8(stg + r * kFcStageLd + c, y);
      }
      __builtin_amdgcn_wave_barrier();
    }
    for (int tt = 0; tt < tn; tt += 2) {
      // two column tiles per pass: independent accumulator chains, all B
      // fragment reads unconditional (rows zero-padded to NCH*32) so they
      // can be issued ahead of the MFMAs; the odd tile may be a dummy
      const bool two = tt + 1 < tn;
      const bf16* wa = ws + ((t0 + tt) * 16 + r16) * ldk + 8 * g;
      const bf16* wb = two ? wa + 16 * ldk : wa;
      f32x4 c0 = {0.f, 0.f, 0.f, 0.f}, c1 = {0.f, 0.f, 0.f, 0.f};
      // all of the pair's B fragments in flight before the first MFMA
      // (left to itself the compiler keeps only ~2 reads ahead, exposing the
      // LDS latency on every MFMA)
      bf16x8 ba[NCH], bb[NCH];
#pragma unroll
      for (int q = 0; q < NCH; ++q) {
        ba[q] = load8(wa + q * 32);
        bb[q] = load8(wb + q * 32);
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int q = 0; q < NCH; ++q) {
        c0 = mma(c0, a[q], ba[q]);
        c1 = mma(c1, a[q], bb[q]);
      }
      epilogue(c0, t0 + tt, tt);
      if (two) epilogue(c1, t0 + tt + 1, tt + 1);
    }
    if (EPI == EPI_LOGITS) continue;
    // wave-private tile -> 16 rows x (tn*16) columns, 16-byte stores (ldc % 8 == 0)
    __builtin_amdgcn_wave_barrier();
    const int c0 = t0 * 16;
    const int ncols = min(tn * 16, cols - c0);  // up to the leading dim (padding columns written as 0)
    bf16* C = static_cast<bf16*>(p.C);
#pragma unroll
    for (int j = 0; j < 4; ++j) {  // 16 rows x 16 vectors of 8 columns, 4 per lane
      const int v = lane + 64 * j;
      const int r = v >> 4, c = (v & 15) * 8;
      const int row = row0 + r;
      if (c < ncols && row < p.M) store8(C + (size_t)row * p.ldc + c0 + c, load8(stg + r * kFcStageLd + c));
    }
    __builtin_amdgcn_wave_barrier();
  }
  if (P && rb + (int)gridDim.x < nrb) load_a(rb + gridDim.x);
  }  // row blocks
  if (dbg && lane == 0) dbg[3] = (long long)__builtin_amdgcn_s_memrealtime();
}

template <int E, int A>
struct EpiTag {
  static constexpr int epi = E, act = A;
};

}  // namespace

bool fc_supported(int N, int K) {
  return N > 0 && K > 0 && K <= kFcMaxChunks * 32 && fc_lds(N, (K + 7) & ~7, K) <= 160 * 1024;
}

void fc_forward(const FcParams& p, hipStream_t s) {
  MCC_CHECK(fc_supported(p.N, p.K), "fc_forward: shape outside the weights-resident regime");
  MCC_CHECK(p.lda % 8 == 0 && p.ldw % 8 == 0 && p.lda >= ((p.K + 7) & ~7) && p.ldw >= ((p.K + 7) & ~7) &&
                (p.epi == EPI_LOGITS || p.ldc % 8 == 0),
            "fc_forward: leading dims must be multiples of 8 covering K");
  if (p.M <= 0) return;
  const FcParams& pl = p;
  // (a column split of a W that fills a CU over blockIdx.y measured slower
  // both ways with 8-wave workgroups -- LeNet-5 FC1 dX 39.6 -> 45.0 us, forward
  // 34.9 -> 47.7 us, profiles/fc_split_ab_r2.txt -- and was removed in round 3)
  const size_t lds = fc_lds(p.N, p.ldw, p.K);
  // persistent (as many workgroups as the LDS lets every CU hold) when W
  // limits the CU to one or two workgroups
  const int per_cu = std::max(1, std::min(8, (int)((160 * 1024) / (lds + 1024))));
  const bool persist = per_cu <= 2;
  const dim3 grid((unsigned)(persist ? std::min(cdiv(p.M, kFcRows), 256 * per_cu) : cdiv(p.M, kFcRows))),
      block(kFcThreads);
  MCC_CHECK(lds <= 160 * 1024, "fc_forward: weights do not fit in LDS");
  const int nchb = fc_nchb(p.K);
  auto go = [&](auto kern) { hipLaunchKernelGGL(kern, grid, block, lds, s, pl); };
  auto by_nch = [&](auto tag) {
    constexpr int EPI = decltype(tag)::epi, ACT = decltype(tag)::act;
    switch (nchb) {
      case 1: (persist ? go(fc_kernel<EPI, ACT, 1, true>) : go(fc_kernel<EPI, ACT, 1, false>)); break;
      case 2: (persist ? go(fc_kernel<EPI, ACT, 2, true>) : go(fc_kernel<EPI, ACT, 2, false>)); break;
      case 4: (persist ? go(fc_kernel<EPI, ACT, 4, true>) : go(fc_kernel<EPI, ACT, 4, false>)); break;
      case 8: (persist ? go(fc_kernel<EPI, ACT, 8, true>) : go(fc_kernel<EPI, ACT, 8, false>)); break;
      default: (persist ? go(fc_kernel<EPI, ACT, 16, true>) : go(fc_kernel<EPI, ACT, 16, false>)); break;
    }
  };
  switch (p.epi) {
    case EPI_BIAS_ACT:
      if (p.act == ACT_RELU) by_nch(EpiTag<EPI_BIAS_ACT, ACT_RELU>{});
      else if (p.act == ACT_TANH) by_nch(EpiTag<EPI_BIAS_ACT, ACT_TANH>{});
      else by_nch(EpiTag<EPI_BIAS_ACT, ACT_NONE>{});
      break;
    case EPI_LOGITS:
      by_nch(EpiTag<EPI_LOGITS, ACT_NONE>{});
      break;
    case EPI_DACT:
      if (p.act == ACT_RELU) by_nch(EpiTag<EPI_DACT, ACT_RELU>{});
      else if (p.act == ACT_TANH) by_nch(EpiTag<EPI_DACT, ACT_TANH>{});
      else by_nch(EpiTag<EPI_DACT, ACT_NONE>{});
      break;
    default:
      MCC_CHECK(false, "fc_forward: unsupported epilogue");
  }
}

}  // namespace gpu
}  // namespace mcc
