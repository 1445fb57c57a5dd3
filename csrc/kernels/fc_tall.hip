// Tall-skinny FC GEMM for a large batch and a long reduction whose weights do
// not fit in LDS: the reference model's FC1 (1568 -> 200, cnn.c:416-428,
// Layer_feedForw_full cnn.c:113-152) forward, and its data gradient
// (200 -> 1568, Layer_feedBack_full cnn.c:154-173) as the same GEMM with the
// W^T copy.
//
//   out[m][n] = epi( sum_k A[m][k] * W[n][k] )   m < M (batch), n < N, k < K
//
// Tile: 128 batch rows x 224 output columns (14 fragments: N = 200 wastes
// 11 %, where the 128x128 implicit-GEMM kernel computed two N tiles and 22 %
// padding), 8 waves = 4 (rows, 32 each) x 2 (columns, 112 each), 14
// v_mfma_f32_16x16x32_bf16 accumulators per wave.  The MFMA orientation is
// transposed -- rows = output columns, columns = batch rows -- so a lane
// holds 4 consecutive outputs of one batch row and stores them as one 8-byte
// write.  K moves in 32-deep stages (A rows then W rows, 24 KB) through a
// 3-deep ring of LDS buffers filled by global->LDS DMA (16 B per lane,
// wave-uniform destination): two stages in flight while one is multiplied,
// one barrier per stage, and every iteration issues the same number of DMAs
// per wave (past K: the zero page; weight pieces wholly past N: none, their
// rows zero-filled once) so the wait is a fixed per-wave vmcnt.  73 KB of LDS:
// two workgroups per CU, whose load / multiply phases interleave (a
// persistent one-workgroup-per-CU variant with a 6-deep ring and deferred
// epilogues measured 36 % slower: at 256 workgroups a CU still busy with the
// previous kernel's tail delays its whole share).  The bf16 forward of the
// 224-column tiles is the exception: a 4-deep ring at one workgroup per CU
// (98 KB, three stages in flight) reads the streamed rows 12 % faster.  Rows are 64 B with the
// 16-byte segments XOR-swizzled by row bit 2 (tswz): every ds_read_b128
// phase covers all 64 banks once.  Batch rows past M (clamped)
// and weight rows past N (the zero page) cost no branch.
// fp32 (exact f32 products, f32 accumulate): the same 64-byte LDS rows hold
// 16 floats, so a stage is 16 deep and a lane's 16-byte fragment read feeds
// four v_mfma_f32_16x16x4_f32 (k = 4g .. 4g + 3); MFMA-bound at 32 cycles
// per instruction.
#include <algorithm>
#include <type_traits>

#include "kernels.h"
#include "mfma.h"

namespace mcc {
namespace gpu {
namespace {

typedef __attribute__((address_space(1))) void gvoid;
typedef __attribute__((address_space(3))) void lvoid;

constexpr int kTT = 512;                 // threads (8 waves)
constexpr int kTM = 128;                 // batch rows per tile
#ifndef MCC_TALL_NS
#define MCC_TALL_NS 4  // ring depth of the bf16 224-column forward (one workgroup per CU)
#endif
constexpr int kTNS = 3;                  // ring depth: 2 stages in flight (bf16 forward: 4, see fc_tall)
constexpr int kTXBytes = kTM * 64;
// NF fragments per wave column: tile width TN = 32 NF output columns (7: 224
// for the ref model's FC1; 4: 128 for LeNet-5's FC1 120), W rows staged per
// stage rounded up to 128 (one DMA round of the 8 waves), LDS per workgroup
template <int NF, int NS = kTNS> struct TallGeom {
  static constexpr int TN = 32 * NF;
  static constexpr int WR = (TN + 127) / 128 * 128;
  static constexpr int DMAS = 1 + WR / 128;  // per wave per stage
  static constexpr int STAGE = kTXBytes + WR * 64;
  static constexpr int LDS = NS * STAGE;     // 3 stages: 73,728 B (NF 7) / 49,152 B (NF 4)
};

__device__ __attribute__((aligned(64))) const unsigned short kTallZero[32] = {0};

// 16-byte segment swizzle of a 64-byte row: physical segment = logical ^
// tswz(row).  ds_read_b128 serves a wave in four 16-lane phases, lanes
// {0-3, 12-15, 20-27}, {4-11, 16-19, 28-31} and the same +32
// (MI355X_MICROARCH.md, LDS table), not 16 consecutive lanes: with lane
// (g, r) reading segment g of row r, `(row >> 2) & 3` put two lanes of every
// phase on the same banks (PMC: 50 % conflict cycles); `2 * ((row >> 2) & 1)`
// gives each phase all 64 banks once.
__device__ __forceinline__ int tswz(int row) { return ((row >> 2) & 1) << 1; }

template <typename T, int NF, int ACT, bool BIAS, int NS>
__global__ void __launch_bounds__(kTT, NS == 3 ? 2 : 1) fc_tall_kernel(FcTallParams p) {
  using Gm = TallGeom<NF, NS>;
  constexpr int kTN = Gm::TN, DM = Gm::DMAS;
  constexpr int EPR = 64 / (int)sizeof(T);  // elements per 64-byte row = K per stage
  constexpr int EPS = 16 / (int)sizeof(T);  // elements per 16-byte segment
  typedef typename std::conditional<sizeof(T) == 2, bf16x8, f32x4>::type V;
  extern __shared__ __attribute__((aligned(16))) char tsm[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // (scalar: the per-wave DMA branches below)
  const int r16 = lane & 15, g = lane >> 4;
  const int wm = wave & 3, wn = wave >> 2;
  // XCD-aware order: consecutive column tiles of one row block share its A
  // rows in the same L2
  const int ntn = (p.N + kTN - 1) / kTN;
  const int nwg = gridDim.x;
  const int q8 = nwg >> 3, r8 = nwg & 7, xc = blockIdx.x & 7;
  const int tile = (xc < r8 ? xc * (q8 + 1) : r8 * (q8 + 1) + (xc - r8) * q8) + (blockIdx.x >> 3);
  const int tm = tile / ntn, tn = tile - tm * ntn;
  const int m0 = tm * kTM, n0 = tn * kTN;
  const T* zero = reinterpret_cast<const T*>(kTallZero);

  // ---- DMA sources: A piece = rows 16 wave .. +15 of the tile, W pieces =
  // rows 16 wave and 128 + 16 wave; lane -> row + (lane >> 2), physical
  // segment lane & 3 ----
  const T* src[DM];
  int sk[DM];
#pragma unroll
  for (int i = 0; i < DM; ++i) {
    const int row = i == 0 ? 16 * wave + (lane >> 2) : 16 * (wave + 8 * (i - 1)) + (lane >> 2);
    const int seg = (lane & 3) ^ tswz(row);
    sk[i] = seg * EPS;
    if (i == 0) {
#ifdef MCC_TALL_BLOCKED  // timing probe: A read as [M/128][K/EPR][128][EPR] blocks (values meaningless)
      src[i] = static_cast<const T*>(p.A) + (size_t)m0 * p.lda + row * EPR + seg * EPS;
#else
      src[i] = static_cast<const T*>(p.A) + (size_t)min(m0 + row, p.M - 1) * p.lda + seg * EPS;
#endif
    } else {
      const int n = n0 + row;
      src[i] = (row < kTN && n < p.N) ? static_cast<const T*>(p.W) + (size_t)n * p.ldw + seg * EPS : nullptr;
    }
  }
  const int nk = (p.K + EPR - 1) / EPR;
  // Weight pieces whose 16 rows all lie past N (or past the tile: N = 200 on
  // 224 / 256-row slots) are zero-filled once per ring slot and never
  // fetched again (they were zero-page DMAs every stage: 3 of the 16 weight
  // pieces of the reference FC1).  The count is fixed per wave, so each
  // wave's stage wait stays an exact vmcnt.
  bool dead[DM];
  int cnt = 1;
#pragma unroll
  for (int i = 0; i < DM; ++i) {
    const int rb = 16 * (wave + 8 * (i - 1));
    dead[i] = i > 0 && (rb >= kTN || n0 + rb >= p.N);
    cnt += (i > 0 && !dead[i]) ? 1 : 0;
#pragma unroll
    for (int sl = 0; sl < NS; ++sl)
      if (dead[i])
        *reinterpret_cast<f32x4*>(tsm + sl * Gm::STAGE + kTXBytes + (wave + 8 * (i - 1)) * 1024 + lane * 16) =
            f32x4{0.f, 0.f, 0.f, 0.f};
  }
  auto stage = [&](int kt) {  // cnt DMAs (past K: the zero page)
    char* dst = tsm + (kt % NS) * Gm::STAGE;
    const int k0 = kt * EPR;
#pragma unroll
    for (int i = 0; i < DM; ++i) {
      if (dead[i]) continue;
#ifdef MCC_TALL_BLOCKED
      const T* s = (src[i] && k0 + sk[i] < p.K) ? src[i] + (i == 0 ? (size_t)kt * kTM * EPR : (size_t)k0) : zero;
#else
      const T* s = (src[i] && k0 + sk[i] < p.K) ? src[i] + k0 : zero;
#endif
      char* d = i == 0 ? dst + wave * 1024 : dst + kTXBytes + (wave + 8 * (i - 1)) * 1024;
      __builtin_amdgcn_global_load_lds((gvoid*)s, (lvoid*)d, 16, 0, 0);
    }
  };

  f32x4 acc[NF][2];
#pragma unroll
  for (int f = 0; f < NF; ++f) acc[f][0] = acc[f][1] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int xrow0 = 32 * wm + r16;          // batch fragment b: A row xrow0 + 16 b
  const int wrow0 = 16 * NF * wn + r16;     // weight fragment f: W row wrow0 + 16 f

#pragma unroll
  for (int i = 0; i < NS - 1; ++i) stage(i);
  for (int kt = 0; kt < nk; ++kt) {
    // NS - 2 stages (DM DMAs each) were issued after stage kt: vmcnt((NS-2)
    // DM) = stage kt landed (in-order retirement); the barrier (an explicit
    // s_barrier: __syncthreads() would drain vmcnt) makes every wave's pieces
    // visible and frees the slot read in iteration kt - 1
    static_assert(NS >= 3 && NS <= 4 && DM <= 3, "the s_waitcnt below");
    const int vm = (NS - 2) * cnt;  // wave-uniform
    if (vm >= 6) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    else if (vm == 5) asm volatile("s_waitcnt vmcnt(5)" ::: "memory");
    else if (vm == 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else if (vm == 3) asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
    else if (vm == 2) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(1)" ::: "memory");
    asm volatile("s_barrier" ::: "memory");
    stage(kt + NS - 1);
    const char* xb_ = tsm + (kt % NS) * Gm::STAGE;
    const char* wb_ = xb_ + kTXBytes;
    V xb[2], wf[NF];
#pragma unroll
    for (int b = 0; b < 2; ++b) {
      const int row = xrow0 + 16 * b;
      xb[b] = *reinterpret_cast<const V*>(xb_ + row * 64 + ((g ^ tswz(row)) << 4));
    }
#pragma unroll
    for (int f = 0; f < NF; ++f) {
      const int row = wrow0 + 16 * f;
      wf[f] = *reinterpret_cast<const V*>(wb_ + row * 64 + ((g ^ tswz(row)) << 4));
    }
    __builtin_amdgcn_sched_barrier(0);  // all fragment reads in flight before the first MFMA
    if constexpr (sizeof(T) == 2) {
#pragma unroll
      for (int f = 0; f < NF; ++f)
#pragma unroll
        for (int b = 0; b < 2; ++b) acc[f][b] = mma(acc[f][b], wf[f], xb[b]);
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int f = 0; f < NF; ++f)
#pragma unroll
          for (int b = 0; b < 2; ++b)
            acc[f][b] = __builtin_amdgcn_mfma_f32_16x16x4f32(wf[f][j], xb[b][j], acc[f][b], 0, 0, 0);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the trailing zero-page DMAs

  // ---- epilogue: C^T[4g + i][r] = out[m = batch col r][n = 4g + i] ----
  T* out = static_cast<T*>(p.out);
#pragma unroll
  for (int f = 0; f < NF; ++f) {
    const int n = n0 + 16 * NF * wn + 16 * f + 4 * g;
    if (n >= p.N) continue;
    float bv[4] = {0.f, 0.f, 0.f, 0.f};
    if (BIAS) {
#pragma unroll
      for (int i = 0; i < 4; ++i) bv[i] = p.bias[n + i];
    }
#pragma unroll
    for (int b = 0; b < 2; ++b) {
      const int m = m0 + 32 * wm + 16 * b + r16;
      if (m >= p.M) continue;
      float v[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float t = acc[f][b][i] + bv[i];
        v[i] = ACT == ACT_RELU ? fmaxf(t, 0.f) : (ACT == ACT_TANH ? tanhf(t) : t);
      }
      if constexpr (sizeof(T) == 2) {
        const uint32_t lo = (uint32_t)__builtin_bit_cast(unsigned short, (bf16)v[0]) |
                            ((uint32_t)__builtin_bit_cast(unsigned short, (bf16)v[1]) << 16);
        const uint32_t hi = (uint32_t)__builtin_bit_cast(unsigned short, (bf16)v[2]) |
                            ((uint32_t)__builtin_bit_cast(unsigned short, (bf16)v[3]) << 16);
        *reinterpret_cast<uint2*>(out + (size_t)m * p.ldo + n) = make_uint2(lo, hi);
      } else {
        *reinterpret_cast<float4*>(out + (size_t)m * p.ldo + n) = make_float4(v[0], v[1], v[2], v[3]);
      }
    }
  }
}

}  // namespace

bool fc_tall_supported(int M, int N, int K) {
  return M > 0 && N > 0 && N % 4 == 0 && K > 0 && K % 8 == 0;
}

void fc_tall(const FcTallParams& p, hipStream_t s) {
  MCC_CHECK(fc_tall_supported(p.M, p.N, p.K), "fc_tall: needs N % 4 == 0 and K % 8 == 0");
  const int va = p.f32 ? 4 : 8;  // elements per 16 bytes
  MCC_CHECK(p.lda % va == 0 && p.lda >= p.K && p.ldw % va == 0 && p.ldw >= p.K && p.ldo % 4 == 0 && p.ldo >= p.N,
            "fc_tall: bad leading dims");
  MCC_CHECK(reinterpret_cast<uintptr_t>(p.A) % 16 == 0 && reinterpret_cast<uintptr_t>(p.W) % 16 == 0 &&
                reinterpret_cast<uintptr_t>(p.out) % (p.f32 ? 16 : 8) == 0,
            "fc_tall: alignment");
  MCC_CHECK(p.act == ACT_NONE || p.bias, "fc_tall: an activation needs the forward (bias) epilogue");
  // narrow layers (N <= 128, e.g. LeNet-5 FC1 120) on 128-column tiles, the
  // rest on 224-column tiles
  // The bf16 forward of the wide (224-column) tiles runs a 4-deep ring at one
  // workgroup per CU (three stages in flight: ref FC1 forward 240 -> 224 us,
  // profiles/fc_tall_ab_r4.txt v1); the data gradients and fp32 keep 3 deep
  // at two per CU (v1 lost there: 290 -> 348 us bf16 dX, 986 -> 1010 fp32).
  auto go = [&](auto t, auto nf) {
    using T = decltype(t);
    constexpr int NF = decltype(nf)::value;
    using Gm = TallGeom<NF>;
    using G4 = TallGeom<NF, MCC_TALL_NS>;
    constexpr bool kDeep = sizeof(T) == 2 && NF == 7;
    const int tiles = ((p.M + kTM - 1) / kTM) * ((p.N + Gm::TN - 1) / Gm::TN);
    const dim3 grid((unsigned)tiles), block(kTT);
    if (!p.bias) {
      hipLaunchKernelGGL((fc_tall_kernel<T, NF, ACT_NONE, false, 3>), grid, block, Gm::LDS, s, p);
      return;
    }
    if constexpr (kDeep) {
      if (p.act == ACT_TANH) hipLaunchKernelGGL((fc_tall_kernel<T, NF, ACT_TANH, true, MCC_TALL_NS>), grid, block, G4::LDS, s, p);
      else if (p.act == ACT_RELU) hipLaunchKernelGGL((fc_tall_kernel<T, NF, ACT_RELU, true, MCC_TALL_NS>), grid, block, G4::LDS, s, p);
      else hipLaunchKernelGGL((fc_tall_kernel<T, NF, ACT_NONE, true, MCC_TALL_NS>), grid, block, G4::LDS, s, p);
      return;
    }
    if (p.act == ACT_TANH) hipLaunchKernelGGL((fc_tall_kernel<T, NF, ACT_TANH, true, 3>), grid, block, Gm::LDS, s, p);
    else if (p.act == ACT_RELU) hipLaunchKernelGGL((fc_tall_kernel<T, NF, ACT_RELU, true, 3>), grid, block, Gm::LDS, s, p);
    else hipLaunchKernelGGL((fc_tall_kernel<T, NF, ACT_NONE, true, 3>), grid, block, Gm::LDS, s, p);
  };
  const bool narrow = p.N <= 128;
  using N4 = std::integral_constant<int, 4>;
  using N7 = std::integral_constant<int, 7>;
  if (p.f32) { if (narrow) go(float{}, N4{}); else go(float{}, N7{}); }
  else { if (narrow) go(bf16{}, N4{}); else go(bf16{}, N7{}); }
}

}  // namespace gpu
}  // namespace mcc
