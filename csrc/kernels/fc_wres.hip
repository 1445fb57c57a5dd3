// FC data gradient with a short reduction and the weights RESIDENT in LDS:
//
//   out[m][n] = epi( sum_k A[m][k] * W[n][k] )   m < M (batch), n < N, k < K <= 224
//   epi: x act'(aux[m][n]) of the previous layer's activation (ReLU / tanh),
//        or plain (the previous stage is a conv whose staging applies its mask)
//
// The shapes: the reference model's FC1 data gradient (200 -> 1568, Layer_feedBack_full,
// /root/reference/cnn.c:154-173), its FC2 data gradient (200 -> 200, x tanh'), and
// LeNet-5 fp32's FC1 / FC2 data gradients (120 -> 400, 84 -> 120 x ReLU').
//
// Why not fc_tall (the K-streaming kernel these ran on): with K = 84 .. 224 a
// 128 x 224 output tile is only 3 .. 7 K-stages deep, so every tile pays the
// DMA ring's fill and drain and re-stages its slice of W -- the ref FC1 dX ran
// at ~2 TB/s of output writes (289 us bf16, 964 us fp32).  Here a persistent
// workgroup owns ONE column slab of W ([TN][K], 97 .. 113 KB of LDS, staged
// once) and walks row blocks of A: the only streamed operand is A, read
// straight from global memory into registers one whole row block ahead (the
// MFMA B operand of a lane is 16 contiguous bytes of one A row, so no LDS
// round trip), and the output tile goes out as the MFMA produces it.
//
// MFMA orientation as fc_tall: rows = output columns n (W fragments from
// LDS), columns = batch rows m (A fragments from registers), so a lane's four
// accumulator values are four consecutive n of one m: 16-byte fp32 stores;
// bf16 pairs two fragments by permlane swaps into one 16-byte store per lane
// (64-byte row segments).  A "k-step" is 64 bytes of a row: bf16 one
// v_mfma_f32_16x16x32_bf16 (lane: 8 k at 8g), fp32 four v_mfma_f32_16x16x4_f32
// (lane: 4 k at 4g + j, j = 0..3 -- a permuted k order, identical for W and A,
// so the products and their f32 accumulation order per lane are those of a
// straight k loop over each lane's quarter).  W rows are RS = 64 KS + 32
// bytes apart: every ds_read_b128 lane group covers the 64 banks once
// (tools/lds_banks.py: RS = 32 mod 64 is conflict-free for this pattern).
//
// Grid: nslab column slabs x J workgroups per slab (nslab J <= 256, one per
// CU); workgroup (s, j) takes row blocks j, j + J, ... of slab s, so the
// nslab workgroups of one j read the same A rows at about the same time, and
// (XCD-aware order) from the same L2.
//
// Measured at B = 163,840 (profiles/fc_wres_r6.txt): ref bf16 FC1 dX 289 ->
// 212 us (8-byte stores: 241; without any output traffic 123-140 us: the
// 514 MB of output and the 7-fold A re-read stay the limit -- 16 waves per
// CU on 112-column slabs, deeper W rings and the XCD order measured no
// better), FC2 dX 69 -> 48 us; ref fp32 FC1 dX 964 -> 807 us (81 % of the f32
// MFMA peak), FC2 dX 230 -> 144 us; LeNet-5 fp32 FC1 dX 184 -> 146 us, FC2
// dX 81 -> 48 us.
#include <algorithm>
#include <type_traits>

#include "kernels.h"
#include "mcc/ab.h"
#include "mfma.h"

namespace mcc {
namespace gpu {
namespace {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

constexpr int kWT = 512;  // 8 waves

// store sink of the epilogue's out-of-range lanes (contents meaningless)
__device__ __attribute__((aligned(16))) float kWresSink[4];

// geometry: NF 16-column W fragments per wave, WN wave columns, MB 16-row
// batch fragments per wave, WM = 8 / WN wave rows
template <int KS, int NF, int WN, int MB> struct WresGeom {
  static constexpr int WM = 8 / WN;
  static constexpr int TN = 16 * NF * WN;  // slab width
  static constexpr int TM = 16 * MB * WM;  // batch rows per block
  static constexpr int RS = 64 * KS + 32;  // LDS row stride (bytes)
  static constexpr int LDS = TN * RS;
};

template <typename T, int KS, int NF, int WN, int MB, int ACT, int PERCU>  // PERCU: workgroups per CU
__global__ void __launch_bounds__(kWT, 2 * PERCU) fc_wres_kernel(FcTallParams p, const void* __restrict__ aux, int ldaux,
                                                        int nslab, int J, int xcd) {
  using Gm = WresGeom<KS, NF, WN, MB>;
  // W fragment ring depth (bf16 with an act' epilogue: 3, its aux registers)
  // (bf16 8 or 12 deep: no change, 212 us on the ref FC1 dX)
  constexpr int D = sizeof(T) == 2 ? (ACT != ACT_NONE ? 3 : 4) : 2;
  constexpr int RS = Gm::RS, TN = Gm::TN, TM = Gm::TM;
  extern __shared__ __attribute__((aligned(16))) char wsm[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r16 = lane & 15, g = lane >> 4;
  const int wn = wave % WN, wm = wave / WN;
  // xcd: workgroups dispatch round-robin over the 8 XCDs (blockIdx % 8), so
  // logical index L = (blockIdx % 8) (grid / 8) + blockIdx / 8 puts the nslab
  // workgroups of one j -- the same A rows -- on one XCD's L2
  const int L = xcd ? (int)(blockIdx.x & 7) * (int)(gridDim.x >> 3) + (int)(blockIdx.x >> 3) : (int)blockIdx.x;
  if (L >= nslab * J) return;  // (workgroup-uniform)
  const int slab = L % nslab, jb = L / nslab;
  const int n0 = slab * TN;
  const int kb = p.K * (int)sizeof(T);  // valid bytes of a row (multiple of 16)

  // ---- W slab -> LDS (zero past K and past N), once ----
  for (int i = tid; i < TN * KS * 4; i += kWT) {
    const int row = i / (KS * 4), seg = i - row * (KS * 4);
    const int n = n0 + row;
    u32x4 v = {0u, 0u, 0u, 0u};
    if (n < p.N && 16 * seg < kb)
      v = *reinterpret_cast<const u32x4*>(static_cast<const char*>(p.W) + ((size_t)n * p.ldw) * sizeof(T) + 16 * seg);
    *reinterpret_cast<u32x4*>(wsm + row * RS + 16 * seg) = v;
  }
  __syncthreads();

  const int nrb = (p.M + TM - 1) / TM;
  const char* wl = wsm + (16 * NF * wn + r16) * RS + 16 * g;  // + f 16 RS + 64 ks

  // A fragments of one row block: [KS][MB] 16-byte pieces
  typedef u32x4 ABuf[KS][MB];
  auto load = [&](ABuf& buf, int rb) {
#pragma unroll
    for (int b = 0; b < MB; ++b) {
#if defined(MCC_WRES_ABL) && MCC_WRES_ABL == 2  // timing ablation: every block reads block 0's rows
      const int m = min(16 * (MB * wm + b) + r16, p.M - 1);
#else
      const int m = min(rb * TM + 16 * (MB * wm + b) + r16, p.M - 1);
#endif
      const char* a = static_cast<const char*>(p.A) + ((size_t)m * p.lda) * sizeof(T) + 16 * g;
      // past K (the last k-step's tail): a clamped in-row address, no branch
      // (a branch per load costs the compiler its vmcnt bookkeeping: it then
      // drains the next block's loads before every multiply); the values are
      // finite row data and meet W's zero columns
#pragma unroll
      for (int ks = 0; ks < KS; ++ks)
        buf[ks][b] = *reinterpret_cast<const u32x4*>(a + min(64 * ks, kb - 16 - 16 * g));
    }
  };

  // the previous layer's activations at this block's outputs (for act'),
  // loaded BEFORE the next block's A fragments: vmcnt retires in order, so
  // the epilogue's wait for them leaves the prefetch in flight
  typedef typename std::conditional<sizeof(T) == 2, uint2, float4>::type AuxV;
  struct AuxBuf { AuxV v[ACT != ACT_NONE ? NF : 1][MB]; };
  auto load_aux = [&](AuxBuf& ax, int rb) {
    if constexpr (ACT != ACT_NONE) {
#pragma unroll
      for (int b = 0; b < MB; ++b) {
        const int m = min(rb * TM + 16 * (MB * wm + b) + r16, p.M - 1);
#pragma unroll
        for (int f = 0; f < NF; ++f) {
          const int n = min(n0 + 16 * (NF * wn + f) + 4 * g, p.N - 4);
          ax.v[f][b] = *reinterpret_cast<const AuxV*>(static_cast<const T*>(aux) + (size_t)m * ldaux + n);
        }
      }
    }
  };

  auto compute = [&](const ABuf& buf, int rb, const AuxBuf& ax) {
    f32x4 acc[NF][MB];
#pragma unroll
    for (int f = 0; f < NF; ++f)
#pragma unroll
      for (int b = 0; b < MB; ++b) acc[f][b] = f32x4{0.f, 0.f, 0.f, 0.f};
    // W fragments stream through a ring of D registers over the flattened
    // (k-step, fragment) sequence, read D - 1 steps ahead; the scheduling
    // barriers keep the compiler from hoisting all KS NF reads (the registers
    // hold the next block's A fragments instead)
    constexpr int Q = KS * NF;
    u32x4 wf[D];
#pragma unroll
    for (int q = 0; q < D - 1; ++q) wf[q] = *reinterpret_cast<const u32x4*>(wl + (q % NF) * 16 * RS + 64 * (q / NF));
#pragma unroll
    for (int q = 0; q < Q; ++q) {
      if (q + D - 1 < Q) {
        const int qn = q + D - 1;
        wf[qn % D] = *reinterpret_cast<const u32x4*>(wl + (qn % NF) * 16 * RS + 64 * (qn / NF));
      }
      __builtin_amdgcn_sched_barrier(0);
      const int ks = q / NF, f = q % NF;
#pragma unroll
      for (int b = 0; b < MB; ++b) {
        if constexpr (sizeof(T) == 2) {
          acc[f][b] = mma(acc[f][b], __builtin_bit_cast(bf16x8, wf[q % D]), __builtin_bit_cast(bf16x8, buf[ks][b]));
        } else {
          const f32x4 a = __builtin_bit_cast(f32x4, wf[q % D]), x = __builtin_bit_cast(f32x4, buf[ks][b]);
#pragma unroll
          for (int j = 0; j < 4; ++j) acc[f][b] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[j], x[j], acc[f][b], 0, 0, 0);
        }
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    // ---- epilogue: C^T[4g + i][r16] = out[m][n + i] ----
    // branch-free: the outputs past M / N go to a sink (a divergent branch
    // here lets the compiler sink the aux loads into it, behind the MFMAs)
    T* out = static_cast<T*>(p.out);
#pragma unroll
    for (int b = 0; b < MB; ++b) {
      const int m = rb * TM + 16 * (MB * wm + b) + r16;
      uint2 pk[NF];  // bf16: this lane's four outputs of fragment f, packed
#pragma unroll
      for (int f = 0; f < NF; ++f) {
        const int n = n0 + 16 * (NF * wn + f) + 4 * g;
        float v[4] = {acc[f][b][0], acc[f][b][1], acc[f][b][2], acc[f][b][3]};
        if constexpr (ACT != ACT_NONE) {
          const AuxV yv = ax.v[f][b];
          float y[4];
          if constexpr (sizeof(T) == 2) {
            y[0] = __builtin_bit_cast(float, yv.x << 16); y[1] = __builtin_bit_cast(float, yv.x & 0xffff0000u);
            y[2] = __builtin_bit_cast(float, yv.y << 16); y[3] = __builtin_bit_cast(float, yv.y & 0xffff0000u);
          } else {
            y[0] = yv.x; y[1] = yv.y; y[2] = yv.z; y[3] = yv.w;
          }
#pragma unroll
          for (int i = 0; i < 4; ++i) v[i] *= act_grad_y(ACT, y[i]);
        }
        if constexpr (sizeof(T) == 2) {
          pk[f].x = (uint32_t)__builtin_bit_cast(unsigned short, (bf16)v[0]) |
                    ((uint32_t)__builtin_bit_cast(unsigned short, (bf16)v[1]) << 16);
          pk[f].y = (uint32_t)__builtin_bit_cast(unsigned short, (bf16)v[2]) |
                    ((uint32_t)__builtin_bit_cast(unsigned short, (bf16)v[3]) << 16);
        } else {
          T* dst = m < p.M && n < p.N ? out + (size_t)m * p.ldo + n : reinterpret_cast<T*>(kWresSink);
#if defined(MCC_WRES_ABL) && MCC_WRES_ABL == 1  // timing ablation: no output traffic
          if (v[0] != 12345.f) dst = reinterpret_cast<T*>(kWresSink);
#endif
          *reinterpret_cast<float4*>(dst) = make_float4(v[0], v[1], v[2], v[3]);
        }
      }
      if constexpr (sizeof(T) == 2) {
        // fragment pairs (f, f + 1) -> one 16-byte store per lane: lane group g
        // (16 lanes) ends up with columns 8g .. 8g + 7 of the pair's 32 (one
        // 64-byte row segment per 4 lanes, half the store instructions of the
        // 8-byte form).  permlane32_swap exchanges lane groups 2,3 of the first
        // operand with groups 0,1 of the second, permlane16_swap groups 1,3 of
        // the first with 0,2 of the second:
        //   (A_g, B_g) -> g0 (A0,A2) g1 (A1,A3) g2 (B0,B2) g3 (B1,B3)
        //              -> g0 (A0,A1) g1 (A2,A3) g2 (B0,B1) g3 (B2,B3)
#pragma unroll
        for (int f = 0; f + 1 < NF; f += 2) {
          uint2 x = pk[f], y = pk[f + 1];
          auto s1 = __builtin_amdgcn_permlane32_swap(x.x, y.x, false, false);
          x.x = s1[0]; y.x = s1[1];
          s1 = __builtin_amdgcn_permlane32_swap(x.y, y.y, false, false);
          x.y = s1[0]; y.y = s1[1];
          // now lane g holds (first, second) = (x, y); swap x of groups 1,3 with y of groups 0,2
          auto s2 = __builtin_amdgcn_permlane16_swap(x.x, y.x, false, false);
          x.x = s2[0]; y.x = s2[1];
          s2 = __builtin_amdgcn_permlane16_swap(x.y, y.y, false, false);
          x.y = s2[0]; y.y = s2[1];
          const int n = n0 + 16 * (NF * wn + f) + 8 * g;
          T* dst = m < p.M && n < p.N ? out + (size_t)m * p.ldo + n : reinterpret_cast<T*>(kWresSink);
#if defined(MCC_WRES_ABL) && MCC_WRES_ABL == 1
          if (x.x != 12345u) dst = reinterpret_cast<T*>(kWresSink);
#endif
          *reinterpret_cast<uint4*>(dst) = make_uint4(x.x, x.y, y.x, y.y);
        }
        if constexpr (NF % 2) {  // the odd last fragment: 8 bytes per lane
          const int n = n0 + 16 * (NF * wn + NF - 1) + 4 * g;
          T* dst = m < p.M && n < p.N ? out + (size_t)m * p.ldo + n : reinterpret_cast<T*>(kWresSink);
          *reinterpret_cast<uint2*>(dst) = pk[NF - 1];
        }
      }
    }
  };

  // row blocks jb, jb + J, ...: two register buffers, the next block's A
  // loads in flight while the current one multiplies.  Every load is issued
  // unconditionally (past the last block: a clamped re-read), so the
  // compiler's vmcnt for a block's fragments counts the other buffer's loads
  // as in flight instead of assuming a path where they were skipped.
  const int cnt = jb < nrb ? (nrb - 1 - jb) / J + 1 : 0;
  auto rbk = [&](int i) { return min(jb + i * J, nrb - 1); };
  ABuf b0, b1;
  if (cnt > 0) load(b0, rbk(0));
  for (int i = 0; i < cnt; i += 2) {
    AuxBuf ax;
    load_aux(ax, rbk(i));
    __builtin_amdgcn_sched_barrier(0);
    load(b1, rbk(i + 1));
    __builtin_amdgcn_sched_barrier(0);
    compute(b0, rbk(i), ax);
    if (i + 1 >= cnt) break;
    load_aux(ax, rbk(i + 1));
    __builtin_amdgcn_sched_barrier(0);
    load(b0, rbk(i + 2));
    __builtin_amdgcn_sched_barrier(0);
    compute(b1, rbk(i + 1), ax);
  }
}

// instantiated shapes: (dtype, k-steps) -> fragments
template <typename T, int KS> struct WresCfg;
// (bf16 at 112-column slabs, MB 1, two workgroups per CU: 238 vs 212 us on the ref FC1 dX)
template <> struct WresCfg<bf16, 7> { static constexpr int NF = 7, WN = 2, MB = 2, PERCU = 1; };    // ref FC1 / FC2 dX (K 200)
template <> struct WresCfg<float, 13> { static constexpr int NF = 7, WN = 1, MB = 1, PERCU = 1; };  // ref fp32 (K 200)
template <> struct WresCfg<float, 8> { static constexpr int NF = 13, WN = 1, MB = 1, PERCU = 1; };  // LeNet-5 fp32 FC1 dX (K 120)
template <> struct WresCfg<float, 6> { static constexpr int NF = 8, WN = 1, MB = 1, PERCU = 1; };   // LeNet-5 fp32 FC2 dX (K 84)

int wres_ks(const FcTallParams& p) { return (p.K * (p.f32 ? 4 : 2) + 63) / 64; }

}  // namespace

bool fc_wres_supported(bool f32, int M, int N, int K, int act) {
  if (M <= 0 || N <= 0 || K <= 0 || N % (f32 ? 4 : 8) || K % (f32 ? 4 : 8) || act < ACT_NONE || act > ACT_TANH)
    return false;
  const int ks = (K * (f32 ? 4 : 2) + 63) / 64;
  return f32 ? (ks == 13 || ks == 8 || ks == 6) : ks == 7;
}

void fc_wres(const FcTallParams& p, const void* aux, int ldaux, hipStream_t s) {
  MCC_CHECK(fc_wres_supported(p.f32, p.M, p.N, p.K, p.act), "fc_wres: unsupported shape");
  const int va = p.f32 ? 4 : 8;
  MCC_CHECK(p.lda % va == 0 && p.lda >= p.K && p.ldw % va == 0 && p.ldw >= p.K && p.ldo % va == 0 && p.ldo >= p.N,
            "fc_wres: bad leading dims");
  MCC_CHECK(reinterpret_cast<uintptr_t>(p.A) % 16 == 0 && reinterpret_cast<uintptr_t>(p.W) % 16 == 0 &&
                reinterpret_cast<uintptr_t>(p.out) % 16 == 0,
            "fc_wres: alignment");
  MCC_CHECK(p.act == ACT_NONE || (aux && ldaux >= p.N), "fc_wres: an activation gradient needs aux");
  auto go = [&](auto t, auto ksc) {
    using T = decltype(t);
    constexpr int KS = decltype(ksc)::value;
    using C = WresCfg<T, KS>;
    using Gm = WresGeom<KS, C::NF, C::WN, C::MB>;
    const int nslab = (p.N + Gm::TN - 1) / Gm::TN;
    const int nrb = (p.M + Gm::TM - 1) / Gm::TM;
    static_assert(C::PERCU * Gm::LDS <= 160 * 1024, "fc_wres: LDS per CU");
    int J = std::max(1, std::min(nrb, 256 * C::PERCU / std::max(1, nslab)));
    int G = nslab * J;
    const int xcd = nslab > 1 && G >= 64 && !ab_flag("wres_noxcd");
    if (xcd) {  // a multiple of 8 workgroups, the same J for every slab
      G &= ~7;
      J = G / nslab;
    }
    const dim3 grid((unsigned)G), block(kWT);
    if (p.act == ACT_RELU)
      hipLaunchKernelGGL((fc_wres_kernel<T, KS, C::NF, C::WN, C::MB, ACT_RELU, C::PERCU>), grid, block, Gm::LDS, s, p, aux, ldaux, nslab, J, xcd);
    else if (p.act == ACT_TANH)
      hipLaunchKernelGGL((fc_wres_kernel<T, KS, C::NF, C::WN, C::MB, ACT_TANH, C::PERCU>), grid, block, Gm::LDS, s, p, aux, ldaux, nslab, J, xcd);
    else
      hipLaunchKernelGGL((fc_wres_kernel<T, KS, C::NF, C::WN, C::MB, ACT_NONE, C::PERCU>), grid, block, Gm::LDS, s, p, aux, ldaux, nslab, J, xcd);
  };
  const int ks = wres_ks(p);
  if (!p.f32) go(bf16{}, std::integral_constant<int, 7>{});
  else if (ks == 13) go(float{}, std::integral_constant<int, 13>{});
  else if (ks == 8) go(float{}, std::integral_constant<int, 8>{});
  else go(float{}, std::integral_constant<int, 6>{});
}

}  // namespace gpu
}  // namespace mcc
