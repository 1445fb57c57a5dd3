// Implicit-GEMM convolution for large images (VGG-11 @ 224^2, bf16, NHWC).
//
// Replaces the explicit im2col + GEMM pair of the large-image path (the im2col
// matrix of a VGG layer is up to 1.9 GB per step and was written and re-read
// once per direction).  Reference math: Layer_feedForw_conv / Layer_feedBack_conv
// (cnn.c:175-247), with the correct OIHW indexing of CUDAcnn.cu:167-195.
//
//   forward   out[m][n]  = act(bias[n] + sum_k X(m, k) W[n][k])
//   data grad dX[m][n]   = sum_k dZ(m, k) Wflip[n][k]   (same kernel: stride-1
//             conv of dZ with pad KS-1-pad and the flipped/transposed weights)
//   weights   dW[co][k]  = sum_m dZ[m][co] X(m, k),  db = dZ^T 1 (ones column)
//
// where m is an output pixel (b, oy, ox), k = (ky*KS + kx)*C + c, and
// X(m, k) = in[b][oy*s - pad + ky][ox*s - pad + kx][c] (0 outside the image)
// is never materialised: each 16-byte piece (8 channels of one tap) of an
// operand tile is fetched straight into LDS by global_load_lds_dwordx4 with a
// per-lane source address; padding taps and tile tails point at a zero page.
//
// gfx950 structure (cdna_hip_programming.md §5): 256 threads = 4 waves (2x2),
// 128x128 output tile per workgroup, BK = 64, two LDS buffers (64 KiB, two
// workgroups per CU), one barrier per K-step, bijective XCD-aware tile order
// (T1).  The LDS images are lane-linear (glds) with the bank swizzle applied
// on the SOURCE address and undone on the read (§5.4 rule 21):
//   * [rows][64] images (128-byte rows, ds_read_b128 fragments): 16-byte slot
//     s of row r holds logical slot s ^ ((r >> 1) & 7) -> conflict-free reads
//     of 16 rows at one k range;
//   * [64][128] images (256-byte rows, ds_read_b64_tr_b16 fragments of the
//     weight gradient, K = pixel axis): slot s of row r holds s ^ f(r),
//     f(r) = 2*(r & 3) + 8*((r >> 3) & 1) -> the 8 rows read by a 32-lane
//     group land on 8 distinct 32-byte bank ranges.
// The forward computes C^T (MFMA A = weights, B = pixels) so a lane's four
// accumulators are four consecutive channels of one pixel: one 8-byte NHWC
// store.  The weight gradient computes dW[co][k] per tile into fp32 split-K
// slabs laid out [k][co] (16-byte stores), reduced by a deterministic pass.
#include "kernels.h"
#include "mcc/ab.h"
#include "mfma.h"

#include <algorithm>

namespace mcc {
namespace gpu {

namespace {

typedef __attribute__((address_space(1))) void gvoid;
typedef __attribute__((address_space(3))) void lvoid;

constexpr int kIgT = 256;  // threads per workgroup
constexpr int kIgBM = 128;
constexpr int kIgBK = 64;
// weight-gradient kernel (128 x 128 tiles): 32-pixel K-steps through a
// LDS ring (igemm_dw_kernel)
constexpr int kDwBK = 32;

// zero page (and a bf16 "1, 0 x 7" piece for the ones column), >= 16 bytes each
__device__ __attribute__((aligned(64))) const unsigned short kIgZero[32] = {0};
__device__ __attribute__((aligned(64))) const unsigned short kIgOnes[32] = {0x3f80};

__device__ __forceinline__ void glds16(const void* src, bf16* lds_wave_base) {
  __builtin_amdgcn_global_load_lds((gvoid*)src, (lvoid*)lds_wave_base, 16, 0, 0);
}

// bijective XCD-aware remap (cdna_hip_programming.md §5, T1): consecutive
// logical tiles land on the same XCD (8 XCDs, blocks dealt round-robin)
__device__ __forceinline__ int xcd_remap(int orig, int nwg) {
  const int q = nwg >> 3, r = nwg & 7, xcd = orig & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (orig >> 3);
}

__device__ __forceinline__ int mdiv(const DivMagic& d, int n) {  // exact n / d (Div in mfma.h)
  const uint32_t u = (uint32_t)n;
  return (int)((u * d.mh + __umulhi(u, d.ml)) >> 8);
}
DivMagic magic(int d) {
  const Div v = Div::host(d);
  DivMagic r;
  r.mh = v.mh; r.ml = v.ml;
  return r;
}

__device__ __forceinline__ int swz64(int row) { return (row >> 1) & 7; }
__device__ __forceinline__ int swz128(int row) { return 2 * (row & 3) + 8 * ((row >> 3) & 1); }

// ---------------------------------------------------------------------------
// forward / data gradient
// ---------------------------------------------------------------------------
// POOL epilogue (round 5): the pooling kernels run the MFMA in the C
// orientation (A = pixels, B = weights), so lane (r16, g) of a fragment holds
// rows 4g..4g+3 -- the four positions of ONE pooling window -- of channel
// r16: the pool and its first-max-wins argmax are three in-lane compares.
// (The C^T layout spread a window over a DPP quad: two exchanges of value
// and index per channel, ~15 VALU per pooled value, which cost VGG-11's
// forward 1.2 ms of 12.3, tools/probes/lenet_phase_probe.py MCC_IG_ABL=1.)
// One bf16 + one argmax byte per lane; 16 lanes = 16 consecutive channels.
template <int A>  // activation kind (with_act); 0 also when there is no bias / activation
__device__ __forceinline__ void pool_window_store(bf16* out, int ldo, uint8_t* out_arg, int N, const f32x4& acc, int mwin,
                                                  int ch, float bias) {
  float mx = acc[0];
  uint32_t a = 0;
  if (acc[1] > mx) { mx = acc[1]; a = 1; }
  if (acc[2] > mx) { mx = acc[2]; a = 2; }
  if (acc[3] > mx) { mx = acc[3]; a = 3; }
  const bf16 o = (bf16)act_c<A>(mx + bias);
  if (A == ACT_RELU && !((float)o > 0.f)) a = 4;  // ReLU-inactive window: argmax byte 4
  out[(size_t)mwin * ldo + ch] = o;
  out_arg[(size_t)mwin * N + ch] = (uint8_t)a;
}

// POOL: fused 2x2/2 max-pool epilogue.  The GEMM rows enumerate (b, py, px,
// pos) so each pooling window is four consecutive rows (pool_window_store);
// the pre-pool conv output is never written.
// U8: the input is the u8 image set (optional sample-index gather, /255 as
// cnn.c:457) with few channels (the first layer): the pixel tile is gathered
// through registers (bytes -> bf16) into the same swizzled LDS image.
// Epilogues branch once on the activation kind (with_act, mfma.h).
// epilogue ablation (timing studies only; tools/build_variant.sh): 2 = no
// bias / activation
#ifndef MCC_IG_ABL
#define MCC_IG_ABL 0
#endif

template <int BN, bool BIAS_ACT, bool POOL, bool U8>
__global__ void __launch_bounds__(kIgT, 2) igemm_conv_kernel(IgemmParams p) {
  constexpr int BM = kIgBM;
  constexpr int AJ = BM * 8 / kIgT;  // glds per thread for the pixel tile (4)
  constexpr int BJ = BN * 8 / kIgT;  // ... and for the weight tile (4 or 2)
  constexpr int IMG = (BM + BN) * kIgBK;  // elements per buffer
  constexpr int FM = 4;              // pixel fragments per wave (64 rows)
  constexpr int FN = BN / 32;        // channel fragments per wave (BN/2 cols)
  constexpr int KT = U8 ? 64 : 0;   // u8: per-k tap table (offset, ky, kx); K <= 64: one K-step,
  constexpr int NB = U8 ? 1 : 2;    // one LDS buffer (higher occupancy for this latency-bound layer)
  __shared__ __attribute__((aligned(16))) bf16 smem[NB * IMG + 2 * KT];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r16 = lane & 15, g = lane >> 4;
  const int wm = wave >> 1, wn = wave & 1;
  int* ktab = reinterpret_cast<int*>(smem + NB * IMG);
  if constexpr (U8) {
    for (int k = tid; k < KT; k += kIgT) {
      int v = -1;  // k >= K: zero
      if (k < p.K) {
        const int tap = k / p.C, c = k - tap * p.C;
        const int ky = tap / p.KS, kx = tap - ky * p.KS;
        v = (((ky * p.W + kx) * p.C + c) << 8) | (ky << 4) | kx;  // offset < 2^22, ky, kx < 16
      }
      ktab[k] = v;
    }
    __syncthreads();
  }

  const int ntn = cdiv(p.N, BN);
  const int nwg = gridDim.x;
  const int tile = xcd_remap(blockIdx.x, nwg);
  const int tn = tile % ntn, tm = tile / ntn;
  const int m0 = tm * BM, n0 = tn * BN;
  const bf16* in = static_cast<const bf16*>(p.in);
  const uint8_t* in8 = static_cast<const uint8_t*>(p.in);
  const bf16* w = static_cast<const bf16*>(p.w);
  const bf16* zero = reinterpret_cast<const bf16*>(kIgZero);

  // ---- per-thread staging geometry (fixed for the whole K loop) ----
  int a_iy[AJ], a_ix[AJ], a_base[AJ], a_seg[AJ];
  const uint8_t* a_img[AJ];
#pragma unroll
  for (int j = 0; j < AJ; ++j) {
    const int s = j * kIgT + tid;
    const int row = s >> 3;
    a_seg[j] = ((s & 7) ^ swz64(row)) * 8;
    // decoded for a clamped row (branch-free: the U8 sample-index loads of
    // all four rows issue together), then invalidated by a select
    const int m = m0 + row;
    const int mc = m < p.M ? m : p.M - 1;
    int b, oy, ox;
    if (POOL) {  // m = ((b*PH + py)*PW + px)*4 + pos
      const int q = mc >> 2, pos = mc & 3;
      b = mdiv(p.div_ohw, q);  // div_ohw = PH*PW here
      const int rq = q - b * (p.OH >> 1) * (p.OW >> 1);
      const int py = mdiv(p.div_ow, rq), px = rq - py * (p.OW >> 1);  // div_ow = PW
      oy = 2 * py + (pos >> 1);
      ox = 2 * px + (pos & 1);
    } else {
      b = mdiv(p.div_ohw, mc);
      const int rem = mc - b * p.OH * p.OW;
      oy = mdiv(p.div_ow, rem);
      ox = rem - oy * p.OW;
    }
    const int iy = oy * p.stride - p.pad, ix = ox * p.stride - p.pad;
    if (U8) {  // image base in a 64-bit pointer (large image sets), pixel offset in a_base
      const int img = p.idx ? p.idx[b] : b;
      a_img[j] = in8 + (size_t)img * p.H * p.W * p.C;
      a_base[j] = (iy * p.W + ix) * p.C;
    } else {
      a_img[j] = in8;
      a_base[j] = ((b * p.H + iy) * p.W + ix) * p.C;
    }
    a_iy[j] = m < p.M ? iy : -(1 << 20);  // fails every bounds test
    a_ix[j] = ix;
    if (m >= p.M) a_base[j] = 0;
  }
  const bf16* b_ptr[BJ];
  int b_k[BJ];
#pragma unroll
  for (int j = 0; j < BJ; ++j) {
    const int s = j * kIgT + tid;
    const int row = s >> 3;
    const int n = n0 + row;
    b_k[j] = ((s & 7) ^ swz64(row)) * 8;
    b_ptr[j] = n < p.N ? w + (size_t)n * p.ldw + b_k[j] : nullptr;
  }

  // U8 runs (p.u8_runs: C = 3, 3x3, pad 1, stride 1, 4-byte aligned rows):
  // pixel row tid (< BM) of the tile gathers its im2col row as three 9-byte
  // image-row runs (k = ky*9 + kx*3 + c), each from three aligned dword loads
  // and two byte-aligns, instead of 32 single-byte loads (27 taps + 5
  // padding); threads BM..2BM-1 write the all-zero K slots 4..7 of row
  // tid - BM.  Dwords outside the image row read as 0, which is exactly the
  // zero padding of the kx = 0 / kx = 2 taps at the left / right border.
  const uint8_t* r_row0 = in8;
  int r_iy = -(1 << 20), r_dv = 0, r_sh = 0;
  if (U8 && p.u8_runs && tid < BM) {
    const int m = m0 + tid;
    if (m < p.M) {
      int b, oy, ox;
      if (POOL) {
        const int q = m >> 2, pos = m & 3;
        b = mdiv(p.div_ohw, q);
        const int rq = q - b * (p.OH >> 1) * (p.OW >> 1);
        const int py = mdiv(p.div_ow, rq), px = rq - py * (p.OW >> 1);
        oy = 2 * py + (pos >> 1);
        ox = 2 * px + (pos & 1);
      } else {
        b = mdiv(p.div_ohw, m);
        const int rem = m - b * p.OH * p.OW;
        oy = mdiv(p.div_ow, rem);
        ox = rem - oy * p.OW;
      }
      const int img = p.idx ? p.idx[b] : b;
      r_row0 = in8 + (size_t)img * p.H * p.W * 3;
      r_iy = oy - 1;
      const int o = 3 * (ox - 1);  // byte offset of tap kx = 0 in its row (-3 at the left border)
      r_dv = o & ~3;
      r_sh = o - r_dv;
    }
  }

  const int nk = cdiv(p.K, kIgBK);  // !U8: C % 32 == 0 (KS = 1: C % 8); pieces at k >= K read the zero page
  auto stage = [&](int kt, int buf) {
    const int k0 = kt * kIgBK;
    bf16* A = smem + buf * IMG;
    bf16* Bw = A + BM * kIgBK;
    if constexpr (U8) {
    if (p.u8_runs) {
      const float sc = 1.0f / 255.0f;
      const int rb = 3 * p.W;  // row bytes
      if (tid < BM) {
        uint32_t qd[3][3];
#pragma unroll
        for (int ky = 0; ky < 3; ++ky) {
          const int iy = r_iy + ky;
          const bool rok = (unsigned)iy < (unsigned)p.H;
          const uint8_t* row = r_row0 + (size_t)(rok ? iy : 0) * rb;
#pragma unroll
          for (int i = 0; i < 3; ++i) {
            const int d = r_dv + 4 * i;
            const bool ok = rok && d >= 0 && d <= rb - 4;
            qd[ky][i] = *reinterpret_cast<const uint32_t*>(row + (ok ? d : 0));  // unconditional (no branch + vmcnt(0))
            qd[ky][i] = ok ? qd[ky][i] : 0u;
          }
        }
        bf16x8 v[4];
#pragma unroll
        for (int ky = 0; ky < 3; ++ky) {
          const uint32_t w0 = __builtin_amdgcn_alignbyte(qd[ky][1], qd[ky][0], r_sh);
          const uint32_t w1 = __builtin_amdgcn_alignbyte(qd[ky][2], qd[ky][1], r_sh);
          const uint32_t w2 = __builtin_amdgcn_alignbyte(0u, qd[ky][2], r_sh);
          const uint32_t wb[3] = {w0, w1, w2};
#pragma unroll
          for (int j = 0; j < 9; ++j) {
            const int k = ky * 9 + j;
            v[k >> 3][k & 7] = (bf16)((float)((wb[j >> 2] >> (8 * (j & 3))) & 0xffu) * sc);
          }
        }
#pragma unroll
        for (int k = 27; k < 32; ++k) v[k >> 3][k & 7] = (bf16)0.f;
#pragma unroll
        for (int ls = 0; ls < 4; ++ls) store8(A + tid * kIgBK + ((ls ^ swz64(tid)) << 3), v[ls]);
      } else {
        const int row = tid - BM;
        bf16x8 z;
#pragma unroll
        for (int e = 0; e < 8; ++e) z[e] = (bf16)0.f;
#pragma unroll
        for (int ls = 4; ls < 8; ++ls) store8(A + row * kIgBK + ((ls ^ swz64(row)) << 3), z);
      }
    } else {
      const float sc = 1.0f / 255.0f;
      uint8_t raw[AJ][8];
      uint32_t inb[AJ] = {};
#pragma unroll
      for (int j = 0; j < AJ; ++j) {
        const int4 t0 = *reinterpret_cast<const int4*>(ktab + k0 + a_seg[j]);
        const int4 t1 = *reinterpret_cast<const int4*>(ktab + k0 + a_seg[j] + 4);
        const int tv[8] = {t0.x, t0.y, t0.z, t0.w, t1.x, t1.y, t1.z, t1.w};
        // every byte load is unconditional (padding taps read byte 0 of the
        // image and are zeroed by a select): a guarded load compiles to a
        // branch + vmcnt(0) per element, 32 serialised memory latencies
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const int t = tv[e];
          const int iy = a_iy[j] + ((t >> 4) & 15), ix = a_ix[j] + (t & 15);
          const bool in = t >= 0 && (unsigned)iy < (unsigned)p.H && (unsigned)ix < (unsigned)p.W;
          raw[j][e] = a_img[j][in ? a_base[j] + (t >> 8) : 0];
          inb[j] |= (uint32_t)in << e;
        }
      }
      // all 32 loads are in flight before the first conversion
#pragma unroll
      for (int j = 0; j < AJ; ++j) {
        bf16x8 v;
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = (bf16)((inb[j] >> e & 1u) ? (float)raw[j][e] * sc : 0.f);
        store8(A + (j * kIgT + tid) * 8, v);
      }
    }
    } else if (p.c_shift >= 6) {
      // C = 2^s >= 64: the 64-deep K-step is one tap, no channel wrap, K % 64
      // == 0; the tap comes from a shift (no runtime division per step) and
      // a piece is 2 adds + 2 bounds tests + its address
      const int tap = k0 >> p.c_shift;
      const int c0 = k0 - (tap << p.c_shift);
      const int ky = p.KS == 3 ? tap / 3 : tap / p.KS, kx = tap - ky * p.KS;
      const int toff = ((ky * p.W + kx) << p.c_shift) + c0;
#pragma unroll
      for (int j = 0; j < AJ; ++j) {
        const int iy = a_iy[j] + ky, ix = a_ix[j] + kx;
        const bool ok = (unsigned)iy < (unsigned)p.H && (unsigned)ix < (unsigned)p.W;
        glds16(ok ? in + (a_base[j] + a_seg[j] + toff) : zero, A + (j * kIgT + wave * 64) * 8);
      }
    } else {
      // C % 32 == 0: a 64-deep K-step spans at most two taps (the second from
      // the piece's channel wrap; C = 32: slots 4..7), both wave-uniform
      const int tap = k0 / p.C;
      const int c0 = k0 - tap * p.C;
      const int ky = tap / p.KS, kx = tap - ky * p.KS;
      const int ky1 = kx + 1 < p.KS ? ky : ky + 1, kx1 = kx + 1 < p.KS ? kx + 1 : 0;
      const int toff = (ky * p.W + kx) * p.C;
      const int toff1 = (ky1 * p.W + kx1) * p.C - p.C;  // channel index c0 + seg - C
#pragma unroll
      for (int j = 0; j < AJ; ++j) {
        const int c = c0 + a_seg[j];
        const bool wrap = c >= p.C;
        const int iy = a_iy[j] + (wrap ? ky1 : ky), ix = a_ix[j] + (wrap ? kx1 : kx);
        const bool ok = k0 + a_seg[j] < p.K && (unsigned)iy < (unsigned)p.H && (unsigned)ix < (unsigned)p.W;
        const bf16* src = ok ? in + (a_base[j] + (wrap ? toff1 : toff) + c) : zero;
        glds16(src, A + (j * kIgT + wave * 64) * 8);
      }
    }
#pragma unroll
    for (int j = 0; j < BJ; ++j) {
      const bf16* src = (b_ptr[j] && (p.c_shift >= 6 || k0 + b_k[j] < p.K)) ? b_ptr[j] + k0 : zero;
      glds16(src, Bw + (j * kIgT + wave * 64) * 8);
    }
  };

  f32x4 acc[FN][FM];
#pragma unroll
  for (int i = 0; i < FN; ++i)
#pragma unroll
    for (int j = 0; j < FM; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  stage(0, 0);
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int buf = NB == 1 ? 0 : (kt & 1);
    if (NB == 2 && kt + 1 < nk) stage(kt + 1, buf ^ 1);
    const bf16* A = smem + buf * IMG;
    const bf16* Bw = A + BM * kIgBK;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int seg = 4 * h + g;
      bf16x8 xa[FM], wb[FN];
#pragma unroll
      for (int f = 0; f < FM; ++f) {
        const int row = wm * 64 + f * 16 + r16;
        xa[f] = load8(A + row * kIgBK + ((seg ^ swz64(row)) << 3));
      }
#pragma unroll
      for (int f = 0; f < FN; ++f) {
        const int row = wn * (BN / 2) + f * 16 + r16;
        wb[f] = load8(Bw + row * kIgBK + ((seg ^ swz64(row)) << 3));
      }
#pragma unroll
      for (int i = 0; i < FN; ++i)
#pragma unroll
        for (int j = 0; j < FM; ++j) acc[i][j] = POOL ? mma(acc[i][j], xa[j], wb[i]) : mma(acc[i][j], wb[i], xa[j]);
    }
    __syncthreads();
  }

  if constexpr (POOL) {  // lane: channel r16, window rows 4g..4g+3 (see pool_window_store)
    bf16* const out = static_cast<bf16*>(p.out);
    uint8_t* const oarg = p.out_arg;
    const int ldo = p.ldo, Mx = p.M, Nx = p.N;
    auto epi = [&](auto ak) {
#pragma unroll
      for (int i = 0; i < FN; ++i) {
        const int ch = n0 + wn * (BN / 2) + i * 16 + r16;
        if (ch >= p.N) continue;
        const float bv = BIAS_ACT && p.bias ? p.bias[ch] : 0.f;
#pragma unroll
        for (int j = 0; j < FM; ++j) {
          const int m = m0 + wm * 64 + j * 16 + 4 * g;
          if (m < Mx) pool_window_store<decltype(ak)::v>(out, ldo, oarg, Nx, acc[i][j], m >> 2, ch, bv);
        }
      }
    };
    if (BIAS_ACT) with_act(p.act, epi); else epi(ActK<0>{});
    return;
  }
  // ---- epilogue: lane holds channels 4g..4g+3 of pixel r16 per fragment ----
  bf16* out = static_cast<bf16*>(p.out);
  const int ldo = p.ldo, Mx = p.M, Nx = p.N;  // registers: the stores below would re-read the kernarg copy
  const bf16* rmask = static_cast<const bf16*>(p.relu_mask);
  auto epi = [&](auto ak) {
    constexpr int A = decltype(ak)::v;
#pragma unroll
    for (int i = 0; i < FN; ++i) {
      const int ch = n0 + wn * (BN / 2) + i * 16 + 4 * g;
      const bool chok = ch < Nx;
      float bv[4] = {0.f, 0.f, 0.f, 0.f};
      if (BIAS_ACT && p.bias && chok) {
#pragma unroll
        for (int e = 0; e < 4; ++e) bv[e] = p.bias[ch + e];
      }
#pragma unroll
      for (int j = 0; j < FM; ++j) {
        const int m = m0 + wm * 64 + j * 16 + r16;
        if (!chok || m >= Mx) continue;
        float v[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = (MCC_IG_ABL & 2) ? acc[i][j][e] : act_c<A>(acc[i][j][e] + bv[e]);
        if (!BIAS_ACT && rmask) {  // data gradient straight to dZ of a ReLU layer: dX * (y > 0)
          const bf16x4 y = *reinterpret_cast<const bf16x4*>(rmask + (size_t)m * ldo + ch);
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = (float)y[e] > 0.f ? v[e] : 0.f;
        }
        *reinterpret_cast<bf16x4*>(out + (size_t)m * ldo + ch) = cvt4(v[0], v[1], v[2], v[3]);
      }
    }
  };
  if constexpr (BIAS_ACT) with_act(p.act, epi);
  else epi(ActK<0>{});
}

// ---------------------------------------------------------------------------
// forward / data gradient on 256-pixel x BC-channel tiles, phase-pipelined
// ---------------------------------------------------------------------------
// The 128x128 kernel above streams 32 KiB of operands per 2.1 MFLOP K-step
// and drains every LDS-DMA at each __syncthreads: on the VGG layers it runs
// at ~30% of the bf16 MFMA peak, bound by the per-CU fetch rate.  Here one
// 512-thread workgroup per CU owns a 256 x BC tile (2x / 1.5x the flops per
// staged byte) and keeps up to three quarter-tiles of DMA in flight across
// its barriers (cdna_hip_programming.md §5 "The 256² 8-phase template"):
//   LDS   2 buffers x [A0 | A1 | B0 | B1], A = weight halves (BC/2 channel
//         rows), B = pixel halves (128 rows), each row 64 k (128 B, swz64);
//   waves 2 (channels) x 4 (pixels); wave (wr, wc) owns channels
//         hA*BC/2 + wr*BC/4 + [0, BC/4) and pixels hB*128 + wc*32 + [0, 32)
//         of each quadrant (hA, hB);
//   phase p0 (A0,B0)  p1 (A0,B1)  p2 (A1,B1)  p3 (A1,B0): the A/B register
//         subtiles are read once per K-tile (p0: A0+B0, p1: B1, p2: A1), and
//         phase p stages quarter p of the NEXT K-tile (A0', B0', B1', A1'),
//         so the counted wait before phase p's barrier retires exactly the
//         quarter that phase reads (one barrier later, rule "read a staged
//         buffer one phase after the wait that retires it").
// Raw s_barrier + counted vmcnt: __syncthreads() would emit vmcnt(0) and drain
// the prefetch (guide §5 "Pipelining across barriers").
template <int N> __device__ __forceinline__ void vm_wait();
#define MCC_VM_WAIT(n) \
  template <> __device__ __forceinline__ void vm_wait<n>() { asm volatile("s_waitcnt vmcnt(" #n ")" ::: "memory"); }
MCC_VM_WAIT(0) MCC_VM_WAIT(1) MCC_VM_WAIT(2) MCC_VM_WAIT(3) MCC_VM_WAIT(4)
#undef MCC_VM_WAIT
__device__ __forceinline__ void raw_barrier() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

constexpr int kBigT = 512;
constexpr int kBigBP = 256;

// K loop of the 256-tile kernels.  Quadrant order (A0,B0) (A0,B1) (A1,B1)
// (A1,B0); phase q reads its new register subtile (rd q: 0 = A0+B0, 1 = B1,
// 2 = A1), runs its MFMAs (mm q) and then stages quarter q of the next K-tile
// (st q: A0', B0', B1', A1'; issued after the MFMA cluster so the staging
// address VALU overlaps the MFMAs in flight -- same issue order, same counted
// waits; round 5: +2-5 %).  GA / GB = glds per thread per A / B quarter.
// One barrier per phase, all waves in step (reads, then MFMAs).  (A staggered
// ping-pong variant, wave group 1 one barrier behind with s_setprio around the
// MFMA clusters, measured slower on VGG-11: 18.41 vs 17.66 ms/step, and was
// removed in round 3.)
#ifndef MCC_IG_PIPE
#define MCC_IG_PIPE 2  // 1: s_setprio around the MFMA clusters (measured slower); 2: stage after them
#endif
template <int GA, int GB, class RD, class ST, class MM>
__device__ __forceinline__ void pipe_loop(int nk, RD&& rd, ST&& st, MM&& mm) {
  constexpr bool kLate = MCC_IG_PIPE & 2;  // stage after the MFMA cluster
  auto mmp = [&](int q) {
    if (MCC_IG_PIPE & 1) __builtin_amdgcn_s_setprio(1);
    mm(q);
    if (MCC_IG_PIPE & 1) __builtin_amdgcn_s_setprio(0);
  };
  st(0, 0); st(0, 1); st(0, 2); st(0, 3);
  {
    for (int kt = 0; kt < nk; ++kt) {
      const bool nx = kt + 1 < nk;
      vm_wait<GA + GB>();  // A0, B0 landed (B1, A1 in flight)
      raw_barrier();
      rd(kt, 0);
      if (!kLate && nx) st(kt + 1, 0);
      mmp(0);
      if (kLate && nx) st(kt + 1, 0);
      if (nx) vm_wait<2 * GA>(); else vm_wait<GA>();  // B1 (A1, A0' in flight)
      raw_barrier();
      rd(kt, 1);
      if (!kLate && nx) st(kt + 1, 1);
      mmp(1);
      if (kLate && nx) st(kt + 1, 1);
      if (nx) vm_wait<GA + GB>(); else vm_wait<0>();  // A1 (A0', B0' in flight)
      raw_barrier();
      rd(kt, 2);
      if (!kLate && nx) st(kt + 1, 2);
      mmp(2);
      if (kLate && nx) st(kt + 1, 2);  // issue order B1', A1' kept (the counted waits)
      if (nx) st(kt + 1, 3);
      mmp(3);
    }
  }
}

template <int BC, bool BIAS_ACT, bool POOL>
__global__ void __launch_bounds__(kBigT, 1) igemm_big_kernel(IgemmParams p) {
  constexpr int BK = kIgBK;
  constexpr int HA = BC / 2, HB = kBigBP / 2;    // rows per A / B half
  constexpr int GA = HA * 8 / kBigT, GB = HB * 8 / kBigT;  // glds per thread per half
  constexpr int QA = HA * BK, QB = HB * BK;        // elements per half image
  constexpr int BUF = 2 * QA + 2 * QB;             // [A0][A1][B0][B1]
  constexpr int FA = HA / 2 / 16;                  // channel fragments per wave per half
  static_assert(GA >= 1 && GB == 2 && FA >= 1, "tile shape");
  __shared__ __attribute__((aligned(16))) bf16 smem[2 * BUF];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r16 = lane & 15, g = lane >> 4;
  const int wr = wave >> 2, wc = wave & 3;

  const int ntn = cdiv(p.N, BC);
  const int tile = xcd_remap(blockIdx.x, gridDim.x);
  const int tn = tile % ntn, tm = tile / ntn;  // neighbours share the pixel tile
  const int m0 = tm * kBigBP, n0 = tn * BC;
  const bf16* in = static_cast<const bf16*>(p.in);
  const bf16* w = static_cast<const bf16*>(p.w);
  const bf16* zero = reinterpret_cast<const bf16*>(kIgZero);

  // pixel pieces: half h, j < GB -> row (j*512 + tid) >> 3 of the half
  int a_iy[2][GB], a_ix[2][GB], a_off[2][GB];
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int j = 0; j < GB; ++j) {
      const int s = j * kBigT + tid;
      const int row = s >> 3;
      const int seg = ((s & 7) ^ swz64(row)) * 8;
      const int m = m0 + h * HB + row;
      const int mc = m < p.M ? m : p.M - 1;
      int b, oy, ox;
      if (POOL) {  // m = ((b*PH + py)*PW + px)*4 + pos
        const int q = mc >> 2, pos = mc & 3;
        b = mdiv(p.div_ohw, q);
        const int rq = q - b * (p.OH >> 1) * (p.OW >> 1);
        const int py = mdiv(p.div_ow, rq), px = rq - py * (p.OW >> 1);
        oy = 2 * py + (pos >> 1);
        ox = 2 * px + (pos & 1);
      } else {
        b = mdiv(p.div_ohw, mc);
        const int rem = mc - b * p.OH * p.OW;
        oy = mdiv(p.div_ow, rem);
        ox = rem - oy * p.OW;
      }
      const int iy = oy * p.stride - p.pad, ix = ox * p.stride - p.pad;
      a_iy[h][j] = m < p.M ? iy : -(1 << 20);  // fails every bounds test
      a_ix[h][j] = ix;
      a_off[h][j] = m < p.M ? ((b * p.H + iy) * p.W + ix) * p.C + seg : 0;
    }
  // weight pieces: half h, j < GA -> channel row (j*512 + tid) >> 3 of the half
  const bf16* w_ptr[2][GA];
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int j = 0; j < GA; ++j) {
      const int s = j * kBigT + tid;
      const int row = s >> 3;
      const int n = n0 + h * HA + row;
      w_ptr[h][j] = n < p.N ? w + (size_t)n * p.ldw + ((s & 7) ^ swz64(row)) * 8 : nullptr;
    }

  auto stage_a = [&](int kt, int h) {
    bf16* dst = smem + (kt & 1) * BUF + h * QA;
    const int k0 = kt * BK;
#pragma unroll
    for (int j = 0; j < GA; ++j)
      glds16(w_ptr[h][j] ? w_ptr[h][j] + k0 : zero, dst + (j * kBigT + wave * 64) * 8);
  };
  auto stage_b = [&](int kt, int h) {
    bf16* dst = smem + (kt & 1) * BUF + 2 * QA + h * QB;
    const int k0 = kt * BK;
    // uniform; C % 64 == 0 (a shift when C is a power of two: no runtime division per step)
    const int tap = p.c_shift >= 0 ? k0 >> p.c_shift : k0 / p.C;
    const int c0 = k0 - tap * p.C;
    const int ky = p.KS == 3 ? tap / 3 : tap / p.KS, kx = tap - ky * p.KS;
    const int toff = (ky * p.W + kx) * p.C + c0;
#pragma unroll
    for (int j = 0; j < GB; ++j) {
      const int iy = a_iy[h][j] + ky, ix = a_ix[h][j] + kx;
      const bool ok = (unsigned)iy < (unsigned)p.H && (unsigned)ix < (unsigned)p.W;
      glds16(ok ? in + (a_off[h][j] + toff) : zero, dst + (j * kBigT + wave * 64) * 8);
    }
  };

  f32x4 acc[2][FA][2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int f = 0; f < FA; ++f)
#pragma unroll
      for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int e = 0; e < 2; ++e) acc[a][f][b][e] = f32x4{0.f, 0.f, 0.f, 0.f};

  bf16x8 fa[FA][2], fb0[2][2], fb1[2][2];  // [frag][k half of the 64-deep step]
  auto read_a = [&](const bf16* img, int h) {
#pragma unroll
    for (int f = 0; f < FA; ++f) {
      const int row = wr * (HA / 2) + f * 16 + r16;
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
        fa[f][ks] = load8(img + h * QA + row * BK + (((4 * ks + g) ^ swz64(row)) << 3));
    }
  };
  auto read_b = [&](const bf16* img, int h, bf16x8 (&fb)[2][2]) {
#pragma unroll
    for (int f = 0; f < 2; ++f) {
      const int row = wc * 32 + f * 16 + r16;
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
        fb[f][ks] = load8(img + 2 * QA + h * QB + row * BK + (((4 * ks + g) ^ swz64(row)) << 3));
    }
  };
  auto mfma_q = [&](int ha, int hb, const bf16x8 (&fb)[2][2]) {
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int f = 0; f < FA; ++f)
#pragma unroll
        for (int e = 0; e < 2; ++e)
          acc[ha][f][hb][e] = POOL ? mma(acc[ha][f][hb][e], fb[e][ks], fa[f][ks]) : mma(acc[ha][f][hb][e], fa[f][ks], fb[e][ks]);
  };

  const int nk = p.K / BK;  // host: K % 64 == 0
  pipe_loop<GA, GB>(
      nk,
      [&](int kt, int q) {
        const bf16* img = smem + (kt & 1) * BUF;
        if (q == 0) { read_a(img, 0); read_b(img, 0, fb0); }
        else if (q == 1) read_b(img, 1, fb1);
        else read_a(img, 1);
      },
      [&](int kt, int q) {
        if (q == 0) stage_a(kt, 0);
        else if (q == 1) stage_b(kt, 0);
        else if (q == 2) stage_b(kt, 1);
        else stage_a(kt, 1);
      },
      [&](int q) {
        if (q == 0) mfma_q(0, 0, fb0);
        else if (q == 1) mfma_q(0, 1, fb1);
        else if (q == 2) mfma_q(1, 1, fb1);
        else mfma_q(1, 0, fb0);
      });

  if constexpr (POOL) {  // lane: channel r16, window rows 4g..4g+3 (see pool_window_store)
    bf16* const out = static_cast<bf16*>(p.out);
    uint8_t* const oarg = p.out_arg;
    const int ldo = p.ldo, Mx = p.M, Nx = p.N;
    auto epi = [&](auto ak) {
#pragma unroll
      for (int ha = 0; ha < 2; ++ha)
#pragma unroll
        for (int f = 0; f < FA; ++f) {
          const int ch = n0 + ha * HA + wr * (HA / 2) + f * 16 + r16;
          if (ch >= p.N) continue;
          const float bv = BIAS_ACT && p.bias ? p.bias[ch] : 0.f;
#pragma unroll
          for (int hb = 0; hb < 2; ++hb)
#pragma unroll
            for (int e2 = 0; e2 < 2; ++e2) {
              const int m = m0 + hb * HB + wc * 32 + e2 * 16 + 4 * g;
              if (m < Mx) pool_window_store<decltype(ak)::v>(out, ldo, oarg, Nx, acc[ha][f][hb][e2], m >> 2, ch, bv);
            }
        }
    };
    if (BIAS_ACT) with_act(p.act, epi); else epi(ActK<0>{});
    return;
  }
  // ---- epilogue: lane holds channels 4g..4g+3 of pixel r16 per fragment ----
  bf16* out = static_cast<bf16*>(p.out);
  const int ldo = p.ldo, Mx = p.M, Nx = p.N;  // registers: the stores below would re-read the kernarg copy
  const bf16* rmask = static_cast<const bf16*>(p.relu_mask);
  auto epi = [&](auto ak) {
    constexpr int A = decltype(ak)::v;
#pragma unroll
    for (int ha = 0; ha < 2; ++ha)
#pragma unroll
      for (int f = 0; f < FA; ++f) {
        const int ch = n0 + ha * HA + wr * (HA / 2) + f * 16 + 4 * g;
        const bool chok = ch < Nx;
        float bv[4] = {0.f, 0.f, 0.f, 0.f};
        if (BIAS_ACT && p.bias && chok) {
#pragma unroll
          for (int e = 0; e < 4; ++e) bv[e] = p.bias[ch + e];
        }
#pragma unroll
        for (int hb = 0; hb < 2; ++hb)
#pragma unroll
          for (int e2 = 0; e2 < 2; ++e2) {
            const int m = m0 + hb * HB + wc * 32 + e2 * 16 + r16;
            if (!chok || m >= Mx) continue;
            float v[4];
#pragma unroll
            for (int e = 0; e < 4; ++e)
              v[e] = (MCC_IG_ABL & 2) ? acc[ha][f][hb][e2][e] : act_c<A>(acc[ha][f][hb][e2][e] + bv[e]);
            if (!BIAS_ACT && rmask) {  // data gradient straight to dZ of a ReLU layer
              const bf16x4 y = *reinterpret_cast<const bf16x4*>(rmask + (size_t)m * ldo + ch);
#pragma unroll
              for (int e = 0; e < 4; ++e) v[e] = (float)y[e] > 0.f ? v[e] : 0.f;
            }
            *reinterpret_cast<bf16x4*>(out + (size_t)m * ldo + ch) = cvt4(v[0], v[1], v[2], v[3]);
          }
      }
  };
  if constexpr (BIAS_ACT) with_act(p.act, epi);
  else epi(ActK<0>{});
}

// ---------------------------------------------------------------------------
// weight gradient (split-K over pixels)
// ---------------------------------------------------------------------------
// Pipeline: K-step ks lands in ring slot (ks - ks0) % NST and is issued
// NST - 1 steps ahead; every step issues exactly JD + JX DMAs per thread (past
// the split: harmless pieces into a slot nobody reads), so "stage ks landed"
// is a fixed `s_waitcnt vmcnt((NST - 2) * (JD + JX))` (in-order retirement)
// followed by an explicit s_barrier -- __syncthreads() would drain the
// lookahead.  The barrier also retires the reads of the slot the next DMA
// overwrites (read one step ago).
// BM = 128: 128 x 128 tiles, 4-deep ring (64 KB); BM = 256 (129..256 output
// channels, e.g. the reference model's FC1: 200): one tile covers every
// output channel, so the streamed X rows are not shared between co tiles and
// each ring slot carries twice the unique HBM bytes (3-deep ring, 72 KB).
// (Round 3 ran 64-pixel steps double-buffered with a full drain per step.)
template <int BM, int NST>
__global__ void __launch_bounds__(kIgT, 2) igemm_dw_kernel(IgemmDwParams p) {
  constexpr int BN = 128, BK = kDwBK;             // co x k x pixels
  constexpr int JD = BK * BM / 8 / kIgT;          // dZ glds per thread per step
  constexpr int JX = BK * BN / 8 / kIgT;          // X glds per thread per step
  constexpr int SD = BM / 8;                      // 16-byte slots per dZ row
  constexpr int IMG = (BM + BN) * BK;
  constexpr int VM = (NST - 2) * (JD + JX);
  constexpr int FM = BM / 32;                     // co fragments per wave
  static_assert(VM == 8 || VM == 6, "the s_waitcnt below");
  __shared__ __attribute__((aligned(16))) bf16 smem[NST * IMG];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r16 = lane & 15, g = lane >> 4;
  const int q = r16 >> 2, pp = r16 & 3;
  const int wm = wave >> 1, wn = wave & 1;

  const int ntm = cdiv(p.Cout, BM), ntn = cdiv(p.kf + 1, BN);
  const int ntiles = ntm * ntn;
  // consecutive ids (one XCD after the remap) = different output tiles of
  // the SAME pixel range: the dZ and X rows they stream are shared in L2
  const int id = xcd_remap(blockIdx.x, gridDim.x);
  const int tile = id % ntiles, split = id / ntiles;
  if (split >= p.splitk) return;
  const int tm = tile % ntm, tn = tile / ntm;
  const int co0 = tm * BM, k0 = tn * BN;
  const int nks = cdiv(p.M, BK);
  const int per = cdiv(nks, p.splitk);
  const int ks0 = split * per, ks1 = min(nks, ks0 + per);

  const bf16* dz = static_cast<const bf16*>(p.dz);
  const bf16* in = static_cast<const bf16*>(p.in);
  const bf16* zero = reinterpret_cast<const bf16*>(kIgZero);
  const bf16* ones = reinterpret_cast<const bf16*>(kIgOnes);

  // per-thread staging geometry: row (pixel within the K-step) and the
  // logical 16-byte slot (8 output channels / 8 im2col columns).  The X
  // row's pixel (b, oy, ox) is decoded once and then advanced by BK pixels
  // per K-step with carries (the K-steps of a split are staged in order), and
  // every source is picked by selects: no per-step divisions, no branches.
  int d_col[JD], dm_[JD];
#pragma unroll
  for (int j = 0; j < JD; ++j) {
    const int s = j * kIgT + tid;
    const int row = s / SD;
    d_col[j] = co0 + ((s % SD) ^ swz128(row)) * 8;
    dm_[j] = ks0 * BK + row;
  }
  // (round 5) the pixel's input corner (iy0, ix0) and element offset pb are
  // carried with (oy, ox): no per-step multiplies (see igemm_dwbig_kernel)
  int m_[JX], oy_[JX], ox_[JX], iy0_[JX], ix0_[JX], pb_[JX];
  int x_ky[JX], x_kx[JX], x_off[JX], x_kind[JX];  // kind: 0 tap, 1 ones, 2 zero
#pragma unroll
  for (int j = 0; j < JX; ++j) {
    const int s = j * kIgT + tid;
    const int row = s >> 4;
    const int ls = (s & 15) ^ swz128(row);
    const int k = k0 + ls * 8;
    if (k < p.kf) {
      const int tap = k / p.C;
      const int c = k - tap * p.C;
      x_ky[j] = tap / p.KS;
      x_kx[j] = tap - x_ky[j] * p.KS;
      x_off[j] = (x_ky[j] * p.W + x_kx[j]) * p.C + c;
      x_kind[j] = 0;
    } else {
      x_off[j] = 0; x_ky[j] = 0; x_kx[j] = 0;
      x_kind[j] = k == p.kf ? 1 : 2;
    }
    const int m = ks0 * BK + row;
    m_[j] = m;
    const int b = mdiv(p.div_ohw, m);
    const int rem = m - b * p.OH * p.OW;
    oy_[j] = mdiv(p.div_ow, rem);
    ox_[j] = rem - oy_[j] * p.OW;
    iy0_[j] = oy_[j] * p.stride - p.pad;
    ix0_[j] = ox_[j] * p.stride - p.pad;
    pb_[j] = ((b * p.H + iy0_[j]) * p.W + ix0_[j]) * p.C;
  }
  const int sW = p.stride * p.W, sC = p.stride * p.C;
  const int inc_x = p.adv_x * sC, inc_c1 = (sW - p.OW * p.stride) * p.C, inc_y = p.adv_y * sW * p.C;
  const int inc_c2 = (p.H - p.OH * p.stride) * p.W * p.C, inc_b = p.adv_b * p.H * p.W * p.C;
  const uint64_t zero_u = reinterpret_cast<uint64_t>(zero), ones_u = reinterpret_cast<uint64_t>(ones);

  auto stage = [&](int buf) {  // the next K-step of this split
    bf16* D = smem + buf * IMG;
    bf16* X = D + BK * BM;
#pragma unroll
    for (int j = 0; j < JD; ++j) {
      const bool mok = dm_[j] < p.M;
      const uint64_t dz_u = reinterpret_cast<uint64_t>(dz + (size_t)dm_[j] * p.ldz + d_col[j]);
      const bf16* dsrc = reinterpret_cast<const bf16*>((mok && d_col[j] < p.Cout) ? dz_u : zero_u);  // piece may span the pad
      glds16(dsrc, D + (j * kIgT + wave * 64) * 8);
      dm_[j] += BK;
    }
#pragma unroll
    for (int j = 0; j < JX; ++j) {
      const bool mok = m_[j] < p.M;
      const int iy = iy0_[j] + x_ky[j], ix = ix0_[j] + x_kx[j];
      const bool tap_ok = mok && x_kind[j] == 0 && (unsigned)iy < (unsigned)p.H && (unsigned)ix < (unsigned)p.W;
      const int off = pb_[j] + x_off[j];  // < 2^31 (host check); unused if !tap_ok
      const uint64_t x_u = reinterpret_cast<uint64_t>(in) + 2 * (uint64_t)(uint32_t)off;
      const uint64_t xs = tap_ok ? x_u : ((mok && x_kind[j] == 1) ? ones_u : zero_u);
      glds16(reinterpret_cast<const bf16*>(xs), X + (j * kIgT + wave * 64) * 8);
      // advance this row by BK pixels
      m_[j] += BK;
      ox_[j] += p.adv_x;
      ix0_[j] += p.adv_x * p.stride;
      pb_[j] += inc_x;
      if (ox_[j] >= p.OW) {
        ox_[j] -= p.OW;
        ix0_[j] -= p.OW * p.stride;
        oy_[j] += 1;
        iy0_[j] += p.stride;
        pb_[j] += inc_c1;
      }
      oy_[j] += p.adv_y;
      iy0_[j] += p.adv_y * p.stride;
      pb_[j] += inc_y;
      if (oy_[j] >= p.OH) {
        oy_[j] -= p.OH;
        iy0_[j] -= p.OH * p.stride;
        pb_[j] += inc_c2;
      }
      pb_[j] += inc_b;
    }
  };

  f32x4 acc[FM][4];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // transpose-read of a [BK][ncols] image: 4 consecutive K rows (pixels) of
  // 16 columns; lane 4q+p of a 16-lane group addresses row kr+q, columns 4p..
  // (address of rows kr + q; rows kr + 4 + q have the same swizzle, so the
  // second read of a fragment takes its offset in the instruction)
  auto tra = [&](const bf16* img, int ncols, int kr, int col0) {  // (inline asm: see tr4_async)
    const int row = kr + q;
    const int col = col0 + 4 * pp;
    return img + row * ncols + (((col >> 3) ^ swz128(row)) << 3) + (col & 7);
  };

  if (ks0 < ks1) {
#pragma unroll
    for (int i = 0; i < NST - 1; ++i) stage(i);
    for (int ks = ks0; ks < ks1; ++ks) {
      const int it = ks - ks0;
      if constexpr (VM == 8) asm volatile("s_waitcnt vmcnt(8)\n\ts_barrier" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(6)\n\ts_barrier" ::: "memory");
      stage((it + NST - 1) % NST);
      const bf16* D = smem + (it % NST) * IMG;
      const bf16* X = D + BK * BM;
#pragma unroll
      for (int h = 0; h < BK / 32; ++h) {
        const int kr = 32 * h + 8 * g;
        bf16x4 al[FM], ah[FM], bl[4], bh[4];
#pragma unroll
        for (int f = 0; f < FM; ++f) {
          const bf16* pa = tra(D, BM, kr, wm * (BM / 2) + f * 16);
          al[f] = tr4_async_at<0>(pa);
          ah[f] = tr4_async_at<8 * BM>(pa);  // + 4 rows
        }
#pragma unroll
        for (int f = 0; f < 4; ++f) {
          const bf16* pb = tra(X, BN, kr, wn * 64 + f * 16);
          bl[f] = tr4_async_at<0>(pb);
          bh[f] = tr4_async_at<8 * BN>(pb);
        }
        lds_wait();
        bf16x8 a[FM], b[4];
#pragma unroll
        for (int f = 0; f < FM; ++f) {
          lds_pin(al[f]);
          lds_pin(ah[f]);
          a[f] = __builtin_shufflevector(al[f], ah[f], 0, 1, 2, 3, 4, 5, 6, 7);
        }
#pragma unroll
        for (int f = 0; f < 4; ++f) {
          lds_pin(bl[f]);
          lds_pin(bh[f]);
          b[f] = __builtin_shufflevector(bl[f], bh[f], 0, 1, 2, 3, 4, 5, 6, 7);
        }
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) acc[i][j] = mma(acc[i][j], a[i], b[j]);
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the DMAs issued past the split
  }

  if (p.direct) {
    // single split, canonical layout (KS == 1, no permutation): write the
    // gradient in place; for a fixed i the 16 lanes of a group cover 16
    // consecutive k of one row: 64-byte runs
    const int kreal = p.kreal > 0 ? p.kreal : p.kf;
#pragma unroll
    for (int i = 0; i < FM; ++i) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int k = k0 + wn * 64 + j * 16 + r16;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int co = co0 + wm * (BM / 2) + i * 16 + 4 * g + e;
          if (co >= p.Cout) continue;
          if (k < kreal) p.gw[(size_t)co * kreal + k] = acc[i][j][e];
          else if (k == p.kf) p.gb[co] = acc[i][j][e];
        }
      }
    }
    return;
  }
  // slab[split][k][co]: lane holds co 4g..4g+3 of column k = r16
  float* slab = p.slab + (size_t)split * p.slab_stride;
#pragma unroll
  for (int i = 0; i < FM; ++i) {
    const int co = co0 + wm * (BM / 2) + i * 16 + 4 * g;
    if (co >= p.Cout) continue;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int k = k0 + wn * 64 + j * 16 + r16;
      if (k > p.kf) continue;
      *reinterpret_cast<f32x4*>(slab + (size_t)k * p.Cout + co) = acc[i][j];
    }
  }
}

// gw[co][c*KK + tap] (+)= sum_s slab[s][tap*C + c][co];  gb[co] from k == kf.
// A workgroup owns 64 consecutive slab floats (16 groups of 4 co); its 16
// waves-lanes per group stride the splits (16 independent 16-byte load
// chains in flight per output group), then the 16 partials are combined in
// LDS in a fixed order: deterministic, latency-parallel over the splits.
__global__ void __launch_bounds__(256) igemm_dw_reduce_kernel(IgemmDwParams p, float* gw, float* gb, float beta) {
  __shared__ f32x4 part[16][17];
  const int grp = threadIdx.x & 15, sl = threadIdx.x >> 4;
  const int64_t total4 = (int64_t)(p.kf + 1) * p.Cout / 4;
  const int64_t e4 = (int64_t)blockIdx.x * 16 + grp;
  f32x4 a0 = {0.f, 0.f, 0.f, 0.f}, a1 = a0;
  if (e4 < total4) {
    const f32x4* src = reinterpret_cast<const f32x4*>(p.slab) + e4;
    const int64_t st4 = p.slab_stride / 4;
    int s = sl;
    for (; s + 16 < p.splitk; s += 32) {
      a0 += src[(size_t)s * st4];
      a1 += src[(size_t)(s + 16) * st4];
    }
    if (s < p.splitk) a0 += src[(size_t)s * st4];
  }
  part[sl][grp] = a0 + a1;
  __syncthreads();
  if (threadIdx.x >= 64) return;
  // 64 threads: output float (grp, lane-in-4)
  const int g4 = threadIdx.x >> 2, c4 = threadIdx.x & 3;
  const int64_t e = ((int64_t)blockIdx.x * 16 + g4) * 4 + c4;
  if (e >= total4 * 4) return;
  float v = 0.f;
#pragma unroll
  for (int q = 0; q < 16; ++q) v += part[q][g4][c4];
  const int k = (int)(e / p.Cout), co = (int)(e - (int64_t)k * p.Cout);
  float* dst;
  const int kreal = p.kreal > 0 ? p.kreal : p.kf;
  if (k < p.kf && k >= kreal) return;
  if (k < p.kf && p.perm_c > 0) {
    const int hw = k / p.perm_c, c = k - hw * p.perm_c;
    dst = gw + (size_t)co * kreal + (size_t)c * p.perm_hw + hw;
  } else if (k < p.kf) {
    const int tap = k / p.C, c = k - tap * p.C;  // KS == 1: tap 0, c = k; row stride kreal
    dst = gw + (size_t)co * kreal + (size_t)c * (p.KS * p.KS) + tap;
  } else {
    dst = gb + co;
  }
  *dst = beta != 0.f ? beta * *dst + v : v;
}

// ---------------------------------------------------------------------------
// weight gradient on BA-channel x 256-column tiles, phase-pipelined
// ---------------------------------------------------------------------------
// Same schedule as igemm_big_kernel (4 phases per 64-pixel K-step, quarter
// tiles staged one K-step ahead, counted vmcnt + raw barriers), with the
// weight-gradient operands: A = dZ [64 pixels][BA/2 channels] halves, B =
// im2col(X) [64 pixels][128 columns] halves, both read transposed
// (ds_read_b64_tr_b16).  The bias column is not a GEMM column here (with
// kf % 256 == 0 it would cost a whole extra tile column): the k0 == 0 tiles
// add db = dZ^T 1 with one extra MFMA against a ones fragment per (phase,
// channel fragment), spread over the four pixel-column waves.
// 128-byte rows (BA = 128): 32-byte chunk c of row r sits at c ^ h(r),
// h(r) = ((r >> 1) & 1) | ((r >> 3) & 1) << 1 -> the 8 rows of one
// transposed read land on 8 distinct 32-byte bank ranges (as swz128 does for
// 256-byte rows).
__device__ __forceinline__ int swz_tr64(int row) { return 2 * (((row >> 1) & 1) | (((row >> 3) & 1) << 1)); }

template <int BA>
__global__ void __launch_bounds__(kBigT, 1) igemm_dwbig_kernel(IgemmDwParams p) {
  constexpr int BK = 64;
  constexpr int CA = BA / 2, CB = 128;            // columns per A / B half
  constexpr int SA = CA / 8, SB = CB / 8;         // 16-byte slots per row
  constexpr int GA = BK * SA / kBigT, GB = BK * SB / kBigT;
  constexpr int QA = BK * CA, QB = BK * CB;
  constexpr int BUF = 2 * QA + 2 * QB;
  constexpr int FA = CA / 2 / 16;                 // channel fragments per wave per half
  static_assert(GA >= 1 && GB == 2 && FA >= 1, "tile shape");
  __shared__ __attribute__((aligned(16))) bf16 smem[2 * BUF];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r16 = lane & 15, g = lane >> 4;
  const int q = r16 >> 2, pp = r16 & 3;
  const int wr = wave >> 2, wc = wave & 3;

  const int ntm = cdiv(p.Cout, BA), ntn = cdiv(p.kf, 2 * CB);
  const int ntiles = ntm * ntn;
  const int id = xcd_remap(blockIdx.x, gridDim.x);
  const int tile = id % ntiles, split = id / ntiles;
  if (split >= p.splitk) return;
  const int tm = tile % ntm, tn = tile / ntm;
  const int co0 = tm * BA, k0 = tn * 2 * CB;
  const int nks = cdiv(p.M, BK);
  const int per = cdiv(nks, p.splitk);
  const int ks0 = split * per, ks1 = min(nks, ks0 + per);

  const bf16* dz = static_cast<const bf16*>(p.dz);
  const bf16* in = static_cast<const bf16*>(p.in);
  const uint64_t zero_u = reinterpret_cast<uint64_t>(kIgZero);
  auto swa = [](int row) { return SA == 16 ? swz128(row) : swz_tr64(row); };

  // dZ pieces: row (pixel in the K-step) and channel offset in the half, per j
  // (host: Cout % BA == 0, so every channel column of the tile exists)
  int da_row[GA], da_col[GA];
#pragma unroll
  for (int j = 0; j < GA; ++j) {
    const int s = j * kBigT + tid;
    const int row = s / SA;
    da_row[j] = row;
    da_col[j] = co0 + ((s % SA) ^ swa(row)) * 8;
  }
  // X pieces: pixel row j (decoded once, advanced per K-step with carries),
  // tap/channel per (half, j) packed as c << 8 | ky << 4 | kx (-1: k >= kf)
  // (round 5) the pixel's input corner (iy0, ix0) and its element offset pb
  // are carried along with (oy, ox) -- no per-step multiplies: a piece was
  // 5 quarter-rate v_mul_lo_u32 (stride, H, W, C) per K-step
  int m_[GB], oy_[GB], ox_[GB], iy0_[GB], ix0_[GB], pb_[GB];
  int x_tap[2][GB], x_off[2][GB];
#pragma unroll
  for (int j = 0; j < GB; ++j) {
    const int s = j * kBigT + tid;
    const int row = s >> 4;
    const int m = ks0 * BK + row;
    m_[j] = m;
    const int b = mdiv(p.div_ohw, m);
    const int rem = m - b * p.OH * p.OW;
    oy_[j] = mdiv(p.div_ow, rem);
    ox_[j] = rem - oy_[j] * p.OW;
    iy0_[j] = oy_[j] * p.stride - p.pad;
    ix0_[j] = ox_[j] * p.stride - p.pad;
    pb_[j] = ((b * p.H + iy0_[j]) * p.W + ix0_[j]) * p.C;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int k = k0 + h * CB + ((s & 15) ^ swz128(row)) * 8;
      if (k < p.kf) {
        const int tap = k / p.C, c = k - tap * p.C;
        const int ky = tap / p.KS, kx = tap - ky * p.KS;
        x_tap[h][j] = (ky << 4) | kx;
        x_off[h][j] = (ky * p.W + kx) * p.C + c;
      } else {
        x_tap[h][j] = -1;
        x_off[h][j] = 0;
      }
    }
  }
  // uniform carry increments of (iy0, ix0, pb)
  const int sW = p.stride * p.W, sC = p.stride * p.C;
  const int inc_x = p.adv_x * sC, inc_c1 = (sW - p.OW * p.stride) * p.C, inc_y = p.adv_y * sW * p.C;
  const int inc_c2 = (p.H - p.OH * p.stride) * p.W * p.C, inc_b = p.adv_b * p.H * p.W * p.C;

  auto stage_a = [&](int ks, int h) {
    bf16* dst = smem + ((ks - ks0) & 1) * BUF + h * QA;
#pragma unroll
    for (int j = 0; j < GA; ++j) {
      const int m = ks * BK + da_row[j];
      const bool ok = m < p.M;
      const uint64_t src = reinterpret_cast<uint64_t>(dz + (size_t)m * p.ldz + da_col[j] + h * CA);
      glds16(reinterpret_cast<const bf16*>(ok ? src : zero_u), dst + (j * kBigT + wave * 64) * 8);
    }
  };
  auto stage_b = [&](int ks, int h) {  // pixel geometry currently decoded for K-step ks
    bf16* dst = smem + ((ks - ks0) & 1) * BUF + 2 * QA + h * QB;
#pragma unroll
    for (int j = 0; j < GB; ++j) {
      const int t = x_tap[h][j];
      const int iy = iy0_[j] + ((t >> 4) & 15), ix = ix0_[j] + (t & 15);
      const bool ok = t >= 0 && m_[j] < p.M && (unsigned)iy < (unsigned)p.H && (unsigned)ix < (unsigned)p.W;
      const int off = pb_[j] + x_off[h][j];  // < 2^31 (host check); unused if !ok
      const uint64_t src = reinterpret_cast<uint64_t>(in) + 2 * (uint64_t)(uint32_t)off;
      glds16(reinterpret_cast<const bf16*>(ok ? src : zero_u), dst + (j * kBigT + wave * 64) * 8);
    }
  };
  auto advance = [&]() {
#pragma unroll
    for (int j = 0; j < GB; ++j) {
      m_[j] += BK;
      ox_[j] += p.adv_x;
      ix0_[j] += p.adv_x * p.stride;
      pb_[j] += inc_x;
      if (ox_[j] >= p.OW) {  // (compiles to selects)
        ox_[j] -= p.OW;
        ix0_[j] -= p.OW * p.stride;
        oy_[j] += 1;
        iy0_[j] += p.stride;
        pb_[j] += inc_c1;
      }
      oy_[j] += p.adv_y;
      iy0_[j] += p.adv_y * p.stride;
      pb_[j] += inc_y;
      if (oy_[j] >= p.OH) {
        oy_[j] -= p.OH;
        iy0_[j] -= p.OH * p.stride;
        pb_[j] += inc_c2;
      }
      pb_[j] += inc_b;
    }
  };

  f32x4 acc[2][FA][2][2], accb[2];
#pragma unroll
  for (int a = 0; a < 2; ++a) {
    accb[a] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int f = 0; f < FA; ++f)
#pragma unroll
      for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int e = 0; e < 2; ++e) acc[a][f][b][e] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  const bool bias_wave = k0 == 0 && wc < FA;  // wave-uniform
  bf16x8 ones;
#pragma unroll
  for (int e = 0; e < 8; ++e) ones[e] = (bf16)1.0f;

  // transposed fragment: 4 consecutive pixel rows of 16 columns per call
  // transposed reads as inline asm (tr4_async): with the builtin the compiler
  // put an s_waitcnt vmcnt(0) in front of every quarter's reads, draining the
  // quarter pipeline's DMA lookahead (measured: the ISA showed vmcnt(4),
  // s_barrier, vmcnt(0) per quarter)
  // Address of the 4-row block at rows 8g + q (ks 0, low half); the other
  // three blocks of a fragment pair (rows + 4, + 32, + 36) have the same
  // swizzle (it depends on row & 3 and row bit 3 only), so they are constant
  // byte offsets in the instruction (tr4_async_at): no v_add per read.
  auto tr_addr = [&](const bf16* img, int ncols, int col0) {
    const int row = 8 * g + q;
    const int col = col0 + 4 * pp;
    const int sw = ncols == 128 ? swz128(row) : swz_tr64(row);
    return img + row * ncols + (((col >> 3) ^ sw) << 3) + (col & 7);
  };
  bf16x8 fa[FA][2], fb0[2][2], fb1[2][2];
  auto read_a = [&](const bf16* img, int h) {
    bf16x4 lo[FA][2], hi[FA][2];
#pragma unroll
    for (int f = 0; f < FA; ++f) {
      const bf16* a0 = tr_addr(img + h * QA, CA, wr * (CA / 2) + f * 16);
      lo[f][0] = tr4_async_at<0>(a0);
      hi[f][0] = tr4_async_at<8 * CA>(a0);
      lo[f][1] = tr4_async_at<64 * CA>(a0);
      hi[f][1] = tr4_async_at<72 * CA>(a0);
    }
    lds_wait();
#pragma unroll
    for (int f = 0; f < FA; ++f)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        lds_pin(lo[f][ks]);
        lds_pin(hi[f][ks]);
        fa[f][ks] = __builtin_shufflevector(lo[f][ks], hi[f][ks], 0, 1, 2, 3, 4, 5, 6, 7);
      }
  };
  auto read_b = [&](const bf16* img, int h, bf16x8 (&fb)[2][2]) {
    bf16x4 lo[2][2], hi[2][2];
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const bf16* b0 = tr_addr(img + 2 * QA + h * QB, CB, wc * 32 + e * 16);
      lo[e][0] = tr4_async_at<0>(b0);
      hi[e][0] = tr4_async_at<8 * CB>(b0);
      lo[e][1] = tr4_async_at<64 * CB>(b0);
      hi[e][1] = tr4_async_at<72 * CB>(b0);
    }
    lds_wait();
#pragma unroll
    for (int e = 0; e < 2; ++e)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        lds_pin(lo[e][ks]);
        lds_pin(hi[e][ks]);
        fb[e][ks] = __builtin_shufflevector(lo[e][ks], hi[e][ks], 0, 1, 2, 3, 4, 5, 6, 7);
      }
  };
  auto mfma_q = [&](int ha, int hb, const bf16x8 (&fb)[2][2]) {
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int f = 0; f < FA; ++f)
#pragma unroll
        for (int e = 0; e < 2; ++e) acc[ha][f][hb][e] = mma(acc[ha][f][hb][e], fa[f][ks], fb[e][ks]);
  };
  auto mfma_bias = [&](int ha) {
    if (!bias_wave) return;
#pragma unroll
    for (int f = 0; f < FA; ++f)
      if (f == wc)
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) accb[ha] = mma(accb[ha], fa[f][ks], ones);
  };

  if (ks0 < ks1)
    pipe_loop<GA, GB>(
        ks1 - ks0,
        [&](int t, int q) {
          const bf16* img = smem + (t & 1) * BUF;
          if (q == 0) { read_a(img, 0); read_b(img, 0, fb0); }
          else if (q == 1) read_b(img, 1, fb1);
          else read_a(img, 1);
        },
        [&](int t, int q) {  // the B quarters use the decoded pixels of K-step t, advanced after B1
          if (q == 0) stage_a(ks0 + t, 0);
          else if (q == 1) stage_b(ks0 + t, 0);
          else if (q == 2) { stage_b(ks0 + t, 1); advance(); }
          else stage_a(ks0 + t, 1);
        },
        [&](int q) {
          if (q == 0) { mfma_q(0, 0, fb0); mfma_bias(0); }
          else if (q == 1) mfma_q(0, 1, fb1);
          else if (q == 2) mfma_q(1, 1, fb1);
          else { mfma_q(1, 0, fb0); mfma_bias(1); }
        });

  if (p.direct) {
    // one split, KS == 1, canonical order: write the gradient in place (the
    // 16 lanes of a group cover 16 consecutive k of one row: 64-byte runs)
    const int kreal = p.kreal > 0 ? p.kreal : p.kf;
#pragma unroll
    for (int ha = 0; ha < 2; ++ha) {
#pragma unroll
      for (int f = 0; f < FA; ++f) {
        const int co = co0 + ha * CA + wr * (CA / 2) + f * 16 + 4 * g;
#pragma unroll
        for (int hb = 0; hb < 2; ++hb)
#pragma unroll
          for (int e = 0; e < 2; ++e) {
            const int k = k0 + hb * CB + wc * 32 + e * 16 + r16;
            if (k < kreal)
#pragma unroll
              for (int i = 0; i < 4; ++i) p.gw[(size_t)(co + i) * kreal + k] = acc[ha][f][hb][e][i];
          }
      }
      if (bias_wave && r16 == 0) {
        const int co = co0 + ha * CA + wr * (CA / 2) + wc * 16 + 4 * g;
#pragma unroll
        for (int i = 0; i < 4; ++i) p.gb[co + i] = accb[ha][i];  // gb: 4-byte alignment only
      }
    }
    return;
  }
  // slab[split][k][co]: lane holds co 4g..4g+3 of column k = r16
  float* slab = p.slab + (size_t)split * p.slab_stride;
#pragma unroll
  for (int ha = 0; ha < 2; ++ha) {
#pragma unroll
    for (int f = 0; f < FA; ++f) {
      const int co = co0 + ha * CA + wr * (CA / 2) + f * 16 + 4 * g;
      if (co >= p.Cout) continue;
#pragma unroll
      for (int hb = 0; hb < 2; ++hb)
#pragma unroll
        for (int e = 0; e < 2; ++e) {
          const int k = k0 + hb * CB + wc * 32 + e * 16 + r16;
          if (k < p.kf) *reinterpret_cast<f32x4*>(slab + (size_t)k * p.Cout + co) = acc[ha][f][hb][e];
        }
    }
    if (bias_wave && r16 == 0) {  // every column of the ones product is db
      const int co = co0 + ha * CA + wr * (CA / 2) + wc * 16 + 4 * g;
      if (co < p.Cout) *reinterpret_cast<f32x4*>(slab + (size_t)p.kf * p.Cout + co) = accb[ha];
    }
  }
}

template <int BN, bool BA, bool POOL, bool U8>
void launch_conv(const IgemmParams& p, hipStream_t s) {
  const int nwg = cdiv(p.M, kIgBM) * cdiv(p.N, BN);
  hipLaunchKernelGGL((igemm_conv_kernel<BN, BA, POOL, U8>), dim3((unsigned)nwg), dim3(kIgT), 0, s, p);
}

}  // namespace

bool igemm_conv_supported(int C, int N, int KS) {
  // 128x128 kernel: C % 32 (a K-step spans <= 2 taps; K padded to 64 with
  // zero pieces) -- a 1x1 "conv" (an FC layer over the batch) has one tap, so
  // 8-channel pieces suffice there (ref FC1 1568 -> 200 and its data gradient,
  // K = 200); the 256-tile kernels additionally need C % 64 (igemm_conv)
  return (KS == 1 ? C % 8 == 0 : C % 32 == 0) && N % 8 == 0 && KS <= 16;
}

void igemm_conv(const IgemmParams& p0, hipStream_t s) {
  IgemmParams p = p0;
  if (p.u8) {
    MCC_CHECK(p.N % 8 == 0 && p.epi_bias_act && p.ldw % 8 == 0 && p.ldw >= p.K && p.K <= 64 && p.KS <= 16 &&
                  (int64_t)p.KS * p.W * p.C < (1 << 22),
              "igemm_conv(u8): bad shapes");
  } else {
    MCC_CHECK(igemm_conv_supported(p.C, p.N, p.KS), "igemm_conv: needs C % 32 == 0 (1x1: C % 8) and N % 8 == 0");
  }
  MCC_CHECK(p.K == p.KS * p.KS * p.C, "igemm_conv: K must be KS*KS*C");
  p.c_shift = -1;
  for (int sh = 0; sh < 31; ++sh)
    if (p.C == (1 << sh)) p.c_shift = sh;
  MCC_CHECK(p.M == p.B * p.OH * p.OW && p.M > 0, "igemm_conv: M must be B*OH*OW");
  MCC_CHECK(p.ldw >= p.K && p.ldw % 8 == 0 && p.ldo >= p.N && p.ldo % 4 == 0, "igemm_conv: bad leading dims");
  MCC_CHECK(!p.relu_mask || (!p.epi_bias_act && !p.pool), "igemm_conv: relu_mask is a data-gradient epilogue");
  MCC_CHECK((int64_t)(p.u8 ? 1 : p.B) * p.H * p.W * p.C < (1ll << 31), "igemm_conv: input exceeds 2^31");
  MCC_CHECK(p.OH == (p.H + 2 * p.pad - p.KS) / p.stride + 1 && p.OW == (p.W + 2 * p.pad - p.KS) / p.stride + 1,
            "igemm_conv: output geometry mismatch");
  if (p.pool) {
    MCC_CHECK(p.OH % 2 == 0 && p.OW % 2 == 0 && p.out_arg && p.epi_bias_act && p.ldo == p.N,
              "igemm_conv: fused pool needs even output dims, argmax buffer, dense output");
    p.div_ohw = magic((p.OH / 2) * (p.OW / 2));
    p.div_ow = magic(p.OW / 2);
  } else {
    p.div_ohw = magic(p.OH * p.OW);
    p.div_ow = magic(p.OW);
  }
  const bool ba = p.epi_bias_act;
  if (p.u8) {
    MCC_CHECK(p.N > 64 || p.N % 8 == 0, "igemm_conv(u8): N");
    const bool runs_ok = !ab_flag("u8_bytes");  // A/B: single-byte staging
    p.u8_runs = runs_ok && p.C == 3 && p.KS == 3 && p.pad == 1 && p.stride == 1 && p.W >= 6 && (p.W * 3) % 4 == 0 &&
                reinterpret_cast<uintptr_t>(p.in) % 4 == 0;
    if (p.pool) {
      if (p.N <= 64) launch_conv<64, true, true, true>(p, s); else launch_conv<128, true, true, true>(p, s);
    } else {
      if (p.N <= 64) launch_conv<64, true, false, true>(p, s); else launch_conv<128, true, false, true>(p, s);
    }
    return;
  }
  // 256-pixel tiles for the wide layers (p.tile = 0: 128x128 kernel only;
  // 128: 256x128 tiles only; -1 = auto, as 1)
  // (round 5: 256x128 tiles for the pooled 128-channel conv2 measured 18.66 k
  // vs 18.70 k img/s with the in-lane pool epilogue; all 128-channel layers
  // on them 16.7 k)
  const int big_mode = p.tile >= 0 ? p.tile : 1;
  // auto: 256x256 tiles where N % 256 == 0 (the 128-channel variant measured
  // slower than the 128x128 kernel on VGG conv2 / conv3-dX: profiles/igemm256_ab_r2.txt)
  if (p.C % 64 == 0 &&
      ((big_mode == 1 && p.N % 256 == 0) || ((big_mode == 128 || big_mode == 256) && p.N % 128 == 0))) {
    const bool c256 = p.N % 256 == 0 && big_mode != 128;
    const int nwg = cdiv(p.M, kBigBP) * (p.N / (c256 ? 256 : 128));
#define MCC_BIG(BC, BA, PL) \
  hipLaunchKernelGGL((igemm_big_kernel<BC, BA, PL>), dim3((unsigned)nwg), dim3(kBigT), 0, s, p)
    if (c256) {
      if (p.pool) MCC_BIG(256, true, true); else if (ba) MCC_BIG(256, true, false); else MCC_BIG(256, false, false);
    } else {
      if (p.pool) MCC_BIG(128, true, true); else if (ba) MCC_BIG(128, true, false); else MCC_BIG(128, false, false);
    }
#undef MCC_BIG
    return;
  }
  if (p.pool) {
    if (p.N <= 64) launch_conv<64, true, true, false>(p, s); else launch_conv<128, true, true, false>(p, s);
  } else if (p.N <= 64) {
    if (ba) launch_conv<64, true, false, false>(p, s); else launch_conv<64, false, false, false>(p, s);
  } else {
    if (ba) launch_conv<128, true, false, false>(p, s); else launch_conv<128, false, false, false>(p, s);
  }
}

// weight-gradient tile: 0 = 128x128 kernel, 128 / 256 = igemm_dwbig_kernel<BA>
static int dw_big_ba(int Cout, int kf, int tile) {
  const int mode = tile >= 0 ? tile : 1;  // 1: auto
  if (mode == 0 || Cout % 128 != 0 || kf < 256 || kf >= (1 << 23)) return 0;  // kernel packs c << 8
  if (mode == 1) return Cout % 256 == 0 ? 256 : 0;  // auto: the 128-channel variant lost to 128x128 (conv2)
  return (Cout % 256 == 0 && mode != 128) ? 256 : 128;
}

// co tile of the 128-column weight-gradient kernel: one tile for 129..256
// output channels (see igemm_dw_kernel)
static int dw_bm(int Cout) { return Cout > 128 ? 256 : 128; }

int igemm_dw_splitk(int M, int Cout, int kf, int tile) {
  const int nks = cdiv(M, kIgBK);
  const int ba = dw_big_ba(Cout, kf, tile);
  if (ba) {
    // one 512-thread workgroup per CU: pick the split count that fills whole
    // rounds of 256 workgroups (>= 8 K-steps per split)
    const int tiles = (Cout / ba) * cdiv(kf, 256);
    const int cap = std::max(1, nks / 8);
    for (int r = 1; r <= 8; ++r) {
      const int sk = std::min(cap, (256 * r) / tiles);
      if (sk >= 1 && (double)tiles * sk >= 0.85 * 256 * r) return sk;
      if (sk >= cap) return std::max(1, sk);
    }
    return std::max(1, std::min(cap, 2048 / tiles));
  }
  const int tiles = cdiv(Cout, dw_bm(Cout)) * cdiv(kf + 1, 128);
  const int nks32 = cdiv(M, kDwBK);
  // BM = 128: ~4 workgroups per CU over the launch; BM = 256 (twice the work
  // per K-step): one round of two per CU -- fewer slabs to write and reduce
  int sk = std::max(1, (dw_bm(Cout) == 256 ? 512 : 1024) / tiles);
  sk = std::min(sk, std::max(1, nks32 / 8));   // >= 8 K-steps per slice (the ring is 4 deep)
  return std::min(sk, 1024);
}

size_t igemm_dw_slab_bytes(int Cout, int kf, int splitk) { return (size_t)splitk * (kf + 1) * Cout * 4; }

void igemm_dw(const IgemmDwParams& p0, float* gw, float* gb, float beta, hipStream_t s) {
  IgemmDwParams p = p0;
  // dz rows are read in 8-channel pieces up to round_up(Cout, 8) <= ldz (pad
  // columns only feed output rows that are never written)
  MCC_CHECK(p.C % 8 == 0 && p.Cout % 4 == 0 && p.kf == p.KS * p.KS * p.C, "igemm_dw: needs C % 8, Cout % 4 == 0");
  MCC_CHECK(p.M == p.B * p.OH * p.OW && p.M > 0 && p.ldz >= ((p.Cout + 7) & ~7) && p.ldz % 8 == 0,
            "igemm_dw: bad shapes");
  MCC_CHECK((int64_t)p.B * p.H * p.W * p.C < (1ll << 31), "igemm_dw: input exceeds 2^31 elements");
  MCC_CHECK(p.splitk >= 1 && p.slab_stride >= (int64_t)(p.kf + 1) * p.Cout, "igemm_dw: bad split/slab");
  MCC_CHECK(p.kreal == 0 || (p.KS == 1 && p.kreal <= p.kf), "igemm_dw: kreal needs KS == 1");
  MCC_CHECK(p.perm_c == 0 || (p.KS == 1 && (int64_t)p.perm_c * p.perm_hw == (p.kreal ? p.kreal : p.kf)),
            "igemm_dw: bad permutation");
  p.div_ohw = magic(p.OH * p.OW);
  p.div_ow = magic(p.OW);
  const int ba = dw_big_ba(p.Cout, p.kf, p.tile);
  {  // +BK output pixels per K-step as (ox, oy, b) increments with carries
    const int bk = ba ? kIgBK : kDwBK;
    const int q = bk / p.OW;
    p.adv_x = bk % p.OW;
    p.adv_y = q % p.OH;
    p.adv_b = q / p.OH;
  }
  p.gw = gw;
  p.gb = gb;
  if (ba) {
    MCC_CHECK(p.KS < 16, "igemm_dw: 256-column kernel packs ky, kx in 4 bits");
    p.direct = p.splitk == 1 && p.KS == 1 && p.perm_c == 0 && beta == 0.f;
    const int nwg = (p.Cout / ba) * cdiv(p.kf, 256) * p.splitk;
    if (ba == 256) hipLaunchKernelGGL((igemm_dwbig_kernel<256>), dim3((unsigned)nwg), dim3(kBigT), 0, s, p);
    else hipLaunchKernelGGL((igemm_dwbig_kernel<128>), dim3((unsigned)nwg), dim3(kBigT), 0, s, p);
    if (p.direct) return;
  } else {
    const int bm = dw_bm(p.Cout);
    const int nwg = cdiv(p.Cout, bm) * cdiv(p.kf + 1, 128) * p.splitk;
    p.direct = p.splitk == 1 && p.KS == 1 && p.perm_c == 0 && beta == 0.f;
    if (bm == 256) hipLaunchKernelGGL((igemm_dw_kernel<256, 3>), dim3((unsigned)nwg), dim3(kIgT), 0, s, p);
    else hipLaunchKernelGGL((igemm_dw_kernel<128, 4>), dim3((unsigned)nwg), dim3(kIgT), 0, s, p);
    if (p.direct) return;
  }
  const int64_t total4 = (int64_t)(p.kf + 1) * p.Cout / 4;  // Cout % 8 == 0
  hipLaunchKernelGGL(igemm_dw_reduce_kernel, dim3((unsigned)((total4 + 15) / 16)), dim3(256), 0, s, p, gw, gb, beta);
}

}  // namespace gpu
}  // namespace mcc
