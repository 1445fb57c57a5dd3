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
// DPP quad permutations (lanes 4q..4q+3): xor 1, xor 2
__device__ __forceinline__ float qswap1(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0xB1, 0xf, 0xf, false));
}
__device__ __forceinline__ float qswap2(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x4E, 0xf, 0xf, false));
}
__device__ __forceinline__ int qswap1i(int v) { return __builtin_amdgcn_mov_dpp(v, 0xB1, 0xf, 0xf, false); }
__device__ __forceinline__ int qswap2i(int v) { return __builtin_amdgcn_mov_dpp(v, 0x4E, 0xf, 0xf, false); }

// POOL: fused 2x2/2 max-pool epilogue.  The GEMM rows enumerate (b, py, px,
// pos) so each pooling window is four consecutive rows = four lanes of one
// DPP quad (the C^T fragment holds pixel r16 in lane r16); the max and its
// first-max-wins argmax (PyTorch order) come out of two quad exchanges, and
// the pre-pool conv output is never written.
// U8: the input is the u8 image set (optional sample-index gather, /255 as
// cnn.c:457) with few channels (the first layer): the pixel tile is gathered
// through registers (bytes -> bf16) into the same swizzled LDS image.
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

  const int nk = cdiv(p.K, kIgBK);  // !U8: host guarantees K % 64 == 0 and C % 64 == 0
  auto stage = [&](int kt, int buf) {
    const int k0 = kt * kIgBK;
    bf16* A = smem + buf * IMG;
    bf16* Bw = A + BM * kIgBK;
    if constexpr (U8) {
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
    } else {
      const int tap = k0 / p.C;  // wave-uniform
      const int c0 = k0 - tap * p.C;
      const int ky = tap / p.KS, kx = tap - ky * p.KS;
      const int toff = (ky * p.W + kx) * p.C + c0;
#pragma unroll
      for (int j = 0; j < AJ; ++j) {
        const int iy = a_iy[j] + ky, ix = a_ix[j] + kx;
        const bool ok = (unsigned)iy < (unsigned)p.H && (unsigned)ix < (unsigned)p.W;
        const bf16* src = ok ? in + (a_base[j] + toff + a_seg[j]) : zero;
        glds16(src, A + (j * kIgT + wave * 64) * 8);
      }
    }
#pragma unroll
    for (int j = 0; j < BJ; ++j) {
      const bf16* src = (b_ptr[j] && (!U8 || k0 + b_k[j] < p.ldw)) ? b_ptr[j] + k0 : zero;
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
        for (int j = 0; j < FM; ++j) acc[i][j] = mma(acc[i][j], wb[i], xa[j]);
    }
    __syncthreads();
  }

  // ---- epilogue: lane holds channels 4g..4g+3 of pixel r16 per fragment ----
  bf16* out = static_cast<bf16*>(p.out);
#pragma unroll
  for (int i = 0; i < FN; ++i) {
    const int ch = n0 + wn * (BN / 2) + i * 16 + 4 * g;
    const bool chok = ch < p.N;
    float bv[4] = {0.f, 0.f, 0.f, 0.f};
    if (BIAS_ACT && p.bias && chok) {
#pragma unroll
      for (int e = 0; e < 4; ++e) bv[e] = p.bias[ch + e];
    }
#pragma unroll
    for (int j = 0; j < FM; ++j) {
      const int m = m0 + wm * 64 + j * 16 + r16;
      float v[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = acc[i][j][e];
      uint32_t arg = 0;
      if constexpr (POOL) {  // every lane of the quad takes part in the exchange
        const int pos = r16 & 3;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          int a = pos;
          float o = qswap1(v[e]);
          int oa = qswap1i(a);
          if (o > v[e] || (o == v[e] && oa < a)) { v[e] = o; a = oa; }
          o = qswap2(v[e]);
          oa = qswap2i(a);
          if (o > v[e] || (o == v[e] && oa < a)) { v[e] = o; a = oa; }
          arg |= (uint32_t)a << (8 * e);
        }
      }
      if (!chok || m >= p.M) continue;
      if (POOL && (r16 & 3) != 0) continue;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        v[e] += bv[e];
        if (BIAS_ACT) v[e] = act_apply(p.act, v[e]);
      }
      const bf16x4 o = {(bf16)v[0], (bf16)v[1], (bf16)v[2], (bf16)v[3]};
      const int orow = POOL ? (m >> 2) : m;
      if (POOL && BIAS_ACT && p.act == ACT_RELU) {  // ReLU-inactive window: argmax byte 4
#pragma unroll
        for (int e = 0; e < 4; ++e)
          if (!((float)o[e] > 0.f)) arg = (arg & ~(0xffu << (8 * e))) | (4u << (8 * e));
      }
      *reinterpret_cast<bf16x4*>(out + (size_t)orow * p.ldo + ch) = o;
      if (POOL) *reinterpret_cast<uint32_t*>(p.out_arg + (size_t)orow * p.N + ch) = arg;
    }
  }
}

// ---------------------------------------------------------------------------
// weight gradient (split-K over pixels)
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(kIgT, 2) igemm_dw_kernel(IgemmDwParams p) {
  constexpr int BM = 128, BN = 128, BK = 64;  // co x k x pixels
  constexpr int J = BK * 16 / kIgT;            // glds per thread per operand (4)
  constexpr int IMG = (BM + BN) * BK;
  __shared__ __attribute__((aligned(16))) bf16 smem[2 * IMG];

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
  // logical 16-byte slot (8 output channels / 8 im2col columns).  The row's
  // pixel (b, oy, ox) is decoded once and then advanced by BK pixels per
  // K-step with carries (the K-steps of a split are staged in order), and
  // every source is picked by selects: no per-step divisions, no branches.
  int d_col[J], m_[J], b_[J], oy_[J], ox_[J];
  int x_ky[J], x_kx[J], x_c[J], x_kind[J];  // kind: 0 tap, 1 ones, 2 zero
#pragma unroll
  for (int j = 0; j < J; ++j) {
    const int s = j * kIgT + tid;
    const int row = s >> 4;
    const int ls = (s & 15) ^ swz128(row);
    d_col[j] = co0 + ls * 8;
    const int k = k0 + ls * 8;
    if (k < p.kf) {
      const int tap = k / p.C;
      x_c[j] = k - tap * p.C;
      x_ky[j] = tap / p.KS;
      x_kx[j] = tap - x_ky[j] * p.KS;
      x_kind[j] = 0;
    } else {
      x_c[j] = 0; x_ky[j] = 0; x_kx[j] = 0;
      x_kind[j] = k == p.kf ? 1 : 2;
    }
    const int m = ks0 * BK + row;
    m_[j] = m;
    b_[j] = mdiv(p.div_ohw, m);
    const int rem = m - b_[j] * p.OH * p.OW;
    oy_[j] = mdiv(p.div_ow, rem);
    ox_[j] = rem - oy_[j] * p.OW;
  }
  const uint64_t zero_u = reinterpret_cast<uint64_t>(zero), ones_u = reinterpret_cast<uint64_t>(ones);

  auto stage = [&](int buf) {  // the next K-step of this split
    bf16* D = smem + buf * IMG;
    bf16* X = D + BK * BM;
#pragma unroll
    for (int j = 0; j < J; ++j) {
      const bool mok = m_[j] < p.M;
      const uint64_t dz_u = reinterpret_cast<uint64_t>(dz + (size_t)m_[j] * p.ldz + d_col[j]);
      const bf16* dsrc = reinterpret_cast<const bf16*>((mok && d_col[j] < p.Cout) ? dz_u : zero_u);  // piece may span the pad
      glds16(dsrc, D + (j * kIgT + wave * 64) * 8);
      const int iy = oy_[j] * p.stride - p.pad + x_ky[j], ix = ox_[j] * p.stride - p.pad + x_kx[j];
      const bool tap_ok = mok && x_kind[j] == 0 && (unsigned)iy < (unsigned)p.H && (unsigned)ix < (unsigned)p.W;
      const int off = ((b_[j] * p.H + iy) * p.W + ix) * p.C + x_c[j];  // < 2^31 (host check); unused if !tap_ok
      const uint64_t x_u = reinterpret_cast<uint64_t>(in) + 2 * (uint64_t)(uint32_t)off;
      const uint64_t xs = tap_ok ? x_u : ((mok && x_kind[j] == 1) ? ones_u : zero_u);
      glds16(reinterpret_cast<const bf16*>(xs), X + (j * kIgT + wave * 64) * 8);
      // advance this row by BK pixels
      m_[j] += BK;
      ox_[j] += p.adv_x;
      const int c1 = ox_[j] >= p.OW ? 1 : 0;
      ox_[j] -= c1 * p.OW;
      oy_[j] += p.adv_y + c1;
      const int c2 = oy_[j] >= p.OH ? 1 : 0;
      oy_[j] -= c2 * p.OH;
      b_[j] += p.adv_b + c2;
    }
  };

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // transpose-read of a [BK][128] image: 4 consecutive K rows (pixels) of
  // 16 columns; lane 4q+p of a 16-lane group addresses row kr+q, columns 4p..
  auto tr = [&](const bf16* img, int kr, int col0) {
    const int row = kr + q;
    const int col = col0 + 4 * pp;
    return tr4(img + row * 128 + (((col >> 3) ^ swz128(row)) << 3) + (col & 7));
  };

  if (ks0 < ks1) {
    stage(0);
    __syncthreads();
    for (int ks = ks0; ks < ks1; ++ks) {
      const int buf = (ks - ks0) & 1;
      if (ks + 1 < ks1) stage(buf ^ 1);
      const bf16* D = smem + buf * IMG;
      const bf16* X = D + BK * BM;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int kr = 32 * h + 8 * g;
        bf16x8 a[4], b[4];
#pragma unroll
        for (int f = 0; f < 4; ++f) {
          const bf16x4 lo = tr(D, kr, wm * 64 + f * 16), hi = tr(D, kr + 4, wm * 64 + f * 16);
          a[f] = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
        }
#pragma unroll
        for (int f = 0; f < 4; ++f) {
          const bf16x4 lo = tr(X, kr, wn * 64 + f * 16), hi = tr(X, kr + 4, wn * 64 + f * 16);
          b[f] = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
        }
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) acc[i][j] = mma(acc[i][j], a[i], b[j]);
      }
      __syncthreads();
    }
  }

  if (p.direct) {
    // single split, canonical layout (KS == 1, no permutation): write the
    // gradient in place; for a fixed i the 16 lanes of a group cover 16
    // consecutive k of one row: 64-byte runs
    const int kreal = p.kreal > 0 ? p.kreal : p.kf;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int k = k0 + wn * 64 + j * 16 + r16;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int co = co0 + wm * 64 + i * 16 + 4 * g + e;
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
  for (int i = 0; i < 4; ++i) {
    const int co = co0 + wm * 64 + i * 16 + 4 * g;
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

template <int BN, bool BA, bool POOL, bool U8>
void launch_conv(const IgemmParams& p, hipStream_t s) {
  const int nwg = cdiv(p.M, kIgBM) * cdiv(p.N, BN);
  hipLaunchKernelGGL((igemm_conv_kernel<BN, BA, POOL, U8>), dim3((unsigned)nwg), dim3(kIgT), 0, s, p);
}

}  // namespace

bool igemm_conv_supported(int C, int N, int KS) {
  return C % 64 == 0 && N % 8 == 0 && (KS * KS * C) % kIgBK == 0;
}

void igemm_conv(const IgemmParams& p0, hipStream_t s) {
  IgemmParams p = p0;
  if (p.u8) {
    MCC_CHECK(p.N % 8 == 0 && p.epi_bias_act && p.ldw % 8 == 0 && p.ldw >= p.K && p.K <= 64 && p.KS <= 16 &&
                  (int64_t)p.KS * p.W * p.C < (1 << 22),
              "igemm_conv(u8): bad shapes");
  } else {
    MCC_CHECK(igemm_conv_supported(p.C, p.N, p.KS), "igemm_conv: needs C % 64 == 0 and N % 8 == 0");
  }
  MCC_CHECK(p.K == p.KS * p.KS * p.C, "igemm_conv: K must be KS*KS*C");
  MCC_CHECK(p.M == p.B * p.OH * p.OW && p.M > 0, "igemm_conv: M must be B*OH*OW");
  MCC_CHECK(p.ldw >= p.K && p.ldw % 8 == 0 && p.ldo >= p.N && p.ldo % 4 == 0, "igemm_conv: bad leading dims");
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
    if (p.pool) {
      if (p.N <= 64) launch_conv<64, true, true, true>(p, s); else launch_conv<128, true, true, true>(p, s);
    } else {
      if (p.N <= 64) launch_conv<64, true, false, true>(p, s); else launch_conv<128, true, false, true>(p, s);
    }
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

int igemm_dw_splitk(int M, int Cout, int kf) {
  const int tiles = cdiv(Cout, 128) * cdiv(kf + 1, 128);
  const int nks = cdiv(M, kIgBK);
  int sk = std::max(1, 1024 / tiles);         // ~4 workgroups per CU in flight
  sk = std::min(sk, std::max(1, nks / 4));    // >= 4 K-steps per slice
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
  {  // +kIgBK output pixels as (ox, oy, b) increments with carries (igemm_dw_kernel)
    const int q = kIgBK / p.OW;
    p.adv_x = kIgBK % p.OW;
    p.adv_y = q % p.OH;
    p.adv_b = q / p.OH;
  }
  const int nwg = cdiv(p.Cout, 128) * cdiv(p.kf + 1, 128) * p.splitk;
  p.direct = p.splitk == 1 && p.KS == 1 && p.perm_c == 0 && beta == 0.f;
  p.gw = gw;
  p.gb = gb;
  hipLaunchKernelGGL(igemm_dw_kernel, dim3((unsigned)nwg), dim3(kIgT), 0, s, p);
  if (p.direct) return;
  const int64_t total4 = (int64_t)(p.kf + 1) * p.Cout / 4;  // Cout % 8 == 0
  hipLaunchKernelGGL(igemm_dw_reduce_kernel, dim3((unsigned)((total4 + 15) / 16)), dim3(256), 0, s, p, gw, gb, beta);
}

}  // namespace gpu
}  // namespace mcc
