// Implicit-GEMM convolution on MFMA for small images (whole image tile in LDS).
//
// Replaces the reference's scalar 6-deep loops (Layer_feedForw_conv,
// cnn.c:175-210; Layer_feedBack_conv, cnn.c:212-247) and its one-thread-per-
// output fp64 CUDA kernel (conv_forward_kernel, CUDAcnn.cu:167-195).
//
// Design (gfx950):
//  * A workgroup stages `imgs` whole input images (with the zero halo) into
//    LDS once, channels padded to 8 ("cvec") so one (kernel-position,
//    8-channel group) im2col fragment is a single 16-byte ds_read.  Staging is
//    vectorised per 8-channel group for every input transform.
//  * GEMM rows are output pixels, ordered by 2x2 pooling window when a max-
//    pool is fused: the 16x16 MFMA C-fragment then gives each lane exactly one
//    window (4 consecutive rows) of one channel, so bias + ReLU + maxpool +
//    argmax is an in-register epilogue (no pre-pool tensor ever hits HBM).
//  * Row -> LDS-offset math is table driven (per-image pixel table in LDS,
//    reciprocal-multiply division) so the MFMA loop is not VALU-bound on
//    index arithmetic.
//  * Backward-data is the same kernel run as a stride-1 conv over the
//    zero-inserted output gradient with flipped/transposed packed weights; the
//    ReLU mask and the max-pool routing are applied while staging (IN_RELU /
//    IN_UNPOOL), so no separate unpool/activation-grad pass exists.
//  * Weight gradient: MFMA with the pixel dimension as the reduction axis,
//    the output-gradient tile staged transposed ([co][pixel]), a ones-column
//    appended to im2col so the bias gradient falls out of the same MFMAs; the
//    four waves split the pixel chunks and are combined in LDS in a fixed
//    order; per-workgroup fp32 slabs are reduced deterministically afterwards.
#include "kernels.h"
#include "mfma.h"

namespace mcc {
namespace gpu {

namespace {

// ---------------------------------------------------------------------------
// Staging.  Every tile is staged in two passes: a vectorised zero fill of the
// whole LDS image (halo, channel padding, images past N), a barrier, then a
// scatter pass over the SOURCE elements only.  The scatter moves channel runs
// with the widest aligned access (16 B / 4 B / 2 B), and each thread issues
// U independent loads before its first LDS store so the global-load latency
// of the (L2-resident) activations overlaps instead of serialising.

constexpr int U = 4;  // loads in flight per thread in the scatter passes

__device__ __forceinline__ int chan_vw(int SC) { return (SC & 7) == 0 ? 8 : ((SC & 1) == 0 ? 2 : 1); }

// The three divisors a scatter pass needs, built once per kernel (they depend
// only on the source geometry, not on the stage's image range):
//   dense / relu: (channel runs CV, SW, SH*SW)
//   unpool:       (channel runs CV, PW, PH*PW)
//   u8:           (SC, words per row, words per image) or, for rows that are
//                 not whole words, (SC, row bytes, SH)
__device__ __forceinline__ int plan_divisor(const StageSrc& s, int which) {
  if (s.mode == IN_U8) {
    const int rb = s.SW * s.SC;
    if (which == 0) return s.SC;
    if ((rb & 3) == 0) return which == 1 ? rb >> 2 : s.SH * (rb >> 2);
    return which == 1 ? rb : s.SH;
  }
  if (which == 0) return s.SC / chan_vw(s.SC);
  if (s.mode == IN_UNPOOL) return which == 1 ? s.PW : s.PH * s.PW;
  return which == 1 ? s.SW : s.SH * s.SW;
}

struct ScatterPlan {
  Div d0, d1, d2;
  __device__ __forceinline__ explicit ScatterPlan(const StageSrc& s)
      : d0(plan_divisor(s, 0)), d1(plan_divisor(s, 1)), d2(plan_divisor(s, 2)) {}
};

template <typename T>
__device__ __forceinline__ void lds_zero(T* p, int n) {
  typedef typename Vec8<T>::type V8;
  V8 z;
#pragma unroll
  for (int j = 0; j < 8; ++j) z[j] = T(0);
  for (int i = threadIdx.x * 8; i < n; i += blockDim.x * 8) store8(p + i, z);
}

__host__ __device__ __forceinline__ int round8(int n) { return (n + 7) & ~7; }

template <typename T, int VW>
__device__ __forceinline__ void ld_run(const T* p, T (&v)[VW]) {
  if constexpr (VW == 8) {
    const auto x = load8(p);
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = x[j];
  } else if constexpr (VW == 2) {
    if constexpr (sizeof(T) == 2) {
      const uint32_t w = *reinterpret_cast<const uint32_t*>(p);
      v[0] = __builtin_bit_cast(T, (unsigned short)(w & 0xffffu));
      v[1] = __builtin_bit_cast(T, (unsigned short)(w >> 16));
    } else {
      const float2 w = *reinterpret_cast<const float2*>(p);
      v[0] = w.x;
      v[1] = w.y;
    }
  } else {
    v[0] = *p;
  }
}

template <typename T, int VW>
__device__ __forceinline__ void st_run(T* p, const T (&v)[VW]) {
  if constexpr (VW == 8) {
    typename Vec8<T>::type x;
#pragma unroll
    for (int j = 0; j < 8; ++j) x[j] = v[j];
    store8(p, x);
  } else if constexpr (VW == 2) {
    if constexpr (sizeof(T) == 2) {
      const uint32_t w = (uint32_t)__builtin_bit_cast(unsigned short, v[0]) |
                         ((uint32_t)__builtin_bit_cast(unsigned short, v[1]) << 16);
      *reinterpret_cast<uint32_t*>(p) = w;
    } else {
      *reinterpret_cast<float2*>(p) = make_float2(v[0], v[1]);
    }
  } else {
    *p = v[0];
  }
}

template <int VW>
__device__ __forceinline__ void ld_arg(const uint8_t* p, uint32_t (&a)[VW]) {
  if constexpr (VW == 8) {
    const uint2 w = *reinterpret_cast<const uint2*>(p);
#pragma unroll
    for (int j = 0; j < 8; ++j) a[j] = ((j < 4 ? w.x : w.y) >> (8 * (j & 3))) & 0xffu;
  } else if constexpr (VW == 2) {
    const uint32_t w = *reinterpret_cast<const unsigned short*>(p);
    a[0] = w & 0xffu;
    a[1] = w >> 8;
  } else {
    a[0] = *p;
  }
}

// Tile coordinate of a source element (zero insertion: s*up + off), -1 if outside.
__device__ __forceinline__ int tile_coord(int sc, const StageSrc& s, int L) {
  const int l = sc * s.up + s.off;
  return (l >= 0 && l < L) ? l : -1;
}

// Where one channel-run of source pixel (sy, sx) lands.  DY=false: the
// NHWC image lds[img][LH][LW][CL]; DY=true: the transposed conv-output
// gradient dys[c][img*OH*OW + y*OW + x] (LH = OH, LW = OW, CL = row stride).
template <bool DY>
__device__ __forceinline__ int dst_index(int img, int ly, int lx, int c, int LH, int LW, int CL) {
  if (DY) return c * CL + (img * LH + ly) * LW + lx;
  return ((img * LH + ly) * LW + lx) * CL + c;
}

template <typename T, int VW, bool RELU, bool DY>
__device__ void scatter_dense(const StageSrc& s, const ScatterPlan& pl, T* lds, int img0, int nimg, int LH, int LW, int CL) {
  const T* src = static_cast<const T*>(s.src);
  const T* ay = static_cast<const T*>(s.aux_y);
  const int CV = s.SC / VW;
  const int spix = s.SH * s.SW;
  const int total = nimg * spix * CV;
  const Div &dcv = pl.d0, &dsw = pl.d1, &dsp = pl.d2;
  for (int e0 = threadIdx.x; e0 < total; e0 += U * blockDim.x) {
    T v[U][VW], y[U][VW];
    int img[U], ly[U], lx[U], c0[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int e = e0 + u * blockDim.x;
      ly[u] = -1;
      if (e < total) {
        const int pix = dcv.div(e), cv = e - pix * CV;
        const int im = dsp.div(pix), rem = pix - im * spix;
        const int sy = dsw.div(rem), sx = rem - sy * s.SW;
        const size_t gi = ((size_t)(img0 + im) * spix + rem) * s.SC + cv * VW;
        ld_run<T, VW>(src + gi, v[u]);
        if (RELU) ld_run<T, VW>(ay + gi, y[u]);
        img[u] = im;
        c0[u] = cv * VW;
        lx[u] = tile_coord(sx, s, LW);
        ly[u] = lx[u] < 0 ? -1 : tile_coord(sy, s, LH);
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (ly[u] < 0) continue;
      if (RELU) {
#pragma unroll
        for (int j = 0; j < VW; ++j) v[u][j] = to_f(y[u][j]) > 0.f ? v[u][j] : T(0);
      }
      if (DY) {
#pragma unroll
        for (int j = 0; j < VW; ++j) lds[dst_index<true>(img[u], ly[u], lx[u], c0[u] + j, LH, LW, CL)] = v[u][j];
      } else {
        st_run<T, VW>(lds + dst_index<false>(img[u], ly[u], lx[u], c0[u], LH, LW, CL), v[u]);
      }
    }
  }
}

// Max-pool + ReLU backward folded into staging: one item per POOLED element
// run; the gradient goes to the argmax position of its 2x2 window when the
// pooled (= post-ReLU) output is positive.  Sparse form: only that position
// is written (the tile was zero-filled).  DENSE form (channel-contiguous
// tiles only): all four window positions are written as vector runs, so a
// tile reused across stages needs no zero fill.
template <typename T, int VW, bool DY, bool DENSE = false>
__device__ void scatter_unpool(const StageSrc& s, const ScatterPlan& pl, T* lds, int img0, int nimg, int LH, int LW, int CL) {
  const T* src = static_cast<const T*>(s.src);
  const T* ay = static_cast<const T*>(s.aux_y);
  const int CV = s.SC / VW;
  const int ppix = s.PH * s.PW;
  const int total = nimg * ppix * CV;
  const Div &dcv = pl.d0, &dpw = pl.d1, &dpp = pl.d2;
  for (int e0 = threadIdx.x; e0 < total; e0 += U * blockDim.x) {
    T d[U][VW], y[U][VW];
    uint32_t a[U][VW];
    int img[U], py[U], px[U], c0[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int e = e0 + u * blockDim.x;
      py[u] = -1;
      if (e < total) {
        const int pix = dcv.div(e), cv = e - pix * CV;
        const int im = dpp.div(pix), rem = pix - im * ppix;
        const size_t gi = ((size_t)(img0 + im) * ppix + rem) * s.SC + cv * VW;
        ld_run<T, VW>(src + gi, d[u]);
        ld_run<T, VW>(ay + gi, y[u]);
        ld_arg<VW>(s.aux_arg + gi, a[u]);
        img[u] = im;
        c0[u] = cv * VW;
        py[u] = dpw.div(rem);
        px[u] = rem - py[u] * s.PW;
      }
    }
    if constexpr (DENSE && !DY) {
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (py[u] < 0) continue;
#pragma unroll
        for (int pos = 0; pos < 4; ++pos) {
          const int lx = tile_coord(2 * px[u] + (pos & 1), s, LW), ly = tile_coord(2 * py[u] + (pos >> 1), s, LH);
          if (lx < 0 || ly < 0) continue;
          T v[VW];
#pragma unroll
          for (int j = 0; j < VW; ++j) v[j] = (a[u][j] == (uint32_t)pos && to_f(y[u][j]) > 0.f) ? d[u][j] : T(0);
          st_run<T, VW>(lds + dst_index<false>(img[u], ly, lx, c0[u], LH, LW, CL), v);
        }
      }
      continue;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (py[u] < 0) continue;
#pragma unroll
      for (int j = 0; j < VW; ++j) {
        if (!(to_f(y[u][j]) > 0.f)) continue;
        const int oy = 2 * py[u] + (int)(a[u][j] >> 1), ox = 2 * px[u] + (int)(a[u][j] & 1);
        const int lx = tile_coord(ox, s, LW), ly = tile_coord(oy, s, LH);
        if (lx < 0 || ly < 0) continue;
        lds[dst_index<DY>(img[u], ly, lx, c0[u] + j, LH, LW, CL)] = d[u][j];
      }
    }
  }
}

// u8 images (optionally gathered through idx), scaled by 1/255 (cnn.c:457).
// Rows are moved as 32-bit words when a row is a whole number of words.
template <typename T>
__device__ void scatter_u8(const StageSrc& s, const ScatterPlan& pl, T* lds, int img0, int nimg, int LH, int LW, int CL) {
  const uint8_t* src = static_cast<const uint8_t*>(s.src);
  const int row_bytes = s.SW * s.SC;
  const float inv = 1.0f / 255.0f;
  const Div& dsc = pl.d0;
  if ((row_bytes & 3) == 0) {
    const int wpr = row_bytes >> 2;
    const int wpi = s.SH * wpr;
    const int total = nimg * wpi;
    const Div &dwpr = pl.d1, &dwpi = pl.d2;
    for (int e0 = threadIdx.x; e0 < total; e0 += U * blockDim.x) {
      uint32_t w[U];
      int img[U], sy[U], wi[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int e = e0 + u * blockDim.x;
        img[u] = -1;
        if (e < total) {
          const int im = dwpi.div(e), rem = e - im * wpi;
          const int y = dwpr.div(rem), ww = rem - y * wpr;
          const int n = img0 + im;
          const int gim = s.idx ? s.idx[n] : n;
          w[u] = *reinterpret_cast<const uint32_t*>(src + ((size_t)gim * s.SH + y) * row_bytes + 4 * ww);
          img[u] = im;
          sy[u] = y;
          wi[u] = ww;
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (img[u] < 0) continue;
        const int ly = tile_coord(sy[u], s, LH);
        if (ly < 0) continue;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int flat = 4 * wi[u] + j;
          const int sx = dsc.div(flat), c = flat - sx * s.SC;
          const int lx = tile_coord(sx, s, LW);
          if (lx < 0) continue;
          lds[((img[u] * LH + ly) * LW + lx) * CL + c] = from_f<T>((float)((w[u] >> (8 * j)) & 0xffu) * inv);
        }
      }
    }
  } else {
    const int total = nimg * s.SH * row_bytes;
    const Div &drb = pl.d1, &dsh = pl.d2;
    for (int e = threadIdx.x; e < total; e += blockDim.x) {
      const int r = drb.div(e), b = e - r * row_bytes;
      const int im = dsh.div(r), y = r - im * s.SH;
      const int n = img0 + im;
      const int gim = s.idx ? s.idx[n] : n;
      const uint8_t v = src[((size_t)gim * s.SH + y) * row_bytes + b];
      const int sx = dsc.div(b), c = b - sx * s.SC;
      const int ly = tile_coord(y, s, LH), lx = tile_coord(sx, s, LW);
      if (ly >= 0 && lx >= 0) lds[((im * LH + ly) * LW + lx) * CL + c] = from_f<T>((float)v * inv);
    }
  }
}

// Scatter pass (after the zero fill + barrier) for an NHWC tile (DY=false) or
// the transposed conv-output gradient (DY=true).
template <typename T, bool DY, bool DENSE = false>
__device__ void stage_scatter(const StageSrc& s, const ScatterPlan& pl, T* lds, int img0, int nimg, int LH, int LW, int CL) {
  const int vw = chan_vw(s.SC);
  switch (s.mode) {
    case IN_U8:
      if (!DY) scatter_u8<T>(s, pl, lds, img0, nimg, LH, LW, CL);
      break;
    case IN_UNPOOL:
      if (vw == 8) scatter_unpool<T, 8, DY, DENSE>(s, pl, lds, img0, nimg, LH, LW, CL);
      else if (vw == 2) scatter_unpool<T, 2, DY, DENSE>(s, pl, lds, img0, nimg, LH, LW, CL);
      else scatter_unpool<T, 1, DY, DENSE>(s, pl, lds, img0, nimg, LH, LW, CL);
      break;
    case IN_RELU:
      if (vw == 8) scatter_dense<T, 8, true, DY>(s, pl, lds, img0, nimg, LH, LW, CL);
      else if (vw == 2) scatter_dense<T, 2, true, DY>(s, pl, lds, img0, nimg, LH, LW, CL);
      else scatter_dense<T, 1, true, DY>(s, pl, lds, img0, nimg, LH, LW, CL);
      break;
    default:
      if (vw == 8) scatter_dense<T, 8, false, DY>(s, pl, lds, img0, nimg, LH, LW, CL);
      else if (vw == 2) scatter_dense<T, 2, false, DY>(s, pl, lds, img0, nimg, LH, LW, CL);
      else scatter_dense<T, 1, false, DY>(s, pl, lds, img0, nimg, LH, LW, CL);
  }
}

// Per-image conv-output pixel -> LDS offset of its top-left tap.  With a fused
// pool the pixel order is (window, position) so a 16-row MFMA tile holds four
// whole 2x2 windows.
__device__ __forceinline__ void pixel_table(int* tab, int rows, bool pool, int OW, int PW, int cs, int LW, int CL) {
  const Div dow(OW), dpw(pool ? PW : 1);
  for (int r = threadIdx.x; r < rows; r += blockDim.x) {
    int oy, ox;
    if (pool) {
      const int win = r >> 2, pos = r & 3;
      const int ph = dpw.div(win), pw = win - ph * PW;
      oy = 2 * ph + (pos >> 1);
      ox = 2 * pw + (pos & 1);
    } else {
      oy = dow.div(r);
      ox = r - oy * OW;
    }
    tab[r] = (oy * cs * LW + ox * cs) * CL;
  }
}

enum FwdEpi : int { FE_POOL = 0, FE_ACT = 1, FE_PLAIN = 2 };

// WL: packed weights staged in LDS (rows padded by 8 elements so the 16 lanes
// of a B-fragment read hit distinct banks); else read from global (L2).
template <typename T, bool CVEC, int MT, int EPI, int ACT, bool WL>
__global__ void __launch_bounds__(256) conv_fwd_kernel(ConvParams p) {
  typedef typename Vec8<T>::type V8;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  T* xs = reinterpret_cast<T*>(smem);
  const int img_elems = p.LH * p.LW * p.CL;
  const int xs_elems = round8(p.imgs * img_elems + 16);
  constexpr bool pool = EPI == FE_POOL;
  const int PH = p.OH >> 1, PW = p.OW >> 1;
  const int rows_per_img = pool ? PH * PW * 4 : p.OH * p.OW;
  const int nk = CVEC ? p.nchunks * 4 : p.nchunks * 32;
  const int ntiles = cdiv(p.Cout, 16);
  const int wrow_ld = p.kpad + 8;
  T* ws = reinterpret_cast<T*>(smem + align16(xs_elems * (int)sizeof(T)));
  float* bias_s = reinterpret_cast<float*>(reinterpret_cast<char*>(ws) +
                                           (WL ? align16(ntiles * 16 * wrow_ld * (int)sizeof(T)) : 0));
  int* ktab = reinterpret_cast<int*>(bias_s + ntiles * 16);
  int* ptab = ktab + ((nk + 3) & ~3);
  const int img0 = blockIdx.x * p.imgs;
  const int nimg = min(p.imgs, p.N - img0);
  const int tid = threadIdx.x;
  const T* wpk = static_cast<const T*>(p.wpk);

  lds_zero(xs, xs_elems);
  if (WL) {
    const int nv = ntiles * 16 * (p.kpad >> 3);
    const int vpr = p.kpad >> 3;
    for (int v = tid; v < nv; v += blockDim.x) {
      const int r = v / vpr, c = (v - r * vpr) * 8;
      store8(ws + r * wrow_ld + c, load8(wpk + (size_t)r * p.kpad + c));
    }
  }
  for (int n = tid; n < ntiles * 16; n += blockDim.x) bias_s[n] = (EPI != FE_PLAIN && n < p.Cout) ? p.bias[n] : 0.f;
  // k -> LDS offset table (relative to a pixel's top-left tap).  Padding
  // entries point at tap 0: their weights are zero, any finite value works.
  const int KK = p.KS * p.KS;
  for (int e = tid; e < nk; e += blockDim.x) {
    int off = 0;
    if (CVEC) {
      const int CG = p.CL >> 3;
      const int kp = e / CG, cg = e - kp * CG;
      if (kp < KK) {
        const int kh = kp / p.KS, kw = kp - kh * p.KS;
        off = (kh * p.LW + kw) * p.CL + cg * 8;
      }
    } else if (e < KK * p.Cin) {
      const int kp = e / p.Cin, c = e - kp * p.Cin;
      const int kh = kp / p.KS, kw = kp - kh * p.KS;
      off = (kh * p.LW + kw) * p.CL + c;
    }
    ktab[e] = off;
  }
  pixel_table(ptab, rows_per_img, pool, p.OW, PW, p.cs, p.LW, p.CL);
  __syncthreads();
  stage_scatter<T, false>(p.in, ScatterPlan(p.in), xs, img0, nimg, p.LH, p.LW, p.CL);
  __syncthreads();

  const int lane = tid & 63, wave = tid >> 6, nwaves = blockDim.x >> 6;
  const int r16 = lane & 15, g = lane >> 4;
  const int M = nimg * rows_per_img;
  const int mtiles = cdiv(M, 16), mgroups = cdiv(mtiles, MT);
  const Div drpi(rows_per_img);
  T* out = static_cast<T*>(p.out);
  const size_t obase = pool ? (size_t)img0 * PH * PW : (size_t)img0 * p.OH * p.OW;

  for (int item = wave; item < ntiles * mgroups; item += nwaves) {
    const int nt = item / mgroups, mg = item - nt * mgroups;
    int base[MT];
#pragma unroll
    for (int t = 0; t < MT; ++t) {
      // rows past M read image 0 (finite, discarded by the epilogue)
      const int r = (mg * MT + t) * 16 + r16;
      const int img = drpi.div(r);
      base[t] = r < M ? img * img_elems + ptab[r - img * rows_per_img] : 0;
    }
    f32x4 acc[MT];
#pragma unroll
    for (int t = 0; t < MT; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
    const T* wrow = WL ? ws + (nt * 16 + r16) * wrow_ld + 8 * g : wpk + (size_t)(nt * 16 + r16) * p.kpad + 8 * g;
    for (int q = 0; q < p.nchunks; ++q) {
      const V8 b = load8(wrow + q * 32);
      if (CVEC) {
        const int ko = ktab[q * 4 + g];
#pragma unroll
        for (int t = 0; t < MT; ++t) acc[t] = mma(acc[t], load8(xs + base[t] + ko), b);
      } else {
        int ko[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) ko[j] = ktab[q * 32 + 8 * g + j];
#pragma unroll
        for (int t = 0; t < MT; ++t) {
          V8 a;
#pragma unroll
          for (int j = 0; j < 8; ++j) a[j] = xs[base[t] + ko[j]];
          acc[t] = mma(acc[t], a, b);
        }
      }
    }
    // Epilogue: rows 4g..4g+3 of each tile belong to this lane, column n.
    const int n = nt * 16 + r16;
    if (n >= p.Cout) continue;
    const float bv = bias_s[n];
#pragma unroll
    for (int t = 0; t < MT; ++t) {
      const int rb = (mg * MT + t) * 16 + 4 * g;
      if (rb >= M) continue;
      float v[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float x = acc[t][i] + bv;
        v[i] = ACT == ACT_RELU ? fmaxf(x, 0.f) : (ACT == ACT_TANH ? tanhf(x) : x);
      }
      if (pool) {
        float best = v[0];
        int arg = 0;
#pragma unroll
        for (int i = 1; i < 4; ++i) {
          const bool gt = v[i] > best;
          best = gt ? v[i] : best;
          arg = gt ? i : arg;
        }
        const size_t o = (obase + (rb >> 2)) * p.Cout + n;
        out[o] = from_f<T>(best);
        // ReLU-inactive window (pooled output <= 0): argmax byte 4, the backward routes nothing
        p.out_arg[o] = (uint8_t)(ACT == ACT_RELU && !(to_f(from_f<T>(best)) > 0.f) ? 4 : arg);
      } else {
        if (rb + 4 <= M) {
#pragma unroll
          for (int i = 0; i < 4; ++i) out[(obase + rb + i) * p.Cout + n] = from_f<T>(v[i]);
        } else {
#pragma unroll
          for (int i = 0; i < 4; ++i)
            if (rb + i < M) out[(obase + rb + i) * p.Cout + n] = from_f<T>(v[i]);
        }
      }
    }
  }
}

// Weight gradient of a conv_small layer, bf16.  Both MFMA operands are
// pixel-major in LDS exactly as staged (no transposes):
//   A = dY^T  from dys[pixel][co]              (row = co,      k = pixel)
//   B = im2col from xs[img][y][x][c4]          (col = (tap,c), k = pixel)
// and each K-fragment (8 pixels) is two transpose reads whose four "rows" are
// four arbitrary pixels (their LDS bases come from a per-pixel table), so the
// im2col gather costs 2 LDS instructions per 16x32 fragment.  The bias
// gradient is the row sum of the A fragments.  Waves split the pixel chunks;
// partial sums are combined in LDS in a fixed order (deterministic).
template <int MTW, int NTW>
__global__ void __launch_bounds__(256) conv_dw_tr_kernel(ConvDwParams p) {
  typedef bf16 T;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int CL = p.CL;  // channel stride of xs (multiple of 4)
  const int img_elems = p.LH * p.LW * CL;
  const int xs_elems = round8(p.imgs * img_elems + 16);
  const int drow = conv_dw_tr_drow(p.cout_pad);
  T* xs = reinterpret_cast<T*>(smem);
  T* dys = reinterpret_cast<T*>(smem + align16(xs_elems * 2));
  int* pixbase = reinterpret_cast<int*>(reinterpret_cast<char*>(dys) + align16(p.ppad * drow * 2));
  int* ptab = pixbase + p.ppad;
  float* red = reinterpret_cast<float*>(smem);  // reused after the main loop

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6, nwaves = blockDim.x >> 6;
  const int r16 = lane & 15, g = lane >> 4;
  const int q = r16 >> 2, pp = r16 & 3;  // transpose-read address role
  const int KK = p.KS * p.KS;
  const int opix = p.OH * p.OW;

  int koff[NTW];
#pragma unroll
  for (int t = 0; t < NTW; ++t) {
    const int c4 = (blockIdx.y * NTW + t) * 16 + 4 * pp;  // first of this lane's 4 columns
    const int kp = c4 / CL, c0 = c4 - kp * CL;
    koff[t] = 0;
    if (kp < KK) {
      const int kh = kp / p.KS, kw = kp - kh * p.KS;
      koff[t] = (kh * p.LW + kw) * CL + c0;
    }
  }
  pixel_table(ptab, opix, false, p.OW, 1, p.cs, p.LW, CL);

  f32x4 acc[MTW][NTW];
  float bsum[MTW];
#pragma unroll
  for (int m = 0; m < MTW; ++m) {
    bsum[m] = 0.f;
#pragma unroll
    for (int t = 0; t < NTW; ++t) acc[m][t] = f32x4{0.f, 0.f, 0.f, 0.f};
  }

  const ScatterPlan plx(p.x), pldy(p.dy);
  // Zero once: every stage rewrites the same interior positions (padding
  // borders, pad channels and pad rows stay zero; UNPOOL staging is dense).
  lds_zero(xs, xs_elems);
  lds_zero(dys, p.ppad * drow);
  __syncthreads();  // ptab
  {
    // stage-invariant pixel -> LDS base table; on a tail stage the rows past
    // its last image read stale (finite) pixels against zeroed dY rows
    const Div dopix(opix);
    const int full = p.imgs * opix;
    for (int pix = tid; pix < p.ppad; pix += blockDim.x) {
      const int img = dopix.div(pix);
      pixbase[pix] = pix < full ? img * img_elems + ptab[pix - img * opix] : 0;
    }
  }
  for (int img0 = blockIdx.x * p.imgs; img0 < p.N; img0 += p.nx * p.imgs) {
    const int nimg = min(p.imgs, p.N - img0);
    const int npix = nimg * opix;
    __syncthreads();  // previous stage fully consumed (and the zero fill done)
    if (nimg < p.imgs) lds_zero(dys + npix * drow, (p.ppad - npix) * drow);  // stale rows of a tail stage
    stage_scatter<T, false>(p.x, plx, xs, img0, nimg, p.LH, p.LW, CL);
    stage_scatter<T, false, true>(p.dy, pldy, dys, img0, nimg, p.OH, p.OW, drow);
    __syncthreads();
    const int nq = cdiv(npix, 32);
    for (int qc = wave; qc < nq; qc += nwaves) {
      // fragment k -> pixel: lane group g reads rows 4g..4g+3 (and +16), so
      // the four groups of a read cover 16 consecutive 32-byte rows
      const int pix1 = qc * 32 + 4 * g + q, pix2 = pix1 + 16;
      const int pb1 = pixbase[pix1], pb2 = pixbase[pix2];
      bf16x8 a[MTW];
#pragma unroll
      for (int m = 0; m < MTW; ++m) {
        const bf16x4 lo = tr4(dys + pix1 * drow + m * 16 + 4 * pp);
        const bf16x4 hi = tr4(dys + pix2 * drow + m * 16 + 4 * pp);
        a[m] = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
#pragma unroll
        for (int j = 0; j < 8; ++j) bsum[m] += (float)a[m][j];
      }
#pragma unroll
      for (int t = 0; t < NTW; ++t) {
        const bf16x4 lo = tr4(xs + pb1 + koff[t]);
        const bf16x4 hi = tr4(xs + pb2 + koff[t]);
        const bf16x8 b = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
#pragma unroll
        for (int m = 0; m < MTW; ++m) acc[m][t] = mma(acc[m][t], a[m], b);
      }
    }
  }
  // bias: lanes r16 hold channel m*16+r16; sum the 4 lane groups
#pragma unroll
  for (int m = 0; m < MTW; ++m) {
    bsum[m] += __shfl_xor(bsum[m], 16);
    bsum[m] += __shfl_xor(bsum[m], 32);
  }
  // Combine the waves in a fixed order: red[MTW*16 rows][NTW*16 + 1 cols].
  const int rcols = NTW * 16 + 1;
  for (int w = 0; w < nwaves; ++w) {
    __syncthreads();
    if (wave == w) {
#pragma unroll
      for (int m = 0; m < MTW; ++m) {
#pragma unroll
        for (int t = 0; t < NTW; ++t)
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            float* d = red + (m * 16 + 4 * g + i) * rcols + t * 16 + r16;
            *d = (w == 0 ? 0.f : *d) + acc[m][t][i];
          }
        if (g == 0) {
          float* d = red + (m * 16 + r16) * rcols + NTW * 16;
          *d = (w == 0 ? 0.f : *d) + bsum[m];
        }
      }
    }
  }
  __syncthreads();
  for (int e = tid; e < p.cout_pad * rcols; e += blockDim.x) {
    const int row = e / rcols, c = e - row * rcols;
    float* srow = p.slab + ((size_t)blockIdx.x * p.cout_pad + row) * p.ncols_pad;
    if (c < NTW * 16) {
      const int col = blockIdx.y * NTW * 16 + c;
      if (col < p.kbias) srow[col] = red[row * rcols + c];
    } else if (blockIdx.y == 0) {
      srow[p.kbias] = red[row * rcols + c];
    }
  }
}

// fp32 / fallback weight gradient (scalar im2col gathers, transposed dY).
template <typename T, bool CVEC, int MTW, int NTW>
__global__ void __launch_bounds__(256) conv_dw_kernel(ConvDwParams p) {
  typedef typename Vec8<T>::type V8;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int img_elems = p.LH * p.LW * p.CL;
  const int xs_elems = round8(p.imgs * img_elems + 16);
  T* xs = reinterpret_cast<T*>(smem);
  const int drow = p.ppad + 8;
  T* dys = reinterpret_cast<T*>(smem + align16(xs_elems * (int)sizeof(T)));
  int* pixbase = reinterpret_cast<int*>(reinterpret_cast<char*>(dys) + align16(p.cout_pad * drow * (int)sizeof(T)));
  int* ptab = pixbase + p.ppad;
  float* red = reinterpret_cast<float*>(smem);  // reused after the main loop

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6, nwaves = blockDim.x >> 6;
  const int r16 = lane & 15, g = lane >> 4;
  const int KK = p.KS * p.KS;
  const int CG = p.CL >> 3;
  const int opix = p.OH * p.OW;

  // im2col column of this lane per owned column tile; padding columns read
  // tap 0 (finite; their dW entries are never used), the bias column reads 1.
  int koff[NTW];
  bool is_bias[NTW];
#pragma unroll
  for (int t = 0; t < NTW; ++t) {
    const int col = (blockIdx.y * NTW + t) * 16 + r16;
    koff[t] = 0;
    is_bias[t] = col == p.kbias;
    if (col < p.kbias) {
      int kp, c;
      if (CVEC) {
        const int G = col >> 3;
        kp = G / CG;
        c = (G - kp * CG) * 8 + (col & 7);
      } else {
        kp = col / p.Cin;
        c = col - kp * p.Cin;
      }
      if (kp < KK) {
        const int kh = kp / p.KS, kw = kp - kh * p.KS;
        koff[t] = (kh * p.LW + kw) * p.CL + c;
      }
    }
  }
  pixel_table(ptab, opix, false, p.OW, 1, p.cs, p.LW, p.CL);

  f32x4 acc[MTW][NTW];
#pragma unroll
  for (int m = 0; m < MTW; ++m)
#pragma unroll
    for (int t = 0; t < NTW; ++t) acc[m][t] = f32x4{0.f, 0.f, 0.f, 0.f};

  const Div dopix(opix);
  const ScatterPlan plx(p.x), pldy(p.dy);
  const T one = T(1);
  for (int img0 = blockIdx.x * p.imgs; img0 < p.N; img0 += p.nx * p.imgs) {
    const int nimg = min(p.imgs, p.N - img0);
    const int npix = nimg * opix;
    __syncthreads();  // previous stage fully consumed
    lds_zero(xs, xs_elems);
    lds_zero(dys, p.cout_pad * drow);
    __syncthreads();
    stage_scatter<T, false>(p.x, plx, xs, img0, nimg, p.LH, p.LW, p.CL);
    stage_scatter<T, true>(p.dy, pldy, dys, img0, nimg, p.OH, p.OW, drow);
    for (int pix = tid; pix < p.ppad; pix += blockDim.x) {
      const int img = dopix.div(pix);
      pixbase[pix] = pix < npix ? img * img_elems + ptab[pix - img * opix] : 0;  // dY is 0 there
    }
    __syncthreads();
    const int nq = cdiv(npix, 32);
    for (int q = wave; q < nq; q += nwaves) {
      int pb[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) pb[j] = pixbase[q * 32 + 8 * g + j];
      V8 a[MTW];
#pragma unroll
      for (int m = 0; m < MTW; ++m) a[m] = load8(dys + (m * 16 + r16) * drow + q * 32 + 8 * g);
#pragma unroll
      for (int t = 0; t < NTW; ++t) {
        V8 b;
#pragma unroll
        for (int j = 0; j < 8; ++j) b[j] = is_bias[t] ? one : xs[pb[j] + koff[t]];
#pragma unroll
        for (int m = 0; m < MTW; ++m) acc[m][t] = mma(acc[m][t], a[m], b);
      }
    }
  }
  // Combine the waves' partial sums in a fixed order (deterministic), then
  // write this workgroup's slab.  red: [MTW*16 rows][NTW*16 cols] fp32.
  const int rcols = NTW * 16;
  for (int w = 0; w < nwaves; ++w) {
    __syncthreads();
    if (wave == w) {
#pragma unroll
      for (int m = 0; m < MTW; ++m)
#pragma unroll
        for (int t = 0; t < NTW; ++t)
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            float* d = red + (m * 16 + 4 * g + i) * rcols + t * 16 + r16;
            *d = (w == 0 ? 0.f : *d) + acc[m][t][i];
          }
    }
  }
  __syncthreads();
  for (int e = tid; e < p.cout_pad * rcols; e += blockDim.x) {
    const int row = e / rcols, c = e - row * rcols;
    const int col = blockIdx.y * rcols + c;
    if (col < p.ncols_pad)
      p.slab[((size_t)blockIdx.x * p.cout_pad + row) * p.ncols_pad + col] = red[row * rcols + c];
  }
}

// grid.x over 32-parameter blocks, 8 partial-sum rows of x per block.
__global__ void __launch_bounds__(256) conv_dw_reduce_kernel(ConvDwReduceParams p) {
  __shared__ float part[8][33];
  const int KK = p.KS * p.KS;
  const int nW = p.Cout * p.Cin * KK;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
  const int j = blockIdx.x * 32 + tx;
  float acc = 0.f;
  int row = 0, col = 0;
  const bool ok = j < nW + p.Cout;
  if (ok) {
    if (j < nW) {
      row = j / (p.Cin * KK);
      const int rem = j - row * p.Cin * KK;
      const int i = rem / KK, kp = rem - i * KK;
      col = kp * p.CG + i;  // CG = channel stride of the dW column layout
    } else {
      row = j - nW;
      col = p.kbias;
    }
    const float* s = p.slab + (size_t)row * p.ncols_pad + col;
    const size_t stride = (size_t)p.cout_pad * p.ncols_pad;
    float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
    int x = ty;
    for (; x + 24 < p.nx; x += 32) {
      a0 += s[(size_t)x * stride];
      a1 += s[(size_t)(x + 8) * stride];
      a2 += s[(size_t)(x + 16) * stride];
      a3 += s[(size_t)(x + 24) * stride];
    }
    for (; x < p.nx; x += 8) a0 += s[(size_t)x * stride];
    acc = (a0 + a1) + (a2 + a3);
  }
  part[ty][tx] = acc;
  __syncthreads();
  if (ty == 0 && ok) {
    float sum = 0.f;
#pragma unroll
    for (int r = 0; r < 8; ++r) sum += part[r][tx];
    float* dst = j < nW ? p.gw + j : p.gb + (j - nW);
    *dst = p.beta != 0.f ? p.beta * *dst + sum : sum;
  }
}

inline size_t a16(size_t b) { return (b + 15) & ~size_t(15); }

constexpr size_t kWeightLdsMax = 48 * 1024;

size_t conv_fwd_weight_lds(size_t es, const ConvParams& p) {
  return (size_t)cdiv(p.Cout, 16) * 16 * (p.kpad + 8) * es;
}

template <typename T, bool CVEC, int EPI, int ACT>
void launch_fwd4(const ConvParams& p, hipStream_t s, size_t lds, bool wl) {
  const dim3 grid((unsigned)cdiv(p.N, p.imgs)), block(256);
  if (wl) hipLaunchKernelGGL((conv_fwd_kernel<T, CVEC, 4, EPI, ACT, true>), grid, block, lds, s, p);
  else hipLaunchKernelGGL((conv_fwd_kernel<T, CVEC, 4, EPI, ACT, false>), grid, block, lds, s, p);
}

template <typename T, bool CVEC>
void launch_fwd_c(const ConvParams& p, hipStream_t s, size_t lds, bool wl) {
  if (!p.bias_act) launch_fwd4<T, CVEC, FE_PLAIN, ACT_NONE>(p, s, lds, wl);
  else if (p.pool == 2) launch_fwd4<T, CVEC, FE_POOL, ACT_RELU>(p, s, lds, wl);
  else if (p.act == ACT_RELU) launch_fwd4<T, CVEC, FE_ACT, ACT_RELU>(p, s, lds, wl);
  else if (p.act == ACT_TANH) launch_fwd4<T, CVEC, FE_ACT, ACT_TANH>(p, s, lds, wl);
  else launch_fwd4<T, CVEC, FE_ACT, ACT_NONE>(p, s, lds, wl);
}

template <typename T>
void launch_conv_fwd(const ConvParams& p, hipStream_t s) {
  const DType dt = sizeof(T) == 2 ? DType::BF16 : DType::F32;
  const size_t lds = conv_forward_lds_bytes(dt, p);
  const bool wl = conv_fwd_weight_lds(sizeof(T), p) <= kWeightLdsMax;
  if (p.cvec) launch_fwd_c<T, true>(p, s, lds, wl);
  else launch_fwd_c<T, false>(p, s, lds, wl);
}

int dw_ntw(int mtw) { return mtw <= 1 ? 16 : (mtw <= 2 ? 8 : (mtw <= 4 ? 4 : 2)); }

template <typename T, bool CVEC>
void launch_conv_dw_c(const ConvDwParams& p, hipStream_t s, size_t lds) {
  const int mtw = p.cout_pad / 16;
  const int ncol_tiles = p.ncols_pad / 16;
  auto go = [&](auto kern, int ntw) {
    const dim3 grid((unsigned)p.nx, (unsigned)cdiv(ncol_tiles, ntw)), block(256);
    hipLaunchKernelGGL(kern, grid, block, lds, s, p);
  };
  // Smallest NTW that covers the column tiles keeps the register footprint low.
  if (mtw <= 1) {
    if (ncol_tiles <= 2) go(conv_dw_kernel<T, CVEC, 1, 2>, 2);
    else if (ncol_tiles <= 4) go(conv_dw_kernel<T, CVEC, 1, 4>, 4);
    else if (ncol_tiles <= 8) go(conv_dw_kernel<T, CVEC, 1, 8>, 8);
    else go(conv_dw_kernel<T, CVEC, 1, 16>, 16);
  } else if (mtw <= 2) go(conv_dw_kernel<T, CVEC, 2, 8>, 8);
  else if (mtw <= 4) go(conv_dw_kernel<T, CVEC, 4, 4>, 4);
  else if (mtw <= 8) go(conv_dw_kernel<T, CVEC, 8, 2>, 2);
  else MCC_CHECK(false, "conv_dw: Cout > 128 not supported by conv_small");
}

int dw_tr_ntw(int mtw, int ncol_tiles) {
  if (mtw <= 1) return ncol_tiles <= 2 ? 2 : (ncol_tiles <= 4 ? 4 : (ncol_tiles <= 8 ? 8 : 16));
  return mtw <= 2 ? 8 : (mtw <= 4 ? 4 : 2);
}

size_t conv_dw_tr_lds(const ConvDwParams& p) {
  const size_t stage = a16((size_t)round8(p.imgs * p.LH * p.LW * p.CL + 16) * 2) +
                       a16((size_t)p.ppad * conv_dw_tr_drow(p.cout_pad) * 2) + (size_t)p.ppad * 4 +
                       (size_t)p.OH * p.OW * 4;
  const size_t red = (size_t)p.cout_pad * (dw_tr_ntw(p.cout_pad / 16, p.kbias / 16) * 16 + 1) * 4;
  return stage > red ? stage : red;
}

void launch_conv_dw_tr(const ConvDwParams& p, hipStream_t s, size_t lds) {
  const int mtw = p.cout_pad / 16;
  const int ncol_tiles = p.kbias / 16;
  const int ntw = dw_tr_ntw(mtw, ncol_tiles);
  const dim3 grid((unsigned)p.nx, (unsigned)cdiv(ncol_tiles, ntw)), block(256);
  auto go = [&](auto kern) { hipLaunchKernelGGL(kern, grid, block, lds, s, p); };
  if (mtw <= 1) {
    if (ntw == 2) go(conv_dw_tr_kernel<1, 2>);
    else if (ntw == 4) go(conv_dw_tr_kernel<1, 4>);
    else if (ntw == 8) go(conv_dw_tr_kernel<1, 8>);
    else go(conv_dw_tr_kernel<1, 16>);
  } else if (mtw <= 2) go(conv_dw_tr_kernel<2, 8>);
  else if (mtw <= 4) go(conv_dw_tr_kernel<4, 4>);
  else if (mtw <= 8) go(conv_dw_tr_kernel<8, 2>);
  else MCC_CHECK(false, "conv_dw: Cout > 128 not supported by conv_small");
}

}  // namespace

size_t conv_forward_lds_bytes(DType t, const ConvParams& p) {
  const size_t es = t == DType::BF16 ? 2 : 4;
  const size_t nk = p.cvec ? (size_t)p.nchunks * 4 : (size_t)p.nchunks * 32;
  const size_t rows = p.pool == 2 ? (size_t)(p.OH / 2) * (p.OW / 2) * 4 : (size_t)p.OH * p.OW;
  const size_t wl = conv_fwd_weight_lds(es, p);
  return a16((size_t)round8(p.imgs * p.LH * p.LW * p.CL + 16) * es) + (wl <= kWeightLdsMax ? a16(wl) : 0) +
         (size_t)cdiv(p.Cout, 16) * 16 * 4 + ((nk + 3) & ~size_t(3)) * 4 + rows * 4;
}

size_t conv_dw_lds_bytes(DType t, const ConvDwParams& p) {
  if (t == DType::BF16) return conv_dw_tr_lds(p);
  const size_t es = 4;
  const size_t stage = a16((size_t)round8(p.imgs * p.LH * p.LW * p.CL + 16) * es) +
                       a16((size_t)p.cout_pad * (p.ppad + 8) * es) + (size_t)p.ppad * 4 + (size_t)p.OH * p.OW * 4;
  const int mtw = p.cout_pad / 16;
  const size_t red = (size_t)p.cout_pad * dw_ntw(mtw) * 16 * 4;
  return stage > red ? stage : red;
}

void conv_forward(DType t, const ConvParams& p, hipStream_t s) {
  MCC_CHECK(p.N > 0 && p.imgs > 0 && p.nchunks > 0, "conv_forward: empty problem");
  MCC_CHECK(!p.cvec || (p.CL % 8) == 0, "conv_forward: cvec needs CL % 8 == 0");
  MCC_CHECK(p.kpad == p.nchunks * 32, "conv_forward: kpad mismatch");
  MCC_CHECK(p.pool == 1 || (p.pool == 2 && p.bias_act && p.out_arg), "conv_forward: bad pool config");
  MCC_CHECK((int64_t)p.imgs * p.LH * p.LW * p.CL < (1 << 24), "conv_forward: tile too large for index math");
  MCC_CHECK(conv_forward_lds_bytes(t, p) <= 160 * 1024, "conv_forward: LDS tile exceeds 160 KiB");
  if (t == DType::BF16) launch_conv_fwd<bf16>(p, s);
  else launch_conv_fwd<float>(p, s);
}

void conv_dw(DType t, const ConvDwParams& p, hipStream_t s) {
  MCC_CHECK(p.N > 0 && p.imgs > 0 && p.nx > 0, "conv_dw: empty problem");
  MCC_CHECK(p.ppad % 32 == 0 && p.ppad >= p.imgs * p.OH * p.OW, "conv_dw: bad ppad");
  MCC_CHECK(p.cout_pad % 16 == 0 && p.ncols_pad % 16 == 0 && p.ncols_pad > p.kbias, "conv_dw: bad padding");
  MCC_CHECK((int64_t)p.imgs * p.LH * p.LW * p.CL < (1 << 24) && (int64_t)p.cout_pad * p.ppad < (1 << 24),
            "conv_dw: tile too large for index math");
  const size_t lds = conv_dw_lds_bytes(t, p);
  MCC_CHECK(lds <= 160 * 1024, "conv_dw: LDS tile exceeds 160 KiB");
  if (t == DType::BF16) {
    MCC_CHECK(p.CL % 4 == 0 && p.kbias % 16 == 0, "conv_dw(bf16): needs the c4 column layout");
    launch_conv_dw_tr(p, s, lds);
  } else {
    if (p.cvec) launch_conv_dw_c<float, true>(p, s, lds);
    else launch_conv_dw_c<float, false>(p, s, lds);
  }
}

void conv_dw_reduce(const ConvDwReduceParams& p, hipStream_t s) {
  const int n = p.Cout * p.Cin * p.KS * p.KS + p.Cout;
  hipLaunchKernelGGL(conv_dw_reduce_kernel, dim3((unsigned)cdiv(n, 32)), dim3(256), 0, s, p);
}

}  // namespace gpu
}  // namespace mcc
