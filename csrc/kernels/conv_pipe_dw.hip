// Weight gradient of the pipelined small-image conv (bf16): dY^T x im2col(X)
// with the pixel axis as the MFMA K dimension, both operands read with
// ds_read_b64_tr_b16; per-workgroup slabs reduced by a two-level
// deterministic sum.  Reference: the dW part of Layer_feedBack_conv
// (cnn.c:212-247).  Design notes: conv_pipe_fwd.hip.
#include "conv_pipe.h"

namespace mcc {
namespace gpu {

namespace {

template <int XM, int DM, int MTW, int NTW, bool WS = false>
__global__ void __launch_bounds__(kT) conv_dw_pipe_kernel(ConvDwPipeParams p) {
  constexpr bool S1 = XM == PM_U8S1;
  constexpr bool PIPE_B = NTW <= 4;  // few column tiles: prefetch B too (else the tiles give the ILP)
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const DwLayout L = dw_layout(p);
  bf16* xs = reinterpret_cast<bf16*>(smem);
  bf16* dys = reinterpret_cast<bf16*>(smem + L.dys_off);
  int* pixbase = reinterpret_cast<int*>(smem + L.pixbase_off);
  int* ptab = reinterpret_cast<int*>(smem + L.ptab_off);
  bf16* ones = reinterpret_cast<bf16*>(smem + L.ones_off);
  float* red = reinterpret_cast<float*>(smem);  // reused after the main loop

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int r16 = lane & 15, g = lane >> 4;
  const int q = r16 >> 2, pp = r16 & 3;  // transpose-read address role
  const int KK = p.KS * p.KS;
  const int opix = p.OH * p.OW;
  const int drow = p.drow;
  const PipeSrc& sx = p.x;
  const PipeSrc& sd = p.dy;

  // Column group (4 columns) of this lane per tile: tile offset relative to
  // a pixel's first tap, or the ones vector for the bias column group.
  int koff[NTW];
  bool kone[NTW];
#pragma unroll
  for (int t = 0; t < NTW; ++t) {
    // first of this lane's 4 columns (WS: this wave's own tiles)
    const int c4 = ((WS ? blockIdx.y * 4 + wave : blockIdx.y) * NTW + t) * 16 + 4 * pp;
    koff[t] = 0;
    kone[t] = c4 == p.kbias;
    if (S1) {
      const int kh = c4 >> 3;
      if (kh < p.KS) koff[t] = kh * sx.LWp + (c4 & 7);
    } else {
      const int kp = c4 / sx.CL, c0 = c4 - kp * sx.CL;
      if (kp < KK) {
        const int kh = kp / p.KS, kw = kp - kh * p.KS;
        koff[t] = (kh * sx.LWp + kw) * sx.CL + c0;
      }
    }
  }

  zero_lds(xs, L.xs_elems);
  zero_lds(dys, p.ppad * drow + 8);
  if (tid < 8) ones[tid] = (bf16)1.0f;
  row_table(ptab, opix, false, p.OW, p.cs, p.ty0, p.tx0, sx.LWp, S1 ? 1 : sx.CL);
  Loader<XM, kT> lx;
  Loader<DM, kT> ld;
  lx.init(sx, p.imgs);
  ld.init(sd, p.imgs);
  int grp = blockIdx.x;
  if (grp < p.ngroups) {
    lx.load(sx, grp * p.imgs, p.N);
    ld.load(sd, grp * p.imgs, p.N);
  }
  __syncthreads();  // ptab
  {
    // stage-invariant pixel -> tile base (S1: already in its shifted copy);
    // rows past the last image of a tail group read stale (finite) pixels
    // against zeroed dY rows
    const int full = p.imgs * opix;
    for (int pix = tid; pix < p.ppad + 32; pix += kT) {
      const int img = pix / opix;
      int b = pix < full ? img * sx.IMG + ptab[pix - img * opix] : 0;
      if (S1) {  // column offsets are multiples of 4: the copy depends on the pixel only
        const int c = b & 3;
        b = c * sx.CS + b - c;
      }
      pixbase[pix] = b;
    }
  }

  f32x4 acc[MTW][NTW];
#pragma unroll
  for (int m = 0; m < MTW; ++m)
#pragma unroll
    for (int t = 0; t < NTW; ++t) acc[m][t] = f32x4{0.f, 0.f, 0.f, 0.f};

  const bf16* onesp = ones;
  auto read_a = [&](int pix1, int pix2, bf16x8 (&a)[MTW]) {
#pragma unroll
    for (int m = 0; m < MTW; ++m) {
      const bf16x4 lo = tr4(dys + pix1 * drow + m * 16 + 4 * pp);
      const bf16x4 hi = tr4(dys + pix2 * drow + m * 16 + 4 * pp);
      a[m] = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
    }
  };
  auto read_b = [&](int pb1, int pb2, int t) {
    const bf16* p1 = kone[t] ? onesp : xs + pb1 + koff[t];
    const bf16* p2 = kone[t] ? onesp : xs + pb2 + koff[t];
    const bf16x4 lo = tr4(p1), hi = tr4(p2);
    return __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
  };

  for (; grp < p.ngroups; grp += gridDim.x) {
    const int img0 = grp * p.imgs;
    const int nimg = min(p.imgs, p.N - img0);
    const int npix = nimg * opix;
    __syncthreads();  // previous group consumed
    lx.store(sx, xs, nimg);
    ld.store(sd, dys, nimg);
    if (nimg < p.imgs) zero_lds(dys + npix * drow, (p.ppad - npix) * drow);  // stale rows of a tail group
    __syncthreads();
    if (grp + (int)gridDim.x < p.ngroups) {
      lx.load(sx, (grp + gridDim.x) * p.imgs, p.N);
      ld.load(sd, (grp + gridDim.x) * p.imgs, p.N);
    }
    const int nq = cdiv(npix, 32);
    // fragment k -> pixel: lane group g reads rows 4g..4g+3 (and +16).
    // Pipelined one pixel chunk deep (pixbase is padded by one chunk).
    constexpr int QS = WS ? 1 : kT / 64;  // chunk step: WS waves walk every chunk
    int qc = WS ? 0 : wave;
    int pix1 = qc * 32 + 4 * g + q;
    int pb1 = 0, pb2 = 0;
    bf16x8 a[MTW], b[NTW];
    if (qc < nq) {
      pb1 = pixbase[pix1];
      pb2 = pixbase[pix1 + 16];
      read_a(pix1, pix1 + 16, a);
      if (PIPE_B) {
#pragma unroll
        for (int t = 0; t < NTW; ++t) b[t] = read_b(pb1, pb2, t);
      }
    }
    for (; qc < nq; qc += QS) {
      const int qn = qc + QS;
      const int pixn = qn * 32 + 4 * g + q;
      const bool more = qn < nq;
      const int pbn1 = more ? pixbase[pixn] : 0, pbn2 = more ? pixbase[pixn + 16] : 0;
      bf16x8 an[MTW], bn[NTW];
      if (more) read_a(pixn, pixn + 16, an);
      if (PIPE_B) {
        if (more) {
#pragma unroll
          for (int t = 0; t < NTW; ++t) bn[t] = read_b(pbn1, pbn2, t);
        }
#pragma unroll
        for (int t = 0; t < NTW; ++t)
#pragma unroll
          for (int m = 0; m < MTW; ++m) acc[m][t] = mma(acc[m][t], a[m], b[t]);
#pragma unroll
        for (int t = 0; t < NTW; ++t) b[t] = bn[t];
      } else {
#pragma unroll
        for (int t = 0; t < NTW; ++t) {
          const bf16x8 bt = read_b(pb1, pb2, t);
#pragma unroll
          for (int m = 0; m < MTW; ++m) acc[m][t] = mma(acc[m][t], a[m], bt);
        }
      }
#pragma unroll
      for (int m = 0; m < MTW; ++m) a[m] = an[m];
      pb1 = pbn1;
      pb2 = pbn2;
    }
  }
  // combine the waves in a fixed order: red[MTW*16 rows][NTW*16 cols]
  // (WS: each wave owns its NTW*16 columns of red[MTW*16][4*NTW*16])
  const int rcols = (WS ? 4 : 1) * NTW * 16;
  if constexpr (WS) {
    __syncthreads();  // red aliases the staged tiles
#pragma unroll
    for (int m = 0; m < MTW; ++m)
#pragma unroll
      for (int t = 0; t < NTW; ++t)
#pragma unroll
        for (int i = 0; i < 4; ++i) red[(m * 16 + 4 * g + i) * rcols + (wave * NTW + t) * 16 + r16] = acc[m][t][i];
  }
  for (int w = 0; w < (WS ? 0 : kT / 64); ++w) {
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
  for (int e = tid; e < p.cout_pad * rcols; e += kT) {
    const int row = e / rcols, c = e - row * rcols;
    const int col = blockIdx.y * rcols + c;
    MCC_DCHECK(row < p.cout_pad && (int)blockIdx.x < p.grid);
    if (col < p.ncols_pad) p.slab[((size_t)blockIdx.x * p.cout_pad + row) * p.ncols_pad + col] = red[e];
  }
}

// Level 1: part[xc][v] = sum of slabs x in chunk xc (v over the whole slab).
__global__ void __launch_bounds__(256) dw_slab_sum_kernel(const float* slab, int nx, int nv, int xs_per,
                                                          float* part) {
  __shared__ float red[4][65];
  const int tv = threadIdx.x & 63, tx = threadIdx.x >> 6;
  const int v = blockIdx.x * 64 + tv;
  const int x0 = blockIdx.y * xs_per, x1 = min(nx, x0 + xs_per);
  float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;  // four loads in flight per thread
  if (v < nv) {
    int x = x0 + tx;
    for (; x + 12 < x1; x += 16) {
      a0 += slab[(size_t)x * nv + v];
      a1 += slab[(size_t)(x + 4) * nv + v];
      a2 += slab[(size_t)(x + 8) * nv + v];
      a3 += slab[(size_t)(x + 12) * nv + v];
    }
    for (; x < x1; x += 4) a0 += slab[(size_t)x * nv + v];
  }
  red[tx][tv] = (a0 + a1) + (a2 + a3);
  __syncthreads();
  if (tx == 0 && v < nv) part[(size_t)blockIdx.y * nv + v] = (red[0][tv] + red[1][tv]) + (red[2][tv] + red[3][tv]);
}

// Level 2: canonical gradient from the chunk partials.
__global__ void __launch_bounds__(256) dw_slab_final_kernel(const float* part, int nxc, int nv, int ncols_pad,
                                                            int kbias, int Cout, int Cin, int KS, int layout,
                                                            int CL, float wscale, float* gw, float* gb) {
  const int KK = KS * KS;
  const int nW = Cout * Cin * KK;
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= nW + Cout) return;
  int row, col;
  if (j < nW) {
    row = j / (Cin * KK);
    const int rem = j - row * Cin * KK;
    const int ci = rem / KK, kp = rem - ci * KK;
    const int kh = kp / KS, kw = kp - kh * KS;
    col = layout == XL_S1 ? kh * 8 + kw : (layout == XL_ROWS ? kp : kp * CL + ci);
  } else {
    row = j - nW;
    col = kbias;
  }
  const int v = row * ncols_pad + col;
  float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;  // fixed order, loads in flight
  int xc = 0;
  for (; xc + 3 < nxc; xc += 4) {
    s0 += part[(size_t)xc * nv + v];
    s1 += part[(size_t)(xc + 1) * nv + v];
    s2 += part[(size_t)(xc + 2) * nv + v];
    s3 += part[(size_t)(xc + 3) * nv + v];
  }
  for (; xc < nxc; ++xc) s0 += part[(size_t)xc * nv + v];
  const float s = (s0 + s1) + (s2 + s3);
  if (j < nW) gw[j] = s * wscale;
  else gb[row] = s;
}

}  // namespace

bool conv_dw_pipe_plan(ConvDwPipeParams& p) {
  PipeSrc& x = p.x;
  PipeSrc& d = p.dy;
  const bool s1 = x.mode == PM_U8S1;
  if (s1 && (p.KS > 8 || p.Cin != 1)) return false;
  if (!s1 && (x.mode != PM_PLAIN || x.SC != p.Cin)) return false;
  if (d.mode == PM_U8S1 || d.SC != p.Cout || p.Cout > 128) return false;
  p.layout = s1 ? XL_S1 : XL_C8;
  if (s1) {
    const int ox = x.offx < 4 ? 4 : (x.offx + 3) & ~3;
    p.tx0 += ox - x.offx;
    x.offx = ox;
  }
  const int LH = std::max(p.ty0 + (p.OH - 1) * p.cs + p.KS, x.offy + (x.SH - 1) * x.up + 1);
  int LWp;
  if (s1) LWp = (std::max(p.tx0 + (p.OW - 1) * p.cs + 8, x.offx + x.SW + 4) + 3) & ~3;
  else LWp = std::max(p.tx0 + (p.OW - 1) * p.cs + p.KS, x.offx + (x.SW - 1) * x.up + 1);
  const int CL = s1 ? 1 : r8h(p.Cin);  // C8 staging writes whole 16-byte pixels
  if (!plan_src(x, p.layout, CL, LH, LWp, 0)) return false;
  x.LWp = LWp;
  x.IMG = LH * LWp * CL;
  p.LH = LH;
  p.cout_pad = r16h(p.Cout);
  // Cout <= 8: 16-byte dY rows; the A fragment's channels 8..15 then read the
  // next row (rows 8..15 of the product are garbage and never reduced)
  p.drow = p.Cout <= 8 ? 8 : conv_dw_tr_drow(p.cout_pad);
  d.up = 1; d.offy = 0; d.offx = 0;
  if (!plan_src(d, XL_C8, p.drow, p.OH, p.OW, 0)) return false;
  d.LWp = p.OW;
  d.IMG = p.OH * p.OW * p.drow;
  const int KK = p.KS * p.KS;
  // bias gradient = the column right after the packed ones (a ones vector in
  // the im2col operand), computed by the same MFMAs
  p.kbias = s1 ? p.KS * 8 : KK * CL;
  p.ncols_pad = r16h(p.kbias + 1);
  // wide outputs (>= 4 row tiles) split the column tiles over the waves when
  // there are enough of them (4 waves x NTW)
  {
    const int mtw = p.cout_pad / 16, nct = p.ncols_pad / 16;
    p.wsplit = mtw >= 4 && nct >= 2 * dw_ntw(mtw, nct) ? 1 : 0;
  }
  const int nix = mode_ni(x.mode) * kT / std::max(1, x.per_img);
  const int nid = mode_ni(d.mode) * kT / std::max(1, d.per_img);
  int imgs = std::max(1, std::min(16, std::min(nix, nid)));
  for (; imgs >= 1; --imgs) {
    p.imgs = imgs;
    p.ppad = r32h(imgs * p.OH * p.OW);
    if (s1) x.CS = r8h(imgs * x.IMG + 8);
    if ((size_t)dw_layout(p).total <= dw_lds_target() || imgs == 1) break;
  }
  if (nix < 1 || nid < 1) return false;
  const DwLayout L = dw_layout(p);
  if ((size_t)L.total > kLdsPerCU) return false;
  p.lds = (size_t)L.total;
  p.ngroups = cdiv(p.N, p.imgs);
  p.grid = std::min(p.ngroups, kCUs * wgs_per_cu(p.lds, dw_wgs_cap()));
  return true;
}

void conv_dw_pipe(const ConvDwPipeParams& pin, hipStream_t st) {
  ConvDwPipeParams p = pin;
  p.ngroups = cdiv(p.N, p.imgs);
  p.grid = std::min(p.ngroups, std::min(pin.grid, kCUs * wgs_per_cu(p.lds, dw_wgs_cap())));
  if (p.grid <= 0) return;
  const int mtw = p.cout_pad / 16;
  const int ncol_tiles = p.ncols_pad / 16;
  const int ntw = dw_ntw(mtw, ncol_tiles);
  const dim3 grid((unsigned)p.grid, (unsigned)cdiv(ncol_tiles, ntw * (p.wsplit ? 4 : 1))), block(kT);
  auto go = [&](auto kern) { hipLaunchKernelGGL(kern, grid, block, p.lds, st, p); };
#define MCC_DW_TILES(XM, DM)                                     \
  if (mtw <= 1) {                                                \
    if (ntw == 2) go(conv_dw_pipe_kernel<XM, DM, 1, 2>);         \
    else if (ntw == 3) go(conv_dw_pipe_kernel<XM, DM, 1, 3>);    \
    else if (ntw == 4) go(conv_dw_pipe_kernel<XM, DM, 1, 4>);    \
    else if (ntw == 8) go(conv_dw_pipe_kernel<XM, DM, 1, 8>);    \
    else if (ntw == 13) go(conv_dw_pipe_kernel<XM, DM, 1, 13>);  \
    else go(conv_dw_pipe_kernel<XM, DM, 1, 16>);                 \
  } else if (mtw <= 2) go(conv_dw_pipe_kernel<XM, DM, 2, 8>);   \
  else if (mtw <= 4) {                                           \
    if (p.wsplit) go(conv_dw_pipe_kernel<XM, DM, 4, 4, true>);   \
    else go(conv_dw_pipe_kernel<XM, DM, 4, 4>);                  \
  } else if (p.wsplit) go(conv_dw_pipe_kernel<XM, DM, 8, 2, true>); \
  else go(conv_dw_pipe_kernel<XM, DM, 8, 2>);
#define MCC_DW_DM(XM)                                            \
  if (p.dy.mode == PM_UNPOOL) { MCC_DW_TILES(XM, PM_UNPOOL) }    \
  else if (p.dy.mode == PM_RELU) { MCC_DW_TILES(XM, PM_RELU) }   \
  else { MCC_DW_TILES(XM, PM_PLAIN) }
  if (p.x.mode == PM_U8S1) { MCC_DW_DM(PM_U8S1) }
  else { MCC_DW_DM(PM_PLAIN) }
#undef MCC_DW_DM
#undef MCC_DW_TILES
}

void dw_slab_reduce(const float* slab, int nx, int cout_pad, int ncols_pad, float* part, int Cout, int Cin, int KS,
                    int layout, int CL, int kbias, float* gw, float* gb, hipStream_t st, float wscale) {
  if (nx <= 0) return;
  const int nv = cout_pad * ncols_pad;
  const int xs_per = 64;
  const int nxc = cdiv(nx, xs_per);
  hipLaunchKernelGGL(dw_slab_sum_kernel, dim3((unsigned)cdiv(nv, 64), (unsigned)nxc), dim3(256), 0, st, slab, nx, nv,
                     xs_per, part);
  const int nout = Cout * Cin * KS * KS + Cout;
  hipLaunchKernelGGL(dw_slab_final_kernel, dim3((unsigned)cdiv(nout, 256)), dim3(256), 0, st, part, nxc, nv, ncols_pad,
                     kbias, Cout, Cin, KS, layout, CL, wscale, gw, gb);
}

void conv_dw_pipe_reduce(const ConvDwPipeParams& pin, float* gw, float* gb, hipStream_t st) {
  ConvDwPipeParams p = pin;
  const int ngroups = cdiv(p.N, p.imgs);
  const int nx = std::min(ngroups, std::min(pin.grid, kCUs * wgs_per_cu(p.lds, dw_wgs_cap())));
  if (nx <= 0) return;
  const int nv = p.cout_pad * p.ncols_pad;
  float* part = p.slab + (size_t)pin.grid * nv;  // after the slabs (scratch sized by the planner's grid)
  dw_slab_reduce(p.slab, nx, p.cout_pad, p.ncols_pad, part, p.Cout, p.Cin, p.KS, p.layout, p.x.CL, p.kbias, gw, gb,
                 st);
}

}  // namespace gpu
}  // namespace mcc
