// Implicit-GEMM convolution on MFMA for small images (whole image tile in LDS).
//
// Replaces the reference's scalar 6-deep loops (Layer_feedForw_conv,
// cnn.c:175-210; Layer_feedBack_conv, cnn.c:212-247) and its one-thread-per-
// output fp64 CUDA kernel (conv_forward_kernel, CUDAcnn.cu:167-195).
//
// Design (gfx950):
//  * A workgroup stages `imgs` whole input images (with the zero halo) into
//    LDS once, channels padded to 8 ("cvec") so one (kernel-position,
//    8-channel group) im2col fragment is a single 16-byte ds_read.
//  * GEMM rows are output pixels, ordered by 2x2 pooling window when a max-
//    pool is fused: the 16x16 MFMA C-fragment then gives each lane exactly one
//    window (4 consecutive rows) of one channel, so bias + ReLU + maxpool +
//    argmax is an in-register epilogue (no pre-pool tensor ever hits HBM).
//  * Backward-data is the same kernel run as a stride-1 conv over the
//    zero-inserted output gradient with flipped/transposed packed weights; the
//    ReLU mask and the max-pool routing are applied while staging (IN_RELU /
//    IN_UNPOOL), so no separate unpool/activation-grad pass exists.
//  * Weight gradient: MFMA with the pixel dimension as the reduction axis,
//    the output-gradient tile staged transposed ([co][pixel]), a ones-column
//    appended to im2col so the bias gradient falls out of the same MFMAs,
//    per-workgroup fp32 slabs reduced deterministically afterwards.
#include "kernels.h"
#include "mfma.h"

namespace mcc {
namespace gpu {

namespace {

__device__ __forceinline__ int align16(int bytes) { return (bytes + 15) & ~15; }

template <typename T>
__device__ __forceinline__ float stage_value(const StageSrc& s, int n, int sy, int sx, int c) {
  switch (s.mode) {
    case IN_U8: {
      const int img = s.idx ? s.idx[n] : n;
      const uint8_t* u = static_cast<const uint8_t*>(s.src);
      return (float)u[(((size_t)img * s.SH + sy) * s.SW + sx) * s.SC + c] * (1.0f / 255.0f);
    }
    case IN_RELU: {
      const size_t i = (((size_t)n * s.SH + sy) * s.SW + sx) * s.SC + c;
      const float y = to_f(static_cast<const T*>(s.aux_y)[i]);
      return y > 0.f ? to_f(static_cast<const T*>(s.src)[i]) : 0.f;
    }
    case IN_UNPOOL: {
      const int py = sy >> 1, px = sx >> 1;
      if (py >= s.PH || px >= s.PW) return 0.f;
      const size_t i = (((size_t)n * s.PH + py) * s.PW + px) * s.SC + c;
      const int pos = ((sy & 1) << 1) | (sx & 1);
      if (s.aux_arg[i] != pos) return 0.f;
      const float y = to_f(static_cast<const T*>(s.aux_y)[i]);
      return y > 0.f ? to_f(static_cast<const T*>(s.src)[i]) : 0.f;
    }
    default:
      return to_f(static_cast<const T*>(s.src)[(((size_t)n * s.SH + sy) * s.SW + sx) * s.SC + c]);
  }
}

// Stage `imgs` images starting at img0 into lds[img][LH][LW][CL] (zero halo,
// zero channel padding, zero rows past N).
template <typename T>
__device__ void stage_tile(const StageSrc& s, T* lds, int img0, int N, int imgs, int LH, int LW, int CL,
                           bool cvec) {
  const int per_img = LH * LW;
  const int total = imgs * per_img;
  const bool vec_plain = cvec && s.mode == IN_PLAIN && (s.SC & 7) == 0;
  for (int e = threadIdx.x; e < total; e += blockDim.x) {
    const int img = e / per_img;
    const int rem = e - img * per_img;
    const int ly = rem / LW;
    const int lx = rem - ly * LW;
    const int n = img0 + img;
    const int ty = ly - s.off, tx = lx - s.off;
    bool valid = n < N && ty >= 0 && tx >= 0;
    int sy = ty, sx = tx;
    if (s.up != 1) {
      valid = valid && (ty % s.up) == 0 && (tx % s.up) == 0;
      sy = ty / s.up;
      sx = tx / s.up;
    }
    valid = valid && sy < s.SH && sx < s.SW;
    T* dst = lds + (size_t)e * CL;
    if (cvec) {
      for (int cg = 0; cg < (CL >> 3); ++cg) {
        typename Vec8<T>::type v;
        if (vec_plain && valid) {
          v = load8(static_cast<const T*>(s.src) + (((size_t)n * s.SH + sy) * s.SW + sx) * s.SC + cg * 8);
        } else {
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const int c = cg * 8 + j;
            v[j] = (valid && c < s.SC) ? from_f<T>(stage_value<T>(s, n, sy, sx, c)) : T(0);
          }
        }
        store8(dst + cg * 8, v);
      }
    } else {
      for (int c = 0; c < CL; ++c) dst[c] = valid ? from_f<T>(stage_value<T>(s, n, sy, sx, c)) : T(0);
    }
  }
}

template <typename T, bool CVEC, int MT>
__global__ void __launch_bounds__(256) conv_fwd_kernel(ConvParams p) {
  typedef typename Vec8<T>::type V8;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  T* xs = reinterpret_cast<T*>(smem);
  const int img_elems = p.LH * p.LW * p.CL;
  const int zoff = p.imgs * img_elems;
  int* ktab = reinterpret_cast<int*>(smem + align16((zoff + 16) * (int)sizeof(T)));
  const int img0 = blockIdx.x * p.imgs;
  const int tid = threadIdx.x;

  // k -> LDS offset table (relative to a pixel's top-left tap); -1 = padding.
  const int nk = CVEC ? p.nchunks * 4 : p.nchunks * 32;
  const int KK = p.KS * p.KS;
  for (int e = tid; e < nk; e += blockDim.x) {
    int off = -1;
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
  stage_tile<T>(p.in, xs, img0, p.N, p.imgs, p.LH, p.LW, p.CL, CVEC);
  if (tid < 16) xs[zoff + tid] = T(0);
  __syncthreads();

  const int lane = tid & 63, wave = tid >> 6, nwaves = blockDim.x >> 6;
  const int r16 = lane & 15, g = lane >> 4;
  const int nimg = min(p.imgs, p.N - img0);
  const bool pool = p.pool == 2;
  const int PH = p.OH >> 1, PW = p.OW >> 1;
  const int rows_per_img = pool ? PH * PW * 4 : p.OH * p.OW;
  const int M = nimg * rows_per_img;
  const int mtiles = cdiv(M, 16), ntiles = cdiv(p.Cout, 16), mgroups = cdiv(mtiles, MT);
  const T* wpk = static_cast<const T*>(p.wpk);
  T* out = static_cast<T*>(p.out);

  for (int item = wave; item < ntiles * mgroups; item += nwaves) {
    const int nt = item / mgroups, mg = item - nt * mgroups;
    int base[MT];
#pragma unroll
    for (int t = 0; t < MT; ++t) {
      const int r = (mg * MT + t) * 16 + r16;
      base[t] = -1;
      if (r < M) {
        const int img = r / rows_per_img;
        const int rem = r - img * rows_per_img;
        int oy, ox;
        if (pool) {
          const int win = rem >> 2, pos = rem & 3;
          const int ph = win / PW, pw = win - ph * PW;
          oy = 2 * ph + (pos >> 1);
          ox = 2 * pw + (pos & 1);
        } else {
          oy = rem / p.OW;
          ox = rem - oy * p.OW;
        }
        base[t] = img * img_elems + (oy * p.cs * p.LW + ox * p.cs) * p.CL;
      }
    }
    f32x4 acc[MT];
#pragma unroll
    for (int t = 0; t < MT; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
    const T* wrow = wpk + (size_t)(nt * 16 + r16) * p.kpad + 8 * g;
    for (int q = 0; q < p.nchunks; ++q) {
      const V8 b = load8(wrow + q * 32);
      if (CVEC) {
        const int ko = ktab[q * 4 + g];
#pragma unroll
        for (int t = 0; t < MT; ++t) {
          const int a_off = (base[t] >= 0 && ko >= 0) ? base[t] + ko : zoff;
          acc[t] = mma(acc[t], load8(xs + a_off), b);
        }
      } else {
        int ko[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) ko[j] = ktab[q * 32 + 8 * g + j];
#pragma unroll
        for (int t = 0; t < MT; ++t) {
          V8 a;
#pragma unroll
          for (int j = 0; j < 8; ++j) a[j] = xs[(base[t] >= 0 && ko[j] >= 0) ? base[t] + ko[j] : zoff];
          acc[t] = mma(acc[t], a, b);
        }
      }
    }
    // Epilogue: rows 4g..4g+3 of each tile belong to this lane, column n.
    const int n = nt * 16 + r16;
    if (n >= p.Cout) continue;
    const float bv = p.bias_act ? p.bias[n] : 0.f;
#pragma unroll
    for (int t = 0; t < MT; ++t) {
      const int rb = (mg * MT + t) * 16 + 4 * g;
      if (rb >= M) continue;
      float v[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) v[i] = p.bias_act ? act_apply(p.act, acc[t][i] + bv) : acc[t][i];
      if (pool) {
        float best = v[0];
        int arg = 0;
#pragma unroll
        for (int i = 1; i < 4; ++i)
          if (v[i] > best) { best = v[i]; arg = i; }
        const size_t o = ((size_t)img0 * PH * PW + (rb >> 2)) * p.Cout + n;
        out[o] = from_f<T>(best);
        p.out_arg[o] = (uint8_t)arg;
      } else {
        const size_t obase = (size_t)img0 * p.OH * p.OW;
#pragma unroll
        for (int i = 0; i < 4; ++i)
          if (rb + i < M) out[(obase + rb + i) * p.Cout + n] = from_f<T>(v[i]);
      }
    }
  }
}

template <typename T, bool CVEC, int MTW, int NTW>
__global__ void __launch_bounds__(256) conv_dw_kernel(ConvDwParams p) {
  typedef typename Vec8<T>::type V8;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int img_elems = p.LH * p.LW * p.CL;
  const int zoff = p.imgs * img_elems;
  T* xs = reinterpret_cast<T*>(smem);
  const int drow = p.ppad + 8;
  T* dys = reinterpret_cast<T*>(smem + align16((zoff + 16) * (int)sizeof(T)));
  int* pixbase = reinterpret_cast<int*>(reinterpret_cast<char*>(dys) + align16(p.cout_pad * drow * (int)sizeof(T)));

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6, nwaves = blockDim.x >> 6;
  const int r16 = lane & 15, g = lane >> 4;
  const int ncol_tiles = p.ncols_pad >> 4;
  const int KK = p.KS * p.KS;
  const int CG = p.CL >> 3;

  int koff[NTW];
  bool is_bias[NTW];
  int ntile_of[NTW];
#pragma unroll
  for (int t = 0; t < NTW; ++t) {
    const int nti = (blockIdx.y * nwaves + wave) * NTW + t;
    ntile_of[t] = nti;
    const int col = nti * 16 + r16;
    koff[t] = -1;
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

  f32x4 acc[MTW][NTW];
#pragma unroll
  for (int m = 0; m < MTW; ++m)
#pragma unroll
    for (int t = 0; t < NTW; ++t) acc[m][t] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int opix = p.OH * p.OW;
  for (int img0 = blockIdx.x * p.imgs; img0 < p.N; img0 += p.nx * p.imgs) {
    __syncthreads();
    stage_tile<T>(p.x, xs, img0, p.N, p.imgs, p.LH, p.LW, p.CL, CVEC);
    if (tid < 16) xs[zoff + tid] = T(0);
    const int nimg = min(p.imgs, p.N - img0);
    const int npix = nimg * opix;
    // dY tile, transposed to [co][pixel] (pixel-contiguous A fragments).
    for (int e = tid; e < p.ppad * p.cout_pad; e += blockDim.x) {
      const int pix = e / p.cout_pad, co = e - pix * p.cout_pad;
      float v = 0.f;
      if (pix < npix && co < p.Cout) {
        const int img = pix / opix, rem = pix - img * opix;
        const int oy = rem / p.OW, ox = rem - oy * p.OW;
        v = stage_value<T>(p.dy, img0 + img, oy, ox, co);
      }
      dys[co * drow + pix] = from_f<T>(v);
    }
    for (int pix = tid; pix < p.ppad; pix += blockDim.x) {
      int b = -1;
      if (pix < npix) {
        const int img = pix / opix, rem = pix - img * opix;
        const int oy = rem / p.OW, ox = rem - oy * p.OW;
        b = img * img_elems + (oy * p.cs * p.LW + ox * p.cs) * p.CL;
      }
      pixbase[pix] = b;
    }
    __syncthreads();
    const int nq = cdiv(npix, 32);
    for (int q = 0; q < nq; ++q) {
      int pb[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) pb[j] = pixbase[q * 32 + 8 * g + j];
      V8 b[NTW];
#pragma unroll
      for (int t = 0; t < NTW; ++t) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float one = is_bias[t] ? 1.f : 0.f;
          b[t][j] = (koff[t] >= 0 && pb[j] >= 0) ? xs[pb[j] + koff[t]] : from_f<T>(one);
        }
      }
#pragma unroll
      for (int m = 0; m < MTW; ++m) {
        const V8 a = load8(dys + (m * 16 + r16) * drow + q * 32 + 8 * g);
#pragma unroll
        for (int t = 0; t < NTW; ++t) acc[m][t] = mma(acc[m][t], a, b[t]);
      }
    }
  }
  // Write this workgroup's partial sums.
#pragma unroll
  for (int m = 0; m < MTW; ++m) {
    if (m * 16 >= p.cout_pad) break;
#pragma unroll
    for (int t = 0; t < NTW; ++t) {
      if (ntile_of[t] >= ncol_tiles) continue;
      const int col = ntile_of[t] * 16 + r16;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int row = m * 16 + 4 * g + i;
        p.slab[((size_t)blockIdx.x * p.cout_pad + row) * p.ncols_pad + col] = acc[m][t][i];
      }
    }
  }
}

__global__ void conv_dw_reduce_kernel(ConvDwReduceParams p) {
  const int KK = p.KS * p.KS;
  const int nW = p.Cout * p.Cin * KK;
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= nW + p.Cout) return;
  int row, col;
  if (j < nW) {
    row = j / (p.Cin * KK);
    const int rem = j - row * p.Cin * KK;
    const int i = rem / KK, kp = rem - i * KK;
    col = p.cvec ? (kp * p.CG + (i >> 3)) * 8 + (i & 7) : kp * p.Cin + i;
  } else {
    row = j - nW;
    col = p.kbias;
  }
  const float* s = p.slab + (size_t)row * p.ncols_pad + col;
  const size_t stride = (size_t)p.cout_pad * p.ncols_pad;
  float acc = 0.f;
  for (int x = 0; x < p.nx; ++x) acc += s[x * stride];
  float* dst = j < nW ? p.gw + j : p.gb + (j - nW);
  *dst = p.beta != 0.f ? p.beta * *dst + acc : acc;
}

inline size_t a16(size_t b) { return (b + 15) & ~size_t(15); }

template <typename T>
void launch_conv_fwd(const ConvParams& p, hipStream_t s) {
  const size_t lds = conv_forward_lds_bytes(sizeof(T) == 2 ? DType::BF16 : DType::F32, p);
  const dim3 grid((unsigned)cdiv(p.N, p.imgs)), block(256);
  if (p.cvec)
    hipLaunchKernelGGL((conv_fwd_kernel<T, true, 4>), grid, block, lds, s, p);
  else
    hipLaunchKernelGGL((conv_fwd_kernel<T, false, 4>), grid, block, lds, s, p);
}

template <typename T, bool CVEC>
void launch_conv_dw_c(const ConvDwParams& p, hipStream_t s, size_t lds) {
  const int mtw = p.cout_pad / 16;
  const int ncol_tiles = p.ncols_pad / 16;
  auto go = [&](auto kern, int ntw) {
    const dim3 grid((unsigned)p.nx, (unsigned)cdiv(ncol_tiles, 4 * ntw)), block(256);
    hipLaunchKernelGGL(kern, grid, block, lds, s, p);
  };
  if (mtw <= 1) go(conv_dw_kernel<T, CVEC, 1, 4>, 4);
  else if (mtw <= 2) go(conv_dw_kernel<T, CVEC, 2, 4>, 4);
  else if (mtw <= 4) go(conv_dw_kernel<T, CVEC, 4, 2>, 2);
  else if (mtw <= 8) go(conv_dw_kernel<T, CVEC, 8, 1>, 1);
  else MCC_CHECK(false, "conv_dw: Cout > 128 not supported by conv_small");
}

}  // namespace

size_t conv_forward_lds_bytes(DType t, const ConvParams& p) {
  const size_t es = t == DType::BF16 ? 2 : 4;
  const size_t nk = p.cvec ? (size_t)p.nchunks * 4 : (size_t)p.nchunks * 32;
  return a16(((size_t)p.imgs * p.LH * p.LW * p.CL + 16) * es) + nk * 4;
}

size_t conv_dw_lds_bytes(DType t, const ConvDwParams& p) {
  const size_t es = t == DType::BF16 ? 2 : 4;
  return a16(((size_t)p.imgs * p.LH * p.LW * p.CL + 16) * es) + a16((size_t)p.cout_pad * (p.ppad + 8) * es) +
         (size_t)p.ppad * 4;
}

void conv_forward(DType t, const ConvParams& p, hipStream_t s) {
  MCC_CHECK(p.N > 0 && p.imgs > 0 && p.nchunks > 0, "conv_forward: empty problem");
  MCC_CHECK(!p.cvec || (p.CL % 8) == 0, "conv_forward: cvec needs CL % 8 == 0");
  MCC_CHECK(p.kpad == p.nchunks * 32, "conv_forward: kpad mismatch");
  MCC_CHECK(p.pool == 1 || (p.pool == 2 && p.bias_act && p.out_arg), "conv_forward: bad pool config");
  MCC_CHECK(conv_forward_lds_bytes(t, p) <= 160 * 1024, "conv_forward: LDS tile exceeds 160 KiB");
  if (t == DType::BF16) launch_conv_fwd<bf16>(p, s);
  else launch_conv_fwd<float>(p, s);
}

void conv_dw(DType t, const ConvDwParams& p, hipStream_t s) {
  MCC_CHECK(p.N > 0 && p.imgs > 0 && p.nx > 0, "conv_dw: empty problem");
  MCC_CHECK(p.ppad % 32 == 0 && p.ppad >= p.imgs * p.OH * p.OW, "conv_dw: bad ppad");
  MCC_CHECK(p.cout_pad % 16 == 0 && p.ncols_pad % 16 == 0 && p.ncols_pad > p.kbias, "conv_dw: bad padding");
  const size_t lds = conv_dw_lds_bytes(t, p);
  MCC_CHECK(lds <= 160 * 1024, "conv_dw: LDS tile exceeds 160 KiB");
  if (t == DType::BF16) {
    if (p.cvec) launch_conv_dw_c<bf16, true>(p, s, lds);
    else launch_conv_dw_c<bf16, false>(p, s, lds);
  } else {
    if (p.cvec) launch_conv_dw_c<float, true>(p, s, lds);
    else launch_conv_dw_c<float, false>(p, s, lds);
  }
}

void conv_dw_reduce(const ConvDwReduceParams& p, hipStream_t s) {
  const int n = p.Cout * p.Cin * p.KS * p.KS + p.Cout;
  hipLaunchKernelGGL(conv_dw_reduce_kernel, dim3((unsigned)cdiv(n, 256)), dim3(256), 0, s, p);
}

}  // namespace gpu
}  // namespace mcc
