// Large-image convolution support (explicit im2col + MFMA GEMM path, used for
// layers whose image does not fit the whole-image LDS kernels, e.g. VGG-11
// at 224x224), plus the standalone 2x2 max-pool and the ReLU / max-pool
// gradient transform for that path.
//
//  im2col        rows = output pixels (n, oy, ox) NHWC order, cols = (kernel
//                position, input channel) — the packed weight K order — with
//                the same source transforms as LDS staging (u8 /255 + index
//                gather, ReLU mask, max-pool routing, zero insertion for the
//                data gradient of strided convs), 16-byte vector moves when
//                the channel count allows.
//  maxpool2      2x2/2 max with argmax byte (first max wins, PyTorch order)
//  grad_xform    dZ = relu' / unpool(dY) materialised at conv-output size for
//                the weight-gradient GEMM.
#include "kernels.h"
#include "mfma.h"

namespace mcc {
namespace gpu {

namespace {

template <typename T>
__device__ __forceinline__ float src_value(const StageSrc& s, int n, int sy, int sx, int c) {
  switch (s.mode) {
    case IN_U8: {
      const int img = s.idx ? s.idx[n] : n;
      return (float)static_cast<const uint8_t*>(s.src)[(((size_t)img * s.SH + sy) * s.SW + sx) * s.SC + c] *
             (1.0f / 255.0f);
    }
    case IN_RELU: {
      const size_t i = (((size_t)n * s.SH + sy) * s.SW + sx) * s.SC + c;
      return to_f(static_cast<const T*>(s.aux_y)[i]) > 0.f ? to_f(static_cast<const T*>(s.src)[i]) : 0.f;
    }
    case IN_UNPOOL: {
      // every window (py, px) holding (sy, sx) whose argmax is this position
      // (one window for a 2x2/2 pool; overlapping pools sum, in window order)
      float acc = 0.f;
      const int py0 = sy >= s.pk ? (sy - s.pk) / s.ps + 1 : 0, px0 = sx >= s.pk ? (sx - s.pk) / s.ps + 1 : 0;
      for (int py = py0; py <= sy / s.ps && py < s.PH; ++py)
        for (int px = px0; px <= sx / s.ps && px < s.PW; ++px) {
          const size_t i = (((size_t)n * s.PH + py) * s.PW + px) * s.SC + c;
          if (s.aux_arg[i] != (sy - py * s.ps) * s.pk + (sx - px * s.ps)) continue;
          const float y = to_f(static_cast<const T*>(s.aux_y)[i]), d = to_f(static_cast<const T*>(s.src)[i]);
          acc += s.act == ACT_RELU ? (y > 0.f ? d : 0.f) : d * act_grad_y(s.act, y);
        }
      return acc;
    }
    case IN_TANH: {
      const size_t i = (((size_t)n * s.SH + sy) * s.SW + sx) * s.SC + c;
      const float y = to_f(static_cast<const T*>(s.aux_y)[i]);
      return to_f(static_cast<const T*>(s.src)[i]) * (1.f - y * y);
    }
    default:
      return to_f(static_cast<const T*>(s.src)[(((size_t)n * s.SH + sy) * s.SW + sx) * s.SC + c]);
  }
}

// One thread per (output pixel, 8-column group).
template <typename T>
__global__ void __launch_bounds__(256) im2col_kernel(Im2colParams p) {
  typedef typename Vec8<T>::type V8;
  const int64_t groups = p.ldk >> 3;
  const int64_t total = (int64_t)p.N * p.OH * p.OW * groups;
  const int K = p.KS * p.KS * p.s.SC;
  T* out = static_cast<T*>(p.out);
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t row = e / groups;
    const int k0 = (int)(e - row * groups) * 8;
    const int64_t pix = row % ((int64_t)p.OH * p.OW);
    const int n = (int)(row / ((int64_t)p.OH * p.OW));
    const int oy = (int)(pix / p.OW), ox = (int)(pix % p.OW);
    V8 v;
    const bool vec = (p.s.SC & 7) == 0 && p.s.mode == IN_PLAIN;
    if (vec && k0 + 8 <= K) {
      const int kp = k0 / p.s.SC, c0 = k0 - kp * p.s.SC;
      const int kh = kp / p.KS, kw = kp - kh * p.KS;
      int ty = oy * p.cs + kh - p.s.off, tx = ox * p.cs + kw - p.s.off;
      bool ok = ty >= 0 && tx >= 0;
      if (p.s.up != 1) {
        ok = ok && ty % p.s.up == 0 && tx % p.s.up == 0;
        ty /= p.s.up;
        tx /= p.s.up;
      }
      ok = ok && ty < p.s.SH && tx < p.s.SW;
      if (ok) {
        v = load8(static_cast<const T*>(p.s.src) + (((size_t)n * p.s.SH + ty) * p.s.SW + tx) * p.s.SC + c0);
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = T(0);
      }
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int k = k0 + j;
        float f = 0.f;
        if (k < K) {
          const int kp = k / p.s.SC, c = k - kp * p.s.SC;
          const int kh = kp / p.KS, kw = kp - kh * p.KS;
          int ty = oy * p.cs + kh - p.s.off, tx = ox * p.cs + kw - p.s.off;
          bool ok = ty >= 0 && tx >= 0;
          if (p.s.up != 1) {
            ok = ok && ty % p.s.up == 0 && tx % p.s.up == 0;
            ty /= p.s.up;
            tx /= p.s.up;
          }
          ok = ok && ty < p.s.SH && tx < p.s.SW;
          if (ok) f = src_value<T>(p.s, n, ty, tx, c);
        }
        v[j] = from_f<T>(f);
      }
    }
    store8(out + (size_t)row * p.ldk + k0, v);
  }
}

template <typename T>
__global__ void __launch_bounds__(256) maxpool2_kernel(const T* __restrict__ in, T* __restrict__ out,
                                                       uint8_t* __restrict__ arg, int N, int H, int W, int C,
                                                       bool post_relu) {
  const int PH = H >> 1, PW = W >> 1;
  const int64_t total = (int64_t)N * PH * PW * C;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
    const int c = (int)(e % C);
    const int64_t r = e / C;
    const int px = (int)(r % PW), py = (int)((r / PW) % PH), n = (int)(r / ((int64_t)PW * PH));
    const size_t b = (((size_t)n * H + 2 * py) * W + 2 * px) * C + c;
    float v[4] = {to_f(in[b]), to_f(in[b + C]), to_f(in[b + (size_t)W * C]), to_f(in[b + (size_t)W * C + C])};
    float best = v[0];
    int a = 0;
#pragma unroll
    for (int i = 1; i < 4; ++i)
      if (v[i] > best) { best = v[i]; a = i; }
    out[e] = from_f<T>(best);
    arg[e] = (uint8_t)(!post_relu || to_f(from_f<T>(best)) > 0.f ? a : 4);  // post-ReLU: 4 = inactive window
  }
}

template <typename T>
__global__ void __launch_bounds__(256) maxpool_kernel(const T* __restrict__ in, T* __restrict__ out,
                                                      uint8_t* __restrict__ arg, int N, int H, int W, int C, int k,
                                                      int st, int PH, int PW) {
  const int64_t total = (int64_t)N * PH * PW * C;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
    const int c = (int)(e % C);
    const int64_t r = e / C;
    const int px = (int)(r % PW), py = (int)((r / PW) % PH), n = (int)(r / ((int64_t)PW * PH));
    float best = 0.f;
    int a = -1;
    for (int dy = 0; dy < k; ++dy)
      for (int dx = 0; dx < k; ++dx) {
        const float v = to_f(in[(((size_t)n * H + py * st + dy) * W + px * st + dx) * C + c]);
        if (a < 0 || v > best) { best = v; a = dy * k + dx; }
      }
    out[e] = from_f<T>(best);
    arg[e] = (uint8_t)a;
  }
}

// dZ at conv-output resolution from the stage-output gradient.
template <typename T>
__global__ void __launch_bounds__(256) grad_xform_kernel(StageSrc s, T* __restrict__ dz, int N) {
  const int64_t total = (int64_t)N * s.SH * s.SW * s.SC;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
    const int c = (int)(e % s.SC);
    const int64_t r = e / s.SC;
    const int x = (int)(r % s.SW), y = (int)((r / s.SW) % s.SH), n = (int)(r / ((int64_t)s.SW * s.SH));
    dz[e] = from_f<T>(src_value<T>(s, n, y, x, c));
  }
}

// bf16, C % 8 == 0: one thread per (pixel, 8 channels), 16-byte moves,
// 32-bit index math (host checks the element count).
__global__ void __launch_bounds__(256) maxpool2_vec_kernel(const bf16* __restrict__ in, bf16* __restrict__ out,
                                                           uint8_t* __restrict__ arg, int N, int H, int W, int C,
                                                           bool post_relu) {
  const int PH = H >> 1, PW = W >> 1, C8 = C >> 3;
  const int total = N * PH * PW * C8;
  for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < total; e += gridDim.x * blockDim.x) {
    const int c8 = e % C8, r = e / C8;
    const int px = r % PW, r2 = r / PW, py = r2 % PH, n = r2 / PH;
    const size_t b = (((size_t)n * H + 2 * py) * W + 2 * px) * C + c8 * 8;
    const bf16x8 v0 = load8(in + b), v1 = load8(in + b + C), v2 = load8(in + b + (size_t)W * C),
                 v3 = load8(in + b + (size_t)W * C + C);
    bf16x8 o;
    uint32_t a0 = 0, a1 = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float best = (float)v0[j];
      uint32_t a = 0;
      if ((float)v1[j] > best) { best = (float)v1[j]; a = 1; }
      if ((float)v2[j] > best) { best = (float)v2[j]; a = 2; }
      if ((float)v3[j] > best) { best = (float)v3[j]; a = 3; }
      o[j] = (bf16)best;
      if (post_relu && !(best > 0.f)) a = 4;  // post-ReLU input: inactive window
      if (j < 4) a0 |= a << (8 * j); else a1 |= a << (8 * (j - 4));
    }
    store8(out + (size_t)r * C + c8 * 8, o);
    *reinterpret_cast<uint2*>(arg + (size_t)r * C + c8 * 8) = make_uint2(a0, a1);
  }
}

// dZ = relu' (IN_RELU) or unpool + relu' (IN_UNPOOL) of dY, bf16, C % 8 == 0.
// UNPOOL: one thread per (pooled pixel, 8 channels) writes the whole 2x2
// window (odd-size borders beyond the last window are written as zero).
__global__ void __launch_bounds__(256) grad_xform_vec_kernel(StageSrc s, bf16* __restrict__ dz, int N) {
  const int C8 = s.SC >> 3;
  const bf16* dy = static_cast<const bf16*>(s.src);
  const bf16* y = static_cast<const bf16*>(s.aux_y);
  if (s.mode == IN_RELU) {
    const int total = N * s.SH * s.SW * C8;
    for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < total; e += gridDim.x * blockDim.x) {
      const bf16x8 d = load8(dy + (size_t)e * 8), yv = load8(y + (size_t)e * 8);
      bf16x8 o;
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = (float)yv[j] > 0.f ? d[j] : (bf16)0.f;
      store8(dz + (size_t)e * 8, o);
    }
    return;
  }
  const int total = N * s.PH * s.PW * C8;
  for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < total; e += gridDim.x * blockDim.x) {
    const int c8 = e % C8, r = e / C8;
    const int px = r % s.PW, r2 = r / s.PW, py = r2 % s.PH, n = r2 / s.PH;
    const bf16x8 d = load8(dy + (size_t)e * 8), yv = load8(y + (size_t)e * 8);
    const uint2 av = *reinterpret_cast<const uint2*>(s.aux_arg + (size_t)e * 8);
    bf16x8 o[4];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const uint32_t a = ((j < 4 ? av.x : av.y) >> (8 * (j & 3))) & 0xffu;
      const bf16 v = (float)yv[j] > 0.f ? d[j] : (bf16)0.f;
#pragma unroll
      for (int q = 0; q < 4; ++q) o[q][j] = a == (uint32_t)q ? v : (bf16)0.f;
    }
    const size_t b = (((size_t)n * s.SH + 2 * py) * s.SW + 2 * px) * s.SC + c8 * 8;
    store8(dz + b, o[0]);
    store8(dz + b + s.SC, o[1]);
    store8(dz + b + (size_t)s.SW * s.SC, o[2]);
    store8(dz + b + (size_t)s.SW * s.SC + s.SC, o[3]);
  }
  // odd borders (conv output row/column past the last full window)
  if ((s.SH & 1) || (s.SW & 1)) {
    const int rows = s.SH & 1, cols = s.SW & 1;
    const int per = (rows ? s.SW : 0) + (cols ? s.SH - rows : 0);
    const int tot = N * per * C8;
    const bf16x8 z = {};
    for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < tot; e += gridDim.x * blockDim.x) {
      const int c8 = e % C8, r = e / C8, n = r / per, k = r - n * per;
      int yy, xx;
      if (rows && k < s.SW) { yy = s.SH - 1; xx = k; }
      else { yy = k - (rows ? s.SW : 0); xx = s.SW - 1; }
      store8(dz + (((size_t)n * s.SH + yy) * s.SW + xx) * s.SC + c8 * 8, z);
    }
  }
}

inline unsigned grid_cap(int64_t n) {
  int64_t b = (n + 255) / 256;
  if (b < 1) b = 1;
  if (b > 65536) b = 65536;
  return (unsigned)b;
}

}  // namespace

void im2col(DType t, const Im2colParams& p, hipStream_t s) {
  MCC_CHECK(p.ldk % 8 == 0 && p.ldk >= p.KS * p.KS * p.s.SC, "im2col: bad ldk");
  const int64_t n = (int64_t)p.N * p.OH * p.OW * (p.ldk / 8);
  if (t == DType::BF16) hipLaunchKernelGGL(im2col_kernel<bf16>, dim3(grid_cap(n)), dim3(256), 0, s, p);
  else hipLaunchKernelGGL(im2col_kernel<float>, dim3(grid_cap(n)), dim3(256), 0, s, p);
}

void maxpool2(DType t, const void* in, void* out, uint8_t* arg, int N, int H, int W, int C, hipStream_t s,
              bool post_relu) {
  const int64_t n = (int64_t)N * (H / 2) * (W / 2) * C;
  if (t == DType::BF16 && C % 8 == 0 && (int64_t)N * H * W * C < (1ll << 31)) {
    hipLaunchKernelGGL(maxpool2_vec_kernel, dim3(grid_cap(n / 8)), dim3(256), 0, s, static_cast<const bf16*>(in),
                       static_cast<bf16*>(out), arg, N, H, W, C, post_relu);
    return;
  }
  if (t == DType::BF16)
    hipLaunchKernelGGL(maxpool2_kernel<bf16>, dim3(grid_cap(n)), dim3(256), 0, s, static_cast<const bf16*>(in),
                       static_cast<bf16*>(out), arg, N, H, W, C, post_relu);
  else
    hipLaunchKernelGGL(maxpool2_kernel<float>, dim3(grid_cap(n)), dim3(256), 0, s, static_cast<const float*>(in),
                       static_cast<float*>(out), arg, N, H, W, C, post_relu);
}

void maxpool(DType t, const void* in, void* out, uint8_t* arg, int N, int H, int W, int C, int k, int stride,
             hipStream_t s) {
  MCC_CHECK(k >= 1 && k <= 15 && stride >= 1 && H >= k && W >= k, "maxpool: bad window");
  const int PH = (H - k) / stride + 1, PW = (W - k) / stride + 1;
  const int64_t n = (int64_t)N * PH * PW * C;
  if (t == DType::BF16)
    hipLaunchKernelGGL(maxpool_kernel<bf16>, dim3(grid_cap(n)), dim3(256), 0, s, static_cast<const bf16*>(in),
                       static_cast<bf16*>(out), arg, N, H, W, C, k, stride, PH, PW);
  else
    hipLaunchKernelGGL(maxpool_kernel<float>, dim3(grid_cap(n)), dim3(256), 0, s, static_cast<const float*>(in),
                       static_cast<float*>(out), arg, N, H, W, C, k, stride, PH, PW);
}

void grad_xform(DType t, const StageSrc& src, void* dz, int N, hipStream_t s) {
  const int64_t n = (int64_t)N * src.SH * src.SW * src.SC;
  if (t == DType::BF16 && src.SC % 8 == 0 && n < (1ll << 31) &&
      (src.mode == IN_RELU || (src.mode == IN_UNPOOL && src.act == ACT_RELU && src.pk == 2 && src.ps == 2 &&
                               src.PH == src.SH / 2 && src.PW == src.SW / 2))) {
    hipLaunchKernelGGL(grad_xform_vec_kernel, dim3(grid_cap(n / 8)), dim3(256), 0, s, src, static_cast<bf16*>(dz), N);
    return;
  }
  if (t == DType::BF16)
    hipLaunchKernelGGL(grad_xform_kernel<bf16>, dim3(grid_cap(n)), dim3(256), 0, s, src, static_cast<bf16*>(dz), N);
  else
    hipLaunchKernelGGL(grad_xform_kernel<float>, dim3(grid_cap(n)), dim3(256), 0, s, src, static_cast<float*>(dz), N);
}

}  // namespace gpu
}  // namespace mcc
