// fp64 executor kernels: the reference's own precision on the GPU.
//
// The reference is fp64 end to end (cnn.c:22-30) and its one GPU kernel is
// an fp64 conv forward, one thread per output (CUDAcnn.cu:167-195).  These
// kernels back GpuNet64 (csrc/engine/net64.cpp), which executes any ModelSpec
// in fp64 with the CPU executor's semantics (csrc/core/cpu_net.cpp), so the
// reference program can be reproduced on an MI355X and diffed against it.
//
// Design: every GEMM-shaped product (conv as im2col x weights, FC, and all
// weight / data gradients) runs on one MFMA kernel, v_mfma_f64_16x16x4_f64
// (CDNA4's fp64 matrix path), over strided operand views, so no transposed
// copies are materialised.  Everything is deterministic: fixed-order split-K
// slabs instead of atomics, gathers instead of scatters (col2im, unpool).
#include <hip/hip_runtime.h>

#include <algorithm>

#include "kernels.h"

namespace mcc {
namespace gpu {

namespace {

using f64x4 = __attribute__((ext_vector_type(4))) double;

constexpr int kTK = 16;
constexpr int kPitch = 80;  // LDS row pitch (doubles): the 4 k rows a 16x16x4 operand read touches sit 128 B apart

__device__ __forceinline__ double act_f(int act, double v) {
  return act == ACT_RELU ? (v > 0.0 ? v : 0.0) : act == ACT_TANH ? tanh(v) : v;
}
// derivative in terms of the activation OUTPUT (cnn.c:52-57)
__device__ __forceinline__ double act_g(int act, double y) {
  return act == ACT_RELU ? (y > 0.0 ? 1.0 : 0.0) : act == ACT_TANH ? 1.0 - y * y : 1.0;
}

__device__ __forceinline__ void g64_store(const Gemm64Params& p, int m, int n, double v) {
  if (p.bias_m) v += p.bias_m[m];
  if (p.bias_n) v += p.bias_n[n];
  v = act_f(p.act, v);
  double* dst = p.P > 0 ? p.C + ((int64_t)(n / p.P) * p.M + m) * p.P + n % p.P : p.C + (int64_t)m * p.ldc + n;
  if (p.accumulate) v += *dst;
  *dst = v;
}

// TS x TS output tile per 256-thread workgroup (TS = 64 or 32); wave w owns
// the (TS/2)^2 quadrant (w >> 1, w & 1) as (TS/32)^2 MFMA blocks.  Operands
// are staged k-major in LDS ([k][m], [k][n]) with register prefetch of the
// next k tile; the global load order follows whichever operand dimension is
// unit-stride.  TS = 32 serves the skinny weight-gradient products (the
// reference model's conv1 dW is 16 x 9 over K = B * 196: a 64-tile computed
// 28x the useful MACs).
template <int TS>
__global__ void __launch_bounds__(256) gemm64_kernel(Gemm64Params p) {
  constexpr int NB = TS / 32;             // MFMA blocks per wave dimension
  constexpr int NL = TS * kTK / 256;      // staged elements per thread per operand
  constexpr int PITCH = TS == 64 ? kPitch : 48;
  __shared__ double As[kTK][PITCH];
  __shared__ double Bs[kTK][PITCH];
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int m0 = blockIdx.y * TS, n0 = blockIdx.x * TS;
  const int64_t kbeg = (int64_t)blockIdx.z * p.kchunk;
  const int64_t kend = kbeg + p.kchunk < p.K ? kbeg + p.kchunk : p.K;
  const bool a_kfast = p.sak == 1, b_nfast = p.sbn == 1;

  double ra[NL], rb[NL];
  auto fetch = [&](int64_t k0) {
#pragma unroll
    for (int j = 0; j < NL; ++j) {
      const int e = t + 256 * j;
      int m, k;
      if (a_kfast) { k = e & 15; m = e >> 4; } else { m = e % TS; k = e / TS; }
      const int64_t gk = k0 + k;
      ra[j] = (m0 + m < p.M && gk < kend) ? p.A[(int64_t)(m0 + m) * p.sam + gk * p.sak] : 0.0;
      int n;
      if (b_nfast) { n = e % TS; k = e / TS; } else { k = e & 15; n = e >> 4; }
      const int64_t gk2 = k0 + k;
      rb[j] = (n0 + n < p.N && gk2 < kend) ? p.B[gk2 * p.sbk + (int64_t)(n0 + n) * p.sbn] : 0.0;
    }
  };
  auto stash = [&]() {
#pragma unroll
    for (int j = 0; j < NL; ++j) {
      const int e = t + 256 * j;
      if (a_kfast) As[e & 15][e >> 4] = ra[j]; else As[e / TS][e % TS] = ra[j];
      if (b_nfast) Bs[e / TS][e % TS] = rb[j]; else Bs[e & 15][e >> 4] = rb[j];
    }
  };

  f64x4 acc[NB][NB];
#pragma unroll
  for (int i = 0; i < NB; ++i)
#pragma unroll
    for (int j = 0; j < NB; ++j) acc[i][j] = f64x4{0.0, 0.0, 0.0, 0.0};
  const int wm = (wave >> 1) * (TS / 2), wn = (wave & 1) * (TS / 2);
  const int r = lane & 15, q = lane >> 4;

  if (kbeg < kend) fetch(kbeg);
  for (int64_t k0 = kbeg; k0 < kend; k0 += kTK) {
    __syncthreads();
    stash();
    __syncthreads();
    if (k0 + kTK < kend) fetch(k0 + kTK);
#pragma unroll
    for (int s = 0; s < kTK / 4; ++s) {
      double a[NB], bb[NB];
#pragma unroll
      for (int i = 0; i < NB; ++i) {
        a[i] = As[4 * s + q][wm + 16 * i + r];
        bb[i] = Bs[4 * s + q][wn + 16 * i + r];
      }
#pragma unroll
      for (int i = 0; i < NB; ++i)
#pragma unroll
        for (int j = 0; j < NB; ++j) acc[i][j] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[i], bb[j], acc[i][j], 0, 0, 0);
    }
  }
  // f64 C/D map: col = lane & 15, row = (lane >> 4) + 4 * reg
#pragma unroll
  for (int i = 0; i < NB; ++i)
#pragma unroll
    for (int j = 0; j < NB; ++j)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int m = m0 + wm + 16 * i + q + 4 * g, n = n0 + wn + 16 * j + r;
        if (m >= p.M || n >= p.N) continue;
        if (p.part) p.part[((int64_t)blockIdx.z * p.M + m) * p.N + n] = acc[i][j][g];
        else g64_store(p, m, n, acc[i][j][g]);
      }
}

// split-K: sum the slabs in slab order, then the epilogue
__global__ void gemm64_reduce_kernel(Gemm64Params p, int nslab) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t MN = (int64_t)p.M * p.N;
  if (e >= MN) return;
  double v = 0.0;
  for (int z = 0; z < nslab; ++z) v += p.part[z * MN + e];
  g64_store(p, (int)(e / p.N), (int)(e % p.N), v);
}

// col[(i*k + kh)*k + kw][b*P + oy*OW + ox] = x[b][i][oy*s - pad + kh][ox*s - pad + kw] (0 outside)
__global__ void im2col64_kernel(Conv64Geom g, const double* x, double* col, int B) {
  const int64_t P = (int64_t)g.OH * g.OW, BP = B * P;
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= (int64_t)g.Ci * g.k * g.k * BP) return;
  const int64_t n = e % BP;
  const int kidx = (int)(e / BP);
  const int kw = kidx % g.k, kh = (kidx / g.k) % g.k, i = kidx / (g.k * g.k);
  const int b = (int)(n / P), pp = (int)(n % P), oy = pp / g.OW, ox = pp % g.OW;
  const int y = oy * g.s - g.pad + kh, xx = ox * g.s - g.pad + kw;
  double v = 0.0;
  if (y >= 0 && y < g.H && xx >= 0 && xx < g.W) v = x[((int64_t)(b * g.Ci + i) * g.H + y) * g.W + xx];
  col[e] = v;
}

// dx[b][i][y][x] = sum over (kh, kw) whose output pixel exists of dcol[(i, kh, kw)][b, oy, ox]
__global__ void col2im64_kernel(Conv64Geom g, const double* dcol, double* dx, int B) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= (int64_t)B * g.Ci * g.H * g.W) return;
  const int xx = (int)(e % g.W), y = (int)((e / g.W) % g.H);
  const int i = (int)((e / ((int64_t)g.W * g.H)) % g.Ci), b = (int)(e / ((int64_t)g.W * g.H * g.Ci));
  const int64_t P = (int64_t)g.OH * g.OW, BP = B * P;
  double v = 0.0;
  for (int kh = 0; kh < g.k; ++kh) {
    const int ty = y + g.pad - kh;
    if (ty < 0 || ty % g.s) continue;
    const int oy = ty / g.s;
    if (oy >= g.OH) continue;
    for (int kw = 0; kw < g.k; ++kw) {
      const int tx = xx + g.pad - kw;
      if (tx < 0 || tx % g.s) continue;
      const int ox = tx / g.s;
      if (ox >= g.OW) continue;
      v += dcol[((int64_t)(i * g.k + kh) * g.k + kw) * BP + (int64_t)b * P + oy * g.OW + ox];
    }
  }
  dx[e] = v;
}

// reference shared-slice weights (defect D1, cnn.c:181,193): every input
// channel reads W[o][0]
__global__ void weff64_kernel(const double* w, double* weff, int C, int Ci, int kk) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= C * Ci * kk) return;
  const int o = e / (Ci * kk), r = e % kk;
  weff[e] = w[(int64_t)o * Ci * kk + r];
}
// ... and their gradient lands in that slice, summed over the input channels
__global__ void fold64_kernel(const double* full, double* gw, int C, int Ci, int kk) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= C * kk) return;
  const int o = e / kk, r = e % kk;
  double v = 0.0;
  for (int i = 0; i < Ci; ++i) v += full[((int64_t)o * Ci + i) * kk + r];
  gw[(int64_t)o * Ci * kk + r] += v;
}

// dzT[o][b*P + p] = err[b][o][p] * act'(y[b][o][p])
__global__ void dz64_kernel(const double* err, const double* y, double* dzT, int B, int C, int P, int act) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= (int64_t)B * C * P) return;
  const int pp = (int)(e % P), o = (int)((e / P) % C), b = (int)(e / ((int64_t)P * C));
  dzT[(int64_t)o * B * P + (int64_t)b * P + pp] = err[e] * act_g(act, y[e]);
}

// gb[o] += sum_n dzT[o][n] in two fixed-order levels: S workgroups per row
// each sum a contiguous chunk (strided partials + a fixed tree) into
// part[o][s], then one thread per row adds its S partials in slab order.
// (One workgroup per row left the reference model's conv1 bias -- 16 rows of
// B * 196 -- on 16 CUs: 5 ms of a 13 ms fp64 step at B = 16384.)
__global__ void __launch_bounds__(256) rowsum64_kernel(const double* dzT, double* part, int64_t n, int64_t chunk) {
  __shared__ double red[256];
  const int row = blockIdx.y, sl = blockIdx.x;
  const double* src = dzT + (int64_t)row * n;
  const int64_t j0 = (int64_t)sl * chunk, j1 = j0 + chunk < n ? j0 + chunk : n;
  double v = 0.0;
  for (int64_t j = j0 + threadIdx.x; j < j1; j += 256) v += src[j];
  red[threadIdx.x] = v;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0) part[(int64_t)row * gridDim.x + sl] = red[0];
}
__global__ void rowsum64_finish_kernel(const double* part, double* gb, int rows, int S) {
  const int o = blockIdx.x * blockDim.x + threadIdx.x;
  if (o >= rows) return;
  double v = 0.0;
  for (int s = 0; s < S; ++s) v += part[(int64_t)o * S + s];
  gb[o] += v;
}

// max pool, first maximum wins (cpu_net.cpp pool_fwd); arg = flat input index
__global__ void pool64_fwd_kernel(Pool64Geom g, const double* x, double* y, int32_t* arg, int B) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= (int64_t)B * g.C * g.OH * g.OW) return;
  const int px = (int)(e % g.OW), py = (int)((e / g.OW) % g.OH);
  const int c = (int)((e / ((int64_t)g.OW * g.OH)) % g.C), b = (int)(e / ((int64_t)g.OW * g.OH * g.C));
  const double* in = x + (int64_t)b * g.C * g.H * g.W;
  int best = -1;
  double bv = 0.0;
  for (int dy = 0; dy < g.k; ++dy)
    for (int dx = 0; dx < g.k; ++dx) {
      const int idx = (c * g.H + py * g.s + dy) * g.W + px * g.s + dx;
      if (best < 0 || in[idx] > bv) { best = idx; bv = in[idx]; }
    }
  y[e] = bv;
  arg[e] = best;
}
// gather form of pe[arg[o]] += er[o]: every window covering the input pixel,
// in output order
__global__ void pool64_bwd_kernel(Pool64Geom g, const double* er, const int32_t* arg, double* dx, int B) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= (int64_t)B * g.C * g.H * g.W) return;
  const int xx = (int)(e % g.W), y = (int)((e / g.W) % g.H);
  const int c = (int)((e / ((int64_t)g.W * g.H)) % g.C), b = (int)(e / ((int64_t)g.W * g.H * g.C));
  const int idx = (c * g.H + y) * g.W + xx;
  const int64_t ob = (int64_t)b * g.C * g.OH * g.OW + (int64_t)c * g.OH * g.OW;
  const int py0 = y >= g.k ? (y - g.k) / g.s + 1 : 0, py1 = min(g.OH - 1, y / g.s);
  const int px0 = xx >= g.k ? (xx - g.k) / g.s + 1 : 0, px1 = min(g.OW - 1, xx / g.s);
  double v = 0.0;
  for (int py = py0; py <= py1; ++py)
    for (int px = px0; px <= px1; ++px) {
      const int64_t o = ob + py * g.OW + px;
      if (arg[o] == idx) v += er[o];
    }
  dx[e] = v;
}

// softmax with max subtraction (cnn.c:125-143); ref_compat: the max starts
// at -1 (defect D10)
__global__ void softmax64_kernel(double* z, int B, int C, bool ref_compat) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  double* r = z + (int64_t)b * C;
  double m = ref_compat ? -1.0 : r[0];
  for (int j = 0; j < C; ++j) m = r[j] > m ? r[j] : m;
  double t = 0.0;
  for (int j = 0; j < C; ++j) { r[j] = exp(r[j] - m); t += r[j]; }
  for (int j = 0; j < C; ++j) r[j] /= t;
}

// err = (p - onehot) * scale (cnn.c:284-286) and per-sample stats
// [-log p_label, mean (p - y)^2 (cnn.c:275-282), argmax == label]
__global__ void out_err64_kernel(const double* p, const int32_t* labels, double* err, double* stats, int B, int C,
                                 double scale) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  const double* r = p + (int64_t)b * C;
  const int lab = labels[b];
  int mj = -1;
  double mse = 0.0;
  for (int j = 0; j < C; ++j) {
    if (mj < 0 || r[mj] < r[j]) mj = j;
    const double e = r[j] - (j == lab ? 1.0 : 0.0);
    mse += e * e;
    if (err) err[(int64_t)b * C + j] = e * scale;
  }
  stats[3 * b + 0] = -log(fmax(r[lab], 1e-300));
  stats[3 * b + 1] = mse / C;
  stats[3 * b + 2] = mj == lab ? 1.0 : 0.0;
}

// device-resident batch: x[b] = dataset[idx[b]] / 255 (cnn.c:457), labels[b] = lab[idx[b]]
__global__ void u8_batch64_kernel(const uint8_t* data, const uint8_t* lab, const int32_t* idx, double* x,
                                  int32_t* labels, int B, int npix) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= (int64_t)B * npix) return;
  const int b = (int)(e / npix), i = (int)(e - (int64_t)b * npix);
  const int src = idx ? idx[b] : b;
  x[e] = (double)data[(int64_t)src * npix + i] / 255.0;
  if (i == 0) labels[b] = lab[src];
}

__global__ void sgd64_kernel(double* w, double* g, double lr, int64_t n) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n) return;
  w[e] -= lr * g[e];
  g[e] = 0.0;
}

unsigned blocks(int64_t n, int t = 256) { return (unsigned)((n + t - 1) / t); }

}  // namespace

void u8_batch64(const uint8_t* data, const uint8_t* lab, const int32_t* idx, double* x, int32_t* labels, int B,
                int npix, hipStream_t s) {
  hipLaunchKernelGGL(u8_batch64_kernel, dim3(blocks((int64_t)B * npix)), dim3(256), 0, s, data, lab, idx, x, labels,
                     B, npix);
}

static int gemm64_tile(int M, int N);

int gemm64_slabs(int M, int N, int64_t K) {
  // enough (tile, slab) workgroups to cover the 256 CUs twice, slabs of at
  // least 256 k; a function of the shape only (deterministic results)
  const int TS = gemm64_tile(M, N);
  const int64_t tiles = (int64_t)((M + TS - 1) / TS) * ((N + TS - 1) / TS);
  int64_t s = 512 / tiles;
  const int64_t kmax = (K + 255) / 256;
  if (s > kmax) s = kmax;
  return s < 1 ? 1 : (int)s;
}

// 32-tiles when either output dimension is at most 32 (skinny weight
// gradients / FC layers with few outputs), else 64-tiles
static int gemm64_tile(int M, int N) { return (M <= 32 || N <= 32) ? 32 : 64; }

void gemm64(const Gemm64Params& p0, double* part, hipStream_t s) {
  Gemm64Params p = p0;
  const int TS = gemm64_tile(p.M, p.N);
  const int nslab = part ? gemm64_slabs(p.M, p.N, p.K) : 1;
  int64_t kc = (p.K + nslab - 1) / nslab;
  kc = (kc + kTK - 1) / kTK * kTK;
  const int z = (int)((p.K + kc - 1) / kc);
  p.kchunk = kc;
  p.part = z > 1 ? part : nullptr;
  dim3 grid((unsigned)((p.N + TS - 1) / TS), (unsigned)((p.M + TS - 1) / TS), (unsigned)(z > 0 ? z : 1));
  if (TS == 32) hipLaunchKernelGGL(gemm64_kernel<32>, grid, dim3(256), 0, s, p);
  else hipLaunchKernelGGL(gemm64_kernel<64>, grid, dim3(256), 0, s, p);
  if (z > 1) hipLaunchKernelGGL(gemm64_reduce_kernel, dim3(blocks((int64_t)p.M * p.N)), dim3(256), 0, s, p, z);
}

void im2col64(const Conv64Geom& g, const double* x, double* col, int B, hipStream_t s) {
  const int64_t n = (int64_t)g.Ci * g.k * g.k * B * g.OH * g.OW;
  hipLaunchKernelGGL(im2col64_kernel, dim3(blocks(n)), dim3(256), 0, s, g, x, col, B);
}
void col2im64(const Conv64Geom& g, const double* dcol, double* dx, int B, hipStream_t s) {
  const int64_t n = (int64_t)B * g.Ci * g.H * g.W;
  hipLaunchKernelGGL(col2im64_kernel, dim3(blocks(n)), dim3(256), 0, s, g, dcol, dx, B);
}
void weff64(const double* w, double* weff, int C, int Ci, int kk, hipStream_t s) {
  hipLaunchKernelGGL(weff64_kernel, dim3(blocks((int64_t)C * Ci * kk)), dim3(256), 0, s, w, weff, C, Ci, kk);
}
void fold64(const double* full, double* gw, int C, int Ci, int kk, hipStream_t s) {
  hipLaunchKernelGGL(fold64_kernel, dim3(blocks((int64_t)C * kk)), dim3(256), 0, s, full, gw, C, Ci, kk);
}
void dz64(const double* err, const double* y, double* dzT, int B, int C, int P, int act, hipStream_t s) {
  hipLaunchKernelGGL(dz64_kernel, dim3(blocks((int64_t)B * C * P)), dim3(256), 0, s, err, y, dzT, B, C, P, act);
}
void rowsum64(const double* dzT, double* gb, int rows, int64_t n, double* part, hipStream_t s) {
  // slabs per row: ~1024 workgroups in all, chunks of at least 4096 (a
  // function of the shape only: deterministic)
  int64_t S = std::max<int64_t>(1, std::min<int64_t>(1024 / std::max(rows, 1), (n + 4095) / 4096));
  const int64_t chunk = (n + S - 1) / S;
  S = (n + chunk - 1) / chunk;
  hipLaunchKernelGGL(rowsum64_kernel, dim3((unsigned)S, (unsigned)rows), dim3(256), 0, s, dzT, part, n, chunk);
  hipLaunchKernelGGL(rowsum64_finish_kernel, dim3(blocks(rows)), dim3(256), 0, s, part, gb, rows, (int)S);
}
void pool64_fwd(const Pool64Geom& g, const double* x, double* y, int32_t* arg, int B, hipStream_t s) {
  hipLaunchKernelGGL(pool64_fwd_kernel, dim3(blocks((int64_t)B * g.C * g.OH * g.OW)), dim3(256), 0, s, g, x, y, arg, B);
}
void pool64_bwd(const Pool64Geom& g, const double* er, const int32_t* arg, double* dx, int B, hipStream_t s) {
  hipLaunchKernelGGL(pool64_bwd_kernel, dim3(blocks((int64_t)B * g.C * g.H * g.W)), dim3(256), 0, s, g, er, arg, dx, B);
}
void softmax64(double* z, int B, int C, bool ref_compat, hipStream_t s) {
  hipLaunchKernelGGL(softmax64_kernel, dim3(blocks(B, 64)), dim3(64), 0, s, z, B, C, ref_compat);
}
void out_err64(const double* p, const int32_t* labels, double* err, double* stats, int B, int C, double scale,
               hipStream_t s) {
  hipLaunchKernelGGL(out_err64_kernel, dim3(blocks(B, 64)), dim3(64), 0, s, p, labels, err, stats, B, C, scale);
}
void sgd64(double* w, double* g, double lr, int64_t n, hipStream_t s) {
  hipLaunchKernelGGL(sgd64_kernel, dim3(blocks(n)), dim3(256), 0, s, w, g, lr, n);
}

}  // namespace gpu
}  // namespace mcc
