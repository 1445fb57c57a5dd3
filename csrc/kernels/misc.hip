// Loss, optimizer and layout kernels.
//
//  softmax_xent : fused softmax + cross-entropy forward+backward + the
//                 reference's logged metrics, replacing the softmax in
//                 Layer_feedForw_full (cnn.c:125-143), the output error
//                 (cnn.c:285-286), Layer_getErrorTotal (cnn.c:275-282) and the
//                 argmax of the test loop (cnn.c:506-515).
//  sgd_update   : one multi-tensor pass over the flat fp32 parameter buffer
//                 (Layer_update, cnn.c:303-314, recursive over every layer).
//  pack_gather  : refresh the packed bf16/fp32 compute copies (MFMA order,
//                 transposed shadows) from the fp32 master after the update.
#include "kernels.h"
#include "mcc/ab.h"
#include "mfma.h"
#include "stats.h"

#include <algorithm>
#include <type_traits>

namespace mcc {
namespace gpu {

namespace {

__global__ void stats_to_f32_kernel(const unsigned long long* s, float* out) {
  if (threadIdx.x < 3) {
    const bool bad = s[kStatNaN] != 0 && threadIdx.x < 2;
    out[threadIdx.x] = bad ? __builtin_nanf("") : threadIdx.x == 2 ? (float)s[2] : (float)((double)s[threadIdx.x] / kStatScale);
  }
}


// Softmax-cross-entropy forward + backward, one thread per sample.  For
// N <= 16 classes (ldl % 4 == 0) the row is held in registers after 16-byte
// loads; the three statistics are reduced per workgroup in LDS and leave as
// one atomic each per workgroup.
template <typename T, int NMAX>
__global__ void __launch_bounds__(256) softmax_xent_kernel(XentParams p) {
  __shared__ float red[3][4];
  const int row = blockIdx.x * blockDim.x + threadIdx.x;
  float loss = 0.f, mse = 0.f, correct = 0.f;
  if (row < p.M) {
    const float* l = p.logits + (size_t)row * p.ldl;
    const int sample = p.labels_idx ? p.labels_idx[row] : row;
    const int label = p.labels[sample];
    float v[NMAX > 0 ? NMAX : 1];
    if constexpr (NMAX > 0) {
#pragma unroll
      for (int j = 0; j < NMAX; j += 4) {
        if (j < p.N) {
          const float4 q = *reinterpret_cast<const float4*>(l + j);
          v[j] = q.x; v[j + 1] = q.y; v[j + 2] = q.z; v[j + 3] = q.w;
        }
      }
    }
    auto at = [&](int j) { return NMAX > 0 ? v[j] : l[j]; };
    float m = at(0);
    int am = 0;
#pragma unroll
    for (int j = 1; j < (NMAX > 0 ? NMAX : 1 << 30); ++j) {
      if (j >= p.N) break;
      if (at(j) > m) { m = at(j); am = j; }  // first max wins (cnn.c:510)
    }
    float sum = 0.f;
#pragma unroll
    for (int j = 0; j < (NMAX > 0 ? NMAX : 1 << 30); ++j) {
      if (j >= p.N) break;
      sum += __expf(at(j) - m);
    }
    const float inv = 1.f / sum;
    loss = __logf(sum) - (at(label) - m);
    correct = (am == label) ? 1.f : 0.f;
    T* d = p.dlogits ? static_cast<T*>(p.dlogits) + (size_t)row * p.ldd : nullptr;
#pragma unroll
    for (int j = 0; j < (NMAX > 0 ? NMAX : 1 << 30); ++j) {
      if (j >= p.N) break;
      const float pj = __expf(at(j) - m) * inv;
      const float e = pj - (j == label ? 1.f : 0.f);
      mse += e * e;
      if (d) d[j] = from_f<T>(e * p.scale);
      if (p.probs) p.probs[(size_t)row * p.N + j] = pj;
    }
    mse /= (float)p.N;
    if (p.pred) p.pred[row] = am;
  }
  // wave reduce (64 lanes), then across the workgroup's waves in LDS
  for (int o = 32; o > 0; o >>= 1) {
    loss += __shfl_xor(loss, o);
    mse += __shfl_xor(mse, o);
    correct += __shfl_xor(correct, o);
  }
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    red[0][w] = loss;
    red[1][w] = mse;
    red[2][w] = correct;
  }
  __syncthreads();
  if (threadIdx.x < 3 && p.stats) {
    const float t = (red[threadIdx.x][0] + red[threadIdx.x][1]) + (red[threadIdx.x][2] + red[threadIdx.x][3]);
    stat_add(p.stats, threadIdx.x, t);
  }
}

// Fused classifier head (XentHeadParams): 128 samples per workgroup, four
// threads per sample.  Each computes the sample's softmax-CE (as
// softmax_xent_kernel<., 16>; statistics counted once), then, without
// writing dlogits, a quarter of the last FC layer's data gradient on the VALU
// (e x W from LDS, N <= 16 FMAs per input feature, fused act') and of the
// H^T image; the weight/bias gradient over the workgroup's 128 rows is
// [e]^T [h | 1] on MFMA (E^T and H^T staged in LDS K(=row)-contiguous, one
// 16-column tile per wave), written as this workgroup's slab.  Replaces
// softmax_xent + last-FC dgrad + split-K dW GEMM (3 launches and the dlogits
// round trip) for small heads (LeNet-5: 84 -> 10; the reference model: 200 -> 10).
constexpr int kHeadRows = 128;
constexpr int kHeadThreads = 512;
// row stride of the transposed E / H images (16-byte aligned rows)
template <typename T>
__host__ __device__ constexpr int head_ld() { return kHeadRows + (sizeof(T) == 2 ? 8 : 4); }
// LDS sized by the input width (16 * NT columns, NT = ceil((Kin + 1) / 16)):
// LeNet-5's 84 -> 10 head needs 36.6 KB, four workgroups per CU, so the
// 1024 workgroups of a 131072-row batch run in one round (a fixed 128-column
// layout took 47.6 KB: three per CU, two rounds; 33.2 -> 31.5 us,
// profiles/xent_head_lds_ab_r2.txt)
__host__ __device__ constexpr int head_nt(int Kin) { return (Kin + 1 + 15) >> 4; }
template <typename T>
__host__ __device__ constexpr int head_lds(int Kin) {
  return 16 * (16 * head_nt(Kin)) * 4 + (16 + 16 * head_nt(Kin)) * head_ld<T>() * (int)sizeof(T);
}

// T = bf16: the bf16 engine's rounding points (weights, dlogits, H through
// bf16); T = float: the fp32 engine, no rounding, the dW tile on f32 MFMA.
// FWD: the head's forward too (hp.bias != nullptr): the logits from the
// cached H chunks (each of the 4 threads of a row sums its K chunks, a quad
// shuffle completes them) -- the last FC layer's separate forward GEMM and its
// logits round trip disappear; the logits are still written when asked for.
template <typename T, bool FWD>
__global__ void __launch_bounds__(kHeadThreads) __attribute__((amdgpu_waves_per_eu(sizeof(T) == 2 ? 4 : 2))) xent_head_kernel(XentHeadParams hp) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  typedef typename Vec8<T>::type V8;
  constexpr bool kB = sizeof(T) == 2;
  constexpr int kHeadLd = head_ld<T>();
  __shared__ float red[3][kHeadThreads / 64];
  const XentParams& p = hp.x;
  const int N = p.N, Kin = hp.Kin;
  const int NT = head_nt(Kin), kw = 16 * NT;  // Ws row stride (floats) = HT rows
  float* Ws = reinterpret_cast<float*>(smem);
  T* E = reinterpret_cast<T*>(smem + 16 * kw * 4);
  T* HT = E + 16 * kHeadLd;
  const int tid = threadIdx.x;
  const int r = tid >> 2, q = tid & 3;
  // weights rounded through bf16, as the packed compute copy of the FC path
  for (int i = tid; i < 16 * kw; i += kHeadThreads) {
    const int n = i / kw, k = i - n * kw;
    const float wv = (n < N && k < Kin) ? hp.w[(size_t)n * Kin + k] : 0.f;
    Ws[i] = kB ? (float)(bf16)wv : wv;
  }
  const int row = blockIdx.x * kHeadRows + r;
  const bool live = row < p.M;
  const T* hrow = static_cast<const T*>(hp.h) + (size_t)row * hp.ldh;
  T* drow = static_cast<T*>(hp.dh) + (size_t)row * hp.ldh;
  const int K8 = (Kin + 7) & ~7;
  // this thread's 8-feature chunks q, q + 4, ... of the row (<= 8 for Kin < 256)
  V8 hc[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int k0 = 8 * q + 32 * i;
    if (live && k0 < K8) {
      hc[i] = load8(hrow + k0);
      if (k0 + 8 > Kin) {  // the row's padding columns (never written: may hold NaN)
#pragma unroll
        for (int j = 0; j < 8; ++j)
          if (k0 + j >= Kin) hc[i][j] = (T)0.f;
      }
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) hc[i][j] = (T)0.f;
    }
  }
  float lg[16];
  if constexpr (FWD) {
    __syncthreads();  // Ws
#pragma unroll
    for (int n = 0; n < 16; ++n) lg[n] = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int k0 = 8 * q + 32 * i;
      if (k0 >= K8) break;
#pragma unroll
      for (int n = 0; n < 16; ++n) {
        if (n >= N) break;
        const f32x4 w0 = *reinterpret_cast<const f32x4*>(Ws + n * kw + k0);
        const f32x4 w1 = *reinterpret_cast<const f32x4*>(Ws + n * kw + k0 + 4);
        float acc = lg[n];  // one sequential f32 fma chain per class
#pragma unroll
        for (int j = 0; j < 4; ++j) acc = __builtin_fmaf((float)hc[i][j], w0[j], acc);
#pragma unroll
        for (int j = 0; j < 4; ++j) acc = __builtin_fmaf((float)hc[i][4 + j], w1[j], acc);
        lg[n] = acc;
      }
    }
#pragma unroll
    for (int n = 0; n < 16; ++n) {
      if (n >= N) break;
      lg[n] += __shfl_xor(lg[n], 1);
      lg[n] += __shfl_xor(lg[n], 2);
      lg[n] += hp.bias[n];
    }
  }
  float loss = 0.f, mse = 0.f, correct = 0.f;
  float e[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) e[j] = 0.f;
  if (live) {
    const int sample = p.labels_idx ? p.labels_idx[row] : row;
    const int label = p.labels[sample];
    float v[16];
    if constexpr (FWD) {
#pragma unroll
      for (int j = 0; j < 16; ++j) v[j] = j < N ? lg[j] : 0.f;
      if (p.logits && q == 0) {
        float* l = const_cast<float*>(p.logits) + (size_t)row * p.ldl;  // the engine's logits buffer
#pragma unroll
        for (int j = 0; j < 16; j += 4)
          if (j < N) *reinterpret_cast<float4*>(l + j) = make_float4(v[j], v[j + 1], v[j + 2], v[j + 3]);
      }
    } else {
      const float* l = p.logits + (size_t)row * p.ldl;
#pragma unroll
      for (int j = 0; j < 16; j += 4) {
        if (j < N) {
          const float4 t4 = *reinterpret_cast<const float4*>(l + j);
          v[j] = t4.x; v[j + 1] = t4.y; v[j + 2] = t4.z; v[j + 3] = t4.w;
        } else {
          v[j] = v[j + 1] = v[j + 2] = v[j + 3] = 0.f;
        }
      }
    }
    float m = v[0];
    int am = 0;
#pragma unroll
    for (int j = 1; j < 16; ++j)
      if (j < N && v[j] > m) { m = v[j]; am = j; }  // first max wins (cnn.c:510)
    float sum = 0.f;
#pragma unroll
    for (int j = 0; j < 16; ++j)
      if (j < N) sum += __expf(v[j] - m);
    const float inv = 1.f / sum;
    float vl = 0.f;
#pragma unroll
    for (int j = 0; j < 16; ++j)
      if (j == label) vl = v[j];
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      if (j < N) {
        const float pj = __expf(v[j] - m) * inv;
        const float d = pj - (j == label ? 1.f : 0.f);
        mse += d * d;
        e[j] = kB ? (float)(bf16)(d * p.scale) : d * p.scale;  // the dlogits of the unfused path
        if (p.probs && q == 0) p.probs[(size_t)row * N + j] = pj;
      }
    }
    if (q == 0) {
      loss = __logf(sum) - (vl - m);
      correct = (am == label) ? 1.f : 0.f;
      mse /= (float)N;
      if (p.pred) p.pred[row] = am;
    } else {
      mse = 0.f;
    }
  }
  if (q == 0) {
#pragma unroll
    for (int j = 0; j < 16; ++j) E[j * kHeadLd + r] = (T)e[j];
  }
  if constexpr (!FWD) __syncthreads();  // Ws

  // data gradient of the head input + the H^T image (row Kin = ones: bias);
  // thread q of a sample owns the 8-feature chunks q, q+4, ...
#pragma unroll
  for (int ic = 0; ic < 8; ++ic) {
    const int k0 = 8 * q + 32 * ic;
    if (k0 >= K8) break;
    const V8 hv = hc[ic];
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int n = 0; n < 16; ++n) {
      if (n >= N) break;
      const f32x4 w0 = *reinterpret_cast<const f32x4*>(Ws + n * kw + k0);
      const f32x4 w1 = *reinterpret_cast<const f32x4*>(Ws + n * kw + k0 + 4);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        acc[i] += e[n] * w0[i];
        acc[4 + i] += e[n] * w1[i];
      }
    }
    V8 o;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int k = k0 + i;
      const float y = (float)hv[i];
      o[i] = k < Kin ? (T)(acc[i] * act_grad_y(hp.act, y)) : (T)0.f;
      HT[k * kHeadLd + r] = (k < Kin && live) ? hv[i] : (T)((k == Kin && live) ? 1.f : 0.f);
    }
    if (live) store8(drow + k0, o);
  }
  if (q == 0)
    for (int k = K8; k < 16 * NT; ++k) HT[k * kHeadLd + r] = (T)((k == Kin && live) ? 1.f : 0.f);
  __syncthreads();

  // weight + bias gradient of the workgroup's rows: wave w computes the
  // 16-column tiles t = w, w + 8 of C[n][k] = sum_rows E[n][row] HT[k][row]
  const int lane = tid & 63, wave = tid >> 6, r16 = lane & 15, g = lane >> 4;
  for (int t = wave; t < NT; t += kHeadThreads / 64) {
    f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < kHeadRows / 32; ++ks) {
      const int kb = ks * 32 + 8 * g;
      acc = mma(acc, load8(E + r16 * kHeadLd + kb), load8(HT + (16 * t + r16) * kHeadLd + kb));
    }
    float* slab = hp.slab + (size_t)blockIdx.x * N * hp.ldp;
    const int k = 16 * t + r16;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int n = 4 * g + i;
      if (n < N && k <= Kin) slab[n * hp.ldp + k] = acc[i];
    }
  }
  // statistics (wave reduce, then across the waves in a fixed order)
  for (int o = 32; o > 0; o >>= 1) {
    loss += __shfl_xor(loss, o);
    mse += __shfl_xor(mse, o);
    correct += __shfl_xor(correct, o);
  }
  if (lane == 0) {
    red[0][wave] = loss;
    red[1][wave] = mse;
    red[2][wave] = correct;
  }
  __syncthreads();
  if (tid < 3 && p.stats) {
    float t = 0.f;
#pragma unroll
    for (int w = 0; w < kHeadThreads / 64; ++w) t += red[tid][w];
    stat_add(p.stats, tid, t);
  }
}

// The bf16 head on the matrix cores.  The VALU head above spends its time on
// per-element work that is all GEMM-shaped: the logits (H W^T), the data
// gradient (E W, 16 FMAs per feature and thread) and the H^T image for dW
// (Kin ds_write_b16 per row).  Here every product is a 16x16x32 MFMA and the
// transposes are ds_read_b64_tr_b16 reads of row-major LDS images:
//   Hs [128][SH]  the workgroup's H rows (16-byte writes; col Kin = 1, the bias)
//   Ws [16][SH]   W in bf16 (the packed forward copy)
//   Es [128][16]  e = (softmax - onehot) * scale, bf16
// Wave w owns rows 16w..16w+15 for the forward, softmax and dgrad:
//   logits C[row][n] = sum_k Hs[row][k] Ws[n][k]        (NT/2 MFMAs, fp32 + bias)
//   softmax-CE across the 16 lanes of a C column group (class = lane & 15)
//   dH^T   C[k][row] = sum_n Ws^T[k][n] Es^T[n][row]    (NT MFMAs, K = 16 of 32 live)
//          -> act' from Hs, 8-byte stores of 4 consecutive features
// and after one barrier the workgroup's dW/db slab, C[n][k] = sum_row Es^T Hs
// (4 MFMAs per 16-column tile, tiles w, w + 8).
constexpr int kHmWaves = kHeadRows / 16;
// KCH = ceil(16 NT / 32): the 32-feature groups of an H row (ref 200 -> 7,
// LeNet-5 84 -> 3).  LDS rows hold all KCH groups (zero past column Kin), so
// the forward's K loop needs no masks; +16 bytes of pad spread b128 rows over
// the banks.
__host__ __device__ constexpr int head_kch(int Kin) { return (16 * head_nt(Kin) + 31) / 32; }
__host__ __device__ constexpr int headm_sh(int Kin) { return 32 * head_kch(Kin) + 8; }
__host__ __device__ constexpr int headm_lds(int Kin) { return (kHeadRows + 16) * headm_sh(Kin) * 2 + kHeadRows * 32; }

__device__ __forceinline__ bf16x8 head_tr8(const bf16* p0, const bf16* p1) {
  return __builtin_shufflevector(tr4(p0), tr4(p1), 0, 1, 2, 3, 4, 5, 6, 7);
}
// row_ror:n within each 16-lane row (DPP, folds into the consuming VALU op):
// four rotations 8, 4, 2, 1 leave a commutative reduction in every lane
template <int N>
__device__ __forceinline__ float ror16(float x) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x), 0x120 + N, 0xF, 0xF, false));
}
template <int N>
__device__ __forceinline__ int ror16(int x) { return __builtin_amdgcn_update_dpp(0, x, 0x120 + N, 0xF, 0xF, false); }
template <int N>
__device__ __forceinline__ void head_argmax_step(float& m, int& am) {
  const float om = ror16<N>(m);
  const int oa = ror16<N>(am);
  const bool take = (om > m) | ((om == m) & (oa < am));  // (branch-free: no exec-mask blocks)
  m = take ? om : m;
  am = take ? oa : am;
}
template <int N>
__device__ __forceinline__ float head_sum_step(float x) { return x + ror16<N>(x); }

// dead-lane store target: one 1 KB slot per resident wave (a whole dead fp32
// dH row fits; a single shared line would take every wave's dead lanes into
// one L2 channel)
constexpr int kHeadSinkSlots = 4096, kHeadSinkSlot = 256;  // floats
__device__ __attribute__((aligned(64))) float kHeadSink[kHeadSinkSlots * kHeadSinkSlot];

// Persistent: workgroup b takes the 128-row tiles b, b + grid, ... and keeps
// its dW/db partial in the MFMA accumulators across them (one slab per
// workgroup).  The next tile's H rows are loaded into registers while this
// tile computes -- one HBM latency per workgroup instead of one per tile.
// Every global load and store is unconditional (clamped rows, dead stores to
// kHeadSink), so the compiler's vmcnt bookkeeping lets the prefetch stay in
// flight across the whole tile.
template <bool FWD, int KCH>
__global__ void __launch_bounds__(kHeadThreads) __attribute__((amdgpu_waves_per_eu(4))) xent_head_mfma_kernel(XentHeadParams hp) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  __shared__ float red[3][kHmWaves];
  constexpr int SH = 32 * KCH + 8;
  const XentParams& p = hp.x;
  const int N = p.N, Kin = hp.Kin, M = p.M;
  const int K8 = (Kin + 7) & ~7;
  const int ntiles = (M + kHeadRows - 1) / kHeadRows;
  bf16* Hs = reinterpret_cast<bf16*>(smem);
  bf16* Ws = Hs + kHeadRows * SH;
  bf16* Es = Ws + 16 * SH;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, g = lane >> 4;
  const bf16x8 z8 = __builtin_bit_cast(bf16x8, f32x4{0.f, 0.f, 0.f, 0.f});
  float* const sink32 = kHeadSink + ((blockIdx.x * kHmWaves + w) & (kHeadSinkSlots - 1)) * kHeadSinkSlot;
  bf16* const sink16 = reinterpret_cast<bf16*>(sink32);

  // H rows of this wave: lane -> row lane & 15, 8-feature chunks (lane >> 4) + 4 it
  const int hr = lane & 15, hq = lane >> 4;  // (16 rows per 16-lane group: conflict-free b128 LDS writes)
  bf16x8 hc[KCH];
  int sidx = 0;  // dataset index of row lane & 15 (labels_idx), prefetched with H
  auto load_h = [&](int tile, int K8) {
    const int row = min(tile * kHeadRows + 16 * w + hr, M - 1);
    const bf16* hrow = static_cast<const bf16*>(hp.h) + (size_t)row * hp.ldh;
#pragma unroll
    for (int it = 0; it < KCH; ++it) hc[it] = load8(hrow + min(8 * (hq + 4 * it), K8 - 8));  // no branch
    if (p.labels_idx) sidx = p.labels_idx[min(tile * kHeadRows + 16 * w + (lane & 15), M - 1)];
  };
  load_h(blockIdx.x, K8);
  // W (bf16 forward copy), once per workgroup: thread -> class tid >> 5, chunk tid & 31
  {
    const int wn = tid >> 5, wc = tid & 31;
    const bf16x8 wv0 = load8(static_cast<const bf16*>(hp.wpk) + (size_t)min(wn, N - 1) * hp.ldw + min(8 * wc, K8 - 8));
    if (8 * wc < 32 * KCH) {
      bf16x8 wv = wv0;
#pragma unroll
      for (int j = 0; j < 8; ++j)
        if (wn >= N || 8 * wc + j >= Kin) wv[j] = (bf16)0.f;
      store8(Ws + wn * SH + 8 * wc, wv);
    }
  }
  float bias[4];  // classes 4g + i (the logits tile is C[class][row])
#pragma unroll
  for (int i = 0; i < 4; ++i) bias[i] = FWD ? hp.bias[min(4 * g + i, N - 1)] : 0.f;
  float loss = 0.f, mse = 0.f, correct = 0.f;
  f32x4 dwacc[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};

  for (int tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const int row0 = tile * kHeadRows + 16 * w;
    // re-materialised per tile: hoisted out of the tile loop, the per-lane
    // masks derived from these (64-bit each, ~300 SGPRs) spill
    int Kin = hp.Kin, K8 = (hp.Kin + 7) & ~7, N = p.N, NT = head_nt(hp.Kin);
    asm volatile("" : "+s"(Kin), "+s"(K8), "+s"(N), "+s"(NT));
    int lane = tid & 63;  // (and every lane-derived index: 64 hoisted k0 + j alone took 56 VGPRs)
    asm volatile("" : "+v"(lane));
    const int g = lane >> 4, r = lane & 15, q4 = r >> 2, p4 = lane & 3, hr = lane & 15, hq = lane >> 4;
    // label (and logits) of row r; this lane's classes are 4g .. 4g + 3
    const int label = (int)p.labels[p.labels_idx ? sidx : min(row0 + r, M - 1)];
    float lgv[4];
    if constexpr (!FWD) {  // (ldl >= N rounded up to 4: host check)
      const float4 l4 = *reinterpret_cast<const float4*>(p.logits + (size_t)min(row0 + r, M - 1) * p.ldl +
                                                         min(4 * g, ((N + 3) & ~3) - 4));
      lgv[0] = l4.x; lgv[1] = l4.y; lgv[2] = l4.z; lgv[3] = l4.w;
    }
    // this tile's H image (dead rows and padding columns zero, column Kin = 1)
    const bool hlive = row0 + hr < M;
#pragma unroll
    for (int it = 0; it < KCH; ++it) {
      const int k0 = 8 * (hq + 4 * it);
      bf16x8 v = (hlive && k0 < K8) ? hc[it] : z8;
      if (k0 + 8 > Kin) {  // padding columns (never written upstream: may hold NaN)
#pragma unroll
        for (int j = 0; j < 8; ++j)
          if (k0 + j >= Kin) v[j] = (bf16)((k0 + j == Kin && hlive) ? 1.f : 0.f);
      }
      store8(Hs + (16 * w + hr) * SH + k0, v);
    }
    load_h(min(tile + (int)gridDim.x, ntiles - 1), K8);  // next tile (the last tile reloads itself)
    __syncthreads();

    const int rw = row0 + r;
    const bool live = rw < M;
    if constexpr (FWD) {  // logits^T: C[class 4g + i][row r] = sum_k W[class][k] H[row][k]
      f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int c = 0; c < KCH; ++c)
        acc = mma(acc, load8(Ws + r * SH + 32 * c + 8 * g), load8(Hs + (16 * w + r) * SH + 32 * c + 8 * g));
#pragma unroll
      for (int i = 0; i < 4; ++i) lgv[i] = 4 * g + i < N ? acc[i] + bias[i] : 0.f;
      float* dst = (p.logits && live && 4 * g < N) ? const_cast<float*>(p.logits) + (size_t)rw * p.ldl + 4 * g : sink32;
      *reinterpret_cast<float4*>(dst) = make_float4(lgv[0], lgv[1], lgv[2], lgv[3]);
    }

    // softmax-CE of row r: this lane's four classes, then the four lanes
    // r, r + 16, r + 32, r + 48 of the row (permlane swaps).  log(sum) is
    // added by lane g = 0, -(v_label - m) by the lane holding the label (the
    // wave sum at the end adds them up).
    {
      float v[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) v[i] = 4 * g + i < N ? lgv[i] : -INFINITY;
      float m = v[0];
      int am = 4 * g;
#pragma unroll
      for (int i = 1; i < 4; ++i) {  // first max wins (cnn.c:510)
        const bool take = v[i] > m;
        m = take ? v[i] : m;
        am = take ? 4 * g + i : am;
      }
      argmax4lanes(m, am);
      float ex[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) ex[i] = 4 * g + i < N ? __expf(v[i] - m) : 0.f;
      const float s = sum4lanes((ex[0] + ex[1]) + (ex[2] + ex[3]));
      const float inv = __builtin_amdgcn_rcpf(s);
      float d[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) d[i] = ex[i] * inv - (4 * g + i == label ? 1.f : 0.f);  // (0 past N)
      const float d2 = sum4lanes((d[0] * d[0] + d[1] * d[1]) + (d[2] * d[2] + d[3] * d[3]));
      const int lq = label & 3;
      const float vl = lq == 0 ? v[0] : lq == 1 ? v[1] : lq == 2 ? v[2] : v[3];
      const bool first = live && g == 0;
      loss += (first ? __logf(s) : 0.f) - ((live && (label >> 2) == g) ? vl - m : 0.f);
      mse += first ? d2 * (1.f / (float)N) : 0.f;
      correct += (first && am == label) ? 1.f : 0.f;
      *((first && p.pred) ? p.pred + rw : reinterpret_cast<int32_t*>(sink32)) = am;
      if (p.probs) {  // (eval only)
#pragma unroll
        for (int i = 0; i < 4; ++i)
          *((live && 4 * g + i < N) ? p.probs + (size_t)rw * N + 4 * g + i : sink32) = ex[i] * inv;
      }
      // the unfused dlogits, bf16: row r, classes 4g .. 4g + 3 (zero past N and for dead rows)
      const float sc = live ? p.scale : 0.f;
      *reinterpret_cast<bf16x4*>(Es + (16 * w + r) * 16 + 4 * g) = cvt4(d[0] * sc, d[1] * sc, d[2] * sc, d[3] * sc);
    }

    // dH^T tile t: C[16t + 4g + i][row r] (this wave's rows; its Es rows were
    // written by this wave: LDS keeps one wave's accesses in order).  Tiles
    // before the last lie below Kin: no masks; a dead row stores to the sink.
    {
      const bf16x8 eb = g < 2 ? load8(Es + (16 * w + r) * 16 + 8 * g) : z8;  // n >= 16: zero
      const int wr = (8 * g + q4) & 15;  // g >= 2: any class row (times the zero half of eb)
      bf16* drp = row0 + r < M ? static_cast<bf16*>(hp.dh) + (size_t)(row0 + r) * hp.ldh : sink16;
      const bf16* hrw = Hs + (16 * w + r) * SH + 4 * g;
      const bf16* wa = Ws + wr * SH + 4 * p4;
      with_act(hp.act, [&](auto ak) {
        constexpr int A = decltype(ak)::v;
        auto tile_dh = [&](int t, auto last) {
          const bf16x8 a = head_tr8(wa + 16 * t, wa + 4 * SH + 16 * t);  // class rows wr, wr + 4
          const f32x4 c = mma(f32x4{0.f, 0.f, 0.f, 0.f}, a, eb);
          const int kc = 16 * t + 4 * g;
          const bf16x4 y = *reinterpret_cast<const bf16x4*>(hrw + 16 * t);
          float o[4];
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const float yv = (float)y[i];
            o[i] = A == 1 ? (yv > 0.f ? c[i] : 0.f) : A == 2 ? c[i] * (1.f - yv * yv) : c[i];
            if constexpr (decltype(last)::value) o[i] = kc + i < Kin ? o[i] : 0.f;
          }
          bf16* dst = drp + kc;
          if constexpr (decltype(last)::value) dst = kc < K8 ? dst : sink16;
          *reinterpret_cast<bf16x4*>(dst) = cvt4(o[0], o[1], o[2], o[3]);
        };
#pragma unroll 1
        for (int t = 0; t < NT - 1; ++t) tile_dh(t, std::false_type{});
        tile_dh(NT - 1, std::true_type{});
      });
    }
    __syncthreads();

    // dW/db of the tile: C[n][k] += sum over its 128 rows of Es^T Hs, tiles
    // t = w, w + 8 (NT <= 16), accumulated over the workgroup's tiles
#pragma unroll
    for (int tt = 0; tt < 2; ++tt) {
      const int t = w + kHmWaves * tt;
      if (t < NT) {
        f32x4 acc = dwacc[tt];
#pragma unroll
        for (int ks = 0; ks < kHeadRows / 32; ++ks) {
          const int rb = 32 * ks + 8 * g + q4;
          const bf16x8 a = head_tr8(Es + rb * 16 + 4 * p4, Es + (rb + 4) * 16 + 4 * p4);
          const bf16x8 b = head_tr8(Hs + rb * SH + 16 * t + 4 * p4, Hs + (rb + 4) * SH + 16 * t + 4 * p4);
          acc = mma(acc, a, b);
        }
        dwacc[tt] = acc;
      }
    }
    __syncthreads();  // Hs / Es free for the next tile
  }
  // one slab per workgroup (dw_reduce sums gridDim.x of them, not one per
  // tile: 2.5x fewer at the reference model's 1,280 tiles)
  {
    const int r = lane & 15;
#pragma unroll
    for (int tt = 0; tt < 2; ++tt) {
      const int t = w + kHmWaves * tt;
      if (t < head_nt(hp.Kin)) {
        float* slab = hp.slab + (size_t)blockIdx.x * p.N * hp.ldp;
        const int k = 16 * t + r;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int n = 4 * g + i;
          if (n < p.N && k <= hp.Kin) slab[n * hp.ldp + k] = dwacc[tt][i];
        }
      }
    }
  }
  for (int o = 32; o > 0; o >>= 1) {
    loss += __shfl_xor(loss, o);
    mse += __shfl_xor(mse, o);
    correct += __shfl_xor(correct, o);
  }
  if (lane == 0) {
    red[0][w] = loss;
    red[1][w] = mse;
    red[2][w] = correct;
  }
  __syncthreads();
  if (tid < 3 && p.stats) {
    float t = 0.f;
#pragma unroll
    for (int v = 0; v < kHmWaves; ++v) t += red[tid][v];
    stat_add(p.stats, tid, t);
  }
}

// The fp32 head on the f32 matrix cores (xent_head_mfma32_kernel): the same
// persistent structure as the bf16 kernel above, no rounding points.  fp32 has
// no transposing LDS read, so the operands that need a transpose use the
// 16x16x4 instruction's own layout (A[r][g], B[g][r]: one value per lane):
//   logits^T  C[class][row]  f32x8 fragments of W and H rows (8 MFMAs per 32 k)
//   dH^T      C[k][row]      A = W^T from a staged [k][16] copy whose columns
//                            are stored in (g, kk) order, so a lane's four
//                            K-steps are one 16-byte read; B = E^T, 4 MFMAs
//   dW, db    C[n][k]        A = E^T, B = H, one ds_read_b32 each per MFMA
// LDS: H [128][32 KCH + 4] fp32 -- KCH <= 7 (the reference model's 200 -> 10
// head: 153 KB, one workgroup per CU; LeNet-5's 84 -> 10: 71 KB, two).
__host__ __device__ constexpr int head32_sh(int Kin) { return 32 * head_kch(Kin) + 4; }
__host__ __device__ constexpr int head32_lds(int Kin) {
  return ((kHeadRows + 16) * head32_sh(Kin) + 16 * head_nt(Kin) * 16 + kHeadRows * 16) * 4;
}

template <bool FWD, int KCH>
__global__ void __launch_bounds__(kHeadThreads) __attribute__((amdgpu_waves_per_eu(KCH <= 4 ? 4 : 2)))
xent_head_mfma32_kernel(XentHeadParams hp) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  __shared__ float red[3][kHmWaves];
  constexpr int SH = 32 * KCH + 4;
  const XentParams& p = hp.x;
  const int N = p.N, Kin = hp.Kin, M = p.M, NT0 = head_nt(Kin);
  const int ntiles = (M + kHeadRows - 1) / kHeadRows;
  float* Hs = reinterpret_cast<float*>(smem);
  float* Ws = Hs + kHeadRows * SH;  // [16][SH]  W rows
  float* WT = Ws + 16 * SH;         // [16 NT][16] W^T, column (g, kk) = class 4kk + g
  float* Es = WT + 16 * NT0 * 16;   // [128][16]
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, g = lane >> 4;
  const f32x4 z4 = f32x4{0.f, 0.f, 0.f, 0.f};
  float* const sink32 = kHeadSink + ((blockIdx.x * kHmWaves + w) & (kHeadSinkSlots - 1)) * kHeadSinkSlot;

  // H rows of this wave: lane -> row lane & 15, 8-feature chunks (lane >> 4) + 4 it
  const int hr = lane & 15, hq = lane >> 4;
  const int K8 = (Kin + 7) & ~7;
  f32x4 hc[KCH][2];
  int sidx = 0;
  auto load_h = [&](int tile, int K8) {
    const int row = min(tile * kHeadRows + 16 * w + hr, M - 1);
    const float* hrow = static_cast<const float*>(hp.h) + (size_t)row * hp.ldh;
#pragma unroll
    for (int it = 0; it < KCH; ++it) {
      const float* q = hrow + min(8 * (hq + 4 * it), K8 - 8);
      hc[it][0] = *reinterpret_cast<const f32x4*>(q);
      hc[it][1] = *reinterpret_cast<const f32x4*>(q + 4);
    }
    if (p.labels_idx) sidx = p.labels_idx[min(tile * kHeadRows + 16 * w + (lane & 15), M - 1)];
  };
  load_h(blockIdx.x, K8);
  // W (fp32 master [N][Kin]) once per workgroup: rows into Ws, the permuted
  // transpose into WT (zero past N / Kin)
  for (int i = tid; i < 16 * 32 * KCH; i += kHeadThreads) {
    const int n = i / (32 * KCH), k = i - n * (32 * KCH);
    const float v = (n < N && k < Kin) ? hp.w[(size_t)n * Kin + k] : 0.f;
    Ws[n * SH + k] = v;
    if (k < 16 * NT0) WT[k * 16 + (n & 3) * 4 + (n >> 2)] = v;
  }
  float bias[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) bias[i] = FWD ? hp.bias[min(4 * g + i, N - 1)] : 0.f;
  float loss = 0.f, mse = 0.f, correct = 0.f;
  f32x4 dwacc[2] = {z4, z4};

  for (int tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const int row0 = tile * kHeadRows + 16 * w;
    int Kin = hp.Kin, K8 = (hp.Kin + 7) & ~7, N = p.N, NT = head_nt(hp.Kin);
    asm volatile("" : "+s"(Kin), "+s"(K8), "+s"(N), "+s"(NT));  // (see xent_head_mfma_kernel)
    int lane = tid & 63;
    asm volatile("" : "+v"(lane));
    const int g = lane >> 4, r = lane & 15, hr = lane & 15, hq = lane >> 4;
    const int label = (int)p.labels[p.labels_idx ? sidx : min(row0 + r, M - 1)];
    float lgv[4];
    if constexpr (!FWD) {
      const float4 l4 = *reinterpret_cast<const float4*>(p.logits + (size_t)min(row0 + r, M - 1) * p.ldl +
                                                         min(4 * g, ((N + 3) & ~3) - 4));
      lgv[0] = l4.x; lgv[1] = l4.y; lgv[2] = l4.z; lgv[3] = l4.w;
    }
    // this tile's H image (dead rows and padding columns zero, column Kin = 1)
    const bool hlive = row0 + hr < M;
#pragma unroll
    for (int it = 0; it < KCH; ++it) {
      const int k0 = 8 * (hq + 4 * it);
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        f32x4 v = (hlive && k0 < K8) ? hc[it][h] : z4;
        const int kb = k0 + 4 * h;
        if (kb + 4 > Kin) {  // padding columns (never written upstream: may hold NaN)
          v.x = kb + 0 < Kin ? v.x : (kb + 0 == Kin && hlive ? 1.f : 0.f);
          v.y = kb + 1 < Kin ? v.y : (kb + 1 == Kin && hlive ? 1.f : 0.f);
          v.z = kb + 2 < Kin ? v.z : (kb + 2 == Kin && hlive ? 1.f : 0.f);
          v.w = kb + 3 < Kin ? v.w : (kb + 3 == Kin && hlive ? 1.f : 0.f);
        }
        *reinterpret_cast<f32x4*>(Hs + (16 * w + hr) * SH + kb) = v;
      }
    }
    load_h(min(tile + (int)gridDim.x, ntiles - 1), K8);  // next tile (the last tile reloads itself)
    __syncthreads();

    const int rw = row0 + r;
    const bool live = rw < M;
    if constexpr (FWD) {  // logits^T: C[class 4g + i][row r]
      f32x4 acc = z4;
#pragma unroll
      for (int c = 0; c < KCH; ++c)
        acc = mma(acc, load8(Ws + r * SH + 32 * c + 8 * g), load8(Hs + (16 * w + r) * SH + 32 * c + 8 * g));
#pragma unroll
      for (int i = 0; i < 4; ++i) lgv[i] = 4 * g + i < N ? acc[i] + bias[i] : 0.f;
      float* dst = (p.logits && live && 4 * g < N) ? const_cast<float*>(p.logits) + (size_t)rw * p.ldl + 4 * g : sink32;
      *reinterpret_cast<float4*>(dst) = make_float4(lgv[0], lgv[1], lgv[2], lgv[3]);
    }
    {  // softmax-CE of row r (as the bf16 kernel; e stays fp32)
      float v[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) v[i] = 4 * g + i < N ? lgv[i] : -INFINITY;
      float m = v[0];
      int am = 4 * g;
#pragma unroll
      for (int i = 1; i < 4; ++i) {  // first max wins (cnn.c:510)
        const bool take = v[i] > m;
        m = take ? v[i] : m;
        am = take ? 4 * g + i : am;
      }
      argmax4lanes(m, am);
      float ex[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) ex[i] = 4 * g + i < N ? __expf(v[i] - m) : 0.f;
      const float s = sum4lanes((ex[0] + ex[1]) + (ex[2] + ex[3]));
      const float inv = 1.f / s;
      float d[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) d[i] = ex[i] * inv - (4 * g + i == label ? 1.f : 0.f);
      const float d2 = sum4lanes((d[0] * d[0] + d[1] * d[1]) + (d[2] * d[2] + d[3] * d[3]));
      const int lq = label & 3;
      const float vl = lq == 0 ? v[0] : lq == 1 ? v[1] : lq == 2 ? v[2] : v[3];
      const bool first = live && g == 0;
      loss += (first ? __logf(s) : 0.f) - ((live && (label >> 2) == g) ? vl - m : 0.f);
      mse += first ? d2 / (float)N : 0.f;
      correct += (first && am == label) ? 1.f : 0.f;
      *((first && p.pred) ? p.pred + rw : reinterpret_cast<int32_t*>(sink32)) = am;
      if (p.probs) {  // (eval only)
#pragma unroll
        for (int i = 0; i < 4; ++i)
          *((live && 4 * g + i < N) ? p.probs + (size_t)rw * N + 4 * g + i : sink32) = ex[i] * inv;
      }
      const float sc = live ? p.scale : 0.f;
      *reinterpret_cast<f32x4*>(Es + (16 * w + r) * 16 + 4 * g) = f32x4{d[0] * sc, d[1] * sc, d[2] * sc, d[3] * sc};
    }

    {  // dH^T tile t: C[16t + 4g + i][row r], K = 16 classes as four 16x16x4 steps
      float eb[4];  // B[g][r] of step kk = E^T[class 4kk + g][row r]
#pragma unroll
      for (int kk = 0; kk < 4; ++kk) eb[kk] = Es[(16 * w + r) * 16 + 4 * kk + g];
      float* drp = row0 + r < M ? static_cast<float*>(hp.dh) + (size_t)(row0 + r) * hp.ldh : sink32;
      const float* hrw = Hs + (16 * w + r) * SH + 4 * g;
      const float* wtl = WT + r * 16 + 4 * g;
      with_act(hp.act, [&](auto ak) {
        constexpr int A = decltype(ak)::v;
        auto tile_dh = [&](int t, auto last) {
          const f32x4 a = *reinterpret_cast<const f32x4*>(wtl + 16 * 16 * t);  // A[r][g] of steps kk = 0..3
          f32x4 c = z4;
#pragma unroll
          for (int kk = 0; kk < 4; ++kk) c = __builtin_amdgcn_mfma_f32_16x16x4f32(a[kk], eb[kk], c, 0, 0, 0);
          const int kc = 16 * t + 4 * g;
          const f32x4 y = *reinterpret_cast<const f32x4*>(hrw + 16 * t);
          f32x4 o;
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            o[i] = A == 1 ? (y[i] > 0.f ? c[i] : 0.f) : A == 2 ? c[i] * (1.f - y[i] * y[i]) : c[i];
            if constexpr (decltype(last)::value) o[i] = kc + i < Kin ? o[i] : 0.f;
          }
          float* dst = drp + kc;
          if constexpr (decltype(last)::value) dst = kc < K8 ? dst : sink32;
          *reinterpret_cast<f32x4*>(dst) = o;
        };
#pragma unroll 1
        for (int t = 0; t < NT - 1; ++t) tile_dh(t, std::false_type{});
        tile_dh(NT - 1, std::true_type{});
      });
    }
    __syncthreads();

    // dW/db: C[n = 4g + i][k = 16t + r] += sum over the 128 rows, four rows per
    // 16x16x4 step; tiles t = w, w + 8 (NT <= 14 here)
#pragma unroll
    for (int tt = 0; tt < 2; ++tt) {
      const int t = w + kHmWaves * tt;
      if (t < NT) {
        f32x4 acc = dwacc[tt];
#pragma unroll 8
        for (int kk = 0; kk < kHeadRows / 4; ++kk) {
          const float a = Es[(4 * kk + g) * 16 + r];
          const float b = Hs[(4 * kk + g) * SH + 16 * t + r];
          acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc, 0, 0, 0);
        }
        dwacc[tt] = acc;
      }
    }
    __syncthreads();  // Hs / Es free for the next tile
  }
  {
    const int r = lane & 15;
#pragma unroll
    for (int tt = 0; tt < 2; ++tt) {
      const int t = w + kHmWaves * tt;
      if (t < head_nt(hp.Kin)) {
        float* slab = hp.slab + (size_t)blockIdx.x * p.N * hp.ldp;
        const int k = 16 * t + r;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int n = 4 * g + i;
          if (n < p.N && k <= hp.Kin) slab[n * hp.ldp + k] = dwacc[tt][i];
        }
      }
    }
  }
  for (int o = 32; o > 0; o >>= 1) {
    loss += __shfl_xor(loss, o);
    mse += __shfl_xor(mse, o);
    correct += __shfl_xor(correct, o);
  }
  if (lane == 0) {
    red[0][w] = loss;
    red[1][w] = mse;
    red[2][w] = correct;
  }
  __syncthreads();
  if (tid < 3 && p.stats) {
    float t = 0.f;
#pragma unroll
    for (int v = 0; v < kHmWaves; ++v) t += red[tid][v];
    stat_add(p.stats, tid, t);
  }
}

// Wide class counts (ImageNet-style heads): one wave per row, lanes stride
// over the classes, shuffle reductions; same outputs and tie rule as above.
template <typename T>
__global__ void __launch_bounds__(256) softmax_xent_wide_kernel(XentParams p) {
  __shared__ float red[3][4];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int row = blockIdx.x * 4 + w;
  float loss = 0.f, mse = 0.f, correct = 0.f;
  if (row < p.M) {
    const float* l = p.logits + (size_t)row * p.ldl;
    const int sample = p.labels_idx ? p.labels_idx[row] : row;
    const int label = p.labels[sample];
    float m = -INFINITY;
    int am = 0x7fffffff;
    for (int j = lane; j < p.N; j += 64) {
      const float x = l[j];
      if (x > m) { m = x; am = j; }
    }
    for (int o = 32; o > 0; o >>= 1) {  // max, smallest index among equal maxima (first max wins)
      const float om = __shfl_xor(m, o);
      const int oa = __shfl_xor(am, o);
      if (om > m || (om == m && oa < am)) { m = om; am = oa; }
    }
    float sum = 0.f;
    for (int j = lane; j < p.N; j += 64) sum += __expf(l[j] - m);
    for (int o = 32; o > 0; o >>= 1) sum += __shfl_xor(sum, o);
    const float inv = 1.f / sum;
    T* d = p.dlogits ? static_cast<T*>(p.dlogits) + (size_t)row * p.ldd : nullptr;
    for (int j = lane; j < p.N; j += 64) {
      const float pj = __expf(l[j] - m) * inv;
      const float e = pj - (j == label ? 1.f : 0.f);
      mse += e * e;
      if (d) d[j] = from_f<T>(e * p.scale);
      if (p.probs) p.probs[(size_t)row * p.N + j] = pj;
    }
    for (int o = 32; o > 0; o >>= 1) mse += __shfl_xor(mse, o);
    mse /= (float)p.N;
    if (lane == 0) {
      loss = __logf(sum) - (l[label] - m);
      correct = am == label ? 1.f : 0.f;
      if (p.pred) p.pred[row] = am;
    } else {
      mse = 0.f;
    }
  }
  for (int o = 32; o > 0; o >>= 1) {
    loss += __shfl_xor(loss, o);
    mse += __shfl_xor(mse, o);
    correct += __shfl_xor(correct, o);
  }
  if (lane == 0) {
    red[0][w] = loss;
    red[1][w] = mse;
    red[2][w] = correct;
  }
  __syncthreads();
  if (threadIdx.x < 3 && p.stats) {
    const float t = (red[threadIdx.x][0] + red[threadIdx.x][1]) + (red[threadIdx.x][2] + red[threadIdx.x][3]);
    stat_add(p.stats, threadIdx.x, t);
  }
}

__global__ void sgd_kernel(float* __restrict__ w, const float* __restrict__ g, float* __restrict__ v, int64_t n,
                           float lr, float mu, float wd) {
  const int64_t n4 = n >> 2;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    f32x4 wv = reinterpret_cast<f32x4*>(w)[i];
    f32x4 gv = reinterpret_cast<const f32x4*>(g)[i];
    if (wd != 0.f) gv += wd * wv;
    if (v) {
      f32x4 vv = reinterpret_cast<f32x4*>(v)[i];
      vv = mu * vv + gv;
      reinterpret_cast<f32x4*>(v)[i] = vv;
      gv = vv;
    }
    reinterpret_cast<f32x4*>(w)[i] = wv - lr * gv;
  }
  for (int64_t i = (n4 << 2) + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    float gi = g[i] + wd * w[i];
    if (v) { v[i] = mu * v[i] + gi; gi = v[i]; }
    w[i] -= lr * gi;
  }
}

template <typename T>
__global__ void pack_kernel(T* __restrict__ dst, const float* __restrict__ src, const int32_t* __restrict__ idx,
                            int64_t n) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const int32_t j = idx[i];
    dst[i] = j >= 0 ? from_f<T>(src[j]) : T(0);
  }
}

// q = n / d for n, d < 2^32 via m = ceil(2^64 / d) (d >= 2; d == 1: m = 0 = identity)
__device__ __forceinline__ uint32_t fdiv(uint32_t n, uint64_t m) {
  return m ? (uint32_t)__umul64hi((uint64_t)n, m) : n;
}

// Fused SGD (+ momentum, weight decay) and packed-copy refresh: one pass over
// the fp32 master parameters writes the updated master, the momentum and
// every packed compute copy (analytic per-stage maps, no index table).
//
// Conv stages of >= kPackTileMin weights run as (32 n x 32 c x KK) tiles:
// the master reads/writes are contiguous (c, tap) runs of each n, the tile is
// kept in LDS, and each copy is written with its unit-stride index (c for
// the forward layouts, n for the data-gradient ones) across the lanes -- a
// coalesced transpose instead of per-element scatters.  Everything else
// (FC copies are row-major like the master, biases, tiny convs) runs
// elementwise in the remaining workgroups.
constexpr int kPackTN = 32, kPackTC = 32, kPackTCp = kPackTC + 2;
constexpr int64_t kPackTileMin = 65536;
constexpr int kPackMaxKK = 9;  // 3x3 and smaller (LDS: 9 x 32 x 34 elements)

template <typename T, bool UPDATE>
__device__ __forceinline__ float sgd_one(const SgdPackParams& p, int64_t i) {
  float w = p.params[i];
  if (UPDATE) {
    float gi = p.grads[i];
    if (p.wd != 0.f) gi += p.wd * w;
    if (p.mom) {
      const float v = p.mu * p.mom[i] + gi;
      p.mom[i] = v;
      gi = v;
    }
    w = w - p.lr * gi;
    p.params[i] = w;
  }
  return w;
}

template <typename T, bool UPDATE>
__global__ void __launch_bounds__(256) sgd_pack_kernel(SgdPackParams p) {
  T* __restrict__ dst = static_cast<T*>(p.packed);
  if ((int)blockIdx.x < p.ntiles) {
    __shared__ T tile[kPackMaxKK * kPackTN * kPackTCp];
    // the tiled stages' tile ranges are contiguous and increasing
    int s = 0;
    for (; s < p.nstages; ++s) {
      const PackStage& q = p.st[s];
      if (q.tile0 < 0) continue;
      const int Nq = (int)(q.nw / ((int64_t)q.inC * q.KS * q.KS));
      if ((int)blockIdx.x < q.tile0 + cdiv(Nq, kPackTN) * cdiv(q.inC, kPackTC)) break;
    }
    const PackStage& st = p.st[s];
    const int KK = st.KS * st.KS, C = st.inC;
    const int N = (int)(st.nw / ((int64_t)C * KK));
    const int tcs = (C + kPackTC - 1) / kPackTC;
    const int t = (int)blockIdx.x - st.tile0, n0 = (t / tcs) * kPackTN, c0 = (t % tcs) * kPackTC;
    const int nn = min(kPackTN, N - n0), cc = min(kPackTC, C - c0);
    // phase 1: master update, (c, tap) runs of each n are contiguous
    const int run = cc * KK;
    for (int e = threadIdx.x; e < nn * run; e += blockDim.x) {
      const int n = e / run, r = e - n * run;
      const int c = r / KK, k = r - c * KK;
      const int64_t i = st.w_off + ((int64_t)(n0 + n) * C + c0) * KK + r;
      tile[(k * kPackTN + n) * kPackTCp + c] = from_f<T>(sgd_one<T, UPDATE>(p, i));
    }
    __syncthreads();
    // phase 2: each copy along its unit-stride index
    for (int m = 0; m < st.nmaps; ++m) {
      const PackMap& mp = st.map[m];
      const bool c_fast = mp.sc == 1;
      const int inner = c_fast ? cc : nn, outer = c_fast ? nn : cc;
      for (int e = threadIdx.x; e < KK * outer * inner; e += blockDim.x) {
        const int k = e / (outer * inner), r = e - k * (outer * inner);
        const int o = r / inner, q = r - o * inner;
        const int n = c_fast ? o : q, c = c_fast ? q : o;
        const int kh = k / st.KS, kw = k - kh * st.KS;
        const int h = mp.flip ? st.KS - 1 - kh : kh, x = mp.flip ? st.KS - 1 - kw : kw;
        dst[mp.base + (int64_t)(n0 + n) * mp.sn + (int64_t)(c0 + c) * mp.sc + (int64_t)h * mp.skh +
            (int64_t)x * mp.skw] = tile[(k * kPackTN + n) * kPackTCp + c];
      }
    }
    return;
  }
  // elementwise part: four consecutive parameters per thread (16-byte master
  // and momentum accesses); an FC row segment's copy leaves as one 8/16-byte
  // store, other packed elements one by one.  A group that straddles a
  // region boundary (bias | weights | tiled weights) goes element by element.
  auto pack_one = [&](const PackStage& st, int64_t i, float w) {
    const uint32_t j = (uint32_t)(i - st.w_off);
    const uint32_t ckk = (uint32_t)(st.inC * st.KS * st.KS), kk = (uint32_t)(st.KS * st.KS);
    const uint32_t n = fdiv(j, st.m_ckk), r = j - n * ckk;
    const uint32_t c = fdiv(r, st.m_kk), r2 = r - c * kk;
    const uint32_t kh = fdiv(r2, st.m_ks), kw = r2 - kh * (uint32_t)st.KS;
    const T v = from_f<T>(w);
    for (int m = 0; m < st.nmaps; ++m) {
      const PackMap& mp = st.map[m];
      const int h = mp.flip ? st.KS - 1 - (int)kh : (int)kh, x = mp.flip ? st.KS - 1 - (int)kw : (int)kw;
      dst[mp.base + (int64_t)n * mp.sn + (int64_t)c * mp.sc + (int64_t)h * mp.skh + (int64_t)x * mp.skw] = v;
    }
  };
  // region of parameter i: 2*stage (the gap before it: biases) or 2*stage + 1 (its weights)
  auto region = [&](int64_t i, int& ss) {
    while (ss < p.nstages && i >= p.st[ss].w_off + p.st[ss].nw) ++ss;
    return 2 * ss + ((ss < p.nstages && i >= p.st[ss].w_off) ? 1 : 0);
  };
  const int64_t stride = (int64_t)(gridDim.x - p.ntiles) * blockDim.x * 4;
  int s = 0;  // monotone per thread: i only grows
  const int64_t lo4 = p.lo & ~int64_t(3);  // the groups stay 16-byte aligned
  for (int64_t i0 = lo4 + ((int64_t)(blockIdx.x - p.ntiles) * blockDim.x + threadIdx.x) * 4; i0 < p.n; i0 += stride) {
    int s3 = s;
    const int r0 = region(i0, s), r3 = region(min(i0 + 3, p.n - 1), s3);
    if (r0 == r3 && (r0 & 1) && p.st[s].tile0 >= 0 && i0 >= p.lo) continue;  // done by the tiles
    if (r0 != r3 || i0 + 3 >= p.n || i0 < p.lo) {
      for (int e = 0; e < 4 && i0 + e < p.n; ++e) {
        if (i0 + e < p.lo) continue;  // the group straddles the range start
        int se = s;
        const int re = region(i0 + e, se);
        if ((re & 1) && p.st[se].tile0 >= 0) continue;
        const float w = sgd_one<T, UPDATE>(p, i0 + e);
        if (re & 1) pack_one(p.st[se], i0 + e, w);
      }
      continue;
    }
    float w[4];
    {
      const float4 w4 = *reinterpret_cast<const float4*>(p.params + i0);
      w[0] = w4.x; w[1] = w4.y; w[2] = w4.z; w[3] = w4.w;
    }
    if (UPDATE) {
      const float4 g4 = *reinterpret_cast<const float4*>(p.grads + i0);
      float g[4] = {g4.x, g4.y, g4.z, g4.w};
      if (p.wd != 0.f) {
#pragma unroll
        for (int e = 0; e < 4; ++e) g[e] += p.wd * w[e];
      }
      if (p.mom) {
        const float4 v4 = *reinterpret_cast<const float4*>(p.mom + i0);
        const float v[4] = {p.mu * v4.x + g[0], p.mu * v4.y + g[1], p.mu * v4.z + g[2], p.mu * v4.w + g[3]};
        *reinterpret_cast<float4*>(p.mom + i0) = make_float4(v[0], v[1], v[2], v[3]);
#pragma unroll
        for (int e = 0; e < 4; ++e) g[e] = v[e];
      }
#pragma unroll
      for (int e = 0; e < 4; ++e) w[e] -= p.lr * g[e];
      *reinterpret_cast<float4*>(p.params + i0) = make_float4(w[0], w[1], w[2], w[3]);
    }
    if (!(r0 & 1)) continue;  // biases: no packed copy
    const PackStage& st = p.st[s];
    if (st.KS == 1 && st.nmaps == 1 && st.map[0].sc == 1) {
      const int64_t j0 = i0 - st.w_off;
      const uint32_t n = fdiv((uint32_t)j0, st.m_ckk), c = (uint32_t)j0 - n * (uint32_t)st.inC;
      const int64_t d = st.map[0].base + (int64_t)n * st.map[0].sn + c;
      if (c + 3 < (uint32_t)st.inC && (d & 3) == 0) {  // one aligned row segment
        if constexpr (sizeof(T) == 2) {
          const bf16x4 v = {(bf16)w[0], (bf16)w[1], (bf16)w[2], (bf16)w[3]};
          *reinterpret_cast<bf16x4*>(dst + d) = v;
        } else {
          *reinterpret_cast<float4*>(dst + d) = make_float4(w[0], w[1], w[2], w[3]);
        }
        continue;
      }
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) pack_one(st, i0 + e, w[e]);
  }
}

__global__ void fill_kernel(float* dst, float v, int64_t n) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) dst[i] = v;
}

template <typename T>
__global__ void cast_kernel(T* dst, const float* src, int64_t n) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) dst[i] = from_f<T>(src[i]);
}

template <typename T>
__global__ void to_f32_kernel(float* dst, const T* src, int64_t n) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) dst[i] = to_f(src[i]);
}

__device__ __forceinline__ uint64_t mix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

__global__ void sample_kernel(int32_t* idx, int B, int64_t lo, int64_t span, uint64_t seed, const uint64_t* step) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  const uint64_t h = mix64(mix64(seed ^ (*step * 0xD1B54A32D192ED03ull)) + (uint64_t)b);
  idx[b] = (int32_t)(lo + (int64_t)(h % (uint64_t)span));
}

__global__ void advance_kernel(uint64_t* step) { *step += 1; }

// sample_kernel + advance_kernel as one launch: step[0] is the counter,
// step[1] a ticket.  Every workgroup reads the counter before it takes a
// ticket; the workgroup that takes the last one advances the counter and
// resets the ticket, so no workgroup can see the advanced value.  (Grid-
// stride over the batch.)
__global__ void __launch_bounds__(256) sample_advance_kernel(int32_t* idx, int B, int64_t lo, int64_t span,
                                                             uint64_t seed, uint64_t* step) {
  __shared__ uint64_t c;
  if (threadIdx.x == 0) c = __hip_atomic_load(step, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();
  const uint64_t cv = c;
  const uint64_t hs = mix64(seed ^ (cv * 0xD1B54A32D192ED03ull));
  for (int b = blockIdx.x * blockDim.x + threadIdx.x; b < B; b += gridDim.x * blockDim.x)
    idx[b] = (int32_t)(lo + (int64_t)(mix64(hs + (uint64_t)b) % (uint64_t)span));
  if (threadIdx.x == 0) {
    const uint64_t t = __hip_atomic_fetch_add(step + 1, 1ull, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    if (t == gridDim.x - 1) {
      __hip_atomic_store(step + 1, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(step, cv + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// Contention probe (tools/probes/cu_contention.py): `nwg` workgroups of 256
// threads that each hold `lds` bytes of LDS and spin for `ticks` wall-clock
// ticks -- a stand-in for an RCCL kernel that occupies CUs while it waits for
// its peers.  Stores only to LDS (the sink is never written in practice).
__global__ void cu_hold_kernel(uint64_t ticks, float* sink) {
  extern __shared__ float hold_lds[];
  const uint64_t t0 = wall_clock64();
  float a = (float)threadIdx.x;
  while (wall_clock64() - t0 < ticks) {
    hold_lds[threadIdx.x] = a;
    a = a * 0.5f + hold_lds[(threadIdx.x + 64) & 255];
  }
  if (a == -1.f) sink[threadIdx.x] = a;
}

// Sequential global windows: at step t the global batch is dataset positions
// t*stride .. t*stride + stride - 1 (mod n), and this rank takes the slice
// starting at `offset` -- world ranks together draw exactly the batch one
// process of the whole global batch would (cnn_dist --sampler seq).
__global__ void seq_sample_kernel(int32_t* idx, int B, int64_t offset, int64_t stride, int64_t n, const uint64_t* step) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  idx[b] = (int32_t)(((int64_t)(*step % (uint64_t)n) * stride + offset + b) % n);
}

__global__ void iota_kernel(int32_t* idx, int B, int64_t start) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b < B) idx[b] = (int32_t)(start + b);
}

inline unsigned grid_for(int64_t n, int per_thread = 1) {
  int64_t b = (n / per_thread + 255) / 256;
  if (b < 1) b = 1;
  if (b > 4096) b = 4096;
  return (unsigned)b;
}

}  // namespace

bool xent_head_supported(int N, int Kin, int ldh) {
  // Kin < 256: at most 16 dW column tiles (two per wave); the reference
  // model's 200 -> 10 head takes 74 KB of LDS, two workgroups per CU
  return N >= 1 && N <= 16 && Kin >= 1 && Kin < 256 && ldh % 8 == 0 && ldh >= Kin;
}

int xent_head_slabs(int M) { return cdiv(M, kHeadRows); }

// workgroups of a persistent head kernel resident at once (occupancy at its
// LDS size x CUs; cached per kernel and size)
static int head_resident(const void* fn, int lds) {
  static const void* c_fn[4] = {};
  static int c_lds[4] = {}, c_fit[4] = {};
  for (int i = 0; i < 4; ++i)
    if (c_fn[i] == fn && c_lds[i] == lds) return c_fit[i];
  int per_cu = 0, dev = 0, cus = 0;
  MCC_CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, kHeadThreads, lds) == hipSuccess &&
                hipGetDevice(&dev) == hipSuccess &&
                hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess,
            "xent_head: occupancy query failed");
  const int fit = std::max(1, per_cu) * std::max(1, cus);
  static int next = 0;
  c_fn[next] = fn; c_lds[next] = lds; c_fit[next] = fit;
  next = (next + 1) & 3;
  return fit;
}

int xent_head(DType t, const XentHeadParams& p, hipStream_t s) {
  MCC_CHECK(p.x.M > 0 && xent_head_supported(p.x.N, p.Kin, p.ldh), "xent_head: needs N <= 16, Kin < 256, ldh % 8 == 0");
  MCC_CHECK((p.bias && !p.x.logits) ||
                (p.x.ldl % 4 == 0 && (reinterpret_cast<uintptr_t>(p.x.logits) & 15) == 0 && p.x.ldl >= ((p.x.N + 3) & ~3)),
            "xent_head: logits rows must be 16-byte aligned");
  MCC_CHECK(p.h && p.dh && p.w && p.slab && p.ldp >= p.Kin + 1 && (reinterpret_cast<uintptr_t>(p.h) & 15) == 0 &&
                (reinterpret_cast<uintptr_t>(p.dh) & 15) == 0,
            "xent_head: bad buffers");
  const dim3 grid((unsigned)xent_head_slabs(p.x.M)), block(kHeadThreads);
  if (t == DType::BF16 && p.wpk && !ab_flag("head_valu")) {  // (returns from inside)
    MCC_CHECK(p.ldw % 8 == 0 && p.ldw >= p.Kin && (reinterpret_cast<uintptr_t>(p.wpk) & 15) == 0,
              "xent_head: packed weights need 16-byte rows");
    // persistent: as many workgroups as fit at once (A/B: MCC_AB=head_tile1, one tile each)
    const int lds = headm_lds(p.Kin), kch = head_kch(p.Kin);
    const int fit = head_resident(reinterpret_cast<const void*>(xent_head_mfma_kernel<true, 8>), lds);
    const dim3 pg(ab_flag("head_tile1") ? grid.x : std::min(grid.x, (unsigned)fit));
    auto go = [&](auto kc) {
      constexpr int KC = decltype(kc)::value;
      if (p.bias) hipLaunchKernelGGL((xent_head_mfma_kernel<true, KC>), pg, block, lds, s, p);
      else hipLaunchKernelGGL((xent_head_mfma_kernel<false, KC>), pg, block, lds, s, p);
    };
    switch (kch) {
      case 1: go(std::integral_constant<int, 1>{}); break;
      case 2: go(std::integral_constant<int, 2>{}); break;
      case 3: go(std::integral_constant<int, 3>{}); break;
      case 4: go(std::integral_constant<int, 4>{}); break;
      case 5: go(std::integral_constant<int, 5>{}); break;
      case 6: go(std::integral_constant<int, 6>{}); break;
      case 7: go(std::integral_constant<int, 7>{}); break;
      default: go(std::integral_constant<int, 8>{}); break;
    }
    return (int)pg.x;
  }
  if (t == DType::F32 && head_kch(p.Kin) <= 7 && !ab_flag("head32_valu")) {
    const int lds = head32_lds(p.Kin);
    const int fit = head_resident(reinterpret_cast<const void*>(xent_head_mfma32_kernel<true, 7>), lds);
    const dim3 pg(ab_flag("head_tile1") ? grid.x : std::min(grid.x, (unsigned)fit));
    auto go = [&](auto kc) {
      constexpr int KC = decltype(kc)::value;
      if (p.bias) hipLaunchKernelGGL((xent_head_mfma32_kernel<true, KC>), pg, block, lds, s, p);
      else hipLaunchKernelGGL((xent_head_mfma32_kernel<false, KC>), pg, block, lds, s, p);
    };
    switch (head_kch(p.Kin)) {
      case 1: go(std::integral_constant<int, 1>{}); break;
      case 2: go(std::integral_constant<int, 2>{}); break;
      case 3: go(std::integral_constant<int, 3>{}); break;
      case 4: go(std::integral_constant<int, 4>{}); break;
      case 5: go(std::integral_constant<int, 5>{}); break;
      case 6: go(std::integral_constant<int, 6>{}); break;
      default: go(std::integral_constant<int, 7>{}); break;
    }
    return (int)pg.x;
  }
  if (t == DType::BF16) {
    if (p.bias) hipLaunchKernelGGL((xent_head_kernel<bf16, true>), grid, block, head_lds<bf16>(p.Kin), s, p);
    else hipLaunchKernelGGL((xent_head_kernel<bf16, false>), grid, block, head_lds<bf16>(p.Kin), s, p);
  } else {
    if (p.bias) hipLaunchKernelGGL((xent_head_kernel<float, true>), grid, block, head_lds<float>(p.Kin), s, p);
    else hipLaunchKernelGGL((xent_head_kernel<float, false>), grid, block, head_lds<float>(p.Kin), s, p);
  }
  return (int)grid.x;
}

void softmax_xent(DType t, const XentParams& p, hipStream_t s) {
  MCC_CHECK(p.M > 0 && p.N > 0, "softmax_xent: empty");
  const dim3 grid((unsigned)cdiv(p.M, 256)), block(256);
  const bool vec = p.N <= 16 && p.ldl % 4 == 0 && (reinterpret_cast<uintptr_t>(p.logits) & 15) == 0;
  if (p.N > 64) {
    const dim3 g4((unsigned)cdiv(p.M, 4));
    if (t == DType::BF16) hipLaunchKernelGGL(softmax_xent_wide_kernel<bf16>, g4, block, 0, s, p);
    else hipLaunchKernelGGL(softmax_xent_wide_kernel<float>, g4, block, 0, s, p);
    return;
  }
  if (t == DType::BF16) {
    if (vec) hipLaunchKernelGGL((softmax_xent_kernel<bf16, 16>), grid, block, 0, s, p);
    else hipLaunchKernelGGL((softmax_xent_kernel<bf16, 0>), grid, block, 0, s, p);
  } else {
    if (vec) hipLaunchKernelGGL((softmax_xent_kernel<float, 16>), grid, block, 0, s, p);
    else hipLaunchKernelGGL((softmax_xent_kernel<float, 0>), grid, block, 0, s, p);
  }
}

void sgd_update(float* params, const float* grads, float* mom, int64_t n, float lr, float mu, float wd,
                hipStream_t s) {
  MCC_CHECK((reinterpret_cast<uintptr_t>(params) & 15) == 0 && (reinterpret_cast<uintptr_t>(grads) & 15) == 0,
            "sgd_update: buffers must be 16-byte aligned");
  hipLaunchKernelGGL(sgd_kernel, dim3(grid_for(n, 4)), dim3(256), 0, s, params, grads, mom, n, lr, mu, wd);
}

void pack_gather(DType t, void* dst, const float* src, const int32_t* idx, int64_t n, hipStream_t s) {
  if (n <= 0) return;
  if (t == DType::BF16)
    hipLaunchKernelGGL(pack_kernel<bf16>, dim3(grid_for(n)), dim3(256), 0, s, static_cast<bf16*>(dst), src, idx, n);
  else
    hipLaunchKernelGGL(pack_kernel<float>, dim3(grid_for(n)), dim3(256), 0, s, static_cast<float*>(dst), src, idx,
                       n);
}

static uint64_t div_magic(uint64_t d) {
  if (d <= 1) return 0;
  // ceil(2^64 / d) = floor((2^64 - 1) / d) + 1 for d not a power of two; exact either way below
  const uint64_t q = ~0ull / d;
  return q + 1;
}

void sgd_pack(DType t, const SgdPackParams& pin, hipStream_t s) {
  if (pin.n <= 0) return;
  MCC_CHECK(pin.nstages <= kMaxPackStages, "sgd_pack: too many weight stages");
  MCC_CHECK(((reinterpret_cast<uintptr_t>(pin.params) | reinterpret_cast<uintptr_t>(pin.grads) |
              reinterpret_cast<uintptr_t>(pin.mom) | reinterpret_cast<uintptr_t>(pin.packed)) & 15) == 0,
            "sgd_pack: buffers must be 16-byte aligned");
  SgdPackParams p = pin;
  p.ntiles = 0;
  for (int i = 0; i < p.nstages; ++i) {
    PackStage& st = p.st[i];
    st.m_ckk = div_magic((uint64_t)st.inC * st.KS * st.KS);
    st.m_kk = div_magic((uint64_t)st.KS * st.KS);
    st.m_ks = div_magic((uint64_t)st.KS);
    // transposing copies of a large conv: tiles (see sgd_pack_kernel)
    bool transposing = false;
    for (int m = 0; m < st.nmaps; ++m) transposing = transposing || st.map[m].sc == 1 || st.map[m].sn == 1;
    const int KK = st.KS * st.KS;
    st.tile0 = -1;
    if (st.nmaps > 0 && st.KS > 1 && KK <= kPackMaxKK && st.nw >= kPackTileMin && transposing &&
        st.nw % ((int64_t)st.inC * KK) == 0) {
      const int N = (int)(st.nw / ((int64_t)st.inC * KK));
      st.tile0 = p.ntiles;
      p.ntiles += cdiv(N, kPackTN) * cdiv(st.inC, kPackTC);
    }
  }
  MCC_CHECK(p.lo >= 0 && p.lo < p.n, "sgd_pack: empty parameter range");
  const dim3 grid((unsigned)(p.ntiles + (int)grid_for(p.n - (p.lo & ~int64_t(3)), 4))), block(256);
  if (t == DType::BF16) {
    if (p.update) hipLaunchKernelGGL((sgd_pack_kernel<bf16, true>), grid, block, 0, s, p);
    else hipLaunchKernelGGL((sgd_pack_kernel<bf16, false>), grid, block, 0, s, p);
  } else {
    if (p.update) hipLaunchKernelGGL((sgd_pack_kernel<float, true>), grid, block, 0, s, p);
    else hipLaunchKernelGGL((sgd_pack_kernel<float, false>), grid, block, 0, s, p);
  }
}

void sample_indices(int32_t* idx, int B, int64_t lo, int64_t hi, uint64_t seed, const uint64_t* step,
                    hipStream_t s) {
  MCC_CHECK(B > 0 && hi > lo, "sample_indices: empty range");
  hipLaunchKernelGGL(sample_kernel, dim3((unsigned)cdiv(B, 256)), dim3(256), 0, s, idx, B, lo, hi - lo, seed, step);
}

void seq_sample_indices(int32_t* idx, int B, int64_t offset, int64_t stride, int64_t n, const uint64_t* step,
                        hipStream_t s) {
  MCC_CHECK(B > 0 && n > 0 && stride > 0 && offset >= 0, "seq_sample_indices: bad range");
  hipLaunchKernelGGL(seq_sample_kernel, dim3((unsigned)cdiv(B, 256)), dim3(256), 0, s, idx, B, offset, stride, n, step);
}

void cu_hold(int nwg, int lds_bytes, double usec, hipStream_t s) {
  MCC_CHECK(nwg >= 1 && nwg <= 4096 && lds_bytes >= 1024 && lds_bytes <= 65536 && usec > 0 && usec < 1e5,
            "cu_hold: bad arguments");
  int dev = 0, khz = 0;
  MCC_CHECK(hipGetDevice(&dev) == hipSuccess &&
                hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev) == hipSuccess,
            "cu_hold: device query failed");
  const uint64_t ticks = (uint64_t)(usec * 1e-3 * (khz > 0 ? khz : 100000));
  hipLaunchKernelGGL(cu_hold_kernel, dim3((unsigned)nwg), dim3(256), (size_t)lds_bytes, s, ticks, nullptr);
}

void sample_indices_advance(int32_t* idx, int B, int64_t lo, int64_t hi, uint64_t seed, uint64_t* step,
                            hipStream_t s) {
  MCC_CHECK(B > 0 && hi > lo, "sample_indices_advance: empty range");
  // few workgroups: the tickets of one launch serialise on one address
  // (640 workgroups took 16 us, twice sample + advance)
  hipLaunchKernelGGL(sample_advance_kernel, dim3((unsigned)std::min(cdiv(B, 256), 64)), dim3(256), 0, s, idx, B, lo,
                     hi - lo, seed, step);
}

void advance_counter(uint64_t* step, hipStream_t s) {
  hipLaunchKernelGGL(advance_kernel, dim3(1), dim3(1), 0, s, step);
}

void iota_i32(int32_t* idx, int B, int64_t start, hipStream_t s) {
  hipLaunchKernelGGL(iota_kernel, dim3((unsigned)cdiv(B, 256)), dim3(256), 0, s, idx, B, start);
}

void fill_f32(float* dst, float v, int64_t n, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(fill_kernel, dim3(grid_for(n)), dim3(256), 0, s, dst, v, n);
}

void cast_f32(DType t, void* dst, const float* src, int64_t n, hipStream_t s) {
  if (n <= 0) return;
  if (t == DType::BF16)
    hipLaunchKernelGGL(cast_kernel<bf16>, dim3(grid_for(n)), dim3(256), 0, s, static_cast<bf16*>(dst), src, n);
  else
    hipLaunchKernelGGL(cast_kernel<float>, dim3(grid_for(n)), dim3(256), 0, s, static_cast<float*>(dst), src, n);
}

void to_f32(DType t, float* dst, const void* src, int64_t n, hipStream_t s) {
  if (n <= 0) return;
  if (t == DType::BF16)
    hipLaunchKernelGGL(to_f32_kernel<bf16>, dim3(grid_for(n)), dim3(256), 0, s, dst, static_cast<const bf16*>(src), n);
  else
    hipLaunchKernelGGL(to_f32_kernel<float>, dim3(grid_for(n)), dim3(256), 0, s, dst, static_cast<const float*>(src),
                       n);
}

void stats_to_f32(const unsigned long long* stats, float* out, hipStream_t s) {
  hipLaunchKernelGGL(stats_to_f32_kernel, dim3(1), dim3(64), 0, s, stats, out);
}

}  // namespace gpu
}  // namespace mcc
