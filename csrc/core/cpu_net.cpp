// CPU reference executor.  See mcc/cpu_net.h for the reference mapping.
#include "mcc/cpu_net.h"
#include "mcc/cpu_kernels.h"

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>

namespace mcc {

// ---------------------------------------------------------------- init ----

static inline uint64_t splitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

static double layer_std(const LayerSpec& L) {
  if (L.init_std > 0) return L.init_std;
  double fan_in = (double)L.nweights / (double)L.C;
  return std::sqrt(2.0 / fan_in);
}

void init_params(const ModelSpec& spec, double* out, uint64_t seed, InitMode mode) {
  std::memset(out, 0, sizeof(double) * spec.nparams);
  if (mode == InitMode::GlibcRef) {
    // Same call order as the reference: srand once, then for every layer in
    // order 4 rand() per weight (Layer_create_conv/full, cnn.c:320-341).
    srand((unsigned)seed);
    for (const auto& L : spec.layers) {
      if (L.nweights == 0) continue;
      const double sd = layer_std(L);
      for (int64_t i = 0; i < L.nweights; ++i) {
        double r = (double)rand() / RAND_MAX;
        r += (double)rand() / RAND_MAX;
        r += (double)rand() / RAND_MAX;
        r += (double)rand() / RAND_MAX;
        out[L.w_off + i] = sd * ((r - 2.0) * 1.724);
      }
    }
    return;
  }
  const double inv = 1.0 / 9007199254740992.0;  // 2^-53
  for (const auto& L : spec.layers) {
    if (L.nweights == 0) continue;
    const double sd = layer_std(L);
    for (int64_t i = 0; i < L.nweights; ++i) {
      uint64_t base = seed * 0x100000001B3ull + (uint64_t)(L.w_off + i) * 4;
      double r = 0;
      for (int j = 0; j < 4; ++j) r += (double)(splitmix64(base + j) >> 11) * inv;
      out[L.w_off + i] = sd * ((r - 2.0) * 1.724);
    }
  }
}

// ------------------------------------------------------------ executor ----

template <typename T>
static inline T act_fwd(Act a, T x) {
  switch (a) {
    case Act::ReLU: return x > T(0) ? x : T(0);
    case Act::Tanh: return std::tanh(x);
    default: return x;
  }
}

// derivative expressed in the activation OUTPUT y (cnn.c:52-57)
template <typename T>
static inline T act_grad(Act a, T y) {
  switch (a) {
    case Act::ReLU: return y > T(0) ? T(1) : T(0);
    case Act::Tanh: return T(1) - y * y;
    default: return T(1);
  }
}

template <typename T>
CpuNet<T>::CpuNet(const ModelSpec& spec, bool ref_compat) : spec_(spec), ref_compat_(ref_compat) {
  params.assign(spec_.nparams, T(0));
  grads.assign(spec_.nparams, T(0));
  acts_.resize(spec_.layers.size());
  errs_.resize(spec_.layers.size());
  pidx_.resize(spec_.layers.size());
  col_.resize(spec_.layers.size());
}

// ------------------------------------------------------------ fast path ----
// Default mode: batched layers over vectorised kernels (cpu_kernels.inc),
// AVX2/FMA build when the CPU has it.

template <typename T>
const CpuKernels<T>& cpu_kernels() {
  static const CpuKernels<T> k = [] {
#if defined(__x86_64__) && defined(__GNUC__)
    __builtin_cpu_init();
    if (__builtin_cpu_supports("avx2") && __builtin_cpu_supports("fma")) return cpu_v3::kernels<T>();
#endif
    return cpu_base::kernels<T>();
  }();
  return k;
}
template const CpuKernels<double>& cpu_kernels<double>();
template const CpuKernels<float>& cpu_kernels<float>();

template <typename T>
void CpuNet<T>::conv_fwd_fast(size_t li, int B) {
  const LayerSpec& L = spec_.layers[li];
  const int Ci = L.inC, H = L.inH, Wd = L.inW, k = L.ks, C = L.C;
  const int P = L.H * L.W;
  const int64_t K = (int64_t)Ci * k * k, BP = (int64_t)B * P;
  std::vector<T>& col = col_[li];
  col.assign((size_t)(K * BP), T(0));
  // im2col over the minibatch: col[(i, kh, kw)][b*P + oy*OW + ox]
  for (int b = 0; b < B; ++b) {
    const T* in = acts_[li - 1].data() + (size_t)b * L.in_nodes();
    for (int i = 0; i < Ci; ++i)
      for (int kh = 0; kh < k; ++kh)
        for (int kw = 0; kw < k; ++kw) {
          T* row = col.data() + ((int64_t)(i * k + kh) * k + kw) * BP + (int64_t)b * P;
          for (int oy = 0; oy < L.H; ++oy) {
            const int y = oy * L.stride - L.pad + kh;
            if (y < 0 || y >= H) continue;
            const T* src = in + ((size_t)i * H + y) * Wd;
            for (int ox = 0; ox < L.W; ++ox) {
              const int x = ox * L.stride - L.pad + kw;
              if (x >= 0 && x < Wd) row[oy * L.W + ox] = src[x];
            }
          }
        }
  }
  const T* W = params.data() + L.w_off;
  const T* bias = params.data() + L.b_off;
  tmp_.resize((size_t)C * BP);
  for (int o = 0; o < C; ++o) std::fill(tmp_.begin() + (size_t)o * BP, tmp_.begin() + (size_t)(o + 1) * BP, bias[o]);
  cpu_kernels<T>().gemm_acc(C, BP, K, W, K, col.data(), BP, tmp_.data(), BP);  // out_t += W col
  // activation, back to [b][o][p]
  for (int b = 0; b < B; ++b) {
    T* out = acts_[li].data() + (size_t)b * L.nnodes();
    for (int o = 0; o < C; ++o) {
      const T* src = tmp_.data() + (size_t)o * BP + (size_t)b * P;
      for (int q = 0; q < P; ++q) out[(size_t)o * P + q] = act_fwd(L.act, src[q]);
    }
  }
}

template <typename T>
void CpuNet<T>::conv_bwd_fast(size_t li, int B, bool need_dx) {
  const LayerSpec& L = spec_.layers[li];
  const int Ci = L.inC, H = L.inH, Wd = L.inW, k = L.ks, C = L.C;
  const int P = L.H * L.W;
  const int64_t K = (int64_t)Ci * k * k, BP = (int64_t)B * P;
  const T* W = params.data() + L.w_off;
  T* gW = grads.data() + L.w_off;
  T* gb = grads.data() + L.b_off;
  // dz_t[o][b*P + q] = err * act'(y)
  tmp_.resize((size_t)C * BP);
  for (int b = 0; b < B; ++b) {
    const T* y = acts_[li].data() + (size_t)b * L.nnodes();
    const T* er = errs_[li].data() + (size_t)b * L.nnodes();
    for (int o = 0; o < C; ++o)
      for (int q = 0; q < P; ++q)
        tmp_[(size_t)o * BP + (size_t)b * P + q] = er[(size_t)o * P + q] * act_grad(L.act, y[(size_t)o * P + q]);
  }
  for (int o = 0; o < C; ++o) {
    T s = 0;
    const T* d = tmp_.data() + (size_t)o * BP;
    for (int64_t j = 0; j < BP; ++j) s += d[j];
    gb[o] += s;
  }
  const CpuKernels<T>& kern = cpu_kernels<T>();
  // gW[C][K] += dz_t[C][BP] col^T[BP][K]
  tmp2_.resize((size_t)(K * BP));
  kern.transpose(col_[li].data(), K, BP, tmp2_.data());
  kern.gemm_acc(C, K, BP, tmp_.data(), BP, tmp2_.data(), K, gW, K);
  if (!need_dx) return;
  // dcol[K][BP] = W^T[K][C] dz_t[C][BP]
  std::vector<T> wt((size_t)(K * C));
  kern.transpose(W, C, K, wt.data());
  tmp2_.assign((size_t)(K * BP), T(0));
  kern.gemm_acc(K, BP, C, wt.data(), C, tmp_.data(), BP, tmp2_.data(), BP);
  // col2im into the input error
  for (int b = 0; b < B; ++b) {
    T* pe = errs_[li - 1].data() + (size_t)b * L.in_nodes();
    std::fill(pe, pe + L.in_nodes(), T(0));
    for (int i = 0; i < Ci; ++i)
      for (int kh = 0; kh < k; ++kh)
        for (int kw = 0; kw < k; ++kw) {
          const T* row = tmp2_.data() + ((int64_t)(i * k + kh) * k + kw) * BP + (int64_t)b * P;
          for (int oy = 0; oy < L.H; ++oy) {
            const int y = oy * L.stride - L.pad + kh;
            if (y < 0 || y >= H) continue;
            T* dst = pe + ((size_t)i * H + y) * Wd;
            for (int ox = 0; ox < L.W; ++ox) {
              const int x = ox * L.stride - L.pad + kw;
              if (x >= 0 && x < Wd) dst[x] += row[oy * L.W + ox];
            }
          }
        }
  }
}

template <typename T>
void CpuNet<T>::fc_fwd_fast(size_t li, int B) {
  const LayerSpec& L = spec_.layers[li];
  const T* W = params.data() + L.w_off;
  const T* bias = params.data() + L.b_off;
  const int64_t nin = L.in_nodes();
  const int C = L.C;
  // W^T [nin][C] so the inner loop runs over the outputs
  tmp_.resize((size_t)(nin * C));
  for (int o = 0; o < C; ++o)
    for (int64_t i = 0; i < nin; ++i) tmp_[(size_t)(i * C + o)] = W[o * nin + i];
  for (int b = 0; b < B; ++b) {
    T* out = acts_[li].data() + (size_t)b * C;
    for (int o = 0; o < C; ++o) out[o] = bias[o];
  }
  // out[B][C] += in[B][nin] W^T[nin][C]
  cpu_kernels<T>().gemm_acc(B, C, nin, acts_[li - 1].data(), nin, tmp_.data(), C, acts_[li].data(), C);
}

template <typename T>
void CpuNet<T>::fc_bwd_fast(size_t li, int B, bool need_dx) {
  const LayerSpec& L = spec_.layers[li];
  const bool last = li + 1 == spec_.layers.size();
  const T* W = params.data() + L.w_off;
  T* gW = grads.data() + L.w_off;
  T* gb = grads.data() + L.b_off;
  const int64_t nin = L.in_nodes();
  const int C = L.C;
  tmp_.resize((size_t)B * C);  // dnet[b][o]
  for (int b = 0; b < B; ++b) {
    const T* y = acts_[li].data() + (size_t)b * C;
    const T* er = errs_[li].data() + (size_t)b * C;
    for (int o = 0; o < C; ++o) tmp_[(size_t)b * C + o] = er[o] * (last ? T(1) : act_grad(L.act, y[o]));
  }
  for (int o = 0; o < C; ++o) {
    T s = 0;
    for (int b = 0; b < B; ++b) s += tmp_[(size_t)b * C + o];
    gb[o] += s;
  }
  const CpuKernels<T>& kern = cpu_kernels<T>();
  // gW[C][nin] += dnet^T[C][B] x[B][nin]
  tmp2_.resize((size_t)B * C);
  kern.transpose(tmp_.data(), B, C, tmp2_.data());
  kern.gemm_acc(C, nin, B, tmp2_.data(), B, acts_[li - 1].data(), nin, gW, nin);
  if (!need_dx) return;
  // pe[B][nin] = dnet[B][C] W[C][nin]
  T* pe = errs_[li - 1].data();
  std::fill(pe, pe + (size_t)B * nin, T(0));
  kern.gemm_acc(B, nin, C, tmp_.data(), C, W, nin, pe, nin);
}

template <typename T>
int64_t CpuNet<T>::widx(const LayerSpec& L, int o, int i, int kh, int kw) const {
  const int k = L.ks;
  if (ref_compat_) return (int64_t)o * L.inC * k * k + kh * k + kw;  // defect D1, cnn.c:181,193
  return (((int64_t)o * L.inC + i) * k + kh) * k + kw;
}
// (the loop-nest conv paths below run in ref-compat mode only: the default
// mode takes conv_fwd_fast / conv_bwd_fast)

template <typename T>
void CpuNet<T>::forward(const T* x, int B) {
  B_ = B;
  const size_t n = spec_.layers.size();
  for (size_t li = 0; li < n; ++li) {
    acts_[li].resize((size_t)B * spec_.layers[li].nnodes());
    errs_[li].resize((size_t)B * spec_.layers[li].nnodes());
  }
  std::memcpy(acts_[0].data(), x, sizeof(T) * acts_[0].size());
  for (size_t li = 1; li < n; ++li) {
    switch (spec_.layers[li].kind) {
      case LayerKind::Conv: conv_fwd(li, B); break;
      case LayerKind::MaxPool: pool_fwd(li, B); break;
      case LayerKind::FC: fc_fwd(li, B); break;
      default: break;
    }
  }
}

template <typename T>
void CpuNet<T>::conv_fwd(size_t li, int B) {
  if (!ref_compat_) { conv_fwd_fast(li, B); return; }
  const LayerSpec& L = spec_.layers[li];
  const T* W = params.data() + L.w_off;
  const T* bias = params.data() + L.b_off;
  const int Ci = L.inC, H = L.inH, Wd = L.inW, k = L.ks;
  for (int b = 0; b < B; ++b) {
    const T* in = acts_[li - 1].data() + (size_t)b * L.in_nodes();
    T* out = acts_[li].data() + (size_t)b * L.nnodes();
    // reference loop nest and summation order (cnn.c:175-210); weights
    // indexed with the reference's shared slice (D1): every input channel
    // reads W[o][0] (widx in ref-compat mode), hoisted out of the MAC loop
    for (int o = 0; o < L.C; ++o) {
      const T* wo = W + widx(L, o, 0, 0, 0);
      for (int oy = 0; oy < L.H; ++oy)
        for (int ox = 0; ox < L.W; ++ox) {
          T v = bias[o];
          const int y0 = oy * L.stride - L.pad, x0 = ox * L.stride - L.pad;
          const int kh0 = std::max(0, -y0), kh1 = std::min(k, H - y0);
          const int kw0 = std::max(0, -x0), kw1 = std::min(k, Wd - x0);
          for (int i = 0; i < Ci; ++i)
            for (int kh = kh0; kh < kh1; ++kh) {
              const T* src = in + ((size_t)i * H + y0 + kh) * Wd + x0;
              const T* w = wo + kh * k;
              for (int kw = kw0; kw < kw1; ++kw) v += src[kw] * w[kw];
            }
          out[((size_t)o * L.H + oy) * L.W + ox] = act_fwd(L.act, v);
        }
    }
  }
}

template <typename T>
void CpuNet<T>::pool_fwd(size_t li, int B) {
  const LayerSpec& L = spec_.layers[li];
  pidx_[li].resize((size_t)B * L.nnodes());
  for (int b = 0; b < B; ++b) {
    const T* in = acts_[li - 1].data() + (size_t)b * L.in_nodes();
    T* out = acts_[li].data() + (size_t)b * L.nnodes();
    int* arg = pidx_[li].data() + (size_t)b * L.nnodes();
    for (int c = 0; c < L.C; ++c)
      for (int py = 0; py < L.H; ++py)
        for (int px = 0; px < L.W; ++px) {
          int best = -1;
          T bv = T(0);
          for (int dy = 0; dy < L.ks; ++dy)
            for (int dx = 0; dx < L.ks; ++dx) {
              const int y = py * L.stride + dy, xx = px * L.stride + dx;
              const int idx = (c * L.inH + y) * L.inW + xx;
              if (best < 0 || in[idx] > bv) { best = idx; bv = in[idx]; }
            }
          const size_t o = ((size_t)c * L.H + py) * L.W + px;
          out[o] = bv;
          arg[o] = best;
        }
  }
}

template <typename T>
void CpuNet<T>::fc_fwd(size_t li, int B) {
  const LayerSpec& L = spec_.layers[li];
  const T* W = params.data() + L.w_off;
  const T* bias = params.data() + L.b_off;
  const int64_t nin = L.in_nodes();
  const bool last = li + 1 == spec_.layers.size();
  if (!ref_compat_) fc_fwd_fast(li, B);
  for (int b = 0; b < B; ++b) {
    const T* in = acts_[li - 1].data() + (size_t)b * nin;
    T* out = acts_[li].data() + (size_t)b * L.C;
    if (ref_compat_)
      for (int o = 0; o < L.C; ++o) {
        T v = bias[o];
        const T* w = W + (size_t)o * nin;
        for (int64_t i = 0; i < nin; ++i) v += in[i] * w[i];
        out[o] = v;
      }
    if (last) {
      // softmax with max subtraction (cnn.c:125-143); ref max starts at -1 (D10)
      T m = ref_compat_ ? T(-1) : out[0];
      for (int o = 0; o < L.C; ++o) m = std::max(m, out[o]);
      T t = 0;
      for (int o = 0; o < L.C; ++o) { out[o] = std::exp(out[o] - m); t += out[o]; }
      for (int o = 0; o < L.C; ++o) out[o] /= t;
    } else {
      for (int o = 0; o < L.C; ++o) out[o] = act_fwd(L.act, out[o]);
    }
  }
}

template <typename T>
StepStats CpuNet<T>::evaluate(const int* labels) const {
  StepStats s;
  const int nc = spec_.num_classes();
  const T* p = acts_.back().data();
  for (int b = 0; b < B_; ++b) {
    const T* pb = p + (size_t)b * nc;
    int mj = -1;
    double mse = 0;
    for (int j = 0; j < nc; ++j) {
      if (mj < 0 || pb[mj] < pb[j]) mj = j;
      const double e = (double)pb[j] - (j == labels[b] ? 1.0 : 0.0);
      mse += e * e;
    }
    s.mse_sum += mse / nc;
    s.loss_sum += -std::log(std::max((double)pb[labels[b]], 1e-300));
    s.correct += (mj == labels[b]);
    s.count += 1;
  }
  return s;
}

template <typename T>
StepStats CpuNet<T>::backward(const int* labels, T scale) {
  StepStats s = evaluate(labels);
  const size_t n = spec_.layers.size();
  const int nc = spec_.num_classes();
  // errors = p - y (cnn.c:285-286), scaled (mean-gradient minibatches)
  T* e = errs_.back().data();
  const T* p = acts_.back().data();
  for (int b = 0; b < B_; ++b)
    for (int j = 0; j < nc; ++j)
      e[(size_t)b * nc + j] = (p[(size_t)b * nc + j] - (j == labels[b] ? T(1) : T(0))) * scale;
  for (size_t li = n - 1; li >= 1; --li) {
    const bool need_dx = li >= 2;  // no error propagation into the input layer
    switch (spec_.layers[li].kind) {
      case LayerKind::Conv: conv_bwd(li, B_, need_dx); break;
      case LayerKind::MaxPool: pool_bwd(li, B_); break;
      case LayerKind::FC: fc_bwd(li, B_, need_dx); break;
      default: break;
    }
  }
  return s;
}

template <typename T>
void CpuNet<T>::fc_bwd(size_t li, int B, bool need_dx) {
  if (!ref_compat_) { fc_bwd_fast(li, B, need_dx); return; }
  const LayerSpec& L = spec_.layers[li];
  const bool last = li + 1 == spec_.layers.size();
  const T* W = params.data() + L.w_off;
  T* gW = grads.data() + L.w_off;
  T* gb = grads.data() + L.b_off;
  const int64_t nin = L.in_nodes();
  std::vector<T> dnet(L.C);
  for (int b = 0; b < B; ++b) {
    const T* y = acts_[li].data() + (size_t)b * L.C;
    const T* er = errs_[li].data() + (size_t)b * L.C;
    const T* x = acts_[li - 1].data() + (size_t)b * nin;
    T* pe = need_dx ? errs_[li - 1].data() + (size_t)b * nin : nullptr;
    if (pe) std::fill(pe, pe + nin, T(0));
    for (int o = 0; o < L.C; ++o) dnet[o] = er[o] * (last ? T(1) : act_grad(L.act, y[o]));
    for (int o = 0; o < L.C; ++o) {
      const T d = dnet[o];
      const T* w = W + (size_t)o * nin;
      T* g = gW + (size_t)o * nin;
      if (pe)
        for (int64_t i = 0; i < nin; ++i) pe[i] += w[i] * d;
      for (int64_t i = 0; i < nin; ++i) g[i] += d * x[i];
      gb[o] += d;
    }
  }
}

template <typename T>
void CpuNet<T>::conv_bwd(size_t li, int B, bool need_dx) {
  if (!ref_compat_) { conv_bwd_fast(li, B, need_dx); return; }
  const LayerSpec& L = spec_.layers[li];
  const T* W = params.data() + L.w_off;
  T* gW = grads.data() + L.w_off;
  T* gb = grads.data() + L.b_off;
  const int Ci = L.inC, H = L.inH, Wd = L.inW, k = L.ks;
  for (int b = 0; b < B; ++b) {
    const T* in = acts_[li - 1].data() + (size_t)b * L.in_nodes();
    const T* y = acts_[li].data() + (size_t)b * L.nnodes();
    const T* er = errs_[li].data() + (size_t)b * L.nnodes();
    T* pe = need_dx ? errs_[li - 1].data() + (size_t)b * L.in_nodes() : nullptr;
    if (pe) std::fill(pe, pe + L.in_nodes(), T(0));
    // reference order (cnn.c:212-247), shared-slice weights (D1) hoisted
    for (int o = 0; o < L.C; ++o) {
      const T* wo = W + widx(L, o, 0, 0, 0);
      T* go = gW + widx(L, o, 0, 0, 0);
      for (int oy = 0; oy < L.H; ++oy)
        for (int ox = 0; ox < L.W; ++ox) {
          const size_t oi = ((size_t)o * L.H + oy) * L.W + ox;
          const T d = er[oi] * act_grad(L.act, y[oi]);
          if (d == T(0)) continue;
          const int y0 = oy * L.stride - L.pad, x0 = ox * L.stride - L.pad;
          const int kh0 = std::max(0, -y0), kh1 = std::min(k, H - y0);
          const int kw0 = std::max(0, -x0), kw1 = std::min(k, Wd - x0);
          for (int i = 0; i < Ci; ++i)
            for (int kh = kh0; kh < kh1; ++kh) {
              const size_t ii0 = ((size_t)i * H + y0 + kh) * Wd + x0;
              const T* w = wo + kh * k;
              T* g = go + kh * k;
              if (pe)
                for (int kw = kw0; kw < kw1; ++kw) {
                  pe[ii0 + kw] += w[kw] * d;
                  g[kw] += d * in[ii0 + kw];
                }
              else
                for (int kw = kw0; kw < kw1; ++kw) g[kw] += d * in[ii0 + kw];
            }
          gb[o] += d;
        }
    }
  }
}

template <typename T>
void CpuNet<T>::pool_bwd(size_t li, int B) {
  const LayerSpec& L = spec_.layers[li];
  for (int b = 0; b < B; ++b) {
    const T* er = errs_[li].data() + (size_t)b * L.nnodes();
    const int* arg = pidx_[li].data() + (size_t)b * L.nnodes();
    T* pe = errs_[li - 1].data() + (size_t)b * L.in_nodes();
    std::fill(pe, pe + L.in_nodes(), T(0));
    for (int64_t o = 0; o < L.nnodes(); ++o) pe[arg[o]] += er[o];
  }
}

template <typename T>
void CpuNet<T>::sgd(T lr) {
  for (int64_t i = 0; i < spec_.nparams; ++i) {
    params[i] -= lr * grads[i];
    grads[i] = T(0);
  }
}

template <typename T>
void CpuNet<T>::zero_grads() {
  std::fill(grads.begin(), grads.end(), T(0));
}

template class CpuNet<double>;
template class CpuNet<float>;

}  // namespace mcc
