// CPU reference executor.  See mcc/cpu_net.h for the reference mapping.
#include "mcc/cpu_net.h"

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
}

template <typename T>
int64_t CpuNet<T>::widx(const LayerSpec& L, int o, int i, int kh, int kw) const {
  const int k = L.ks;
  if (ref_compat_) return (int64_t)o * L.inC * k * k + kh * k + kw;  // defect D1, cnn.c:181,193
  return (((int64_t)o * L.inC + i) * k + kh) * k + kw;
}

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
  const LayerSpec& L = spec_.layers[li];
  const T* W = params.data() + L.w_off;
  const T* bias = params.data() + L.b_off;
  const int Ci = L.inC, H = L.inH, Wd = L.inW, k = L.ks;
  for (int b = 0; b < B; ++b) {
    const T* in = acts_[li - 1].data() + (size_t)b * L.in_nodes();
    T* out = acts_[li].data() + (size_t)b * L.nnodes();
    for (int o = 0; o < L.C; ++o)
      for (int oy = 0; oy < L.H; ++oy)
        for (int ox = 0; ox < L.W; ++ox) {
          T v = bias[o];
          const int y0 = oy * L.stride - L.pad, x0 = ox * L.stride - L.pad;
          for (int i = 0; i < Ci; ++i)
            for (int kh = 0; kh < k; ++kh) {
              const int y = y0 + kh;
              if (y < 0 || y >= H) continue;
              for (int kw = 0; kw < k; ++kw) {
                const int xx = x0 + kw;
                if (xx < 0 || xx >= Wd) continue;
                v += in[((size_t)i * H + y) * Wd + xx] * W[widx(L, o, i, kh, kw)];
              }
            }
          out[((size_t)o * L.H + oy) * L.W + ox] = act_fwd(L.act, v);
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
  for (int b = 0; b < B; ++b) {
    const T* in = acts_[li - 1].data() + (size_t)b * nin;
    T* out = acts_[li].data() + (size_t)b * L.C;
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
    for (int o = 0; o < L.C; ++o)
      for (int oy = 0; oy < L.H; ++oy)
        for (int ox = 0; ox < L.W; ++ox) {
          const size_t oi = ((size_t)o * L.H + oy) * L.W + ox;
          const T d = er[oi] * act_grad(L.act, y[oi]);
          if (d == T(0)) continue;
          const int y0 = oy * L.stride - L.pad, x0 = ox * L.stride - L.pad;
          for (int i = 0; i < Ci; ++i)
            for (int kh = 0; kh < k; ++kh) {
              const int yy = y0 + kh;
              if (yy < 0 || yy >= H) continue;
              for (int kw = 0; kw < k; ++kw) {
                const int xx = x0 + kw;
                if (xx < 0 || xx >= Wd) continue;
                const size_t ii = ((size_t)i * H + yy) * Wd + xx;
                const int64_t wi = widx(L, o, i, kh, kw);
                if (pe) pe[ii] += W[wi] * d;
                gW[wi] += d * in[ii];
              }
            }
          gb[o] += d;
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
