// CPU reference executor (fp64 or fp32): the correctness oracle that needs no
// GPU and no torch, and the engine behind the `cnn` / `cnnmpi` programs.
//
// Semantics follow the reference layer functions:
//   FC fwd + tanh / softmax      cnn.c:113-152
//   FC bwd                       cnn.c:154-173
//   conv fwd + ReLU              cnn.c:175-210
//   conv bwd                     cnn.c:212-247
//   output error p - y           cnn.c:284-286
//   logged error (MSE of p - y)  cnn.c:275-282
//   SGD update                   cnn.c:303-314
// Differences: conv weights are indexed [o][i][kh][kw]
// (defect D1 fixed) unless `ref_compat` is set, in which case the reference's
// shared-slice indexing (q = o*Cin*k*k + kh*k + kw, cnn.c:181,193) is used so
// the output can be diffed against the original program.  Max-pool is an
// addition (no reference counterpart).
#pragma once

#include <vector>

#include "mcc/model.h"

namespace mcc {

struct StepStats {
  double loss_sum = 0;   // sum over samples of -log p[label]
  double mse_sum = 0;    // sum over samples of mean((p - onehot)^2)  (cnn.c:275)
  int64_t correct = 0;   // argmax == label, first max wins (cnn.c:508-513)
  int64_t count = 0;
};

enum class InitMode : int {
  GlibcRef = 0,  // srand(seed); w = std * nrnd() with nrnd = (4 rand()/RAND_MAX - 2)*1.724 (cnn.c:46-49)
  Fast = 1,      // counter-based (splitmix64) Irwin-Hall, same distribution, O(1) per element
};

// Fill a canonical flat parameter vector.  Biases are zero (cnn.c:60-94 calloc).
// std per layer = LayerSpec::init_std, or sqrt(2/fan_in) when init_std == 0.
void init_params(const ModelSpec& spec, double* out, uint64_t seed, InitMode mode);

template <typename T>
class CpuNet {
 public:
  explicit CpuNet(const ModelSpec& spec, bool ref_compat = false);

  const ModelSpec& spec() const { return spec_; }
  int64_t nparams() const { return spec_.nparams; }
  bool ref_compat() const { return ref_compat_; }

  std::vector<T> params;  // canonical flat
  std::vector<T> grads;   // canonical flat, accumulated (u_weights/u_biases)

  // x: [B][C*H*W] in CHW order, already normalised to [0,1].
  void forward(const T* x, int B);
  const T* probs() const { return acts_.back().data(); }
  // Backward from integer labels.  dlogits = (p - onehot) * scale; grads +=.
  // Also computes the loss / metric / accuracy of the current forward.
  StepStats backward(const int* labels, T scale);
  // Evaluate stats without backward.
  StepStats evaluate(const int* labels) const;
  // params -= lr * grads; grads = 0  (Layer_update, cnn.c:303-314)
  void sgd(T lr);
  void zero_grads();

 private:
  // Default mode runs batched, cache-blocked kernels (im2col over the whole
  // minibatch + axpy-form GEMMs that vectorise; FC weights blocked to stay in
  // L2 across the batch).  --ref-compat keeps the per-sample reference loop
  // nests below, so its log stays byte-identical to cnn.c.
  void conv_fwd_fast(size_t li, int B);
  void conv_bwd_fast(size_t li, int B, bool need_dx);
  void fc_fwd_fast(size_t li, int B);
  void fc_bwd_fast(size_t li, int B, bool need_dx);
  void conv_fwd(size_t li, int B);
  void conv_bwd(size_t li, int B, bool need_dx);
  void pool_fwd(size_t li, int B);
  void pool_bwd(size_t li, int B);
  void fc_fwd(size_t li, int B);
  void fc_bwd(size_t li, int B, bool need_dx);
  int64_t widx(const LayerSpec& L, int o, int i, int kh, int kw) const;

  ModelSpec spec_;
  bool ref_compat_;
  int B_ = 0;
  std::vector<std::vector<T>> acts_;   // per layer outputs [B][nnodes]
  std::vector<std::vector<T>> errs_;   // per layer dL/d(output) [B][nnodes]
  std::vector<std::vector<int>> pidx_; // maxpool argmax (flat input index)
  std::vector<std::vector<T>> col_;    // fast path: im2col [K][B*P] of each conv layer (kept for backward)
  std::vector<T> tmp_, tmp2_;          // fast path scratch
};

extern template class CpuNet<double>;
extern template class CpuNet<float>;

}  // namespace mcc
