// GpuNet64 implementation: fp64 layer schedule over the f64.hip kernels.
// Layer semantics follow csrc/core/cpu_net.cpp one for one (which cites the
// reference lines): conv = im2col x W on the fp64 MFMA GEMM with bias and
// activation in its epilogue, FC = X x W^T likewise, backward = dZ^T panels
// feeding three strided GEMM views (dW, dX / dcol) plus col2im and unpool
// gathers.
#include "mcc/net64.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <string>

#include "kernels.h"

namespace mcc {

#define HIP_OK(expr)                                                                                    \
  do {                                                                                                  \
    hipError_t _e = (expr);                                                                             \
    if (_e != hipSuccess)                                                                               \
      throw Error(std::string("HIP error: ") + hipGetErrorString(_e) + " at " + __FILE__ + ":" +        \
                  std::to_string(__LINE__));                                                            \
  } while (0)

namespace {

gpu::Conv64Geom conv_geom(const LayerSpec& L) {
  return gpu::Conv64Geom{L.inC, L.inH, L.inW, L.ks, L.stride, L.pad, L.H, L.W};
}
gpu::Pool64Geom pool_geom(const LayerSpec& L) {
  return gpu::Pool64Geom{L.C, L.inH, L.inW, L.ks, L.stride, L.H, L.W};
}
int act_kind(Act a) { return a == Act::ReLU ? gpu::ACT_RELU : a == Act::Tanh ? gpu::ACT_TANH : gpu::ACT_NONE; }

// split-K slabs never exceed 512 tiles' worth of 64x64 outputs (gemm64_slabs)
constexpr int64_t kPartDoubles = 512LL * 64 * 64;

}  // namespace

GpuNet64::GpuNet64(const ModelSpec& spec, bool ref_compat, int max_batch, int device)
    : spec_(spec), ref_compat_(ref_compat), max_batch_(max_batch), device_(device) {
  MCC_CHECK(max_batch > 0, "GpuNet64: max_batch must be positive");
  if (device_ >= 0) HIP_OK(hipSetDevice(device_));
  HIP_OK(hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking));
  const size_t n = spec_.layers.size();
  const int64_t Bm = max_batch;
  // arena layout: [params grads | per-layer act, err | conv col | pool arg | scratch]
  std::vector<std::pair<void**, size_t>> plan;
  auto add = [&](void** slot, size_t bytes) { plan.emplace_back(slot, (bytes + 255) & ~size_t(255)); };
  add(reinterpret_cast<void**>(&params_), 8 * (size_t)spec_.nparams);
  add(reinterpret_cast<void**>(&grads_), 8 * (size_t)spec_.nparams);
  act_.assign(n, nullptr);
  err_.assign(n, nullptr);
  col_.assign(n, nullptr);
  arg_.assign(n, nullptr);
  int64_t dz = 0, dcol = 0, weff = 0;
  for (size_t li = 0; li < n; ++li) {
    const LayerSpec& L = spec_.layers[li];
    add(reinterpret_cast<void**>(&act_[li]), 8 * (size_t)(Bm * L.nnodes()));
    add(reinterpret_cast<void**>(&err_[li]), 8 * (size_t)(Bm * L.nnodes()));
    if (L.kind == LayerKind::Conv) {
      const int64_t K = (int64_t)L.inC * L.ks * L.ks, BP = Bm * L.H * L.W;
      add(reinterpret_cast<void**>(&col_[li]), 8 * (size_t)(K * BP));
      dz = std::max(dz, L.C * BP);
      dcol = std::max(dcol, K * BP);
      weff = std::max(weff, L.C * K);
    } else if (L.kind == LayerKind::MaxPool) {
      add(reinterpret_cast<void**>(&arg_[li]), 4 * (size_t)(Bm * L.nnodes()));
    } else if (L.kind == LayerKind::FC) {
      dz = std::max(dz, (int64_t)L.C * Bm);
    }
  }
  add(reinterpret_cast<void**>(&dz_), 8 * (size_t)dz);
  add(reinterpret_cast<void**>(&dcol_), 8 * (size_t)std::max<int64_t>(dcol, 1));
  add(reinterpret_cast<void**>(&weff_), 8 * (size_t)std::max<int64_t>(weff, 1));
  add(reinterpret_cast<void**>(&wfull_), 8 * (size_t)std::max<int64_t>(weff, 1));
  add(reinterpret_cast<void**>(&part_), 8 * (size_t)kPartDoubles);
  add(reinterpret_cast<void**>(&stats_), 8 * 3 * (size_t)Bm);
  add(reinterpret_cast<void**>(&labels_), 4 * (size_t)Bm);
  bytes_ = 0;
  for (auto& e : plan) bytes_ += e.second;
  HIP_OK(hipMalloc(reinterpret_cast<void**>(&arena_), bytes_));
  size_t off = 0;
  for (auto& e : plan) {
    *e.first = arena_ + off;
    off += e.second;
  }
  HIP_OK(hipMemsetAsync(arena_, 0, bytes_, stream_));
  HIP_OK(hipStreamSynchronize(stream_));
}

GpuNet64::~GpuNet64() {
  if (stream_) (void)hipStreamSynchronize(stream_);
  if (arena_) (void)hipFree(arena_);
  if (stream_) (void)hipStreamDestroy(stream_);
}

void GpuNet64::set_params(const double* host) {
  HIP_OK(hipMemcpyAsync(params_, host, 8 * (size_t)spec_.nparams, hipMemcpyHostToDevice, stream_));
  HIP_OK(hipStreamSynchronize(stream_));
}
void GpuNet64::get_params(double* host) const {
  HIP_OK(hipMemcpyAsync(host, params_, 8 * (size_t)spec_.nparams, hipMemcpyDeviceToHost, stream_));
  HIP_OK(hipStreamSynchronize(stream_));
}
void GpuNet64::set_grads(const double* host) {
  HIP_OK(hipMemcpyAsync(grads_, host, 8 * (size_t)spec_.nparams, hipMemcpyHostToDevice, stream_));
  HIP_OK(hipStreamSynchronize(stream_));
}
void GpuNet64::get_grads(double* host) const {
  HIP_OK(hipMemcpyAsync(host, grads_, 8 * (size_t)spec_.nparams, hipMemcpyDeviceToHost, stream_));
  HIP_OK(hipStreamSynchronize(stream_));
}

void GpuNet64::forward(const double* x, int B) {
  MCC_CHECK(B > 0 && B <= max_batch_, "GpuNet64::forward: batch out of range");
  HIP_OK(hipMemcpyAsync(act_[0], x, 8 * (size_t)B * spec_.input_nodes(), hipMemcpyHostToDevice, stream_));
  HIP_OK(hipStreamSynchronize(stream_));  // the caller may refill x right away
  forward_device(act_[0], B);
}

void GpuNet64::forward_device(const double* x, int B) {
  MCC_CHECK(B > 0 && B <= max_batch_, "GpuNet64::forward: batch out of range");
  B_ = B;
  if (x != act_[0])
    HIP_OK(hipMemcpyAsync(act_[0], x, 8 * (size_t)B * spec_.input_nodes(), hipMemcpyDeviceToDevice, stream_));
  const size_t n = spec_.layers.size();
  for (size_t li = 1; li < n; ++li) {
    const LayerSpec& L = spec_.layers[li];
    const double* W = params_ + L.w_off;
    const double* bias = params_ + L.b_off;
    if (L.kind == LayerKind::Conv) {
      const gpu::Conv64Geom g = conv_geom(L);
      const int kk = L.ks * L.ks, P = L.H * L.W;
      const int64_t K = (int64_t)L.inC * kk;
      gpu::im2col64(g, act_[li - 1], col_[li], B, stream_);
      if (ref_compat_) {
        gpu::weff64(W, weff_, L.C, L.inC, kk, stream_);
        W = weff_;
      }
      gpu::Gemm64Params p;
      p.M = L.C; p.N = B * P; p.K = K;
      p.A = W; p.sam = K; p.sak = 1;
      p.B = col_[li]; p.sbk = (int64_t)B * P; p.sbn = 1;
      p.C = act_[li]; p.P = P;
      p.bias_m = bias; p.act = act_kind(L.act);
      gpu::gemm64(p, part_, stream_);
    } else if (L.kind == LayerKind::MaxPool) {
      gpu::pool64_fwd(pool_geom(L), act_[li - 1], act_[li], arg_[li], B, stream_);
    } else if (L.kind == LayerKind::FC) {
      const bool last = li + 1 == n;
      const int64_t nin = L.in_nodes();
      gpu::Gemm64Params p;
      p.M = B; p.N = L.C; p.K = nin;
      p.A = act_[li - 1]; p.sam = nin; p.sak = 1;
      p.B = W; p.sbk = 1; p.sbn = nin;
      p.C = act_[li]; p.ldc = L.C;
      p.bias_n = bias; p.act = last ? gpu::ACT_NONE : act_kind(L.act);
      gpu::gemm64(p, part_, stream_);
      if (last) gpu::softmax64(act_[li], B, L.C, ref_compat_, stream_);
    }
  }
  HIP_OK(hipGetLastError());
}

const double* GpuNet64::probs() {
  const int nc = spec_.num_classes();
  host_probs_.resize((size_t)B_ * nc);
  HIP_OK(hipMemcpyAsync(host_probs_.data(), act_.back(), 8 * host_probs_.size(), hipMemcpyDeviceToHost, stream_));
  HIP_OK(hipStreamSynchronize(stream_));
  return host_probs_.data();
}

void GpuNet64::upload_labels(const int* labels) {
  HIP_OK(hipMemcpyAsync(labels_, labels, 4 * (size_t)B_, hipMemcpyHostToDevice, stream_));
  HIP_OK(hipStreamSynchronize(stream_));
}

StepStats GpuNet64::read_stats() {
  host_stats_.resize(3 * (size_t)B_);
  HIP_OK(hipMemcpyAsync(host_stats_.data(), stats_, 8 * host_stats_.size(), hipMemcpyDeviceToHost, stream_));
  HIP_OK(hipStreamSynchronize(stream_));
  StepStats s;
  for (int b = 0; b < B_; ++b) {  // sample order, as CpuNet::evaluate
    s.loss_sum += host_stats_[3 * b];
    s.mse_sum += host_stats_[3 * b + 1];
    s.correct += host_stats_[3 * b + 2] != 0.0;
    s.count += 1;
  }
  return s;
}

StepStats GpuNet64::evaluate(const int* labels) {
  MCC_CHECK(B_ > 0, "GpuNet64::evaluate before forward");
  upload_labels(labels);
  gpu::out_err64(act_.back(), labels_, nullptr, stats_, B_, spec_.num_classes(), 0.0, stream_);
  return read_stats();
}

void GpuNet64::forward_u8(const uint8_t* data, const uint8_t* labels, const int32_t* idx, int B) {
  MCC_CHECK(B > 0 && B <= max_batch_, "GpuNet64::forward_u8: bad batch");
  const int npix = (int)spec_.input_nodes();
  // the input layer's activation buffer holds the normalised batch
  gpu::u8_batch64(data, labels, idx, act_[0], labels_, B, npix, stream_);
  forward_device(act_[0], B);
}

StepStats GpuNet64::backward(const int* labels, double scale) {
  MCC_CHECK(B_ > 0, "GpuNet64::backward before forward");
  upload_labels(labels);
  backward_device(scale);
  return read_stats();
}

void GpuNet64::backward_device(double scale) {
  MCC_CHECK(B_ > 0, "GpuNet64::backward before forward");
  const int B = B_;
  const size_t n = spec_.layers.size();
  gpu::out_err64(act_.back(), labels_, err_.back(), stats_, B, spec_.num_classes(), scale, stream_);
  for (size_t li = n - 1; li >= 1; --li) {
    const LayerSpec& L = spec_.layers[li];
    const bool need_dx = li >= 2;  // no error into the input layer (CpuNet::backward)
    const double* W = params_ + L.w_off;
    double* gW = grads_ + L.w_off;
    double* gb = grads_ + L.b_off;
    if (L.kind == LayerKind::Conv) {
      const gpu::Conv64Geom g = conv_geom(L);
      const int kk = L.ks * L.ks, P = L.H * L.W;
      const int64_t K = (int64_t)L.inC * kk, BP = (int64_t)B * P;
      gpu::dz64(err_[li], act_[li], dz_, B, L.C, P, act_kind(L.act), stream_);
      gpu::rowsum64(dz_, gb, L.C, BP, part_, stream_);
      // gW[C][K] += dZ^T[C][BP] col^T[BP][K]
      gpu::Gemm64Params p;
      p.M = L.C; p.N = (int)K; p.K = BP;
      p.A = dz_; p.sam = BP; p.sak = 1;
      p.B = col_[li]; p.sbk = 1; p.sbn = BP;
      if (ref_compat_) {
        p.C = wfull_; p.ldc = K;
        gpu::gemm64(p, part_, stream_);
        gpu::fold64(wfull_, gW, L.C, L.inC, kk, stream_);
      } else {
        p.C = gW; p.ldc = K; p.accumulate = true;
        gpu::gemm64(p, part_, stream_);
      }
      if (need_dx) {
        if (ref_compat_) {
          gpu::weff64(W, weff_, L.C, L.inC, kk, stream_);
          W = weff_;
        }
        // dcol[K][BP] = W^T[K][C] dZ^T[C][BP]
        gpu::Gemm64Params d;
        d.M = (int)K; d.N = (int)BP; d.K = L.C;
        d.A = W; d.sam = 1; d.sak = K;
        d.B = dz_; d.sbk = BP; d.sbn = 1;
        d.C = dcol_; d.ldc = BP;
        gpu::gemm64(d, part_, stream_);
        gpu::col2im64(g, dcol_, err_[li - 1], B, stream_);
      }
    } else if (L.kind == LayerKind::MaxPool) {
      gpu::pool64_bwd(pool_geom(L), err_[li], arg_[li], err_[li - 1], B, stream_);
    } else if (L.kind == LayerKind::FC) {
      const bool last = li + 1 == n;
      const int64_t nin = L.in_nodes();
      gpu::dz64(err_[li], act_[li], dz_, B, L.C, 1, last ? gpu::ACT_NONE : act_kind(L.act), stream_);
      gpu::rowsum64(dz_, gb, L.C, B, part_, stream_);
      // gW[C][nin] += dZ^T[C][B] X[B][nin]
      gpu::Gemm64Params p;
      p.M = L.C; p.N = (int)nin; p.K = B;
      p.A = dz_; p.sam = B; p.sak = 1;
      p.B = act_[li - 1]; p.sbk = nin; p.sbn = 1;
      p.C = gW; p.ldc = nin; p.accumulate = true;
      gpu::gemm64(p, part_, stream_);
      if (need_dx) {
        // dX[B][nin] = dZ[B][C] W[C][nin]
        gpu::Gemm64Params d;
        d.M = B; d.N = (int)nin; d.K = L.C;
        d.A = dz_; d.sam = 1; d.sak = B;
        d.B = W; d.sbk = nin; d.sbn = 1;
        d.C = err_[li - 1]; d.ldc = nin;
        gpu::gemm64(d, part_, stream_);
      }
    }
  }
  HIP_OK(hipGetLastError());
}

void GpuNet64::sgd(double lr) {
  gpu::sgd64(params_, grads_, lr, spec_.nparams, stream_);
  HIP_OK(hipGetLastError());
}

void GpuNet64::zero_grads() {
  HIP_OK(hipMemsetAsync(grads_, 0, 8 * (size_t)spec_.nparams, stream_));
}

}  // namespace mcc
