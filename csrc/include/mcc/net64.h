// GpuNet64: the reference's precision (fp64, cnn.c:22-30) on the MI355X.
//
// The reference's GPU code is one fp64 conv-forward kernel offloaded per call
// with cudaMalloc/cudaMemcpy around it (CUDAcnn.cu:167-218, never compiled in
// its Makefile).  GpuNet64 runs the WHOLE network in fp64 on the GPU --
// forward, backward, SGD -- with exactly the CPU executor's semantics
// (mcc/cpu_net.h: output error p - y, tanh/ReLU derivatives in the output,
// first-max pooling, the D1 shared-slice conv weights and the D10 softmax max
// in --ref-compat mode), so `cnn_hip --dtype fp64 [--ref-compat]` reproduces
// the reference program's log line for line (tests/test_gpu_fp64.py).
//
// Layouts are the canonical ones of CpuNet (activations [B][C][H][W],
// parameters one flat fp64 vector [W0 b0 W1 b1 ...]); every buffer is
// allocated once for `max_batch`.  The GEMM-shaped work runs on the fp64
// MFMA kernel of f64.hip; results are deterministic (no atomics).
#pragma once

#include <hip/hip_runtime_api.h>

#include <vector>

#include "mcc/cpu_net.h"
#include "mcc/model.h"

namespace mcc {

class GpuNet64 {
 public:
  GpuNet64(const ModelSpec& spec, bool ref_compat, int max_batch, int device = -1);
  ~GpuNet64();
  GpuNet64(const GpuNet64&) = delete;
  GpuNet64& operator=(const GpuNet64&) = delete;

  const ModelSpec& spec() const { return spec_; }
  int64_t nparams() const { return spec_.nparams; }
  bool ref_compat() const { return ref_compat_; }
  int max_batch() const { return max_batch_; }
  int batch() const { return B_; }  // of the last forward
  hipStream_t stream() const { return stream_; }
  double* device_params() const { return params_; }
  double* device_grads() const { return grads_; }
  size_t device_bytes() const { return bytes_; }

  // host <-> device, synchronous
  void set_params(const double* host);
  void get_params(double* host) const;
  void set_grads(const double* host);
  void get_grads(double* host) const;

  // x: host [B][C*H*W] (CHW, normalised), B <= max_batch
  void forward(const double* x, int B);
  // same, x already on the device
  void forward_device(const double* x, int B);
  // probabilities of the last forward, copied to the host (synchronises)
  const double* probs();
  // errors = (p - onehot) * scale, grads += (CpuNet::backward); stats of the
  // current forward.  labels: host int[B].
  StepStats backward(const int* labels, double scale);
  StepStats evaluate(const int* labels);
  void sgd(double lr);  // params -= lr * grads; grads = 0
  // Device-resident training step pieces without host synchronisation (the
  // throughput path, bench.py --dtype fp64): forward of the u8 dataset rows
  // idx[0..B) (/255 in fp64), and the backward with the labels gathered on the
  // device; per-sample stats stay on the device (device_stats).
  void forward_u8(const uint8_t* data, const uint8_t* labels, const int32_t* idx, int B);
  void backward_device(double scale);
  const double* device_stats() const { return stats_; }
  void zero_grads();

 private:
  void upload_labels(const int* labels);
  StepStats read_stats();

  ModelSpec spec_;
  bool ref_compat_;
  int max_batch_;
  int device_ = -1;
  int B_ = 0;
  hipStream_t stream_ = nullptr;
  size_t bytes_ = 0;
  char* arena_ = nullptr;
  double* params_ = nullptr;
  double* grads_ = nullptr;
  std::vector<double*> act_, err_, col_;
  std::vector<int32_t*> arg_;
  double *dz_ = nullptr, *dcol_ = nullptr, *weff_ = nullptr, *wfull_ = nullptr, *part_ = nullptr;
  double* stats_ = nullptr;
  int32_t* labels_ = nullptr;
  std::vector<double> host_probs_, host_stats_;
};

}  // namespace mcc
