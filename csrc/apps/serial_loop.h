// The reference program's serial train/test loop (cnn.c:406-531), shared by
// `cnn` (CpuNet on the host, fp64 / fp32) and `cnn_hip --dtype fp64`
// (GpuNet64: the same arithmetic on the MI355X), so both print the same log
// and a GPU run at the reference precision can be diffed line by line
// against the CPU one (tests/test_gpu_fp64.py).
//
// Net must provide forward(const T*, int B), backward(const int*, T scale) ->
// StepStats, evaluate(const int*) -> StepStats and sgd(T); parameters move
// through net_set_params / net_get_params (found by argument-dependent
// lookup, defined next to each Net).
#pragma once

#include <chrono>
#include <cmath>
#include <cstdio>
#include <memory>
#include <vector>

#include "cli.h"
#include "mcc/cpu_net.h"
#include "mcc/io.h"

namespace mcc {

template <typename T>
void net_set_params(CpuNet<T>& n, const std::vector<double>& p) {
  for (size_t i = 0; i < p.size(); ++i) n.params[i] = (T)p[i];
}
template <typename T>
std::vector<double> net_get_params(CpuNet<T>& n) {
  return std::vector<double>(n.params.begin(), n.params.end());
}

// make_net(spec) -> std::unique_ptr<Net>
template <typename T, typename MakeNet>
int run_serial(const CliArgs& a, const char* program, MakeNet make_net) {
  IdxFile tr_img, tr_lab;
  ModelSpec spec;
  std::vector<double> loaded;
  // Reference order: srand(0) then model creation (cnn.c:413-428), then IDX load.
  if (!a.load.empty()) {
    try { spec = load_weights(a.load, loaded); } catch (const Error& e) { std::fprintf(stderr, "%s\n", e.what()); return 111; }
    srand(a.seed);
  } else {
    spec = make_model(a.model);
  }
  auto net_ptr = make_net(spec);
  auto& net = *net_ptr;
  {
    std::vector<double> p(spec.nparams);
    if (a.load.empty()) init_params(spec, p.data(), a.seed, InitMode::GlibcRef);
    else p = loaded;
    net_set_params(net, p);
  }
  const int C = spec.input().C, H = spec.input().H, W = spec.input().W;
  const int64_t in_nodes = spec.input_nodes();
  try {
    tr_img = load_idx(a.train_images, spec);
    tr_lab = load_idx(a.train_labels, spec);
  } catch (const Error& e) {
    std::fprintf(stderr, "%s\n", e.what());
    return 111;
  }
  if (tr_img.item_size() != in_nodes || tr_lab.count() < tr_img.count()) {
    std::fprintf(stderr, "train set shape does not match the model input %dx%dx%d\n", C, H, W);
    return 111;
  }
  int64_t N = tr_img.count();
  if (a.max_train > 0 && a.max_train < N) N = a.max_train;

  // u8 NHWC image -> CHW float / 255 (cnn.c:457)
  auto load_x = [&](const IdxFile& f, int64_t i, T* x) {
    const uint8_t* src = f.data.data() + (size_t)i * in_nodes;
    for (int c = 0; c < C; ++c)
      for (int y = 0; y < H; ++y)
        for (int xx = 0; xx < W; ++xx) x[((size_t)c * H + y) * W + xx] = (T)(src[((size_t)y * W + xx) * C + c] / 255.0);
  };

  std::fprintf(stderr, "training...\n");
  const auto t0 = std::chrono::steady_clock::now();
  double etotal = 0;
  const int64_t total = (int64_t)a.epochs * N;
  if (a.ref_compat) {
    std::vector<T> x(in_nodes);
    for (int64_t i = 0; i < total; ++i) {
      const int64_t index = rand() % N;
      load_x(tr_img, index, x.data());
      net.forward(x.data(), 1);
      const int label = tr_lab.data[index];
      StepStats s = net.backward(&label, (T)1);
      etotal += s.mse_sum;
      if (i % a.batch == 0) net.sgd((T)(a.lr / a.batch));
      if (i % a.log_every == 0) {
        std::fprintf(stderr, "i=%lld, error=%.4f\n", (long long)i, etotal / 1000);
        etotal = 0;
      }
    }
  } else {
    const int B = a.batch;
    std::vector<T> x((size_t)B * in_nodes);
    std::vector<int> labels(B);
    for (int64_t i = 0; i < total; i += B) {
      const int nb = (int)std::min<int64_t>(B, total - i);
      for (int b = 0; b < nb; ++b) {
        const int64_t index = rand() % N;
        load_x(tr_img, index, x.data() + (size_t)b * in_nodes);
        labels[b] = tr_lab.data[index];
      }
      net.forward(x.data(), nb);
      StepStats s = net.backward(labels.data(), (T)(1.0 / nb));
      net.sgd((T)a.lr);
      etotal += s.mse_sum;
      const int64_t mark = ((i + a.log_every - 1) / a.log_every) * a.log_every;
      if (mark < i + nb) {
        std::fprintf(stderr, "i=%lld, error=%.4f\n", (long long)mark, etotal / 1000);
        etotal = 0;
      }
    }
  }
  const double train_s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();

  IdxFile te_img, te_lab;
  try {
    te_img = load_idx(a.test_images, spec);
    te_lab = load_idx(a.test_labels, spec);
  } catch (const Error& e) {
    std::fprintf(stderr, "%s\n", e.what());
    return 111;
  }
  if (te_img.item_size() != in_nodes || te_lab.count() < te_img.count()) return 111;
  std::fprintf(stderr, "testing...\n");
  const int64_t ntests = te_img.count();
  int64_t ncorrect = 0;
  const auto t1 = std::chrono::steady_clock::now();
  const int EB = 256;
  std::vector<T> x((size_t)EB * in_nodes);
  std::vector<int> labels(EB);
  for (int64_t i = 0; i < ntests; i += EB) {
    const int nb = (int)std::min<int64_t>(EB, ntests - i);
    for (int b = 0; b < nb; ++b) {
      load_x(te_img, i + b, x.data() + (size_t)b * in_nodes);
      labels[b] = te_lab.data[i + b];
    }
    net.forward(x.data(), nb);
    ncorrect += net.evaluate(labels.data()).correct;
    for (int64_t j = i; j < i + nb; ++j)
      if (j % 1000 == 0) std::fprintf(stderr, "i=%lld\n", (long long)j);
  }
  const double test_s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t1).count();
  std::fprintf(stderr, "ntests=%lld, ncorrect=%lld\n", (long long)ntests, (long long)ncorrect);
  if (!a.save.empty()) {
    std::vector<double> p = net_get_params(net);
    try { save_weights(a.save, spec, p.data()); } catch (const Error& e) { std::fprintf(stderr, "%s\n", e.what()); return 111; }
  }
  if (!a.log_json.empty()) {
    FILE* f = a.log_json == "-" ? stdout : std::fopen(a.log_json.c_str(), "w");
    if (f) {
      std::fprintf(f,
                   "{\"program\": \"%s\", \"model\": \"%s\", \"dtype\": \"%s\", \"train_samples\": %lld, "
                   "\"train_s\": %.6f, \"train_img_per_s\": %.3f, \"test_img_per_s\": %.3f, \"ntests\": %lld, "
                   "\"ncorrect\": %lld}\n",
                   program, spec.name.c_str(), sizeof(T) == 8 ? "fp64" : "fp32", (long long)total, train_s,
                   total / std::max(train_s, 1e-9), ntests / std::max(test_s, 1e-9), (long long)ntests,
                   (long long)ncorrect);
      if (f != stdout) std::fclose(f);
    }
  }
  return 0;
}

}  // namespace mcc
