// Model graph description: the MI355X framework's replacement for the
// reference's doubly-linked `struct Layer` list (cnn.c:15-43, Layer_create*
// at cnn.c:60-94 and :316-342).
//
// A model is a flat vector of LayerSpec (input first).  Shapes are inferred
// from the geometry (the reference hard-codes conv output H/W, cnn.c:329 —
// here they are derived and checked).  Parameters of all layers live in ONE
// flat fp32 buffer in layer order: [W0 b0 W1 b1 ...].  That makes the data-
// parallel gradient sync a handful of contiguous buckets instead of the
// reference's per-layer MPI_Allreduce calls (cnnmpi.c:487-498).
//
// Canonical parameter layouts (identical to the reference and to PyTorch):
//   conv weight  [Cout][Cin][KH][KW]   (OIHW, cnn.c:335)
//   fc weight    [out][in]             (cnn.c:320) with `in` in C,H,W order
//   bias         [out]
// The GPU engine keeps packed bf16/fp32 copies in its own (MFMA-friendly)
// orders; the canonical fp32 master copy is what is all-reduced, updated and
// saved.
#pragma once

#include <string>
#include <vector>

#include "mcc/common.h"

namespace mcc {

enum class LayerKind : int { Input = 0, Conv = 1, MaxPool = 2, FC = 3 };
enum class Act : int { None = 0, ReLU = 1, Tanh = 2, Softmax = 3 };

const char* layer_kind_name(LayerKind k);
const char* act_name(Act a);

struct LayerSpec {
  LayerKind kind = LayerKind::Input;
  // Output shape in C,H,W semantics (GPU storage is NHWC).
  int C = 0, H = 1, W = 1;
  // Conv / pool geometry.
  int ks = 0, stride = 1, pad = 0;
  Act act = Act::None;
  double init_std = 0.1;  // reference init: std * nrnd() (cnn.c:49,325)
  // Derived by ModelSpec::finalize().
  int inC = 0, inH = 0, inW = 0;  // input shape
  int64_t w_off = -1, b_off = -1, nweights = 0, nbiases = 0;
  int64_t nnodes() const { return (int64_t)C * H * W; }
  int64_t in_nodes() const { return (int64_t)inC * inH * inW; }
};

struct ModelSpec {
  std::string name;
  std::vector<LayerSpec> layers;
  int64_t nparams = 0;

  // Shape inference, validation and flat parameter offsets.
  void finalize();
  const LayerSpec& input() const { return layers.front(); }
  const LayerSpec& output() const { return layers.back(); }
  int num_classes() const { return layers.back().C; }
  int64_t input_nodes() const { return layers.front().nnodes(); }
  std::string describe() const;
  // Forward MACs per sample (for FLOP accounting in benches).
  int64_t macs_per_sample() const;
};

// Data-parallel gradient buckets.  "Stages" are the parameterised layers in
// order (exactly the GPU engine's fused stages: a max-pool has no parameters
// and is fused into the conv before it).  Buckets walk the stages from the
// LAST one (first to finish in backward) and cut whenever the gradient bytes
// reach `bucket_bytes`; each bucket is a contiguous range of the flat buffer.
// Stage 0 (the last to finish) always gets a bucket of its own, so the big
// collective overlaps its weight-gradient kernel.
struct Bucket {
  int stage_hi = 0, stage_lo = 0;  // inclusive, stage_hi >= stage_lo
  int64_t off = 0, count = 0;      // elements of the flat fp32 gradient
};
std::vector<Bucket> plan_buckets(const ModelSpec& spec, int64_t bucket_bytes);

// Builders used by the model zoo and by the text spec parser.
struct ModelBuilder {
  ModelSpec m;
  explicit ModelBuilder(std::string name, int C, int H, int W);
  ModelBuilder& conv(int cout, int ks, int stride, int pad, Act act, double std = 0.1);
  ModelBuilder& maxpool(int k = 2, int stride = 2);
  ModelBuilder& fc(int out, Act act, double std = 0.1);
  ModelSpec build();
};

// Model zoo.
//   "ref"    : the reference network, cnn.c:416-428
//   "lenet5" : LeNet-5 on 28x28x1 (BASELINE.json headline config)
//   "cifar3" : 3x[conv3x3+ReLU+pool] 3->32->64->128, FC 2048->256->10 (32x32x3)
//   "vgg11"  : VGG-11 (config A) on 224x224x3, FC 25088->4096->4096->1000
ModelSpec make_model(const std::string& name);
std::vector<std::string> model_names();

// Text spec, one layer per line or ';'-separated:
//   input C H W | conv COUT kK sS pP ACT | pool K [S] | fc OUT ACT
ModelSpec parse_model_spec(const std::string& text, const std::string& name = "custom");

}  // namespace mcc
