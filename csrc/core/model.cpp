// Model graph: shape inference, parameter layout, model zoo, spec parser.
// Reference counterpart: Layer_create_input/full/conv (cnn.c:316-342) and the
// hard-coded topology in main (cnn.c:416-428).
#include "mcc/model.h"

#include <sstream>

namespace mcc {

const char* layer_kind_name(LayerKind k) {
  switch (k) {
    case LayerKind::Input: return "input";
    case LayerKind::Conv: return "conv";
    case LayerKind::MaxPool: return "maxpool";
    case LayerKind::FC: return "fc";
  }
  return "?";
}

const char* act_name(Act a) {
  switch (a) {
    case Act::None: return "none";
    case Act::ReLU: return "relu";
    case Act::Tanh: return "tanh";
    case Act::Softmax: return "softmax";
  }
  return "?";
}

void ModelSpec::finalize() {
  MCC_CHECK(!layers.empty() && layers[0].kind == LayerKind::Input, "model must start with an input layer");
  int64_t off = 0;
  for (size_t i = 0; i < layers.size(); ++i) {
    LayerSpec& L = layers[i];
    if (i == 0) {
      MCC_CHECK(L.C > 0 && L.H > 0 && L.W > 0, "bad input shape");
      L.inC = L.C; L.inH = L.H; L.inW = L.W;
      continue;
    }
    const LayerSpec& P = layers[i - 1];
    L.inC = P.C; L.inH = P.H; L.inW = P.W;
    switch (L.kind) {
      case LayerKind::Conv: {
        MCC_CHECK(L.ks > 0 && L.stride > 0 && L.pad >= 0, "bad conv geometry");
        MCC_CHECK(P.kind != LayerKind::FC, "conv after fc is not supported");
        L.H = (L.inH + 2 * L.pad - L.ks) / L.stride + 1;
        L.W = (L.inW + 2 * L.pad - L.ks) / L.stride + 1;
        MCC_CHECK(L.H > 0 && L.W > 0, "conv output is empty");
        L.nweights = (int64_t)L.C * L.inC * L.ks * L.ks;
        L.nbiases = L.C;
        break;
      }
      case LayerKind::MaxPool: {
        MCC_CHECK(L.ks > 0 && L.stride > 0, "bad pool geometry");
        L.C = L.inC;
        L.H = (L.inH - L.ks) / L.stride + 1;  // floor mode (PyTorch default)
        L.W = (L.inW - L.ks) / L.stride + 1;
        MCC_CHECK(L.H > 0 && L.W > 0, "pool output is empty");
        L.nweights = 0;
        L.nbiases = 0;
        break;
      }
      case LayerKind::FC: {
        MCC_CHECK(L.C > 0, "fc needs >0 outputs");
        L.H = 1; L.W = 1;
        L.nweights = (int64_t)L.C * P.nnodes();
        L.nbiases = L.C;
        break;
      }
      default:
        MCC_CHECK(false, "input layer in the middle of a model");
    }
    if (L.nweights > 0) {
      L.w_off = off; off += L.nweights;
      L.b_off = off; off += L.nbiases;
    }
  }
  MCC_CHECK(layers.back().kind == LayerKind::FC && layers.back().act == Act::Softmax,
            "last layer must be fc+softmax (the reference objective, cnn.c:125-143)");
  for (size_t i = 1; i + 1 < layers.size(); ++i)
    MCC_CHECK(layers[i].act != Act::Softmax, "softmax only on the last layer");
  nparams = off;
}

std::string ModelSpec::describe() const {
  std::ostringstream os;
  os << name << " (" << nparams << " params)\n";
  for (size_t i = 0; i < layers.size(); ++i) {
    const LayerSpec& L = layers[i];
    os << "  [" << i << "] " << layer_kind_name(L.kind) << " " << L.C << "x" << L.H << "x" << L.W;
    if (L.kind == LayerKind::Conv) os << " k" << L.ks << " s" << L.stride << " p" << L.pad;
    if (L.kind == LayerKind::MaxPool) os << " k" << L.ks << " s" << L.stride;
    if (L.kind != LayerKind::Input && L.kind != LayerKind::MaxPool) os << " " << act_name(L.act);
    os << "\n";
  }
  return os.str();
}

int64_t ModelSpec::macs_per_sample() const {
  int64_t macs = 0;
  for (const auto& L : layers) {
    if (L.kind == LayerKind::Conv) macs += L.nnodes() * L.inC * L.ks * L.ks;
    if (L.kind == LayerKind::FC) macs += L.nweights;
  }
  return macs;
}

std::vector<Bucket> plan_buckets(const ModelSpec& spec, int64_t bucket_bytes) {
  std::vector<const LayerSpec*> stages;
  for (const auto& L : spec.layers)
    if (L.nweights > 0) stages.push_back(&L);
  std::vector<Bucket> out;
  Bucket cur;
  bool open = false;
  for (int s = (int)stages.size() - 1; s >= 0; --s) {
    const LayerSpec& L = *stages[s];
    if (!open) { cur = Bucket(); cur.stage_hi = s; open = true; }
    cur.stage_lo = s;
    cur.count += L.nweights + L.nbiases;
    cur.off = L.w_off;
    // Stage 0 finishes LAST in backward, so whatever shares its bucket waits
    // for it and only the final collective is exposed: cut before it so the
    // rest of the gradient is reduced while stage 0's dW kernel runs and the
    // exposed tail is one small (latency-bound) all-reduce.
    if (cur.count * 4 >= bucket_bytes || s <= 1) {
      out.push_back(cur);
      open = false;
    }
  }
  return out;
}

ModelBuilder::ModelBuilder(std::string name, int C, int H, int W) {
  m.name = std::move(name);
  LayerSpec in;
  in.kind = LayerKind::Input;
  in.C = C; in.H = H; in.W = W;
  m.layers.push_back(in);
}

ModelBuilder& ModelBuilder::conv(int cout, int ks, int stride, int pad, Act act, double std) {
  LayerSpec L;
  L.kind = LayerKind::Conv;
  L.C = cout; L.ks = ks; L.stride = stride; L.pad = pad; L.act = act; L.init_std = std;
  m.layers.push_back(L);
  return *this;
}

ModelBuilder& ModelBuilder::maxpool(int k, int stride) {
  LayerSpec L;
  L.kind = LayerKind::MaxPool;
  L.ks = k; L.stride = stride;
  m.layers.push_back(L);
  return *this;
}

ModelBuilder& ModelBuilder::fc(int out, Act act, double std) {
  LayerSpec L;
  L.kind = LayerKind::FC;
  L.C = out; L.act = act; L.init_std = std;
  m.layers.push_back(L);
  return *this;
}

ModelSpec ModelBuilder::build() {
  m.finalize();
  return m;
}

std::vector<std::string> model_names() { return {"ref", "lenet5", "cifar3", "vgg11"}; }

ModelSpec make_model(const std::string& name) {
  if (name == "ref") {
    // cnn.c:416-428: conv(1->16,3x3,s2,p1)+ReLU, conv(16->32,3x3,s2,p1)+ReLU,
    // fc 1568->200 tanh, fc 200->200 tanh, fc 200->10 softmax; std 0.1.
    return ModelBuilder("ref", 1, 28, 28)
        .conv(16, 3, 2, 1, Act::ReLU)
        .conv(32, 3, 2, 1, Act::ReLU)
        .fc(200, Act::Tanh)
        .fc(200, Act::Tanh)
        .fc(10, Act::Softmax)
        .build();
  }
  if (name == "lenet5") {
    // LeNet-5 for 28x28 MNIST (padding 2 on conv1 keeps the classic 32x32
    // receptive geometry): 6x28x28 -> pool 6x14x14 -> 16x10x10 -> pool 16x5x5
    // -> fc 400->120->84->10.  Init std scaled by fan-in (He) so it trains.
    return ModelBuilder("lenet5", 1, 28, 28)
        .conv(6, 5, 1, 2, Act::ReLU, 0.0)
        .maxpool(2, 2)
        .conv(16, 5, 1, 0, Act::ReLU, 0.0)
        .maxpool(2, 2)
        .fc(120, Act::ReLU, 0.0)
        .fc(84, Act::ReLU, 0.0)
        .fc(10, Act::Softmax, 0.0)
        .build();
  }
  if (name == "cifar3") {
    return ModelBuilder("cifar3", 3, 32, 32)
        .conv(32, 3, 1, 1, Act::ReLU, 0.0).maxpool(2, 2)
        .conv(64, 3, 1, 1, Act::ReLU, 0.0).maxpool(2, 2)
        .conv(128, 3, 1, 1, Act::ReLU, 0.0).maxpool(2, 2)
        .fc(256, Act::ReLU, 0.0)
        .fc(10, Act::Softmax, 0.0)
        .build();
  }
  if (name == "vgg11") {
    // VGG-11 (Simonyan & Zisserman config A) on 224x224x3.
    return ModelBuilder("vgg11", 3, 224, 224)
        .conv(64, 3, 1, 1, Act::ReLU, 0.0).maxpool(2, 2)
        .conv(128, 3, 1, 1, Act::ReLU, 0.0).maxpool(2, 2)
        .conv(256, 3, 1, 1, Act::ReLU, 0.0)
        .conv(256, 3, 1, 1, Act::ReLU, 0.0).maxpool(2, 2)
        .conv(512, 3, 1, 1, Act::ReLU, 0.0)
        .conv(512, 3, 1, 1, Act::ReLU, 0.0).maxpool(2, 2)
        .conv(512, 3, 1, 1, Act::ReLU, 0.0)
        .conv(512, 3, 1, 1, Act::ReLU, 0.0).maxpool(2, 2)
        .fc(4096, Act::ReLU, 0.0)
        .fc(4096, Act::ReLU, 0.0)
        .fc(1000, Act::Softmax, 0.0)
        .build();
  }
  throw Error("unknown model '" + name + "' (known: ref, lenet5, cifar3, vgg11)");
}

static Act parse_act(const std::string& s) {
  if (s == "relu") return Act::ReLU;
  if (s == "tanh") return Act::Tanh;
  if (s == "softmax") return Act::Softmax;
  if (s == "none" || s == "linear") return Act::None;
  throw Error("unknown activation '" + s + "'");
}

ModelSpec parse_model_spec(const std::string& text, const std::string& name) {
  std::string t = text;
  for (char& ch : t)
    if (ch == ';') ch = '\n';
  std::istringstream lines(t);
  std::string line;
  bool have_input = false;
  ModelBuilder* b = nullptr;
  ModelBuilder storage(name, 1, 1, 1);
  while (std::getline(lines, line)) {
    std::istringstream ls(line);
    std::string kw;
    if (!(ls >> kw) || kw[0] == '#') continue;
    if (kw == "input") {
      int C, H, W;
      MCC_CHECK(bool(ls >> C >> H >> W), "input C H W");
      storage = ModelBuilder(name, C, H, W);
      b = &storage;
      have_input = true;
      continue;
    }
    MCC_CHECK(have_input, "spec must start with 'input C H W'");
    if (kw == "conv") {
      int cout = 0, k = 3, s = 1, p = 0;
      Act act = Act::ReLU;
      MCC_CHECK(bool(ls >> cout), "conv COUT");
      std::string tok;
      while (ls >> tok) {
        if (tok[0] == 'k') k = std::stoi(tok.substr(1));
        else if (tok[0] == 's') s = std::stoi(tok.substr(1));
        else if (tok[0] == 'p') p = std::stoi(tok.substr(1));
        else act = parse_act(tok);
      }
      b->conv(cout, k, s, p, act, 0.0);
    } else if (kw == "pool" || kw == "maxpool") {
      int k = 2, s = -1;
      ls >> k;
      if (!(ls >> s)) s = k;
      b->maxpool(k, s);
    } else if (kw == "fc") {
      int out = 0;
      std::string a = "relu";
      MCC_CHECK(bool(ls >> out), "fc OUT");
      ls >> a;
      b->fc(out, parse_act(a), 0.0);
    } else {
      throw Error("unknown layer keyword '" + kw + "'");
    }
  }
  MCC_CHECK(b != nullptr, "empty model spec");
  return b->build();
}

}  // namespace mcc
