// IDX + weight-file I/O and the synthetic data generator (see mcc/io.h).
#include "mcc/io.h"

#include <algorithm>
#include <cstring>
#include <fstream>
#include <memory>

namespace mcc {

static uint32_t be32(const uint8_t* p) {
  return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | (uint32_t)p[3];
}

IdxFile idx_read(const std::string& path) {
  std::unique_ptr<FILE, int (*)(FILE*)> fp(fopen(path.c_str(), "rb"), fclose);
  if (!fp) throw Error("cannot open IDX file '" + path + "'");
  uint8_t hdr[4];
  if (fread(hdr, 1, 4, fp.get()) != 4) throw Error("short IDX header in '" + path + "'");
  // {u16 magic == 0, u8 type == 0x08, u8 ndims}  (cnn.c:355-363)
  if (hdr[0] != 0 || hdr[1] != 0) throw Error("bad IDX magic in '" + path + "'");
  if (hdr[2] != 0x08) throw Error("IDX type is not unsigned byte in '" + path + "'");
  if (hdr[3] < 1) throw Error("IDX ndims < 1 in '" + path + "'");
  IdxFile f;
  f.dims.resize(hdr[3]);
  std::vector<uint8_t> raw(4 * (size_t)hdr[3]);
  if (fread(raw.data(), 1, raw.size(), fp.get()) != raw.size()) throw Error("short IDX dims in '" + path + "'");
  uint64_t nbytes = 1;
  for (int i = 0; i < hdr[3]; ++i) {
    f.dims[i] = be32(&raw[4 * i]);
    nbytes *= f.dims[i];
  }
  f.data.resize(nbytes);
  if (nbytes && fread(f.data.data(), 1, nbytes, fp.get()) != nbytes)
    throw Error("short IDX payload in '" + path + "'");
  return f;
}

void check_labels(const IdxFile& labels, int64_t n, int num_classes, const std::string& what) {
  n = std::min<int64_t>(n, (int64_t)labels.data.size());
  for (int64_t i = 0; i < n; ++i)
    if (labels.data[i] >= num_classes)
      throw Error(what + ": label " + std::to_string((int)labels.data[i]) + " at index " + std::to_string(i) +
                  " is not a class of the model (" + std::to_string(num_classes) + " classes)");
}

void idx_write(const std::string& path, const std::vector<uint32_t>& dims, const uint8_t* data) {
  std::unique_ptr<FILE, int (*)(FILE*)> fp(fopen(path.c_str(), "wb"), fclose);
  if (!fp) throw Error("cannot create IDX file '" + path + "'");
  uint8_t hdr[4] = {0, 0, 0x08, (uint8_t)dims.size()};
  fwrite(hdr, 1, 4, fp.get());
  uint64_t nbytes = 1;
  for (uint32_t d : dims) {
    uint8_t b[4] = {(uint8_t)(d >> 24), (uint8_t)(d >> 16), (uint8_t)(d >> 8), (uint8_t)d};
    fwrite(b, 1, 4, fp.get());
    nbytes *= d;
  }
  if (nbytes && fwrite(data, 1, nbytes, fp.get()) != nbytes) throw Error("short write to '" + path + "'");
}

static inline uint64_t mix(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

void synth_dataset(int64_t N, int C, int H, int W, int num_classes, uint64_t seed,
                   std::vector<uint8_t>& images, std::vector<uint8_t>& labels) {
  images.resize((size_t)N * C * H * W);
  labels.resize(N);
  const int bands = num_classes;
  for (int64_t n = 0; n < N; ++n) {
    uint64_t s = mix(seed * 0x9E3779B97F4A7C15ull + (uint64_t)n);
    const int label = (int)(s % (uint64_t)num_classes);
    labels[n] = (uint8_t)label;
    // stripe rows: for 28x28 and 10 classes, rows 2+2l .. 3+2l
    const double scale = (double)H / 28.0;
    int r0 = (int)((2 + 2 * (label % 10)) * scale);
    int r1 = (int)((4 + 2 * (label % 10)) * scale);
    if (bands > 10) {  // more classes than stripes: add a column band
      r0 = (int)((double)(label % 10) * H / 10.0);
      r1 = r0 + std::max(1, H / 14);
    }
    const int cband = bands > 10 ? (label / 10) % std::max(1, W / 4) : -1;
    uint8_t* img = images.data() + (size_t)n * C * H * W;
    uint64_t r = s;
    for (int y = 0; y < H; ++y)
      for (int x = 0; x < W; ++x)
        for (int c = 0; c < C; ++c) {
          r = mix(r);
          int v = (int)(r % 40);
          bool on = (y >= r0 && y < r1);
          if (cband >= 0) on = on && (x / 4 == cband || x / 4 == cband + 1);
          if (on) v = 220;
          img[((size_t)y * W + x) * C + c] = (uint8_t)v;
        }
  }
}

// ------------------------------------------------------------ weights ----

static const char kMagic[8] = {'M', 'C', 'N', 'N', 'W', 0, 0, 0};
static const uint32_t kByteOrder = 0x01020304u;

static int32_t ref_ltype(LayerKind k) {
  switch (k) {
    case LayerKind::Input: return 0;
    case LayerKind::FC: return 1;
    case LayerKind::Conv: return 2;
    case LayerKind::MaxPool: return 3;
  }
  return -1;
}

void save_weights(const std::string& path, const ModelSpec& spec, const double* params) {
  std::ofstream os(path, std::ios::binary);
  if (!os) throw Error("cannot create weight file '" + path + "'");
  auto w32 = [&](int32_t v) { os.write(reinterpret_cast<const char*>(&v), 4); };
  auto w64 = [&](int64_t v) { os.write(reinterpret_cast<const char*>(&v), 8); };
  os.write(kMagic, 8);
  w32(2);
  w32((int32_t)kByteOrder);
  w32((int32_t)spec.layers.size());
  w64(spec.nparams);
  for (const auto& L : spec.layers) {
    w32(ref_ltype(L.kind));
    w32(L.C); w32(L.W); w32(L.H);
    w32(L.ks); w32(L.pad); w32(L.stride); w32((int32_t)L.act);
    w64(L.nbiases); w64(L.nweights);
  }
  for (const auto& L : spec.layers) {
    if (L.nbiases) os.write(reinterpret_cast<const char*>(params + L.b_off), 8 * L.nbiases);
    if (L.nweights) os.write(reinterpret_cast<const char*>(params + L.w_off), 8 * L.nweights);
  }
  if (!os) throw Error("write failed for '" + path + "'");
}

ModelSpec load_weights(const std::string& path, std::vector<double>& params) {
  std::ifstream is(path, std::ios::binary);
  if (!is) throw Error("cannot open weight file '" + path + "'");
  char magic[8];
  is.read(magic, 8);
  if (!is || std::memcmp(magic, kMagic, 8) != 0) throw Error("not an MCNNW weight file: '" + path + "'");
  auto r32 = [&]() { int32_t v; is.read(reinterpret_cast<char*>(&v), 4); return v; };
  auto r64 = [&]() { int64_t v; is.read(reinterpret_cast<char*>(&v), 8); return v; };
  const int32_t version = r32();
  if (version == 0x02000000 || version == 0x01000000) throw Error("big-endian MCNNW file: '" + path + "'");
  if (version != 1 && version != 2) throw Error("unsupported MCNNW version");
  if (version >= 2 && (uint32_t)r32() != kByteOrder) throw Error("bad MCNNW byte-order mark in '" + path + "'");
  const int32_t nl = r32();
  const int64_t np = r64();
  if (!is || nl < 2 || nl > 4096) throw Error("corrupt MCNNW header");
  ModelSpec spec;
  spec.name = "loaded";
  std::vector<int64_t> stored_nb, stored_nw;
  std::vector<int32_t> stored_shape;
  for (int i = 0; i < nl; ++i) {
    LayerSpec L;
    const int32_t t = r32();
    L.C = r32(); L.W = r32(); L.H = r32();
    L.ks = r32(); L.pad = r32(); L.stride = r32();
    const int32_t act = r32();
    if (act < (int32_t)Act::None || act > (int32_t)Act::Softmax) throw Error("corrupt MCNNW activation");
    L.act = (Act)act;
    stored_shape.insert(stored_shape.end(), {L.C, L.W, L.H});
    stored_nb.push_back(r64());
    stored_nw.push_back(r64());
    if (L.C < 1 || L.W < 1 || L.H < 1 || L.C > (1 << 20) || L.W > (1 << 16) || L.H > (1 << 16))
      throw Error("corrupt MCNNW layer shape");
    switch (t) {
      case 0: L.kind = LayerKind::Input; break;
      case 1: L.kind = LayerKind::FC; break;
      case 2: L.kind = LayerKind::Conv; break;
      case 3: L.kind = LayerKind::MaxPool; break;
      default: throw Error("corrupt MCNNW layer type");
    }
    spec.layers.push_back(L);
  }
  if (!is) throw Error("truncated MCNNW layer table");
  spec.finalize();
  if (spec.nparams != np) throw Error("MCNNW parameter count mismatch");
  for (int i = 0; i < nl; ++i)
    if (spec.layers[i].nbiases != stored_nb[i] || spec.layers[i].nweights != stored_nw[i] ||
        spec.layers[i].C != stored_shape[3 * i] || spec.layers[i].W != stored_shape[3 * i + 1] ||
        spec.layers[i].H != stored_shape[3 * i + 2])
      throw Error("MCNNW layer " + std::to_string(i) + ": stored shape / parameter counts do not match its geometry");
  params.assign(np, 0.0);
  for (const auto& L : spec.layers) {
    if (L.nbiases) is.read(reinterpret_cast<char*>(params.data() + L.b_off), 8 * L.nbiases);
    if (L.nweights) is.read(reinterpret_cast<char*>(params.data() + L.w_off), 8 * L.nweights);
  }
  if (!is) throw Error("truncated MCNNW payload");
  if (is.peek() != std::char_traits<char>::eof()) throw Error("trailing bytes after the MCNNW payload");
  return spec;
}

}  // namespace mcc
