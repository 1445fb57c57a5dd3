// GpuNet implementation: model lowering, arena, packing tables, schedule.
#include "mcc/engine.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <sstream>

#include "kernels.h"
#include "mcc/ab.h"

#include <cstdlib>

namespace mcc {

#define HIP_OK(expr)                                                                                    \
  do {                                                                                                  \
    hipError_t _e = (expr);                                                                             \
    if (_e != hipSuccess)                                                                               \
      throw Error(std::string("HIP error: ") + hipGetErrorString(_e) + " at " + __FILE__ + ":" +        \
                  std::to_string(__LINE__));                                                            \
  } while (0)

struct GpuNet::Stage {
  enum Kind { CONV, FC } kind = CONV;
  int li = 0;            // spec layer index of the conv / fc layer
  bool pooled = false;   // fused 2x2/2 maxpool
  int act = gpu::ACT_NONE;
  bool last = false;
  bool head = false;  // last FC: backward fused into the loss kernel (xent_head)
  bool cvec = true;      // conv input gathered in 8-channel vectors
  int inC = 0, inH = 1, inW = 1;
  int C = 0, OH = 1, OW = 1;   // conv grid (pre-pool)
  int outH = 1, outW = 1;      // stage output spatial (pooled)
  int64_t in_elems = 0, out_elems = 0;  // per-sample NHWC elements
  int in_ld = 0, out_ld = 0;   // FC row strides (elements)
  int KS = 1, stride = 1, pad = 0;
  int64_t w_off = 0, b_off = 0, nw = 0, nb = 0;
  // buffers
  void* act_buf = nullptr;
  uint8_t* arg_buf = nullptr;
  void* grad_buf = nullptr;
  // packed weight offsets (elements into packed_)
  int64_t pk_fwd = -1, pk_dx = -1;
  // conv geometry
  int CL = 0, nchunks = 0, kpad = 0;        // forward
  int CLd = 0, nchunks_d = 0, kpad_d = 0;   // data-gradient (transposed) form
  bool cvec_d = true;
  int imgs_fwd = 1, imgs_dx = 1, imgs_dw = 1, ppad = 32, kbias = 0, ncols_pad = 16, cout_pad = 16;
  int CLdw = 0;  // channel stride of the weight-gradient column layout
  int nx_dw = 1;  // dW workgroup columns (each reduces a strided subset of image groups)
  // fc geometry
  int Kin = 0, Nout = 0, permC = 0, permHW = 0, ldp = 0;
  // large-image conv (explicit im2col + MFMA GEMM) when the image tile does
  // not fit the whole-image LDS kernels
  bool big = false;
  bool dz_fused = false;  // big ReLU stage whose dZ the next stage's dX epilogue writes
  bool generic = false;  // tanh conv / pool after a non-ReLU conv / non-2x2 pool: im2col or igemm path + grad_xform
  int pk = 2, ps = 2;    // pooled: window / stride
  int kgem = 0, kgem_d = 0;      // im2col row strides (fwd/dW, data grad)
  // implicit-GEMM kernels (igemm.hip) per direction of a large-image conv;
  // the explicit im2col + GEMM path remains for what they do not cover
  // (the u8 input layer, C % 64 != 0, strided data gradients, fp32)
  bool ig_fwd = false, ig_dw = false, ig_dx = false;
  bool ig_dw0 = false;  // stage 0: im2col rows through the implicit-GEMM dW kernel
  bool c0dw = false;    // stage 0, pooled 3x3: dW straight from pooled dY / argmax (conv0_dw.hip)
  gpu::Conv0DwParams pc0;
  bool ig_pool = false; // forward max-pool fused into the implicit-GEMM epilogue
  // large FC layers (VGG heads): no W^T shadow (the data gradient reads the
  // forward copy K-major) and the weight gradient on the implicit-GEMM dW
  // kernel as a 1x1 "conv" over the batch
  bool fc_big = false, fc_igdw = false;
  // wide FC at a large batch (CIFAR-3conv FC1 2048 -> 256, ref FC1
  // 1568 -> 200): forward / data gradient as a 1x1 implicit-GEMM "conv" over
  // the batch (igemm.hip) instead of the generic tiled GEMM
  bool fc_ig = false, fc_igdx = false;
  // ... narrow enough (Nout <= 224) for one tile row of the tall-skinny FC
  // kernel (fc_tall.hip: ref FC1 1568 -> 200), forward / data gradient
  bool fc_tall = false, fc_tall_dx = false;
  // ... short reduction (K <= 224): the data gradient on the W-resident
  // kernel (fc_wres.hip), x act' of an FC predecessor (wres_act)
  bool fc_wres = false;
  int wres_act = 0;
  void* conv_buf = nullptr;      // pre-pool conv output (big + pooled)
  void* dz_buf = nullptr;        // pre-activation gradient at conv-output size (big)
  // persistent pipelined kernels (bf16 small-image layers; geometry planned
  // for max_batch, pointers and batch filled per call)
  bool pipe_fwd = false, pipe_dx = false, pipe_dw = false;
  gpu::ConvPipeParams pf, pdx;
  gpu::ConvDwPipeParams pdw;
  // single-channel first layer: row-chunked weight gradient (conv_rows.hip)
  bool rows_dw = false;
  gpu::ConvDwRowsParams prw;
  // fp32 small pooled convs: direct VALU kernels (conv_direct.hip) for the
  // forward (direct_fwd), the weight gradient (direct1: single-channel first
  // layer; direct_dw: the 6 -> 16 conv) and the data gradient (direct_dx)
  bool direct_fwd = false, direct1 = false, direct_dx = false, direct_dw = false;
  gpu::Conv1DirectParams pd1;
  // u8 RGB first layer (3x3 pad 1, ReLU, 2x2 pool), bf16: row-worker forward (conv_u8.hip)
  bool u8fwd = false;
  bool c2k = false;  // CIFAR-3conv conv2 kernels (cifar_c2.hip)
  bool c2bwd = false;  // ... and their backward (dX / dW from the pooled dY + argmax)
  bool c3k = false;  // CIFAR-3conv conv3 kernels (cifar_c3.hip): forward, dX, dW (no grad_xform)
};

static inline int r8(int x) { return (x + 7) & ~7; }
static inline int r16(int x) { return (x + 15) & ~15; }
static inline int r32(int x) { return (x + 31) & ~31; }
// Split-K factor for a weight-gradient GEMM [M x N] reduced over K rows:
// aim for ~512 workgroups of 64x64 tiles, each slice >= 128 rows.
static inline int dw_splitk(int M, int N, int64_t K, int target = 512) {
  const int64_t tiles = ceil_div(M, 64) * ceil_div(N, 64);
  int64_t sk = std::max<int64_t>(1, std::min<int64_t>(target / std::max<int64_t>(1, tiles), K / 64));
  return (int)std::min<int64_t>(sk, 256);
}
// FC weight gradients on the generic GEMM: fp32 aims at ~5 workgroups per CU
// (its one-chunk register prefetch leaves each workgroup latency-bound)
static inline int fc_dw_splitk(int M, int N, int64_t K, DType t) {
  return dw_splitk(M, N, K, t == DType::F32 ? 1280 : 512);
}

static inline int act_kind(Act a) {
  switch (a) {
    case Act::ReLU: return gpu::ACT_RELU;
    case Act::Tanh: return gpu::ACT_TANH;
    default: return gpu::ACT_NONE;
  }
}

GpuNet::GpuNet(const ModelSpec& spec, DType dtype, int max_batch, int device)
    : spec_(spec), dtype_(dtype), max_batch_(max_batch), device_(device) {
  MCC_CHECK(dtype == DType::BF16 || dtype == DType::F32, "GpuNet: dtype must be bf16 or fp32");
  MCC_CHECK(max_batch > 0, "GpuNet: max_batch > 0");
  // Kernels index activations with 32-bit element offsets; channel counts are
  // padded up to 16 in the packed layouts, so bound the padded tensor size.
  for (const LayerSpec& l : spec.layers)
    MCC_CHECK((int64_t)max_batch * ((l.C + 15) / 16 * 16) * l.H * l.W < (1ll << 31),
              "GpuNet: max_batch too large for 32-bit activation indexing");
  // A/B switches (mcc/ab.h, MCC_AB=...)
  no_igemm_ = ab_flag("no_igemm");       // im2col + GEMM instead of the implicit GEMM
  // dW side stream: opt-in (MCC_AB=side_stream).  Measured on MI355X (one GPU,
  // bench.py): CIFAR-3conv 2.27 -> 2.17 ms/step, but LeNet-5 0.452 -> 0.502 and
  // VGG-11 12.14 -> 12.40: the persistent conv kernels are sized to own every
  // CU, so a concurrent dW kernel steals their slots and stretches both.
  no_side_ = !ab_flag("side_stream");
  if (device_ >= 0) HIP_OK(hipSetDevice(device_));
  else HIP_OK(hipGetDevice(&device_));
  build();
  if (!no_side_) {
    HIP_OK(hipStreamCreateWithFlags(&wstream_, hipStreamNonBlocking));
    fork_ev_.resize(stages_.size());
    for (auto& e : fork_ev_) HIP_OK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    HIP_OK(hipEventCreateWithFlags(&join_ev_, hipEventDisableTiming));
  }
}

GpuNet::~GpuNet() {
  for (auto e : fork_ev_) (void)hipEventDestroy(e);
  if (join_ev_) (void)hipEventDestroy(join_ev_);
  if (wstream_) (void)hipStreamDestroy(wstream_);
  for (Stage* st : stages_) delete st;
  if (arena_) (void)hipFree(arena_);
  if (mom_) (void)hipFree(mom_);
}

void* GpuNet::arena_alloc(size_t bytes) {
  const size_t a = (arena_used_ + 255) & ~size_t(255);
  arena_used_ = a + bytes;
  return arena_ ? arena_ + a : reinterpret_cast<void*>(a + 1);  // sizing pass returns dummies
}

// Plan the persistent pipelined kernels for a small-image bf16 conv stage.
// Each direction falls back to conv_small when the planner declines it.
void GpuNet::plan_pipe(Stage& st, bool first) {
  const int dy_mode = st.pooled ? gpu::PM_UNPOOL : (st.act == gpu::ACT_RELU ? gpu::PM_RELU : gpu::PM_PLAIN);
  const int dyH = st.pooled ? st.outH : st.OH, dyW = st.pooled ? st.outW : st.OW;
  const bool x_ok = first ? st.inC == 1 : true;
  const int x_mode = first ? gpu::PM_U8S1 : gpu::PM_PLAIN;
  if (x_ok && (st.inC == 1 || st.cvec)) {
    gpu::ConvPipeParams& p = st.pf;
    p.N = max_batch_; p.Cin = st.inC; p.OH = st.OH; p.OW = st.OW; p.cs = st.stride; p.KS = st.KS; p.Cout = st.C;
    p.epi = st.pooled ? 0 : 1; p.act = st.act;
    p.in.mode = x_mode; p.in.SH = st.inH; p.in.SW = st.inW; p.in.SC = st.inC;
    p.in.up = 1; p.in.offy = st.pad; p.in.offx = st.pad;
    st.pipe_fwd = gpu::conv_pipe_plan(p);
    // the C8 layout is conv_small's cvec packing; S1 has its own (see pack table)
    if (st.pipe_fwd && p.layout == gpu::XL_C8)
      st.pipe_fwd = st.cvec && st.CL == ((st.inC + 7) & ~7) && st.nchunks == p.nchunks;
  }
  if (!first && st.cvec_d) {
    gpu::ConvPipeParams& p = st.pdx;
    p.N = max_batch_; p.Cin = st.C; p.OH = st.inH; p.OW = st.inW; p.cs = 1; p.KS = st.KS; p.Cout = st.inC;
    p.epi = 2; p.act = gpu::ACT_NONE;
    p.in.mode = dy_mode; p.in.SH = dyH; p.in.SW = dyW; p.in.SC = st.C;
    p.in.up = st.stride; p.in.offy = st.KS - 1 - st.pad; p.in.offx = st.KS - 1 - st.pad;
    st.pipe_dx = gpu::conv_pipe_plan(p) && p.layout == gpu::XL_C8 && st.CLd == ((st.C + 7) & ~7) &&
                 st.nchunks_d == p.nchunks;
  }
  if (first && st.inC == 1) {
    gpu::ConvDwRowsParams& p = st.prw;
    p.N = max_batch_; p.SH = st.inH; p.SW = st.inW; p.OH = st.OH; p.OW = st.OW; p.KS = st.KS; p.pad = st.pad;
    p.Cout = st.C;
    p.dmode = st.pooled ? gpu::PM_UNPOOL : gpu::PM_RELU;
    p.DH = dyH; p.DW = dyW;
    st.rows_dw = st.stride == 1 && (st.pooled || st.act == gpu::ACT_RELU) && gpu::conv_dw_rows_plan(p);
  }
  if (x_ok && !st.rows_dw) {
    gpu::ConvDwPipeParams& p = st.pdw;
    p.N = max_batch_; p.Cin = st.inC; p.OH = st.OH; p.OW = st.OW; p.cs = st.stride; p.KS = st.KS; p.Cout = st.C;
    p.x.mode = x_mode; p.x.SH = st.inH; p.x.SW = st.inW; p.x.SC = st.inC;
    p.x.up = 1; p.x.offy = st.pad; p.x.offx = st.pad;
    p.dy.mode = dy_mode; p.dy.SH = dyH; p.dy.SW = dyW; p.dy.SC = st.C;
    st.pipe_dw = gpu::conv_dw_pipe_plan(p);
  }
}

void GpuNet::build() {
  const size_t es = dtype_size(dtype_);
  // ---- lower the layer list into fused stages ----
  const auto& L = spec_.layers;
  for (size_t i = 1; i < L.size(); ++i) {
    const LayerSpec& l = L[i];
    Stage* st = new Stage();
    st->li = (int)i;
    st->act = act_kind(l.act);
    st->inC = l.inC; st->inH = l.inH; st->inW = l.inW;
    st->w_off = l.w_off; st->b_off = l.b_off; st->nw = l.nweights; st->nb = l.nbiases;
    if (l.kind == LayerKind::Conv) {
      st->kind = Stage::CONV;
      st->C = l.C; st->OH = l.H; st->OW = l.W;
      st->KS = l.ks; st->stride = l.stride; st->pad = l.pad;
      st->outH = l.H; st->outW = l.W;
      MCC_CHECK(l.act == Act::ReLU || l.act == Act::None || l.act == Act::Tanh,
                "GPU conv supports relu/tanh/none activations");
      // the pipelined / whole-image kernels fold the ReLU mask into their
      // staging; tanh convs and pools after a non-ReLU conv take the
      // implicit-GEMM / im2col path, whose separate grad_xform pass applies
      // act' (and the unpool) for any activation
      st->generic = l.act != Act::ReLU && !(l.act == Act::None && !(i + 1 < L.size() && L[i + 1].kind == LayerKind::MaxPool));
      if (i + 1 < L.size() && L[i + 1].kind == LayerKind::MaxPool) {
        const LayerSpec& pl = L[i + 1];
        MCC_CHECK(pl.ks <= 15, "GPU engine: max-pool windows up to 15x15");
        st->pooled = true;
        st->pk = pl.ks; st->ps = pl.stride;
        if (pl.ks != 2 || pl.stride != 2) st->generic = true;  // standalone k x k / s pool + gather unpool
        st->outH = pl.H; st->outW = pl.W;
        ++i;
      }
    } else if (l.kind == LayerKind::FC) {
      st->kind = Stage::FC;
      st->C = l.C;
      st->Nout = l.C;
      st->Kin = (int)l.in_nodes();
      if (l.inH * l.inW > 1) { st->permC = l.inC; st->permHW = l.inH * l.inW; }
    } else {
      delete st;
      throw Error("GPU engine: max-pool must directly follow a conv");
    }
    stages_.push_back(st);
  }
  MCC_CHECK(!stages_.empty() && stages_[0]->kind == Stage::CONV, "GPU engine: first layer must be a conv");
  stages_.back()->last = true;
  MCC_CHECK(stages_.back()->kind == Stage::FC, "GPU engine: last stage must be fc+softmax");

  // ---- per-stage geometry ----
  for (size_t s = 0; s < stages_.size(); ++s) {
    Stage& st = *stages_[s];
    st.in_elems = (int64_t)st.inC * st.inH * st.inW;
    if (st.kind == Stage::CONV) {
      st.out_elems = (int64_t)st.C * st.outH * st.outW;
      st.cvec = st.inC >= 4;
      st.CL = st.cvec ? r8(st.inC) : st.inC;
      const int KK = st.KS * st.KS;
      st.nchunks = st.cvec ? (int)ceil_div((int64_t)KK * (st.CL / 8), 4) : (int)ceil_div((int64_t)KK * st.inC, 32);
      st.kpad = st.nchunks * 32;
      st.cvec_d = st.C >= 4;
      st.CLd = st.cvec_d ? r8(st.C) : st.C;
      st.nchunks_d = st.cvec_d ? (int)ceil_div((int64_t)KK * (st.CLd / 8), 4) : (int)ceil_div((int64_t)KK * st.C, 32);
      st.kpad_d = st.nchunks_d * 32;
      const int LH = (st.OH - 1) * st.stride + st.KS, LW = (st.OW - 1) * st.stride + st.KS;
      const int img_b = LH * LW * st.CL * (int)es;
      st.imgs_fwd = std::max(1, std::min(16, 40960 / img_b));
      const int LHd = st.inH + st.KS - 1, LWd = st.inW + st.KS - 1;
      st.imgs_dx = std::max(1, std::min(16, 40960 / (LHd * LWd * st.CLd * (int)es)));
      st.cout_pad = r16(st.C);
      int dw_img_b;
      if (dtype_ == DType::BF16) {
        // transpose-read dW kernel: channels padded to 4, columns (tap, c4),
        // bias gradient in its own column after the 16-aligned K columns
        st.CLdw = (st.inC + 3) & ~3;
        st.kbias = r16(KK * st.CLdw);
        st.ncols_pad = st.kbias + 16;
        dw_img_b = LH * LW * st.CLdw * (int)es + gpu::conv_dw_tr_drow(st.cout_pad) * st.OH * st.OW * (int)es;
      } else {
        st.CLdw = st.CL;
        st.kbias = KK * st.CL;
        st.ncols_pad = r16(st.kbias + 1);
        dw_img_b = img_b + st.cout_pad * st.OH * st.OW * (int)es;
      }
      st.imgs_dw = std::max(1, std::min(16, 65536 / dw_img_b));
      st.ppad = r32(st.imgs_dw * st.OH * st.OW);
      // enough workgroups for ~4 per CU on 256 CUs (the dW kernel is latency
      // bound on its staging loads); fewer when a batch has fewer groups
      st.nx_dw = (int)std::min<int64_t>(ceil_div(max_batch_, st.imgs_dw), dtype_ == DType::BF16 ? 1024 : 512);
      // whole-image LDS kernels if one image fits comfortably; else im2col + GEMM
      const int64_t lds_cap = 120 * 1024;
      st.big = st.OH * st.OW > 4096 || st.cout_pad > 128 || (int64_t)img_b > lds_cap ||
               (int64_t)LHd * LWd * st.CLd * (int64_t)es > lds_cap || (int64_t)dw_img_b > lds_cap || st.generic;
      MCC_CHECK(!st.generic || st.C % 8 == 0, "GPU engine: tanh convs / pools after a non-ReLU conv need Cout % 8 == 0");
      // small images with wide channels (C % 64, Cout % 8, stride 1) go to the
      // 128x128 / 256-tile MFMA kernels (the whole-image LDS kernels
      // measured slower there).  CIFAR-3conv conv3 (64 -> 128): 3.91 -> 4.32 M img/s; conv2
      // (32 -> 64) measured slower on igemm (3.83 M), so C % 64 only.
      const int ig_cmod = ab_flag("ig32") ? 32 : 64;
      if (!st.big && s > 0 && dtype_ == DType::BF16 && !no_igemm_ && st.stride == 1 &&
          st.inC % ig_cmod == 0 && st.C % 64 == 0 &&
          gpu::igemm_conv_supported(st.inC, st.C, st.KS) && gpu::igemm_conv_supported(st.C, st.inC, st.KS))
        st.big = true;
      st.kgem = r8(KK * st.inC);
      st.kgem_d = r8(KK * st.C);
      if (st.big) MCC_CHECK(st.C % 8 == 0, "im2col conv path needs Cout % 8 == 0");
      st.ig_dw0 = st.big && dtype_ == DType::BF16 && !no_igemm_ && s == 0 && st.C % 8 == 0 &&
                  (int64_t)max_batch_ * st.OH * st.OW < (1ll << 31);
      // first layer forward: u8 gather through registers (K = KS*KS*inC small)
      if (st.ig_dw0 && st.KS * st.KS * st.inC <= 64) st.ig_fwd = true;
      // first layer weight gradient straight from the pooled dY / argmax
      if (st.ig_dw0 && st.ig_fwd && st.pooled && st.pk == 2 && st.ps == 2 && st.act == gpu::ACT_RELU && st.KS == 3 &&
          st.stride == 1 && st.pad == 1) {
        gpu::Conv0DwParams& c = st.pc0;
        c.B = max_batch_; c.H = st.OH; c.W = st.OW; c.C = st.inC; c.PH = st.outH; c.PW = st.outW; c.Cout = st.C;
        st.c0dw = st.OH == st.inH && st.OW == st.inW && gpu::conv0_dw_supported(c);
        if (st.c0dw) st.ig_dw0 = false;
      }
      if (st.big && dtype_ == DType::BF16 && !no_igemm_ && s > 0) {
        st.ig_fwd = gpu::igemm_conv_supported(st.inC, st.C, st.KS);
        st.ig_dw = st.inC % 8 == 0;
        st.ig_dx = st.stride == 1 && gpu::igemm_conv_supported(st.C, st.inC, st.KS);
      }
      st.ig_pool = st.ig_fwd && st.pooled && st.pk == 2 && st.ps == 2 && st.OH % 2 == 0 && st.OW % 2 == 0;
      // 64 -> 128 3x3 pooled ReLU convs on 8 x 8 output tiles (CIFAR-3conv
      // conv3 at 8x8, VGG-11 conv2 at 112x112): dedicated kernels over the
      // implicit GEMM, same packed weights ([C][kgem] / [inC][kgem_d],
      // k = tap * channels + c) and output layouts
      st.c3k = st.big && dtype_ == DType::BF16 && s > 0 && !no_igemm_ && !ab_flag("no_c3k") && st.pooled &&
               st.pk == 2 && st.ps == 2 && st.kgem == 576 && st.kgem_d == 1152 &&
               gpu::cifar_c3_supported(st.inC, st.inH, st.inW, st.C, st.KS, st.stride, st.pad,
                                       st.act == gpu::ACT_RELU, st.pooled);
      if (!st.big && dtype_ == DType::BF16) plan_pipe(st, s == 0);
      // CIFAR-3conv conv2 (32 -> 64 at 16x16, pooled ReLU): dedicated kernels
      // (cifar_c2.hip) over the pipelined small-image ones; same packed
      // weights ([r16(C)][kpad], k = tap * 32 + c) and output layouts
      st.c2k = !st.big && dtype_ == DType::BF16 && s > 0 && !ab_flag("no_c2k") && st.cvec && st.CL == 32 &&
               st.kpad == 288 && st.pk == 2 && st.ps == 2 &&
               gpu::cifar_c2_supported(st.inC, st.inH, st.inW, st.C, st.KS, st.stride, st.pad, st.act == gpu::ACT_RELU,
                                       st.pooled);
      st.c2bwd = st.c2k && st.CLd == 64 && st.kpad_d == 576 && !ab_flag("no_c2bwd");
      if (!st.big && dtype_ == DType::F32 && st.pooled && st.stride == 1 &&
          (s == 0 || st.inC > 1)) {
        gpu::Conv1DirectParams& d = st.pd1;
        d.N = max_batch_; d.H = st.inH; d.W = st.inW; d.Cin = st.inC; d.KS = st.KS; d.pad = st.pad; d.C = st.C;
        d.OH = st.OH; d.OW = st.OW; d.PH = st.outH; d.PW = st.outW;
        st.direct_fwd = gpu::conv_direct_fwd_supported(d);
        st.direct1 = s == 0 && gpu::conv1_direct_dw_supported(d);
        st.direct_dx = s > 0 && gpu::conv_direct_dx_supported(d);
        st.direct_dw = s > 0 && gpu::conv_direct_dw_supported(d);
        if (s > 0 && !st.direct_dx) st.direct_fwd = false;  // the packed copies are then the generic ones
      }
      if (s == 0 && dtype_ == DType::BF16 && st.inC == 3 && st.KS == 3 && st.stride == 1 && st.pad == 1 &&
          st.pooled && st.pk == 2 && st.ps == 2 && st.act == gpu::ACT_RELU && !ab_flag("no_u8fwd")) {
        gpu::U8ConvParams u;
        u.N = max_batch_; u.H = st.inH; u.W = st.inW; u.Cout = st.C;
        st.u8fwd = st.OH == st.inH && st.OW == st.inW && gpu::u8conv_fwd_supported(u);
        // small images (CIFAR): the first layer's dW from the pooled dY / argmax too
        if (st.u8fwd && !st.big) {
          gpu::Conv0DwParams& c = st.pc0;
          c.B = max_batch_; c.H = st.OH; c.W = st.OW; c.C = st.inC; c.PH = st.outH; c.PW = st.outW; c.Cout = st.C;
          st.c0dw = gpu::conv0_dw_supported(c);
        }
      }
    } else {
      st.out_elems = st.Nout;
      st.out_ld = r8(st.Nout);
      st.ldp = r8(st.Kin + 1);
      st.fc_big = (int64_t)st.Nout * st.Kin >= (1 << 20) &&
                  !(dtype_ == DType::BF16 && gpu::fc_supported(st.Kin, st.Nout));
    }
    if (s > 0) {
      const Stage& pv = *stages_[s - 1];
      MCC_CHECK(pv.out_elems == st.in_elems, "stage shape mismatch");
      if (st.kind == Stage::FC) st.in_ld = pv.kind == Stage::FC ? pv.out_ld : (int)pv.out_elems;
    }
    if (st.kind == Stage::FC) MCC_CHECK(st.in_ld % 8 == 0, "fc input leading dim must be a multiple of 8");
    if (st.kind == Stage::FC && dtype_ == DType::BF16 && !st.last && !st.fc_big && !no_igemm_ &&
        max_batch_ >= 8192 && st.Kin % 8 == 0 && st.Nout % 8 == 0 && st.Kin >= 512 &&
        st.in_ld == st.Kin && st.out_ld == st.Nout && !gpu::fc_supported(st.Nout, st.Kin)) {
      st.fc_ig = gpu::igemm_conv_supported(st.Kin, st.Nout, 1);
      // data gradient: pv's act' is a ReLU mask (FC) or nothing (conv: its staging applies it)
      const Stage* pv = s > 0 ? stages_[s - 1] : nullptr;
      st.fc_igdx = st.fc_ig && pv &&
                   (pv->kind == Stage::CONV || pv->act == gpu::ACT_RELU || pv->act == gpu::ACT_NONE) &&
                   gpu::igemm_conv_supported(st.Nout, st.Kin, 1);
      st.fc_tall = st.fc_ig && st.Nout <= 224 && gpu::fc_tall_supported(max_batch_, st.Nout, st.Kin);
      st.fc_tall_dx = st.fc_tall && st.fc_igdx && (pv->kind == Stage::CONV || pv->act == gpu::ACT_NONE) &&
                      gpu::fc_tall_supported(max_batch_, st.Kin, st.Nout);
    }
    // fp32 tall-skinny FC (ref FC1 1568 -> 200, LeNet-5 FC1 400 -> 120 at a
    // large batch): exact f32 MFMA, same tiles
    // (also the narrow FC2s: LeNet-5 120 -> 84 writes 84 of its 88-column
    // rows, as the generic GEMM did; ref 200 -> 200)
    if (st.kind == Stage::FC && dtype_ == DType::F32 && !st.last && !st.fc_big && max_batch_ >= 8192 && s > 0 &&
        st.Nout <= 224 && st.Kin >= 64 && st.Kin % 8 == 0 && st.in_ld == st.Kin && st.out_ld >= st.Nout &&
        st.out_ld % 4 == 0 && gpu::fc_tall_supported(max_batch_, st.Nout, st.Kin)) {
      const Stage* pv = stages_[s - 1];
      st.fc_tall = true;
      st.fc_tall_dx = (pv->kind == Stage::CONV || pv->act == gpu::ACT_NONE) &&
                      gpu::fc_tall_supported(max_batch_, st.Kin, st.Nout);
    }
    // FC data gradient with W resident in LDS (ref FC1 / FC2, LeNet-5 fp32 FC1 /
    // FC2): the W^T copy [Kin][out_ld] as a per-workgroup column slab
    if (st.kind == Stage::FC && s > 0 && !st.fc_big && max_batch_ >= 8192 && !ab_flag("no_wres") &&
        (dtype_ == DType::F32 || dtype_ == DType::BF16) && st.out_ld % 8 == 0 && st.in_ld % 8 == 0) {
      const Stage* pv = stages_[s - 1];
      st.wres_act = pv->kind == Stage::FC ? pv->act : gpu::ACT_NONE;
      st.fc_wres = gpu::fc_wres_supported(dtype_ == DType::F32, max_batch_, st.Kin, st.Nout, st.wres_act);
    }
    st.head = st.kind == Stage::FC && st.last && s > 0 && !(dtype_ == DType::F32 && ab_flag("no_head32")) &&
              gpu::xent_head_supported(st.Nout, st.Kin, st.in_ld);
    // FC weight gradient on the implicit-GEMM dW kernel (a 1x1 "conv" over the
    // batch, C = in_ld with the pad columns dropped by the reduce)
    if (st.kind == Stage::FC)
      st.fc_igdw = dtype_ == DType::BF16 && !no_igemm_ && s > 0 && st.Nout % 4 == 0 && st.out_ld % 8 == 0 &&
                   st.in_ld % 8 == 0 && st.in_ld >= st.Kin && (int64_t)st.Nout * st.Kin >= 8192;
  }

  // ---- LeNet-5 conv block (lenet.hip): conv1 + pool + conv2 + pool as ONE
  // forward kernel and ONE fused backward kernel (conv2 dW, conv2 dX and the
  // unpooled conv1 dW per image, dY1 never leaves LDS).  MCC_AB=no_lenet keeps
  // the per-layer pipelined kernels (MCC_AB=no_lenet).
  {
    lenet_ = false;
    if (dtype_ == DType::BF16 && stages_.size() >= 3 && !ab_flag("no_lenet")) {
      const Stage& a = *stages_[0];
      const Stage& b = *stages_[1];
      auto pool_relu = [](const Stage& x) {
        return x.kind == Stage::CONV && x.act == gpu::ACT_RELU && x.pooled && x.pk == 2 && x.ps == 2 && !x.generic &&
               !x.big && x.stride == 1 && x.KS == 5;
      };
      lenet_ = pool_relu(a) && pool_relu(b) && a.inC == 1 && a.inH == 28 && a.inW == 28 && a.C == 6 && a.pad == 2 &&
               b.inC == 6 && b.C == 16 && b.pad == 0;
    }
  }
  // ---- reference-model conv block (refnet.hip; fp32: refnet_f32.hip): conv
  // 1->16 and 16->32, 3x3 stride 2 pad 1 ReLU on 28x28, fused forward and
  // fused backward (recomputed conv1, sub-pixel conv2 dX).
  {
    refblk_ = false;
    if (stages_.size() >= 3) {
      const Stage& a = *stages_[0];
      const Stage& b = *stages_[1];
      auto s2 = [](const Stage& x) {
        return x.kind == Stage::CONV && x.act == gpu::ACT_RELU && !x.pooled && !x.generic && !x.big && x.stride == 2 &&
               x.KS == 3 && x.pad == 1;
      };
      refblk_ = s2(a) && s2(b) && a.inC == 1 && a.inH == 28 && a.inW == 28 && a.C == 16 && b.inC == 16 &&
                b.inH == 14 && b.C == 32 && stages_[2]->kind == Stage::FC;
    }
  }
  // ---- LeNet-5 classifier chain (lenet_fc.hip): FC 400 -> 120 -> 84 -> 10
  // forward, softmax-CE and backward in one kernel launched by loss();
  // MCC_AB=no_fcchain keeps the per-layer FC kernels + the fused head.
  {
    fcchain_ = false;
    if (lenet_ && stages_.size() == 5 && !ab_flag("no_fcchain")) {
      const Stage& f1 = *stages_[2];
      const Stage& f2 = *stages_[3];
      const Stage& f3 = *stages_[4];
      fcchain_ = f1.kind == Stage::FC && f2.kind == Stage::FC && f3.kind == Stage::FC && f3.last &&
                 f1.act == gpu::ACT_RELU && f2.act == gpu::ACT_RELU &&
                 gpu::lenet_fc_supported(f1.Kin, f1.Nout, f2.Nout, f3.Nout) && f1.in_ld == f1.Kin &&
                 f2.Kin == f1.Nout && f3.Kin == f2.Nout;
    }
  }

  // ---- data gradient straight into dZ (no grad_xform pass) ----
  // A big stage whose input is a ReLU big conv writes that stage's dZ in its
  // implicit-GEMM data-gradient epilogue: dX * (y > 0) for an unpooled conv
  // (VGG-11 conv3/5/7), optionally the 2x2 unpool by the stored argmax for a
  // pooled one (conv2/4/6); the separate grad_xform pass re-reads dX (and y /
  // argmax) and re-writes dZ.
  {
    // ReLU mask only: an unpool in the same epilogue (four scattered 8-byte
    // stores per fragment) cost more in the dX kernel than the grad_xform pass
    // it replaced (VGG-11 B=512: off 15.61k, mask-only 15.77k, mask+unpool
    // 15.46k img/s) and was removed in round 3.  MCC_AB=no_dz_fuse: off.
    const bool on = !ab_flag("no_dz_fuse");
    for (size_t s = 1; on && s < stages_.size(); ++s) {
      Stage& cur = *stages_[s];
      Stage& pv = *stages_[s - 1];
      // (not for a conv0_dw first layer: its weight gradient reads the pooled dY itself)
      // (not when cur runs the cifar_c3 kernels: their dX is a plain store of dY)
      pv.dz_fused = cur.kind == Stage::CONV && cur.big && cur.ig_dx && !cur.c3k && pv.kind == Stage::CONV && pv.big &&
                    !pv.c0dw &&
                    !pv.pooled && pv.act == gpu::ACT_RELU && dtype_ == DType::BF16 &&
                    pv.C == cur.inC;
    }
  }

  // ---- packed weight table ----
  std::vector<int32_t> idx;
  auto reserve = [&](int64_t n) {
    int64_t off = (int64_t)idx.size();
    idx.resize(off + ((n + 15) & ~int64_t(15)), -1);
    return off;
  };
  for (Stage* sp : stages_) {
    Stage& st = *sp;
    if (st.kind == Stage::CONV && st.big) {
      const int KK = st.KS * st.KS;
      // im2col GEMM operands: forward [C][kgem], k = kp*inC + ci; data
      // gradient [inC][kgem_d], k = kp*C + co with flipped taps
      st.pk_fwd = reserve((int64_t)st.C * st.kgem);
      for (int n = 0; n < st.C; ++n)
        for (int kp = 0; kp < KK; ++kp)
          for (int c = 0; c < st.inC; ++c)
            idx[st.pk_fwd + (int64_t)n * st.kgem + kp * st.inC + c] =
                (int32_t)(st.w_off + ((int64_t)n * st.inC + c) * KK + kp);
      if (&st != stages_[0]) {
        st.pk_dx = reserve((int64_t)st.inC * st.kgem_d);
        for (int ci = 0; ci < st.inC; ++ci)
          for (int kp = 0; kp < KK; ++kp)
            for (int co = 0; co < st.C; ++co)
              idx[st.pk_dx + (int64_t)ci * st.kgem_d + kp * st.C + co] =
                  (int32_t)(st.w_off + ((int64_t)co * st.inC + ci) * KK + (KK - 1 - kp));
      }
    } else if (st.kind == Stage::CONV && st.pipe_fwd && st.pf.layout == gpu::XL_S1) {
      // single-channel pipelined forward: [r16(C)][kpad], k = kh*8 + kw (kw < KS)
      // (pair: columns 8 + n hold the right pixel of a pair, taps shifted by one)
      st.pk_fwd = reserve((int64_t)r16(st.C) * st.pf.kpad);
      for (int n = 0; n < st.C; ++n)
        for (int kh = 0; kh < st.KS; ++kh)
          for (int kw = 0; kw < st.KS; ++kw) {
            const int32_t src = (int32_t)(st.w_off + ((int64_t)n * st.KS + kh) * st.KS + kw);
            idx[st.pk_fwd + (int64_t)n * st.pf.kpad + kh * 8 + kw] = src;
            if (st.pf.pair) idx[st.pk_fwd + (int64_t)(8 + n) * st.pf.kpad + kh * 8 + kw + st.pf.pair] = src;
          }
    } else if (st.kind == Stage::CONV && st.direct_fwd) {
      // fp32 direct kernels: tap-major [inC][KK][C] (forward) and flipped
      // tap-major [C][KK][inC] (data gradient): channel pairs are adjacent
      // words, loaded as one scalar pair per packed FMA
      const int KK = st.KS * st.KS;
      st.pk_fwd = reserve((int64_t)st.inC * KK * st.C);
      for (int n = 0; n < st.C; ++n)
        for (int c = 0; c < st.inC; ++c)
          for (int kp = 0; kp < KK; ++kp)
            idx[st.pk_fwd + ((int64_t)c * KK + kp) * st.C + n] = (int32_t)(st.w_off + ((int64_t)n * st.inC + c) * KK + kp);
      if (st.direct_dx) {
        st.pk_dx = reserve((int64_t)st.C * KK * st.inC);
        for (int n = 0; n < st.C; ++n)
          for (int c = 0; c < st.inC; ++c)
            for (int kp = 0; kp < KK; ++kp)
              idx[st.pk_dx + ((int64_t)n * KK + (KK - 1 - kp)) * st.inC + c] =
                  (int32_t)(st.w_off + ((int64_t)n * st.inC + c) * KK + kp);
      }
    } else if (st.kind == Stage::CONV) {
      const int KK = st.KS * st.KS;
      // forward: [r16(C)][kpad], k = (kp, cgroup, c8) or (kp, c)
      st.pk_fwd = reserve((int64_t)r16(st.C) * st.kpad);
      for (int n = 0; n < st.C; ++n)
        for (int k = 0; k < st.kpad; ++k) {
          int kp, c;
          if (st.cvec) { const int G = k >> 3, CG = st.CL / 8; kp = G / CG; c = (G % CG) * 8 + (k & 7); }
          else { kp = k / st.inC; c = k % st.inC; }
          if (kp >= KK || c >= st.inC) continue;
          const int kh = kp / st.KS, kw = kp % st.KS;
          idx[st.pk_fwd + (int64_t)n * st.kpad + k] = (int32_t)(st.w_off + (((int64_t)n * st.inC + c) * st.KS + kh) * st.KS + kw);
        }
      if (&st != stages_[0]) {
        // data gradient: [r16(inC)][kpad_d], input channels = conv outputs, flipped taps
        st.pk_dx = reserve((int64_t)r16(st.inC) * st.kpad_d);
        for (int ci = 0; ci < st.inC; ++ci)
          for (int k = 0; k < st.kpad_d; ++k) {
            int kp, co;
            if (st.cvec_d) { const int G = k >> 3, CG = st.CLd / 8; kp = G / CG; co = (G % CG) * 8 + (k & 7); }
            else { kp = k / st.C; co = k % st.C; }
            if (kp >= KK || co >= st.C) continue;
            const int kh = st.KS - 1 - kp / st.KS, kw = st.KS - 1 - kp % st.KS;
            idx[st.pk_dx + (int64_t)ci * st.kpad_d + k] =
                (int32_t)(st.w_off + (((int64_t)co * st.inC + ci) * st.KS + kh) * st.KS + kw);
          }
      }
    } else {
      auto perm = [&](int k) { return k; };  // device order == activation order (see set_params)
      const int ldk = r8(st.Kin);
      st.pk_fwd = reserve((int64_t)st.Nout * ldk);
      for (int n = 0; n < st.Nout; ++n)
        for (int k = 0; k < st.Kin; ++k)
          idx[st.pk_fwd + (int64_t)n * ldk + k] = (int32_t)(st.w_off + (int64_t)n * st.Kin + perm(k));
      if (&st != stages_[0] && !st.fc_big) {
        st.pk_dx = reserve((int64_t)st.Kin * st.out_ld);
        for (int k = 0; k < st.Kin; ++k)
          for (int n = 0; n < st.Nout; ++n)
            idx[st.pk_dx + (int64_t)k * st.out_ld + n] = (int32_t)(st.w_off + (int64_t)n * st.Kin + perm(k));
      }
    }
  }
  packed_count_ = (int64_t)idx.size();

  // ---- analytic maps of the same packed layouts (fused SGD + pack) ----
  // Each weight stage's copies as (base, strides, flip) of its canonical
  // (n, c, kh, kw) index; verified below against the table, entry by entry.
  pack_.nstages = 0;
  bool maps_ok = (int)stages_.size() <= gpu::kMaxPackStages;
  if (ab_flag("no_fused_pack")) maps_ok = false;  // A/B: the gather-table path
  for (Stage* sp : stages_) {
    if (!maps_ok) break;
    const Stage& st = *sp;
    gpu::PackStage& ps = pack_.st[pack_.nstages++];
    ps.w_off = st.w_off; ps.nw = st.nw; ps.nmaps = 0;
    auto add = [&](int64_t base, int sn, int sc, int skh, int skw, int flip) {
      gpu::PackMap& m = ps.map[ps.nmaps++];
      m.base = base; m.sn = sn; m.sc = sc; m.skh = skh; m.skw = skw; m.flip = flip;
    };
    if (st.kind == Stage::FC) {
      ps.inC = st.Kin; ps.KS = 1;
      add(st.pk_fwd, r8(st.Kin), 1, 0, 0, 0);
      if (st.pk_dx >= 0) add(st.pk_dx, 1, st.out_ld, 0, 0, 0);
    } else {
      ps.inC = st.inC; ps.KS = st.KS;
      const int KS = st.KS;
      if (st.big) {
        add(st.pk_fwd, st.kgem, 1, KS * st.inC, st.inC, 0);
        if (st.pk_dx >= 0) add(st.pk_dx, 1, st.kgem_d, KS * st.C, st.C, 1);
      } else if (st.direct_fwd) {
        const int KK = KS * KS;
        add(st.pk_fwd, 1, KK * st.C, KS * st.C, st.C, 0);
        if (st.pk_dx >= 0) add(st.pk_dx, KK * st.inC, 1, KS * st.inC, st.inC, 1);
      } else if (st.pipe_fwd && st.pf.layout == gpu::XL_S1) {
        add(st.pk_fwd, st.pf.kpad, 0, 8, 1, 0);
        if (st.pf.pair) add(st.pk_fwd + 8 * (int64_t)st.pf.kpad + st.pf.pair, st.pf.kpad, 0, 8, 1, 0);
      } else {
        const int CLx = st.cvec ? st.CL : st.inC;
        add(st.pk_fwd, st.kpad, 1, KS * CLx, CLx, 0);
        if (st.pk_dx >= 0) {
          const int CLd = st.cvec_d ? st.CLd : st.C;
          add(st.pk_dx, 1, st.kpad_d, KS * CLd, CLd, 1);
        }
      }
    }
  }
  if (maps_ok) {
    int64_t covered = 0;
    for (int si = 0; si < pack_.nstages && maps_ok; ++si) {
      const gpu::PackStage& ps = pack_.st[si];
      const int KK = ps.KS * ps.KS;
      for (int64_t j = 0; j < ps.nw && maps_ok; ++j) {
        const int64_t n = j / ((int64_t)ps.inC * KK), r = j % ((int64_t)ps.inC * KK);
        const int c = (int)(r / KK), kh = (int)(r % KK) / ps.KS, kw = (int)(r % KK) % ps.KS;
        for (int m = 0; m < ps.nmaps; ++m) {
          const gpu::PackMap& mp = ps.map[m];
          const int h = mp.flip ? ps.KS - 1 - kh : kh, x = mp.flip ? ps.KS - 1 - kw : kw;
          const int64_t pos = mp.base + n * mp.sn + (int64_t)c * mp.sc + (int64_t)h * mp.skh + (int64_t)x * mp.skw;
          if (pos < 0 || pos >= packed_count_ || idx[pos] != ps.w_off + j) { maps_ok = false; break; }
          ++covered;
        }
      }
    }
    int64_t used = 0;
    for (int32_t v : idx) used += v >= 0;
    maps_ok = maps_ok && covered == used;
  }
  fused_pack_ = maps_ok;

  // ---- arena: sizing pass then real pass ----
  const int Bm = max_batch_;
  size_t scratch = 0;
  col_bytes_ = 0;
  for (Stage* sp : stages_) {
    const Stage& st = *sp;
    if (st.kind == Stage::CONV && st.big) {
      const int KK = st.KS * st.KS;
      const int64_t rows = (int64_t)Bm * st.OH * st.OW;
      if (!st.ig_fwd || (!st.ig_dw && !st.c0dw)) col_bytes_ = std::max(col_bytes_, es * (size_t)rows * st.kgem);
      if (st.c0dw) scratch = std::max(scratch, gpu::conv0_dw_slab_bytes(st.pc0));
      if (sp != stages_[0] && !st.ig_dx)
        col_bytes_ = std::max(col_bytes_, es * (size_t)Bm * st.inH * st.inW * st.kgem_d);
      if (st.c3k) scratch = std::max(scratch, gpu::cifar_c3_dw_scratch_bytes());
      if (st.ig_dw0) {
        const int sk = gpu::igemm_dw_splitk((int)rows, st.C, st.kgem);
        scratch = std::max(scratch, gpu::igemm_dw_slab_bytes(st.C, st.kgem, sk));
      } else if (st.ig_dw) {
        MCC_CHECK(rows < (1ll << 31), "igemm dW: too many pixels per batch");
        const int sk = gpu::igemm_dw_splitk((int)rows, st.C, KK * st.inC);
        scratch = std::max(scratch, gpu::igemm_dw_slab_bytes(st.C, KK * st.inC, sk));
      } else {
        const int sk = dw_splitk(st.C, KK * st.inC + 1, rows);
        scratch = std::max(scratch, (size_t)sk * st.C * r8(KK * st.inC + 1) * 4);
      }
    } else if (st.kind == Stage::CONV) {
      scratch = std::max(scratch, (size_t)st.nx_dw * st.cout_pad * st.ncols_pad * 4);
      if (st.rows_dw) scratch = std::max(scratch, gpu::conv_dw_rows_scratch_bytes(st.prw));
      if (st.direct1) scratch = std::max(scratch, gpu::conv1_direct_slab_bytes(st.pd1));
      if (st.direct_dw) scratch = std::max(scratch, gpu::conv_direct_dw_slab_bytes(st.pd1));
      if (st.c0dw) scratch = std::max(scratch, gpu::conv0_dw_slab_bytes(st.pc0));
      if (st.c2bwd) scratch = std::max(scratch, gpu::cifar_c2_dw_scratch_bytes());
      if (st.pipe_dw) {
        const size_t nv = (size_t)st.pdw.cout_pad * st.pdw.ncols_pad;
        scratch = std::max(scratch, (st.pdw.grid + ceil_div(st.pdw.grid, 16)) * nv * 4);
      }
    } else if (st.head) {
      scratch = std::max(scratch, (size_t)gpu::xent_head_slabs(Bm) * st.Nout * st.ldp * 4);
    } else if (st.fc_igdw) {
      scratch = std::max(scratch, gpu::igemm_dw_slab_bytes(st.Nout, st.in_ld, gpu::igemm_dw_splitk(Bm, st.Nout, st.in_ld)));
    } else {
      scratch = std::max(scratch, (size_t)fc_dw_splitk(st.Nout, st.Kin + 1, Bm, dtype_) * st.Nout * st.ldp * 4);
      if (dtype_ == DType::F32)
        scratch = std::max(scratch, (size_t)gpu::fc_dw32_splitk(st.Nout, st.Kin, Bm) * st.Nout * st.ldp * 4);
    }
  }
  for (Stage* sp : stages_) {
    const Stage& st = *sp;
    if (st.kind != Stage::FC) continue;
    const int ld = st.last ? r8(spec_.num_classes()) : st.out_ld;
    // the split count is not monotonic in the batch (VGG-11 FC1 at max batch
    // 1024: sk 4 x 1024 rows, at 768: sk 6 x 768 rows): size for every batch
    // forward() can see
    size_t need = 0;
    for (int b = 1; b <= Bm; ++b)
      need = std::max(need, (size_t)gpu::gemm_fwd_splitk(b, st.Nout, st.Kin) * b * ld * 4);
    scratch = std::max(scratch, need);
  }
  if (lenet_) scratch = std::max(scratch, gpu::lenet_slab_bytes());
  if (fcchain_) scratch = std::max(scratch, gpu::lenet_fc_slab_bytes(Bm));
  if (refblk_) scratch = std::max(scratch, gpu::ref_slab_bytes(dtype_ == DType::F32));
  scratch_bytes_ = scratch;
  for (int pass = 0; pass < 2; ++pass) {
    arena_used_ = 0;
    params_ = static_cast<float*>(arena_alloc(4 * (size_t)spec_.nparams));
    grads_ = static_cast<float*>(arena_alloc(4 * (size_t)spec_.nparams));
    stats_ = static_cast<unsigned long long*>(arena_alloc(64));
    logits_ld_ = r8(spec_.num_classes());
    logits_ = static_cast<float*>(arena_alloc(4 * (size_t)Bm * logits_ld_));
    packed_ = arena_alloc(es * (size_t)packed_count_);
    pack_idx_ = fused_pack_ ? nullptr : static_cast<int32_t*>(arena_alloc(4 * (size_t)packed_count_));
    scratch_ = static_cast<float*>(arena_alloc(scratch_bytes_));
    col_ = col_bytes_ ? arena_alloc(col_bytes_) : nullptr;
    for (Stage* sp : stages_) {
      Stage& st = *sp;
      const int64_t per = st.kind == Stage::FC ? st.out_ld : st.out_elems;
      // the LeNet block keeps conv1's pooled output HWC-8 and its argmax planar
      const bool l0 = lenet_ && sp == stages_[0];
      st.act_buf = arena_alloc(es * (size_t)Bm * (l0 ? std::max<int64_t>(per, gpu::lenet_y1_elems()) : per));
      st.grad_buf = arena_alloc(es * (size_t)Bm * per);
      st.arg_buf = st.pooled ? static_cast<uint8_t*>(arena_alloc(
                                   (size_t)Bm * (l0 ? std::max<int64_t>(per, gpu::lenet_a1_bytes()) : per)))
                             : nullptr;
      if (st.kind == Stage::CONV && st.big) {
        const size_t conv_elems = (size_t)Bm * st.OH * st.OW * st.C;
        st.conv_buf = st.pooled && !st.ig_pool ? arena_alloc(es * conv_elems) : nullptr;
        st.dz_buf = arena_alloc(es * conv_elems);
      }
    }
    if (pass == 0) {
      arena_bytes_ = arena_used_ + 256;
      HIP_OK(hipMalloc(reinterpret_cast<void**>(&arena_), arena_bytes_));
      HIP_OK(hipMemset(arena_, 0, arena_bytes_));
    }
  }
  if (!fused_pack_) HIP_OK(hipMemcpy(pack_idx_, idx.data(), 4 * idx.size(), hipMemcpyHostToDevice));
  pack_.packed = packed_;
  pack_.params = params_;
  pack_.grads = grads_;
  pack_.n = spec_.nparams;
}

std::string GpuNet::plan() const {
  std::ostringstream os;
  if (lenet_) os << "[lenet block: stages 0+1 fused fwd (lenet_fwd) and bwd (lenet_bwd)]\n";
  if (fcchain_) os << "[lenet fc chain: stages 2-4 fwd + softmax-CE + bwd in one kernel (lenet_fc)]\n";
  if (refblk_) os << "[ref block: stages 0+1 fused fwd (ref_fwd) and bwd (ref_bwd: recomputed conv1, sub-pixel dX)]\n";
  os << "GpuNet(" << spec_.name << ", " << dtype_name(dtype_) << ", max_batch=" << max_batch_
     << ", arena=" << (arena_bytes_ >> 20) << " MiB, " << (fused_pack_ ? "fused sgd+pack" : "sgd + pack table")
     << ")\n";
  for (size_t s = 0; s < stages_.size(); ++s) {
    const Stage& st = *stages_[s];
    if (st.kind == Stage::CONV) {
      os << "  [" << s << "] conv " << st.inC << "x" << st.inH << "x" << st.inW << " -> " << st.C << "x" << st.OH << "x"
         << st.OW << (st.pooled ? " +maxpool" : "") << " k" << st.KS << "s" << st.stride << "p" << st.pad
         << (st.big ? (st.c3k ? " c3k[fwd dx dw]" : st.ig_fwd ? " igemm" : " im2col+gemm")
                    : (st.cvec ? " lds-cvec" : " lds-scalar"))
         << (st.c0dw ? " dw:pooled-direct" : "") << (st.dz_fused ? " dz<-next-dx" : "")
         << (st.generic ? " generic" : "") << " chunks=" << st.nchunks
         << " imgs=" << st.imgs_fwd << "/"
         << st.imgs_dx << "/" << st.imgs_dw;
      if (st.pipe_fwd || st.pipe_dx || st.pipe_dw || st.rows_dw) {
        os << " pipe[";
        if (st.pipe_fwd) os << "fwd:" << (st.pf.layout == gpu::XL_S1 ? (st.pf.pair == 2 ? "s1w" : st.pf.pair ? "s1p" : "s1") : "c8") << "x" << st.pf.imgs << "/g" << st.pf.grid << " ";
        if (st.pipe_dx) os << "dx:x" << st.pdx.imgs << "/g" << st.pdx.grid << " ";
        if (st.pipe_dw) os << "dw:x" << st.pdw.imgs << "/g" << st.pdw.grid;
        if (st.rows_dw) os << "dw:rows x" << st.prw.imgs << "/g" << st.prw.grid;
        os << "]";
      }
      if (st.direct_fwd || st.direct1 || st.direct_dx || st.direct_dw)
        os << " direct-f32[" << (st.direct_fwd ? "fwd" : "") << (st.direct1 || st.direct_dw ? " dw" : "")
           << (st.direct_dx ? " dx" : "") << "]";
      if (st.u8fwd) os << " u8fwd" << (st.c0dw && !st.big ? " dw:pooled-direct" : "");
      if (st.c2k) os << (st.c2bwd ? " c2k[fwd dx dw]" : " c2k[fwd]");
      os << "\n";
    } else {
      os << "  [" << s << "] fc " << st.Kin << " -> " << st.Nout << (st.last ? " (logits)" : "")
         << (st.permC ? " nhwc-flatten" : "")
         << (st.fc_tall ? (st.fc_tall_dx && !st.fc_wres ? " tall[fwd dx]" : " tall[fwd]")
                        : st.fc_ig ? (st.fc_igdx ? " igemm[fwd dx]" : " igemm[fwd]") : "")
         << (st.fc_wres ? " wres[dx]" : "") << (st.head ? " head[softmax-CE fused]" : "") << "\n";
    }
  }
  return os.str();
}

// Device parameter layout: the canonical reference layouts (cnn.c:318-342)
// except the weight of an FC layer fed by a conv, whose columns are kept in
// the activation (NHWC-flatten) order k = hw*C + c instead of the canonical
// CHW order c*HW + hw: its packed copy is then a straight cast and its weight
// gradient needs no scatter.  The host API speaks canonical order only.
void GpuNet::to_device_order(const float* canon, float* dev) const {
  std::copy(canon, canon + spec_.nparams, dev);
  for (const Stage* sp : stages_) {
    const Stage& st = *sp;
    if (st.kind != Stage::FC || st.permC <= 0) continue;
    for (int n = 0; n < st.Nout; ++n) {
      const float* src = canon + st.w_off + (int64_t)n * st.Kin;
      float* dst = dev + st.w_off + (int64_t)n * st.Kin;
      for (int hw = 0; hw < st.permHW; ++hw)
        for (int c = 0; c < st.permC; ++c) dst[hw * st.permC + c] = src[c * st.permHW + hw];
    }
  }
}

void GpuNet::to_canonical_order(const float* dev, float* canon) const {
  std::copy(dev, dev + spec_.nparams, canon);
  for (const Stage* sp : stages_) {
    const Stage& st = *sp;
    if (st.kind != Stage::FC || st.permC <= 0) continue;
    for (int n = 0; n < st.Nout; ++n) {
      const float* src = dev + st.w_off + (int64_t)n * st.Kin;
      float* dst = canon + st.w_off + (int64_t)n * st.Kin;
      for (int hw = 0; hw < st.permHW; ++hw)
        for (int c = 0; c < st.permC; ++c) dst[c * st.permHW + hw] = src[hw * st.permC + c];
    }
  }
}

void GpuNet::set_params(const float* host) {
  std::vector<float> d((size_t)spec_.nparams);
  to_device_order(host, d.data());
  HIP_OK(hipMemcpy(params_, d.data(), 4 * (size_t)spec_.nparams, hipMemcpyHostToDevice));
  pack(nullptr);
  HIP_OK(hipDeviceSynchronize());
}

void GpuNet::get_params(float* host) const {
  HIP_OK(hipDeviceSynchronize());
  std::vector<float> d((size_t)spec_.nparams);
  HIP_OK(hipMemcpy(d.data(), params_, 4 * (size_t)spec_.nparams, hipMemcpyDeviceToHost));
  to_canonical_order(d.data(), host);
}

void GpuNet::get_grads(float* host) const {
  HIP_OK(hipDeviceSynchronize());
  std::vector<float> d((size_t)spec_.nparams);
  HIP_OK(hipMemcpy(d.data(), grads_, 4 * (size_t)spec_.nparams, hipMemcpyDeviceToHost));
  to_canonical_order(d.data(), host);
}

void GpuNet::pack(hipStream_t s) {
  if (fused_pack_) {
    gpu::SgdPackParams p = pack_;
    p.update = false;
    gpu::sgd_pack(dtype_, p, s);
  } else {
    gpu::pack_gather(dtype_, packed_, params_, pack_idx_, packed_count_, s);
  }
}

void GpuNet::zero_stats(hipStream_t s) { HIP_OK(hipMemsetAsync(stats_, 0, 32, s)); }

// standalone max-pool of a conv stage's output (conv_buf -> act_buf, argmax)
void GpuNet::pool_fwd(Stage& st, int B, hipStream_t s) {
  if (st.pk == 2 && st.ps == 2)
    gpu::maxpool2(dtype_, st.conv_buf, st.act_buf, st.arg_buf, B, st.OH, st.OW, st.C, s, st.act == gpu::ACT_RELU);
  else
    gpu::maxpool(dtype_, st.conv_buf, st.act_buf, st.arg_buf, B, st.OH, st.OW, st.C, st.pk, st.ps, s);
}

void GpuNet::forward(const uint8_t* images, const int32_t* idx, int B, hipStream_t s) {
  MCC_CHECK(B > 0 && B <= max_batch_, "forward: batch exceeds max_batch");
  B_ = B;
  images_ = images;
  idx_ = idx;
  head_done_ = false;
  fc_pending_ = false;
  fc_bwd_done_ = false;
  forward_stages(0, true, s);
}

// The LeNet-5 classifier chain (lenet_fc.hip) runs its forward inside the
// fused forward+loss+backward kernel that loss(backward = true) launches, so
// forward() stops after the conv block and leaves the FC forward pending.
// Anything that needs the FC outputs without that kernel (loss(backward =
// false), get_logits) runs the per-layer FC forward first.
void GpuNet::flush_forward(hipStream_t s) const {
  if (!fc_pending_) return;
  fc_pending_ = false;
  const_cast<GpuNet*>(this)->forward_stages(pending_from_, false, s);
}

void GpuNet::forward_stages(size_t first, bool defer_fc, hipStream_t s) {
  const int B = B_;
  const uint8_t* images = images_;
  const int32_t* idx = idx_;
  const size_t es = dtype_size(dtype_);
  for (size_t si = first; si < stages_.size(); ++si) {
    Stage& st = *stages_[si];
    if (fcchain_ && defer_fc && si >= 2) {
      fc_pending_ = true;
      pending_from_ = 2;
      return;
    }
    // the last FC layer of a fused softmax-CE head: its forward runs inside
    // the head kernel that loss(backward = true) launches (xent_head FWD).
    // fp32: ref 63 + 107 -> 152 us, LeNet-5 36 + 57 -> 88 us.  bf16 only with
    // the MFMA head: the VALU head's logits cost more than the MFMA forward
    // they replace (ref 20 + 76 -> 102 us)
    if (defer_fc && st.head && si + 1 == stages_.size() && !ab_flag("no_head_fwd") &&
        (dtype_ == DType::F32 || !ab_flag("head_valu"))) {
      fc_pending_ = true;
      pending_from_ = si;
      return;
    }
    if (lenet_ && si <= 1) {
      if (si == 1) continue;  // produced with stage 0
      const Stage& s1 = *stages_[1];
      gpu::LenetFwdParams f;
      f.B = B; f.x = images; f.idx = idx;
      f.w1 = params_ + st.w_off; f.b1 = params_ + st.b_off; f.w2 = params_ + s1.w_off; f.b2 = params_ + s1.b_off;
      f.y1 = st.act_buf; f.a1 = st.arg_buf; f.y2 = s1.act_buf; f.a2 = s1.arg_buf;
      gpu::lenet_forward(f, s);
      continue;
    }
    if (refblk_ && si <= 1) {
      if (si == 1) continue;  // produced with stage 0 (stage 0's own output is never stored)
      const Stage& s1 = *stages_[1];
      gpu::RefFwdParams f;
      f.B = B; f.x = images; f.idx = idx; f.f32 = dtype_ == DType::F32;
      f.w1 = params_ + st.w_off; f.b1 = params_ + st.b_off; f.w2 = params_ + s1.w_off; f.b2 = params_ + s1.b_off;
      f.y2 = s1.act_buf;
      gpu::ref_forward(f, s);
      continue;
    }
    if (st.u8fwd) {
      gpu::U8ConvParams u;
      u.N = B; u.H = st.inH; u.W = st.inW; u.Cout = st.C;
      u.x = images; u.idx = idx;
      u.w = params_ + st.w_off; u.bias = params_ + st.b_off;
      u.out = static_cast<uint16_t*>(st.act_buf); u.out_arg = st.arg_buf;
      gpu::u8conv_forward(u, s);
      continue;
    }
    if (st.kind == Stage::CONV && st.c3k) {
      gpu::CifarC3Params c;
      c.B = B;
      c.x = stages_[si - 1]->act_buf;
      c.w = static_cast<const char*>(packed_) + es * st.pk_fwd; c.ldw = st.kgem;
      c.bias = params_ + st.b_off;
      c.y = st.act_buf; c.arg = st.arg_buf;
      c.H = st.inH; c.W = st.inW;
      gpu::cifar_c3_forward(c, s);
      continue;
    }
    if (st.kind == Stage::CONV && st.big && st.ig_fwd) {
      // implicit GEMM with bias+ReLU epilogue -> 2x2 max-pool
      gpu::IgemmParams g;
      g.B = B; g.H = st.inH; g.W = st.inW; g.C = st.inC;
      g.OH = st.OH; g.OW = st.OW; g.KS = st.KS; g.stride = st.stride; g.pad = st.pad;
      g.M = B * st.OH * st.OW; g.N = st.C; g.K = st.KS * st.KS * st.inC;
      g.in = si > 0 ? stages_[si - 1]->act_buf : nullptr;
      g.w = static_cast<const char*>(packed_) + es * st.pk_fwd; g.ldw = st.kgem;
      g.bias = params_ + st.b_off; g.epi_bias_act = true; g.act = st.act;
      g.out = st.pooled && !st.ig_pool ? st.conv_buf : st.act_buf; g.ldo = st.C;
      g.pool = st.ig_pool; g.out_arg = st.arg_buf;
      if (si == 0) { g.u8 = true; g.in = images; g.idx = idx; }
      gpu::igemm_conv(g, s);
      if (st.pooled && !st.ig_pool) pool_fwd(st, B, s);
    } else if (st.kind == Stage::CONV && st.big) {
      // im2col (input transform fused) -> GEMM with bias+ReLU epilogue -> 2x2 max-pool
      gpu::Im2colParams ic;
      ic.N = B; ic.OH = st.OH; ic.OW = st.OW; ic.KS = st.KS; ic.cs = st.stride; ic.ldk = st.kgem;
      ic.s.SH = st.inH; ic.s.SW = st.inW; ic.s.SC = st.inC; ic.s.off = st.pad; ic.s.up = 1;
      if (si == 0) { ic.s.mode = gpu::IN_U8; ic.s.src = images; ic.s.idx = idx; }
      else { ic.s.mode = gpu::IN_PLAIN; ic.s.src = stages_[si - 1]->act_buf; }
      ic.out = col_;
      gpu::im2col(dtype_, ic, s);
      gpu::GemmParams g;
      g.M = B * st.OH * st.OW; g.N = st.C; g.K = st.KS * st.KS * st.inC;
      g.A = col_; g.lda = st.kgem;
      g.B = static_cast<const char*>(packed_) + es * st.pk_fwd; g.ldb = st.kgem;
      g.epi = gpu::EPI_BIAS_ACT; g.act = st.act; g.bias = params_ + st.b_off;
      g.C = st.pooled ? st.conv_buf : st.act_buf; g.ldc = st.C;
      gpu::gemm(dtype_, g, s);
      if (st.pooled) pool_fwd(st, B, s);
    } else if (st.kind == Stage::CONV && st.direct_fwd) {
      gpu::Conv1DirectParams p = st.pd1;
      p.N = B;
      if (si == 0) { p.x = images; p.idx = idx; }
      else p.xf = static_cast<const float*>(stages_[si - 1]->act_buf);
      p.wt = reinterpret_cast<const float*>(packed_) + st.pk_fwd; p.bias = params_ + st.b_off;
      p.out = static_cast<float*>(st.act_buf); p.out_arg = st.arg_buf;
      gpu::conv_direct_forward(p, s);
    } else if (st.kind == Stage::CONV && st.c2k) {
      gpu::CifarC2Params c;
      c.B = B;
      c.x = stages_[si - 1]->act_buf;
      c.w = static_cast<const char*>(packed_) + es * st.pk_fwd; c.ldw = st.kpad;
      c.bias = params_ + st.b_off;
      c.y = st.act_buf; c.arg = st.arg_buf;
      gpu::cifar_c2_forward(c, s);
    } else if (st.kind == Stage::CONV && st.pipe_fwd) {
      gpu::ConvPipeParams p = st.pf;
      p.N = B;
      if (si == 0) { p.in.src = images; p.in.idx = idx; }
      else p.in.src = stages_[si - 1]->act_buf;
      p.wpk = static_cast<const char*>(packed_) + es * st.pk_fwd;
      p.bias = params_ + st.b_off;
      p.out = st.act_buf; p.out_arg = st.arg_buf;
      gpu::conv_pipe_forward(p, s);
    } else if (st.kind == Stage::CONV) {
      gpu::ConvParams p;
      p.N = B; p.imgs = st.imgs_fwd;
      p.Cin = st.inC; p.CL = st.CL; p.cvec = st.cvec;
      p.LH = (st.OH - 1) * st.stride + st.KS; p.LW = (st.OW - 1) * st.stride + st.KS;
      p.OH = st.OH; p.OW = st.OW; p.cs = st.stride; p.KS = st.KS;
      p.Cout = st.C; p.nchunks = st.nchunks; p.kpad = st.kpad;
      p.pool = st.pooled ? 2 : 1; p.act = st.act; p.bias_act = true;
      p.in.SH = st.inH; p.in.SW = st.inW; p.in.SC = st.inC; p.in.off = st.pad; p.in.up = 1;
      if (si == 0) { p.in.mode = gpu::IN_U8; p.in.src = images; p.in.idx = idx; }
      else { p.in.mode = gpu::IN_PLAIN; p.in.src = stages_[si - 1]->act_buf; }
      p.wpk = static_cast<const char*>(packed_) + es * st.pk_fwd;
      p.bias = params_ + st.b_off;
      p.out = st.act_buf; p.out_arg = st.arg_buf;
     
      gpu::conv_forward(dtype_, p, s);
    } else if (st.fc_tall) {
      const Stage& pv = *stages_[si - 1];
      gpu::FcTallParams t;
      t.M = B; t.N = st.Nout; t.K = st.Kin; t.f32 = dtype_ == DType::F32;
      t.A = pv.act_buf; t.lda = st.in_ld;
      t.W = static_cast<const char*>(packed_) + es * st.pk_fwd; t.ldw = r8(st.Kin);
      t.bias = params_ + st.b_off; t.act = st.act;
      t.out = st.act_buf; t.ldo = st.out_ld;
      gpu::fc_tall(t, s);
    } else if (st.fc_ig) {
      const Stage& pv = *stages_[si - 1];
      gpu::IgemmParams g;
      g.B = B; g.H = 1; g.W = 1; g.C = st.Kin;
      g.OH = 1; g.OW = 1; g.KS = 1; g.stride = 1; g.pad = 0;
      g.M = B; g.N = st.Nout; g.K = st.Kin;
      g.in = pv.act_buf;
      g.w = static_cast<const char*>(packed_) + es * st.pk_fwd; g.ldw = r8(st.Kin);
      g.bias = params_ + st.b_off; g.epi_bias_act = true; g.act = st.act;
      g.out = st.act_buf; g.ldo = st.out_ld;
      gpu::igemm_conv(g, s);
    } else if (dtype_ == DType::BF16 && gpu::fc_supported(st.Nout, st.Kin)) {
      const Stage& pv = *stages_[si - 1];
      gpu::FcParams p;
      p.M = B; p.N = st.Nout; p.K = st.Kin;
      p.A = pv.act_buf; p.lda = st.in_ld;
      p.W = static_cast<const char*>(packed_) + es * st.pk_fwd; p.ldw = r8(st.Kin);
      p.bias = params_ + st.b_off;
      if (st.last) { p.epi = gpu::EPI_LOGITS; p.Cf = logits_; p.ldc = logits_ld_; }
      else { p.epi = gpu::EPI_BIAS_ACT; p.act = st.act; p.C = st.act_buf; p.ldc = st.out_ld; }
      gpu::fc_forward(p, s);
    } else {
      const Stage& pv = *stages_[si - 1];
      gpu::GemmParams p;
      p.M = B; p.N = st.Nout; p.K = st.Kin;
      p.A = pv.act_buf; p.lda = st.in_ld;
      p.B = static_cast<const char*>(packed_) + es * st.pk_fwd; p.ldb = r8(st.Kin);
      p.bias = params_ + st.b_off;
      if (st.last) { p.epi = gpu::EPI_LOGITS; p.Cf = logits_; p.ldc = logits_ld_; }
      else { p.epi = gpu::EPI_BIAS_ACT; p.act = st.act; p.C = st.act_buf; p.ldc = st.out_ld; }
      int sk = gpu::gemm_fwd_splitk(B, st.Nout, st.Kin);
      // (build() sizes the scratch for every B <= max_batch; the clamp only
      // guards a future change of the split rule)
      while (sk > 1 && (size_t)sk * B * p.ldc * 4 > scratch_bytes_) --sk;
      gpu::gemm_splitk_fwd(dtype_, p, scratch_, sk, s);
    }
  }
}

void GpuNet::loss(const uint8_t* labels, const int32_t* idx, float grad_scale, bool backward, hipStream_t s,
                  int32_t* pred) {
  MCC_CHECK(B_ > 0, "loss: call forward first");
  const Stage& last = *stages_.back();
  if (fcchain_ && fc_pending_ && backward) {
    // forward + softmax-CE + backward of the three FC layers in one kernel;
    // the weight gradients land in grads_ through a fixed-order slab reduce
    const Stage& s1 = *stages_[1];
    const Stage& f1 = *stages_[2];
    const Stage& f2 = *stages_[3];
    const Stage& f3 = *stages_[4];
    const size_t es = dtype_size(dtype_);
    gpu::LenetFcParams f;
    f.B = B_;
    f.y = s1.act_buf; f.ldy = f1.in_ld;
    f.w1 = static_cast<const char*>(packed_) + es * f1.pk_fwd; f.ldw1 = r8(f1.Kin);
    f.w2 = static_cast<const char*>(packed_) + es * f2.pk_fwd; f.ldw2 = r8(f2.Kin);
    f.w3 = static_cast<const char*>(packed_) + es * f3.pk_fwd; f.ldw3 = r8(f3.Kin);
    f.b1 = params_ + f1.b_off; f.b2 = params_ + f2.b_off; f.b3 = params_ + f3.b_off;
    f.labels = labels; f.idx = idx;
    f.scale = grad_scale;
    f.logits = logits_; f.ldl = logits_ld_;
    f.pred = pred;
    f.stats = stats_;
    f.dy = s1.grad_buf; f.ldd = f1.in_ld;
    f.slab = scratch_;
    gpu::lenet_fc(f, grads_ + f1.w_off, s);
    fc_pending_ = false;
    fc_bwd_done_ = true;
    return;
  }
  const bool head_fwd = backward && last.head && fc_pending_ && pending_from_ + 1 == stages_.size();
  if (!head_fwd) flush_forward(s);
  gpu::XentParams p;
  p.M = B_; p.N = spec_.num_classes();
  p.logits = logits_; p.ldl = logits_ld_;
  p.labels_idx = idx; p.labels = labels;
  p.dlogits = backward ? last.grad_buf : nullptr; p.ldd = last.out_ld;
  p.scale = grad_scale;
  p.stats = stats_;
  p.pred = pred;
  if (backward && last.head) {
    // softmax-CE + the last FC layer's dX, dW, db in one kernel; the per-
    // workgroup dW slabs are summed in a fixed order by dw_reduce
    const Stage& pv = *stages_[stages_.size() - 2];
    gpu::XentHeadParams h;
    h.x = p;
    h.x.dlogits = nullptr;
    h.h = pv.act_buf; h.ldh = last.in_ld;
    h.w = params_ + last.w_off; h.Kin = last.Kin;
    h.act = pv.kind == Stage::FC ? pv.act : gpu::ACT_NONE;  // conv masks are applied by its staging
    h.dh = pv.grad_buf;
    h.slab = scratch_; h.ldp = last.ldp;
    if (dtype_ == DType::BF16) {  // the MFMA head reads the packed forward copy
      h.wpk = static_cast<const char*>(packed_) + 2 * last.pk_fwd;
      h.ldw = r8(last.Kin);
    }
    if (head_fwd) {  // the head computes (and writes) the logits itself
      h.bias = params_ + last.b_off;
      fc_pending_ = false;
    }
    const int slabs = gpu::xent_head(dtype_, h, s);
    gpu::DwReduceParams r;
    r.S = slabs; r.Nout = last.Nout; r.kfeat = last.Kin; r.ldp = last.ldp; r.part = scratch_;
    r.partial_stride = (int64_t)last.Nout * last.ldp;
    r.gw = grads_ + last.w_off; r.gb = grads_ + last.b_off;
    r.permC = 0; r.permHW = 0;  // device order (see set_params)
    gpu::dw_reduce(r, s);
    head_done_ = true;
    return;
  }
  gpu::softmax_xent(dtype_, p, s);
}

void GpuNet::backward(int hi, int lo, hipStream_t s) {
  MCC_CHECK(B_ > 0, "backward: call forward + loss first");
  MCC_CHECK(hi >= lo && lo >= 0 && hi < (int)stages_.size(), "backward: bad stage range");
  const int B = B_;
  const size_t es = dtype_size(dtype_);
  const hipStream_t s_main = s;
  bool forked = false;
  for (int si = hi; si >= lo; --si) {
    Stage& st = *stages_[si];
    s = s_main;
    if (fc_bwd_done_ && si >= 2) continue;  // done by loss() (lenet_fc)
    if (lenet_ && si <= 1) {
      // stage 1 runs the fused block backward (both stages' dW, db); stage 0 is then done
      if (si == 0) continue;
      if (forked) {  // the block kernel uses scratch_ on the main stream
        HIP_OK(hipEventRecord(join_ev_, wstream_));
        HIP_OK(hipStreamWaitEvent(s_main, join_ev_, 0));
        forked = false;
      }
      const Stage& s0 = *stages_[0];
      gpu::LenetBwdParams b;
      b.B = B; b.x = images_; b.idx = idx_;
      b.w2 = params_ + st.w_off;
      b.dy2 = st.grad_buf; b.a2 = st.arg_buf; b.y1 = s0.act_buf; b.a1 = s0.arg_buf;
      b.slab = scratch_;
      b.gw1 = grads_ + s0.w_off; b.gb1 = grads_ + s0.b_off; b.gw2 = grads_ + st.w_off; b.gb2 = grads_ + st.b_off;
      gpu::lenet_backward(b, s_main);
      continue;
    }
    if (refblk_ && si <= 1) {
      if (si == 0) continue;
      if (forked) {
        HIP_OK(hipEventRecord(join_ev_, wstream_));
        HIP_OK(hipStreamWaitEvent(s_main, join_ev_, 0));
        forked = false;
      }
      const Stage& s0 = *stages_[0];
      gpu::RefBwdParams b;
      b.B = B; b.x = images_; b.idx = idx_; b.f32 = dtype_ == DType::F32;
      b.w1 = params_ + s0.w_off; b.b1 = params_ + s0.b_off; b.w2 = params_ + st.w_off;
      b.y2 = st.act_buf; b.dy2 = st.grad_buf;
      b.slab = scratch_;
      b.gw1 = grads_ + s0.w_off; b.gb1 = grads_ + s0.b_off; b.gw2 = grads_ + st.w_off; b.gb2 = grads_ + st.b_off;
      gpu::ref_backward(b, s_main);
      continue;
    }
    // Side stream for this stage's weight gradient when the two directions
    // share no scratch: every path except the im2col fallbacks of the
    // large-image conv (col_ is shared by their dW and dX).  All dW work is
    // serialised on wstream_, so scratch_ (split-K slabs) stays single-user;
    // the dX kernels never touch scratch_.
    const bool side = wstream_ && !(st.kind == Stage::CONV && st.big &&
                                    !((st.ig_dw || st.ig_dw0 || st.c0dw) && (st.ig_dx || si == 0)));
    hipStream_t ws = s_main;
    if (!side && forked) {  // this stage's dW uses scratch_ on the main stream: drain the side stream first
      HIP_OK(hipEventRecord(join_ev_, wstream_));
      HIP_OK(hipStreamWaitEvent(s_main, join_ev_, 0));
      forked = false;
    }
    auto fork = [&]() {
      if (!side) return;
      HIP_OK(hipEventRecord(fork_ev_[si], s_main));
      HIP_OK(hipStreamWaitEvent(wstream_, fork_ev_[si], 0));
      ws = wstream_;
      forked = true;
    };
    if (st.kind == Stage::CONV) {
      gpu::StageSrc dy;
      dy.mode = st.pooled ? gpu::IN_UNPOOL
                          : (st.act == gpu::ACT_RELU ? gpu::IN_RELU : st.act == gpu::ACT_TANH ? gpu::IN_TANH : gpu::IN_PLAIN);
      dy.act = st.act;
      dy.pk = st.pk; dy.ps = st.ps;
      dy.src = st.grad_buf; dy.aux_y = st.act_buf; dy.aux_arg = st.arg_buf;
      dy.SH = st.OH; dy.SW = st.OW; dy.SC = st.C; dy.PH = st.outH; dy.PW = st.outW;
      if (st.big) {
        const int KK = st.KS * st.KS;
        const int kf = KK * st.inC;
        if (st.c0dw) {  // first layer: dW from the pooled dY / argmax directly (no dZ, no im2col)
          fork();
          gpu::Conv0DwParams c = st.pc0;
          c.B = B; c.x = images_; c.idx = idx_;
          c.dy = static_cast<const uint16_t*>(st.grad_buf); c.arg = st.arg_buf;
          c.slab = scratch_;
          gpu::conv0_dw(c, grads_ + st.w_off, grads_ + st.b_off, ws);
          continue;
        }
        if (st.c3k) {  // dX / dW straight from the pooled dY and argmax (no dZ pass)
          fork();
          gpu::CifarC3BwdParams c;
          c.B = B; c.dy = st.grad_buf; c.arg = st.arg_buf; c.x = stages_[si - 1]->act_buf;
          c.slab = scratch_;
          c.H = st.inH; c.W = st.inW;
          gpu::cifar_c3_dw(c, grads_ + st.w_off, grads_ + st.b_off, ws);
          c.wd = static_cast<const char*>(packed_) + es * st.pk_dx; c.ldw = st.kgem_d;
          c.dx = stages_[si - 1]->grad_buf;
          gpu::cifar_c3_dx(c, s);
          continue;
        }
        // dZ = relu'/unpool(dY) at conv-output size
        if (!st.dz_fused) gpu::grad_xform(dtype_, dy, st.dz_buf, B, s);  // else written by the next stage's dX
        fork();
        if (st.ig_dw0) {
          // stage 0 (u8 input, few channels): the explicit im2col rows as a 1x1
          // "conv" through the implicit-GEMM dW kernel (split-K over the pixels)
          gpu::Im2colParams ic;
          ic.N = B; ic.OH = st.OH; ic.OW = st.OW; ic.KS = st.KS; ic.cs = st.stride; ic.ldk = st.kgem;
          ic.s.SH = st.inH; ic.s.SW = st.inW; ic.s.SC = st.inC; ic.s.off = st.pad; ic.s.up = 1;
          ic.s.mode = gpu::IN_U8; ic.s.src = images_; ic.s.idx = idx_;
          ic.out = col_;
          gpu::im2col(dtype_, ic, ws);
          gpu::IgemmDwParams w;
          w.B = B * st.OH * st.OW; w.H = 1; w.W = 1; w.C = st.kgem;
          w.OH = 1; w.OW = 1; w.KS = 1; w.stride = 1; w.pad = 0;
          w.M = w.B; w.Cout = st.C; w.kf = st.kgem; w.kreal = kf;
          w.perm_c = st.inC; w.perm_hw = KK;  // k = kp*inC + ci  ->  ci*KK + kp
          w.dz = st.dz_buf; w.ldz = st.C; w.in = col_;
          w.splitk = gpu::igemm_dw_splitk(w.M, st.C, st.kgem);
          w.slab = scratch_; w.slab_stride = (int64_t)(st.kgem + 1) * st.C;
          MCC_CHECK(gpu::igemm_dw_slab_bytes(st.C, st.kgem, w.splitk) <= scratch_bytes_, "igemm dW0 scratch too small");
          gpu::igemm_dw(w, grads_ + st.w_off, grads_ + st.b_off, 0.f, ws);
        }
        if (st.ig_dw) {
          // dW, db: implicit GEMM over the pixels (split-K slabs + ordered reduce)
          gpu::IgemmDwParams w;
          w.B = B; w.H = st.inH; w.W = st.inW; w.C = st.inC;
          w.OH = st.OH; w.OW = st.OW; w.KS = st.KS; w.stride = st.stride; w.pad = st.pad;
          w.M = B * st.OH * st.OW; w.Cout = st.C; w.kf = kf;
          w.dz = st.dz_buf; w.ldz = st.C; w.in = stages_[si - 1]->act_buf;
          w.splitk = gpu::igemm_dw_splitk(w.M, st.C, kf);
          w.slab = scratch_; w.slab_stride = (int64_t)(kf + 1) * st.C;
          MCC_CHECK(gpu::igemm_dw_slab_bytes(st.C, kf, w.splitk) <= scratch_bytes_, "igemm dW scratch too small");
          gpu::igemm_dw(w, grads_ + st.w_off, grads_ + st.b_off, 0.f, ws);
        }
        // dW, db = dZ^T [im2col(X) | 1]  (split-K over B*OH*OW)
        if (!st.ig_dw && !st.ig_dw0) {
        gpu::Im2colParams ic;
        ic.N = B; ic.OH = st.OH; ic.OW = st.OW; ic.KS = st.KS; ic.cs = st.stride; ic.ldk = st.kgem;
        ic.s.SH = st.inH; ic.s.SW = st.inW; ic.s.SC = st.inC; ic.s.off = st.pad; ic.s.up = 1;
        if (si == 0) { ic.s.mode = gpu::IN_U8; ic.s.src = images_; ic.s.idx = idx_; }
        else { ic.s.mode = gpu::IN_PLAIN; ic.s.src = stages_[si - 1]->act_buf; }
        ic.out = col_;
        gpu::im2col(dtype_, ic, s);
        gpu::GemmParams w;
        const int64_t rows = (int64_t)B * st.OH * st.OW;
        w.M = st.C; w.N = kf + 1; w.K = (int)rows;
        w.A = st.dz_buf; w.lda = st.C; w.ta = true;
        w.B = col_; w.ldb = st.kgem; w.tb = true; w.ones_col = kf;
        w.epi = gpu::EPI_PARTIAL; w.Cf = scratch_; w.ldc = r8(kf + 1);
        w.splitk = dw_splitk(st.C, kf + 1, rows);
        w.partial_stride = (int64_t)st.C * w.ldc;
        MCC_CHECK((size_t)w.splitk * w.partial_stride * 4 <= scratch_bytes_, "big conv dW scratch too small");
        gpu::gemm(dtype_, w, s);
        gpu::DwReduceParams r;
        r.S = w.splitk; r.Nout = st.C; r.kfeat = kf; r.ldp = w.ldc; r.part = scratch_;
        r.partial_stride = w.partial_stride;
        r.gw = grads_ + st.w_off; r.gb = grads_ + st.b_off;
        r.permC = st.inC; r.permHW = KK;  // k = kp*inC + ci  ->  ci*KK + kp
        gpu::dw_reduce(r, s);
        }
        if (si > 0 && st.ig_dx) {
          // dX = stride-1 conv of dZ with the flipped weights (pad KS-1-pad)
          gpu::IgemmParams d;
          d.B = B; d.H = st.OH; d.W = st.OW; d.C = st.C;
          d.OH = st.inH; d.OW = st.inW; d.KS = st.KS; d.stride = 1; d.pad = st.KS - 1 - st.pad;
          d.M = B * st.inH * st.inW; d.N = st.inC; d.K = KK * st.C;
          d.in = st.dz_buf;
          d.w = static_cast<const char*>(packed_) + es * st.pk_dx; d.ldw = st.kgem_d;
          d.epi_bias_act = false;
          d.out = stages_[si - 1]->grad_buf; d.ldo = st.inC;
          if (stages_[si - 1]->dz_fused) {  // dZ of the ReLU stage below: masked / unpooled in the epilogue
            const Stage& pv = *stages_[si - 1];
            d.out = pv.dz_buf;
            d.relu_mask = pv.act_buf;
          }
          gpu::igemm_conv(d, s);
        } else if (si > 0) {
          // dX = im2col(zero-inserted dZ) x flipped W^T
          gpu::Im2colParams id;
          id.N = B; id.OH = st.inH; id.OW = st.inW; id.KS = st.KS; id.cs = 1; id.ldk = st.kgem_d;
          id.s.mode = gpu::IN_PLAIN; id.s.src = st.dz_buf;
          id.s.SH = st.OH; id.s.SW = st.OW; id.s.SC = st.C; id.s.off = st.KS - 1 - st.pad; id.s.up = st.stride;
          id.out = col_;
          gpu::im2col(dtype_, id, s);
          gpu::GemmParams d;
          d.M = B * st.inH * st.inW; d.N = st.inC; d.K = KK * st.C;
          d.A = col_; d.lda = st.kgem_d;
          d.B = static_cast<const char*>(packed_) + es * st.pk_dx; d.ldb = st.kgem_d;
          d.epi = gpu::EPI_DACT; d.act = gpu::ACT_NONE;
          d.C = stages_[si - 1]->grad_buf; d.ldc = st.inC;
          gpu::gemm(dtype_, d, s);
        }
        continue;
      }
      fork();
      if (st.direct1) {
        gpu::Conv1DirectParams w = st.pd1;
        w.N = B; w.x = images_; w.idx = idx_;
        w.dy = static_cast<const float*>(st.grad_buf); w.arg = st.arg_buf;
        w.slab = scratch_;
        gpu::conv1_direct_dw(w, grads_ + st.w_off, grads_ + st.b_off, ws);
      } else if (st.c0dw) {  // small-image first layer (CIFAR): as the large-image path
        gpu::Conv0DwParams c = st.pc0;
        c.B = B; c.x = images_; c.idx = idx_;
        c.dy = static_cast<const uint16_t*>(st.grad_buf); c.arg = st.arg_buf;
        c.slab = scratch_;
        gpu::conv0_dw(c, grads_ + st.w_off, grads_ + st.b_off, ws);
      } else if (st.direct_dw) {
        gpu::Conv1DirectParams w = st.pd1;
        w.N = B; w.xf = static_cast<const float*>(stages_[si - 1]->act_buf);
        w.dy = static_cast<const float*>(st.grad_buf); w.arg = st.arg_buf;
        w.slab = scratch_;
        gpu::conv_direct_dw(w, grads_ + st.w_off, grads_ + st.b_off, ws);
      } else if (st.rows_dw) {
        gpu::ConvDwRowsParams w = st.prw;
        w.N = B;
        w.x = images_; w.idx = idx_;
        w.dy = st.grad_buf; w.aux_y = st.act_buf; w.aux_arg = st.arg_buf;
        w.slab = scratch_;
        gpu::conv_dw_rows(w, grads_ + st.w_off, grads_ + st.b_off, ws);
      } else if (st.c2bwd) {
        gpu::CifarC2BwdParams c;
        c.B = B; c.dy = st.grad_buf; c.arg = st.arg_buf; c.x = stages_[si - 1]->act_buf;
        c.slab = scratch_;
        gpu::cifar_c2_dw(c, grads_ + st.w_off, grads_ + st.b_off, ws);
      } else if (st.pipe_dw) {
        gpu::ConvDwPipeParams w = st.pdw;
        w.N = B;
        if (si == 0) { w.x.src = images_; w.x.idx = idx_; }
        else w.x.src = stages_[si - 1]->act_buf;
        w.dy.src = st.grad_buf; w.dy.aux_y = st.act_buf; w.dy.aux_arg = st.arg_buf;
        w.slab = scratch_;
        gpu::conv_dw_pipe(w, ws);
        gpu::conv_dw_pipe_reduce(w, grads_ + st.w_off, grads_ + st.b_off, ws);
      }
      if (st.c2bwd) {
        gpu::CifarC2BwdParams c;
        c.B = B; c.dy = st.grad_buf; c.arg = st.arg_buf;
        c.wd = static_cast<const char*>(packed_) + es * st.pk_dx; c.ldw = st.kpad_d;
        c.dx = stages_[si - 1]->grad_buf;
        gpu::cifar_c2_dx(c, s);
      } else       if (st.pipe_dx && si > 0) {
        gpu::ConvPipeParams p = st.pdx;
        p.N = B;
        p.in.src = st.grad_buf; p.in.aux_y = st.act_buf; p.in.aux_arg = st.arg_buf;
        p.wpk = static_cast<const char*>(packed_) + es * st.pk_dx;
        p.out = stages_[si - 1]->grad_buf;
        gpu::conv_pipe_forward(p, s);
      }
      const bool dw_done = st.pipe_dw || st.rows_dw || st.direct1 || st.direct_dw || st.c0dw || st.c2bwd;
      if (dw_done && (st.pipe_dx || st.c2bwd || si == 0)) continue;
      // weight gradient
      if (!dw_done) {
      gpu::ConvDwParams w;
      w.N = B; w.imgs = st.imgs_dw;
      w.nx = (int)std::min<int64_t>(ceil_div(B, st.imgs_dw), st.nx_dw);
      w.Cin = st.inC; w.CL = st.CLdw; w.cvec = st.cvec;
      w.LH = (st.OH - 1) * st.stride + st.KS; w.LW = (st.OW - 1) * st.stride + st.KS;
      w.OH = st.OH; w.OW = st.OW; w.cs = st.stride; w.KS = st.KS; w.Cout = st.C;
      w.kbias = st.kbias; w.ncols_pad = st.ncols_pad; w.cout_pad = st.cout_pad; w.ppad = st.ppad;
      w.x.SH = st.inH; w.x.SW = st.inW; w.x.SC = st.inC; w.x.off = st.pad; w.x.up = 1;
      if (si == 0) { w.x.mode = gpu::IN_U8; w.x.src = images_; w.x.idx = idx_; }
      else { w.x.mode = gpu::IN_PLAIN; w.x.src = stages_[si - 1]->act_buf; }
      w.dy = dy;
      w.slab = scratch_;
      MCC_CHECK((size_t)w.nx * w.cout_pad * w.ncols_pad * 4 <= scratch_bytes_, "conv dW scratch too small");
     
      gpu::conv_dw(dtype_, w, ws);
      gpu::ConvDwReduceParams r;
      r.nx = w.nx; r.Cout = st.C; r.Cin = st.inC; r.KS = st.KS; r.CG = st.CLdw; r.cvec = st.cvec;
      r.cout_pad = st.cout_pad; r.ncols_pad = st.ncols_pad; r.kbias = st.kbias;
      r.slab = scratch_; r.gw = grads_ + st.w_off; r.gb = grads_ + st.b_off;
      gpu::conv_dw_reduce(r, ws);
      }
      // data gradient into the previous stage's output gradient
      if (si > 0 && st.direct_dx) {
        gpu::Conv1DirectParams p = st.pd1;
        p.N = B; p.wd = reinterpret_cast<const float*>(packed_) + st.pk_dx;
        p.dy = static_cast<const float*>(st.grad_buf); p.arg = st.arg_buf;
        gpu::conv_direct_dx(p, static_cast<float*>(stages_[si - 1]->grad_buf), s);
      } else if (si > 0 && !st.pipe_dx) {
        gpu::ConvParams p;
        p.N = B; p.imgs = st.imgs_dx;
        p.Cin = st.C; p.CL = st.CLd; p.cvec = st.cvec_d;
        p.LH = st.inH + st.KS - 1; p.LW = st.inW + st.KS - 1;
        p.OH = st.inH; p.OW = st.inW; p.cs = 1; p.KS = st.KS;
        p.Cout = st.inC; p.nchunks = st.nchunks_d; p.kpad = st.kpad_d;
        p.pool = 1; p.bias_act = false;
        p.in = dy;
        p.in.off = st.KS - 1 - st.pad; p.in.up = st.stride;
        p.wpk = static_cast<const char*>(packed_) + es * st.pk_dx;
        p.out = stages_[si - 1]->grad_buf;
       
        gpu::conv_forward(dtype_, p, s);
      }
    } else {
      const Stage& pv = *stages_[si - 1];
      if (st.head && head_done_) continue;  // done by loss() (xent_head)
      fork();
      if (st.fc_igdw) {
        gpu::IgemmDwParams w;
        w.B = B; w.H = 1; w.W = 1; w.C = st.in_ld;
        w.OH = 1; w.OW = 1; w.KS = 1; w.stride = 1; w.pad = 0;
        w.M = B; w.Cout = st.Nout; w.kf = st.in_ld; w.kreal = st.Kin;
        w.dz = st.grad_buf; w.ldz = st.out_ld; w.in = pv.act_buf;
        w.splitk = gpu::igemm_dw_splitk(B, st.Nout, st.in_ld);
        w.slab = scratch_; w.slab_stride = (int64_t)(st.in_ld + 1) * st.Nout;
        MCC_CHECK(gpu::igemm_dw_slab_bytes(st.Nout, st.in_ld, w.splitk) <= scratch_bytes_, "fc dW scratch too small");
        gpu::igemm_dw(w, grads_ + st.w_off, grads_ + st.b_off, 0.f, ws);
      } else if (dtype_ == DType::F32 && !ab_flag("no_fc_dw32") &&
                 gpu::fc_dw32_supported(st.Nout, st.Kin, st.out_ld, st.in_ld)) {
        // fp32 skinny-output weight gradient: all Nout rows per workgroup
        gpu::FcDw32Params w;
        w.M = st.Nout; w.N = st.Kin; w.K = B;
        w.dz = static_cast<const float*>(st.grad_buf); w.ldz = st.out_ld;
        w.x = static_cast<const float*>(pv.act_buf); w.ldx = st.in_ld;
        w.slab = scratch_; w.ldp = st.ldp;
        w.splitk = gpu::fc_dw32_splitk(st.Nout, st.Kin, B);
        w.slab_stride = (int64_t)st.Nout * st.ldp;
        MCC_CHECK((size_t)w.splitk * w.slab_stride * 4 <= scratch_bytes_, "fc dW scratch too small");
        gpu::fc_dw32(w, ws);
        gpu::DwReduceParams r;
        r.S = w.splitk; r.Nout = st.Nout; r.kfeat = st.Kin; r.ldp = st.ldp; r.part = scratch_;
        r.partial_stride = w.slab_stride;
        r.gw = grads_ + st.w_off; r.gb = grads_ + st.b_off;
        r.permC = 0; r.permHW = 0;
        gpu::dw_reduce(r, ws);
      } else {
      // weight + bias gradient: [Nout][Kin+1] = dZ^T [X | 1], split-K over the batch
      gpu::GemmParams w;
      w.M = st.Nout; w.N = st.Kin + 1; w.K = B;
      w.A = st.grad_buf; w.lda = st.out_ld; w.ta = true;
      w.B = pv.act_buf; w.ldb = st.in_ld; w.tb = true; w.ones_col = st.Kin;
      w.epi = gpu::EPI_PARTIAL; w.Cf = scratch_; w.ldc = st.ldp;
      const int sk = fc_dw_splitk(st.Nout, st.Kin + 1, B, dtype_);
      w.splitk = sk;
      w.partial_stride = (int64_t)st.Nout * st.ldp;
      gpu::gemm(dtype_, w, ws);
      gpu::DwReduceParams r;
      r.S = sk; r.Nout = st.Nout; r.kfeat = st.Kin; r.ldp = st.ldp; r.part = scratch_;
      r.partial_stride = w.partial_stride;
      r.gw = grads_ + st.w_off; r.gb = grads_ + st.b_off;
      r.permC = 0; r.permHW = 0;  // device order (see set_params)
      gpu::dw_reduce(r, ws);
      }
      // data gradient
      if (si > 0 && st.fc_wres) {
        gpu::FcTallParams t;
        t.M = B; t.N = st.Kin; t.K = st.Nout; t.f32 = dtype_ == DType::F32;
        t.A = st.grad_buf; t.lda = st.out_ld;
        t.W = static_cast<const char*>(packed_) + es * st.pk_dx; t.ldw = st.out_ld;  // W^T [Kin][out_ld]
        t.act = st.wres_act;  // x act'(pv output); a conv predecessor's staging applies its own mask
        t.out = pv.grad_buf; t.ldo = st.in_ld;
        gpu::fc_wres(t, pv.act_buf, st.in_ld, s);
      } else if (si > 0 && st.fc_tall_dx) {
        gpu::FcTallParams t;
        t.M = B; t.N = st.Kin; t.K = st.Nout; t.f32 = dtype_ == DType::F32;
        t.A = st.grad_buf; t.lda = st.out_ld;
        t.W = static_cast<const char*>(packed_) + es * st.pk_dx; t.ldw = st.out_ld;  // W^T [Kin][out_ld]
        t.bias = nullptr; t.act = gpu::ACT_NONE;  // pv is a conv (its staging applies the ReLU mask) or linear
        t.out = pv.grad_buf; t.ldo = st.in_ld;
        gpu::fc_tall(t, s);
      } else if (si > 0 && st.fc_igdx) {
        gpu::IgemmParams g;
        g.B = B; g.H = 1; g.W = 1; g.C = st.Nout;
        g.OH = 1; g.OW = 1; g.KS = 1; g.stride = 1; g.pad = 0;
        g.M = B; g.N = st.Kin; g.K = st.Nout;
        g.in = st.grad_buf;
        g.w = static_cast<const char*>(packed_) + es * st.pk_dx; g.ldw = st.out_ld;  // W^T [Kin][out_ld]
        g.epi_bias_act = false;
        g.relu_mask = pv.kind == Stage::FC && pv.act == gpu::ACT_RELU ? pv.act_buf : nullptr;
        g.out = pv.grad_buf; g.ldo = st.in_ld;
        gpu::igemm_conv(g, s);
      } else if (si > 0 && dtype_ == DType::BF16 && gpu::fc_supported(st.Kin, st.Nout)) {
        gpu::FcParams d;
        d.M = B; d.N = st.Kin; d.K = st.Nout;
        d.A = st.grad_buf; d.lda = st.out_ld;
        d.W = static_cast<const char*>(packed_) + es * st.pk_dx; d.ldw = st.out_ld;
        d.epi = gpu::EPI_DACT;
        d.act = pv.kind == Stage::FC ? pv.act : gpu::ACT_NONE;  // conv masks are applied by its staging
        d.aux = pv.act_buf; d.ldaux = st.in_ld;
        d.C = pv.grad_buf; d.ldc = st.in_ld;
        gpu::fc_forward(d, s);
      } else if (si > 0) {
        gpu::GemmParams d;
        d.M = B; d.N = st.Kin; d.K = st.Nout;
        d.A = st.grad_buf; d.lda = st.out_ld;
        if (st.fc_big) {  // the forward copy [Nout][r8(Kin)] read K-major
          d.B = static_cast<const char*>(packed_) + es * st.pk_fwd; d.ldb = r8(st.Kin); d.tb = true;
        } else {
          d.B = static_cast<const char*>(packed_) + es * st.pk_dx; d.ldb = st.out_ld;
        }
        d.epi = gpu::EPI_DACT;
        d.act = pv.kind == Stage::FC ? pv.act : gpu::ACT_NONE;  // conv masks are applied by its staging
        d.aux = pv.act_buf; d.ldaux = st.in_ld;
        d.C = pv.grad_buf; d.ldc = st.in_ld;
        gpu::gemm(dtype_, d, s);
      }
    }
  }
  if (forked) {
    HIP_OK(hipEventRecord(join_ev_, wstream_));
    HIP_OK(hipStreamWaitEvent(s_main, join_ev_, 0));
  }
}

void GpuNet::ensure_momentum() {
  if (mom_) return;
  HIP_OK(hipMalloc(reinterpret_cast<void**>(&mom_), 4 * (size_t)spec_.nparams));
  HIP_OK(hipMemset(mom_, 0, 4 * (size_t)spec_.nparams));
}

void GpuNet::sgd(float lr, float momentum, float weight_decay, hipStream_t s) {
  if (momentum != 0.f) ensure_momentum();
  if (fused_pack_) {  // update + packed-copy refresh in one pass
    gpu::SgdPackParams p = pack_;
    p.update = true;
    p.mom = momentum != 0.f ? mom_ : nullptr;
    p.lr = lr; p.mu = momentum; p.wd = weight_decay;
    gpu::sgd_pack(dtype_, p, s);
    return;
  }
  gpu::sgd_update(params_, grads_, momentum != 0.f ? mom_ : nullptr, spec_.nparams, lr, momentum, weight_decay, s);
  pack(s);
}

void GpuNet::sgd_range(float lr, float momentum, float weight_decay, int64_t off, int64_t count, hipStream_t s) {
  MCC_CHECK(off >= 0 && count > 0 && off + count <= spec_.nparams, "sgd_range: bad parameter range");
  bool lo_ok = false, hi_ok = false;  // whole stages only: [w_off of one, end of another]
  for (const Stage* st : stages_) {
    if (st->nw + st->nb == 0) continue;
    lo_ok = lo_ok || st->w_off == off;
    hi_ok = hi_ok || st->w_off + st->nw + st->nb == off + count;
  }
  MCC_CHECK(lo_ok && hi_ok, "sgd_range: range must start and end at stage boundaries");
  if (momentum != 0.f) ensure_momentum();
  if (fused_pack_) {
    gpu::SgdPackParams p = pack_;
    p.nstages = 0;  // the weight stages inside the range (sorted by w_off, as pack_)
    for (int i = 0; i < pack_.nstages; ++i)
      if (pack_.st[i].w_off >= off && pack_.st[i].w_off < off + count) p.st[p.nstages++] = pack_.st[i];
    p.lo = off;
    p.n = off + count;
    p.update = true;
    p.mom = momentum != 0.f ? mom_ : nullptr;
    p.lr = lr; p.mu = momentum; p.wd = weight_decay;
    gpu::sgd_pack(dtype_, p, s);
    return;
  }
  gpu::sgd_update(params_ + off, grads_ + off, momentum != 0.f ? mom_ + off : nullptr, count, lr, momentum,
                  weight_decay, s);
  pack(s);  // (the table path refreshes every copy: idempotent)
}

void GpuNet::stage_param_range(int stage, int64_t& off, int64_t& count) const {
  const Stage& st = *stages_.at(stage);
  off = st.w_off;
  count = st.nw + st.nb;
}

const void* GpuNet::stage_output(int stage, int64_t& per_sample, const uint8_t** argmax) const {
  const Stage& st = *stages_.at(stage);
  // Stage 0 of a fused conv block keeps a kernel-private layout (LeNet: Y1
  // HWC-8 + planar argmax codes) or is never written (ref block: conv1 is
  // recomputed in the backward); its buffer is not the standard NCHW output.
  MCC_CHECK(!((lenet_ || refblk_) && stage == 0),
            "stage_output: stage 0 is internal to the fused conv block (no standard-layout output)");
  // the fused LeNet classifier chain keeps FC1 / FC2 activations in LDS when
  // it ran forward + backward in one kernel (loss() of a training step)
  MCC_CHECK(!(fcchain_ && fc_bwd_done_ && (stage == 2 || stage == 3)),
            "stage_output: FC activations of the fused classifier chain were not written (training step)");
  MCC_CHECK(!(fc_pending_ && (size_t)stage >= pending_from_),
            "stage_output: the FC forward is still pending (call flush_forward)");
  per_sample = st.out_elems;
  if (argmax) *argmax = st.pooled ? st.arg_buf : nullptr;
  return st.act_buf;
}

std::vector<GpuBucket> GpuNet::buckets(int64_t bucket_bytes) const {
  std::vector<GpuBucket> out;
  for (const Bucket& b : plan_buckets(spec_, bucket_bytes)) {
    GpuBucket g;
    g.stage_hi = b.stage_hi; g.stage_lo = b.stage_lo; g.off = b.off; g.count = b.count;
    // A fused conv block (lenet_bwd / ref_bwd) produces stage 0's and stage
    // 1's gradients in ONE kernel that runs after every later stage's
    // backward (LeNet-5: the FC chain's gradients are final when loss()
    // returns).  Cut the bucket that spans the block boundary so the later
    // stages' all-reduce (LeNet-5: 96 % of the gradient bytes) is issued
    // BEFORE the block's backward kernel and overlaps it on RCCL's stream;
    // the block's own small bucket is the only collective left after it.
    if ((lenet_ || refblk_) && b.stage_hi >= 2 && b.stage_lo <= 1) {
      int64_t off2 = 0, cnt2 = 0;
      stage_param_range(2, off2, cnt2);
      GpuBucket hi = g, lo = g;
      hi.stage_lo = 2; hi.off = off2; hi.count = b.off + b.count - off2;
      lo.stage_hi = 1; lo.count = off2 - b.off;
      out.push_back(hi);
      g = lo;
    }
    // ... and stage 0 joins the block's bucket (same kernel; a separate
    // stage-0 bucket would only add another latency-bound collective)
    if ((lenet_ || refblk_) && b.stage_hi == 0 && !out.empty() && out.back().stage_lo == 1 &&
        b.off + b.count == out.back().off) {
      out.back().stage_lo = 0;
      out.back().off = b.off;
      out.back().count += b.count;
      continue;
    }
    out.push_back(g);
  }
  return out;
}

}  // namespace mcc
