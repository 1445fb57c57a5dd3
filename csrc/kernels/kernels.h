// Host-visible launch API of the gfx950 kernels.  Pure C++ (no device code)
// so the engine, the pybind module and the native drivers can call into the
// kernels without being compiled as HIP translation units.
//
// Activation layout on the GPU is NHWC ("channels-last"): the MFMA epilogue
// of a 16x16 tile holds 16 consecutive output channels per pixel, so NHWC
// makes every store a contiguous run, and 8-channel groups become single
// 16-byte LDS reads in the implicit-GEMM gather.
#pragma once

#include <hip/hip_runtime_api.h>

#include <cstdint>

#include "mcc/common.h"

namespace mcc {
namespace gpu {

enum InMode : int {
  IN_PLAIN = 0,   // src is T NHWC
  IN_U8 = 1,      // src is u8 NHWC images (optionally gathered by idx), scaled 1/255
  IN_RELU = 2,    // value = (aux_y > 0) ? src : 0          (ReLU backward, no pool)
  IN_UNPOOL = 3,  // value = (argmax == pos) ? act'(aux_y) * src_pooled : 0  (2x2 maxpool + act backward, act in
                  // StageSrc::act; ReLU: argmax 4 also marks an inactive window)
  IN_TANH = 4,    // value = (1 - aux_y^2) * src                 (tanh backward, no pool)
};

enum ActKind : int { ACT_NONE = 0, ACT_RELU = 1, ACT_TANH = 2 };

// Source description for staging an NHWC tile into LDS.  The LDS tile
// coordinate j maps to source coordinate (j - off) / up when that is an
// integer in range, else zero: forward conv uses off = pad, up = 1; the
// data-gradient of a strided conv uses off = KS-1-pad, up = stride (zero
// insertion) and runs as a stride-1 conv with flipped weights.
struct StageSrc {
  int mode = IN_PLAIN;
  const void* src = nullptr;     // T* or uint8_t*
  const int32_t* idx = nullptr;  // IN_U8: optional per-image index
  const void* aux_y = nullptr;   // IN_RELU/IN_UNPOOL: layer output (T)
  const uint8_t* aux_arg = nullptr;  // IN_UNPOOL: argmax (pos in 2x2 window; 4 = ReLU-inactive window)
  int SH = 0, SW = 0, SC = 0;    // conv-grid dims of the source (pre-pool for UNPOOL)
  int PH = 0, PW = 0;            // IN_UNPOOL: pooled dims of src/aux tensors
  int off = 0, up = 1;
  int act = 1;                   // IN_UNPOOL: activation of the pooled conv (ActKind; default ReLU)
  int pk = 2, ps = 2;            // IN_UNPOOL: pool window / stride (argmax = dy * pk + dx in the window)
};

// Implicit-GEMM conv over small images staged whole in LDS ("conv_small").
// Rows = output pixels (pool-window ordered when pool==2), cols = output
// channels, K = (kernel position, input channel) in the packed order.
struct ConvParams {
  int N = 0;          // images in the batch
  int imgs = 1;       // images per workgroup
  int Cin = 0;        // staged channels (real)
  int CL = 0;         // LDS channel stride: round_up(Cin, 8) (cvec) or Cin (scalar)
  bool cvec = true;   // 8-channel vector gather (else scalar gather)
  int LH = 0, LW = 0; // LDS tile dims per image
  int OH = 0, OW = 0; // conv output dims
  int cs = 1;         // conv stride (in LDS coordinates)
  int KS = 1;
  int Cout = 0;
  int nchunks = 0;    // K chunks of 32
  int kpad = 0;       // packed K row length = nchunks*32
  int pool = 1;       // 1 or 2 (fused 2x2/2 maxpool)
  int act = ACT_RELU;
  bool bias_act = true;  // false: plain store (data-gradient form)
  StageSrc in;
  const void* wpk = nullptr;    // packed weights [round_up(Cout,16)][kpad], T
  const float* bias = nullptr;  // fp32 canonical bias [Cout]
  void* out = nullptr;          // T NHWC [N][OH'][OW'][Cout]
  uint8_t* out_arg = nullptr;   // pool argmax [N][PH][PW][Cout]: position 0..3 in the 2x2 window
                                // (first max wins), or 4 where the pooled ReLU output is <= 0 —
                                // the max-pool + ReLU backward then needs only dY and this byte
};

// Weight gradient of a conv_small layer: slab[x][co][col] partial sums over
// the images of workgroup column x; col < kbias are packed K entries and
// col == kbias is the bias gradient (a ones-column in the im2col operand).
struct ConvDwParams {
  int N = 0, imgs = 1, nx = 1;
  int Cin = 0, CL = 0;
  bool cvec = true;
  int LH = 0, LW = 0, OH = 0, OW = 0, cs = 1, KS = 1, Cout = 0;
  int kbias = 0;       // first column after the packed K entries
  int ncols_pad = 0;   // round_up(kbias + 1, 16)
  int cout_pad = 0;    // round_up(Cout, 16)
  int ppad = 0;        // pixels per stage, padded to 32
  StageSrc x;          // forward input of the layer
  StageSrc dy;         // gradient w.r.t. the conv output (via RELU/UNPOOL)
  float* slab = nullptr;  // [nx][cout_pad][ncols_pad]
};

// Row stride (elements) of the pixel-major dY tile of the bf16 transpose-read
// dW kernel.  32-byte rows are conflict-free for its 4-rows-per-lane-group
// reads; wider rows get 16 B of skew.
constexpr int conv_dw_tr_drow(int cout_pad) { return cout_pad == 16 ? 16 : cout_pad + 8; }

// Sum the dW slabs over x and scatter into the canonical fp32 gradient.
struct ConvDwReduceParams {
  int nx = 0, Cout = 0, Cin = 0, KS = 1, CG = 1;
  bool cvec = true;
  int cout_pad = 0, ncols_pad = 0, kbias = 0;
  const float* slab = nullptr;
  float* gw = nullptr;  // canonical [Cout][Cin][KS][KS]
  float* gb = nullptr;  // [Cout]
  float beta = 0.f;     // grad = beta*grad + sum (0 overwrites)
};

// ---------------------------------------------------------------------------
// Persistent, pipelined small-image convolution ("conv_pipe", bf16).
//
// A workgroup keeps its weights, index tables and zeroed LDS tiles for the
// whole launch and walks image groups blockIdx.x, +gridDim.x, ...; while it
// computes group g the global loads of group g+1 are already in flight
// (register prefetch, written to LDS after the next barrier).  Per-thread
// staging geometry is computed once, so the per-group staging is a few loads
// and 16-byte LDS writes per item.  Outputs go through an LDS tile and leave
// as coalesced 16-byte stores.
enum PipeMode : int {
  PM_U8S1 = 0,    // u8 single-channel images -> four shifted bf16 copies (see below)
  PM_PLAIN = 1,   // bf16 NHWC
  PM_RELU = 2,    // bf16 NHWC masked by (aux_y > 0)
  PM_UNPOOL = 3,  // pooled bf16 NHWC routed to the argmax of its 2x2 window (argmax 4: ReLU-inactive, nothing routed)
};
enum PipeLayout : int {
  // Cin == 1: copy c (c = 0..3) holds tile[j + c] at j, so any 4 consecutive
  // tile elements are one aligned 8-byte read from copy (e & 3).  K runs over
  // (kernel row, 8 taps), two 8-byte reads per 8-wide K fragment.
  XL_S1 = 0,
  XL_C8 = 1,  // NHWC, channels padded to a multiple of 8: one 16-byte read per fragment
  XL_ROWS = 2,  // conv_dw_rows: Cin == 1, tap-packed columns kh*KS + kw
};

struct PipeSrc {
  int mode = PM_PLAIN;
  const void* src = nullptr;
  const int32_t* idx = nullptr;      // PM_U8S1: optional per-image dataset index
  const void* aux_y = nullptr;       // PM_RELU / PM_UNPOOL
  const uint8_t* aux_arg = nullptr;  // PM_UNPOOL
  int SH = 0, SW = 0, SC = 0;        // source grid (PM_UNPOOL: the pooled grid)
  int up = 1, offy = 0, offx = 0;    // tile coordinate = (conv-grid coordinate) * up + off
  // filled by the planners
  int RW = 0;       // channels per staged item (PM_U8S1: 4 pixels)
  int per_img = 0;  // items per image
  int LWp = 0;      // destination tile row stride (pixels)
  int CL = 0;       // destination channel stride (elements)
  int IMG = 0;      // destination elements per image
  int CS = 0;       // XL_S1: elements between the shifted copies
};

// Forward conv (bias + act [+ 2x2 max-pool]) or data gradient (plain).
struct ConvPipeParams {
  int N = 0;
  int Cin = 0, OH = 0, OW = 0, cs = 1, KS = 1, Cout = 0;
  int ty0 = 0, tx0 = 0;  // tile coordinate of output pixel (0,0)'s first tap
  int epi = 0;           // 0 = pool, 1 = bias+act, 2 = plain (see FwdEpi)
  int act = ACT_RELU;
  PipeSrc in;
  const void* wpk = nullptr;  // packed bf16 weights [round_up(Cout,16)][kpad]
  const float* bias = nullptr;
  void* out = nullptr;
  uint8_t* out_arg = nullptr;
  // planner outputs
  int layout = XL_C8, imgs = 1, ngroups = 0, grid = 0, LH = 0;
  int nchunks = 0, kpad = 0;
  // XL_S1 with Cout <= 8: an MFMA row is a horizontal PAIR of output pixels;
  // columns 0..7 are the left pixel's channels, 8..15 the right one's (its
  // taps shifted by one inside the 8-wide K window).  Packed weights:
  // [16][kpad], col n < 8: k = kh*8 + kw; col 8 + n: k = kh*8 + kw + pair.
  // pair == 2 (pooled, KS <= 6): rows are the four positions of a 2x2 window
  // and columns 8.. compute the window two pixels to the right (taps shifted
  // by two), so the max-pool is in-lane.
  int pair = 0;
  size_t lds = 0;
  uint32_t rows_mh = 0, rows_ml = 0;  // division magic for the GEMM rows per image (set at launch)
};
// Geometry for a layer (N may be the maximum batch); false when the layer is
// outside what the pipelined kernels cover (the caller keeps conv_small).
bool conv_pipe_plan(ConvPipeParams& p);
void conv_pipe_forward(const ConvPipeParams& p, hipStream_t s);

// Weight gradient: slab[x][co][col], x = workgroup (grid), col < kbias the
// packed columns (XL_S1: kh*8 + kw; XL_C8: (kh*KS + kw)*CL + c), col ==
// kbias the bias gradient.
struct ConvDwPipeParams {
  int N = 0;
  int Cin = 0, OH = 0, OW = 0, cs = 1, KS = 1, Cout = 0;
  int ty0 = 0, tx0 = 0;
  PipeSrc x;   // layer input (tile with halo)
  PipeSrc dy;  // output gradient at the conv grid, pixel-major [pix][drow]
  float* slab = nullptr;
  // planner outputs
  int layout = XL_C8, imgs = 1, ngroups = 0, grid = 0, LH = 0;
  int cout_pad = 0, drow = 0, kbias = 0, ncols_pad = 0, ppad = 0;
  // wsplit: the 4 waves own different column tiles and each walks every
  // pixel chunk (wide-Cout layers: the staged group is shared by 4x more
  // columns; otherwise the waves split the pixel chunks of the same tiles)
  int wsplit = 0;
  size_t lds = 0;
};
bool conv_dw_pipe_plan(ConvDwPipeParams& p);
void conv_dw_pipe(const ConvDwPipeParams& p, hipStream_t s);
// Reduce the slabs of conv_dw_pipe into the canonical fp32 gradient.
void conv_dw_pipe_reduce(const ConvDwPipeParams& p, float* gw, float* gb, hipStream_t s);
// Deterministic two-level reduce of per-workgroup dW slabs [nx][cout_pad][ncols_pad]
// (chunk partials in `part`, ceil(nx/64) * cout_pad * ncols_pad floats) into
// gw[Cout][Cin][KS][KS] / gb[Cout]; `layout` names the slab column order.
// wscale multiplies the weight columns (not the bias), e.g. a 1/255 input scale
// the kernel left out of its operand.
void dw_slab_reduce(const float* slab, int nx, int cout_pad, int ncols_pad, float* part, int Cout, int Cin, int KS,
                    int layout, int CL, int kbias, float* gw, float* gb, hipStream_t s, float wscale = 1.f);

// Row-chunked weight gradient of a single-channel (u8) stride-1 first layer
// (conv_rows.hip): M = output channels, N = tap-packed kernel positions + a
// ones column (bias), K = one 32-pixel output row; dZ staged channel-planar
// with the max-pool / ReLU backward applied while staging, the input as four
// shifted bf16 copies.  Persistent over image groups; fp32 slab per
// workgroup, then dw_slab_reduce.
// fp32 small conv with fused ReLU + 2x2/2 max-pool, direct VALU form
// (conv_direct.hip): forward for the LeNet-class shapes (Cin 1 -> 6, 6 -> 16,
// 5x5) and the single-channel layer's weight gradient.  Canonical fp32
// weights [C][Cin][KS][KS] and bias are read directly (no packed copy).
struct Conv1DirectParams {
  int N = 0, H = 0, W = 0, Cin = 1, KS = 5, pad = 0, C = 0, OH = 0, OW = 0, PH = 0, PW = 0;
  const uint8_t* x = nullptr;     // u8 images [.][H][W][Cin] (when xf is null)
  const int32_t* idx = nullptr;   // optional per-image dataset index
  const float* xf = nullptr;      // fp32 NHWC input [N][H][W][Cin] (a previous layer)
  const float* wt = nullptr;      // forward: tap-major weights [Cin][KS*KS][C] (packed copy)
  const float* wd = nullptr;      // data gradient: flipped tap-major [C][KS*KS][Cin], wd[i][t][c] = w[i][c][KK-1-t]
  const float* bias = nullptr;
  float* out = nullptr;           // forward: pooled [N][PH][PW][C]
  uint8_t* out_arg = nullptr;     //          argmax (4: ReLU-inactive window)
  const float* dy = nullptr;      // weight gradient: pooled output gradient [N][PH][PW][C]
  const uint8_t* arg = nullptr;   //                  its argmax bytes
  float* slab = nullptr;          //                  [grid][C][Cin*KS*KS + 1] partial sums
};
bool conv_direct_fwd_supported(const Conv1DirectParams& p);
bool conv1_direct_dw_supported(const Conv1DirectParams& p);
size_t conv1_direct_slab_bytes(const Conv1DirectParams& p);
void conv_direct_forward(const Conv1DirectParams& p, hipStream_t s);
// data gradient of the 6 -> 16 5x5 pooled conv into dX [N][H][W][Cin] from
// the pooled dY / argmax (p.dy, p.arg) and the canonical weights p.w
bool conv_direct_dx_supported(const Conv1DirectParams& p);
void conv_direct_dx(const Conv1DirectParams& p, float* dx, hipStream_t s);
void conv1_direct_dw(const Conv1DirectParams& p, float* gw, float* gb, hipStream_t s);
// weight gradient of the 6 -> 16 5x5 pooled conv from its fp32 NHWC input
// (p.xf) and the pooled dY / argmax
bool conv_direct_dw_supported(const Conv1DirectParams& p);
size_t conv_direct_dw_slab_bytes(const Conv1DirectParams& p);
void conv_direct_dw(const Conv1DirectParams& p, float* gw, float* gb, hipStream_t s);
// LeNet-5 shapes: sparse (argmax-only) fp32 weight gradients, slab layout of
// conv1_direct_dw's reduce (lenet_f32.hip); used by conv1_direct_dw /
// conv_direct_dw unless MCC_AB=f32_dense_dw
int lenet32_dw1_grid(int N);
int lenet32_dw2_grid(int N);
void lenet32_dw1(const Conv1DirectParams& p, hipStream_t s);
void lenet32_dw2(const Conv1DirectParams& p, hipStream_t s);
void lenet32_conv2_fwd(const Conv1DirectParams& p, hipStream_t s);  // LeNet-5 conv2 forward on f32 MFMA

// Forward of the u8 RGB first conv (C = 3, 3x3, stride 1, pad 1, bias + ReLU
// + 2x2/2 max-pool fused), bf16 MFMA, output pooled NHWC [N][H/2][W/2][Cout]
// + argmax bytes (4: ReLU-inactive window) (conv_u8.hip)
struct U8ConvParams {
  int N = 0, H = 0, W = 0, Cout = 0;
  const uint8_t* x = nullptr;     // u8 images [.][H][W][3]
  const int32_t* idx = nullptr;   // optional per-image dataset index
  const float* w = nullptr;       // canonical fp32 weights [Cout][3][3][3] (rounded to bf16 in-kernel)
  const float* bias = nullptr;
  uint16_t* out = nullptr;       // bf16 bits
  uint8_t* out_arg = nullptr;
};
bool u8conv_fwd_supported(const U8ConvParams& p);
void u8conv_forward(const U8ConvParams& p, hipStream_t s);

// Weight gradient of a large-image first conv (u8 input, C <= 3, 3x3, stride
// 1, pad 1, fused ReLU + 2x2/2 max-pool, Cout <= 64), bf16 (conv0_dw.hip):
// GEMM operands built in LDS from the pooled dY / argmax and the u8 images.
struct Conv0DwParams {
  int B = 0, H = 0, W = 0, C = 0, PH = 0, PW = 0, Cout = 0;
  const uint8_t* x = nullptr;     // u8 images [.][H][W][C]
  const int32_t* idx = nullptr;   // optional per-image dataset index
  const uint16_t* dy = nullptr;   // pooled output gradient, bf16 bits [B][PH][PW][Cout]
  const uint8_t* arg = nullptr;   // argmax (4: ReLU-inactive window)
  float* slab = nullptr;          // per-workgroup partials (conv0_dw_slab_bytes)
};
bool conv0_dw_supported(const Conv0DwParams& p);
size_t conv0_dw_slab_bytes(const Conv0DwParams& p);
void conv0_dw(const Conv0DwParams& p, float* gw, float* gb, hipStream_t s);

// LeNet-5 conv block (lenet.hip): conv1 1->6 5x5 pad 2 + ReLU + 2x2 pool and
// conv2 6->16 5x5 + ReLU + 2x2 pool on 28x28 u8 images, bf16.  Layouts:
// y1 [B][14][14][8] bf16 (channels 6..7 zero), a1 [B][6][14][16] u8,
// y2 [B][25][16] bf16, a2 [B][25][16] u8 (argmax 0..3 in the window, or 4 =
// ReLU-inactive window).  Weights are read from the fp32 master (canonical).
struct LenetFwdParams {
  int B = 0;
  const uint8_t* x = nullptr;     // u8 dataset [N][28][28]
  const int32_t* idx = nullptr;   // [B] sample indices (nullable)
  const float *w1 = nullptr, *b1 = nullptr, *w2 = nullptr, *b2 = nullptr;
  void* y1 = nullptr;
  uint8_t* a1 = nullptr;
  void* y2 = nullptr;
  uint8_t* a2 = nullptr;
};
struct LenetBwdParams {
  int B = 0;
  const uint8_t* x = nullptr;
  const int32_t* idx = nullptr;
  const float* w2 = nullptr;      // fp32 master W2 (canonical)
  const void* dy2 = nullptr;      // [B][25][16] gradient of the pooled conv2 output
  const uint8_t* a2 = nullptr;
  const void* y1 = nullptr;
  const uint8_t* a1 = nullptr;
  float* slab = nullptr;          // lenet_slab_bytes()
  float *gw1 = nullptr, *gb1 = nullptr, *gw2 = nullptr, *gb2 = nullptr;  // canonical gradients (written)
};
// LeNet-5 classifier chain (lenet_fc.hip): FC 400 -> 120 ReLU -> 84 ReLU -> 10
// + softmax-CE forward AND backward in one persistent kernel, bf16 weights
// (the packed [out][ld] compute copies), fp32 accumulation.  Writes the fp32
// logits / predictions (optional), the loss statistics, the bf16 gradient of
// the FC input and -- through per-workgroup slabs and a fixed-order reduce --
// the canonical gradients of the three layers (W1 b1 W2 b2 W3 b3, contiguous,
// 59,134 floats starting at `grads`).
struct LenetFcParams {
  int B = 0;
  const void* y = nullptr; int ldy = 0;          // FC input [B][ldy] bf16 (features in device order)
  const void *w1 = nullptr, *w2 = nullptr, *w3 = nullptr;  // packed bf16 [out][ldw]
  int ldw1 = 0, ldw2 = 0, ldw3 = 0;
  const float *b1 = nullptr, *b2 = nullptr, *b3 = nullptr;  // fp32 master biases
  const uint8_t* labels = nullptr;
  const int32_t* idx = nullptr;                  // label of row b = labels[idx[b]] (nullable)
  float scale = 1.f;                             // dlogits scale (1 / global batch)
  float* logits = nullptr; int ldl = 0;          // optional fp32 logits
  int32_t* pred = nullptr;                       // optional argmax
  unsigned long long* stats = nullptr;           // loss / mse / correct (fixed point)
  void* dy = nullptr; int ldd = 0;               // gradient of the FC input [B][ldd] bf16
  float* slab = nullptr;                         // lenet_fc_slab_bytes(max batch)
};
bool lenet_fc_supported(int kin, int n1, int n2, int n3);
size_t lenet_fc_slab_bytes(int max_batch);
int lenet_fc_grad_count();
void lenet_fc(const LenetFcParams& p, float* grads, hipStream_t s);

int lenet_bwd_grid();
size_t lenet_slab_bytes();
int lenet_y1_elems();   // per image
int lenet_a1_bytes();   // per image
void lenet_forward(const LenetFwdParams& p, hipStream_t s);
void lenet_backward(const LenetBwdParams& p, hipStream_t s);

// Reference-model conv block (refnet.hip): conv1 1->16 3x3 s2 p1 + ReLU and
// conv2 16->32 3x3 s2 p1 + ReLU on 28x28 u8 images (cnn.c:416-428), bf16.
// Forward writes only Y2 [B][49][32] (NHWC, the FC input); the backward
// recomputes conv1 per image and produces dW1, db1, dW2, db2.
struct RefFwdParams {
  int B = 0;
  bool f32 = false;  // fp32 block (refnet_f32.hip): y2 / dy2 are fp32
  const uint8_t* x = nullptr;
  const int32_t* idx = nullptr;
  const float *w1 = nullptr, *b1 = nullptr, *w2 = nullptr, *b2 = nullptr;  // fp32 masters (canonical OIHW)
  void* y2 = nullptr;  // bf16 [B][49][32]
};
struct RefBwdParams {
  int B = 0;
  bool f32 = false;
  const uint8_t* x = nullptr;
  const int32_t* idx = nullptr;
  const float *w1 = nullptr, *b1 = nullptr, *w2 = nullptr;
  const void* y2 = nullptr;   // bf16 [B][49][32] (ReLU mask of conv2)
  const void* dy2 = nullptr;  // bf16 [B][49][32] gradient of Y2
  float* slab = nullptr;      // ref_slab_bytes()
  float *gw1 = nullptr, *gb1 = nullptr, *gw2 = nullptr, *gb2 = nullptr;  // canonical gradients (written)
};
size_t ref_slab_bytes(bool f32 = false);
void ref_forward(const RefFwdParams& p, hipStream_t s);
void ref_backward(const RefBwdParams& p, hipStream_t s);
// fp32 kernels (refnet_f32.hip); ref_forward / ref_backward dispatch on p.f32
size_t ref32_slab_bytes();
void ref32_forward(const RefFwdParams& p, hipStream_t s);
void ref32_backward(const RefBwdParams& p, hipStream_t s);

struct ConvDwRowsParams {
  int N = 0, SH = 0, SW = 0, OH = 0, OW = 0, KS = 1, pad = 0, Cout = 0;
  const uint8_t* x = nullptr;        // u8 images [*][SH][SW]
  const int32_t* idx = nullptr;      // optional per-image dataset index
  int dmode = PM_UNPOOL;             // PM_UNPOOL (2x2/2 pool + ReLU) or PM_RELU
  const void* dy = nullptr;          // bf16 NHWC [N][DH][DW][Cout]
  const void* aux_y = nullptr;       // bf16 NHWC layer output (ReLU mask)
  const uint8_t* aux_arg = nullptr;  // PM_UNPOOL argmax bytes
  int DH = 0, DW = 0;                // dY grid (pooled for PM_UNPOOL)
  float* slab = nullptr;             // scratch (conv_dw_rows_scratch_bytes)
  // planner outputs
  int A = 0, Pw = 0, LH = 0, CS = 0, ximg = 0, dplane = 0, dzimg = 0, KK = 0, ntiles = 0;
  int m0 = 0, nblk = 0, imgs = 1, ngroups = 0, grid = 0;
  size_t lds = 0;
};
bool conv_dw_rows_plan(ConvDwRowsParams& p);
size_t conv_dw_rows_scratch_bytes(const ConvDwRowsParams& p);
void conv_dw_rows(const ConvDwRowsParams& p, float* gw, float* gb, hipStream_t s);

enum GemmEpi : int {
  EPI_BIAS_ACT = 0,  // C = act(acc + bias[n])  (T)
  EPI_LOGITS = 1,    // Cf = acc + bias[n]      (fp32)
  EPI_DACT = 2,      // C = acc * act'(aux[m][n]) (T), or plain when act == ACT_NONE
  EPI_PARTIAL = 3,   // Cf[z][m][n] = acc       (fp32 split-K partial)
};

// C[M][N] = A[M][K] * B[N][K]^T; ta: A stored [K][M]; tb: B stored [K][N].
struct GemmParams {
  int M = 0, N = 0, K = 0;
  const void* A = nullptr; int lda = 0; bool ta = false;
  const void* B = nullptr; int ldb = 0; bool tb = false;
  int ones_col = -1;        // B row n == ones_col reads 1.0 (bias-grad column)
  int epi = EPI_BIAS_ACT;
  int act = ACT_NONE;
  const float* bias = nullptr;
  const void* aux = nullptr; int ldaux = 0;
  void* C = nullptr; int ldc = 0;   // T output
  float* Cf = nullptr;              // fp32 output (logits / partials)
  int splitk = 1;                   // gridDim.z
  int64_t partial_stride = 0;       // elements between split-K partials
};

// Weights-resident FC GEMM (bf16, fc.hip): C[M][N] = epi(A[M][K] W[N][K]^T)
// for N*K small enough that W lives in one CU's LDS (fc_supported).
// Epilogues: EPI_BIAS_ACT (C bf16), EPI_LOGITS (Cf fp32, ldc), EPI_DACT
// (C = acc * act'(aux), aux = the activation OUTPUT of the producing layer).
struct FcParams {
  int M = 0, N = 0, K = 0;
  const void* A = nullptr; int lda = 0;
  const void* W = nullptr; int ldw = 0;
  int epi = EPI_BIAS_ACT;
  int act = ACT_NONE;
  const float* bias = nullptr;
  const void* aux = nullptr; int ldaux = 0;
  void* C = nullptr; int ldc = 0;
  float* Cf = nullptr;
  long long* dbg = nullptr;  // diagnostics: per-wave phase timestamps [grid][4 waves][4]
};
bool fc_supported(int N, int K);
void fc_forward(const FcParams& p, hipStream_t s);



// Reduce split-K partials of a weight gradient into the canonical grad:
// gw[n*Kc + perm(k)] (k < kfeat), gb[n] (k == kfeat).
struct DwReduceParams {
  int S = 1, Nout = 0, kfeat = 0, ldp = 0;
  const float* part = nullptr;  // [S][Nout][ldp]
  int64_t partial_stride = 0;
  float* gw = nullptr;
  float* gb = nullptr;
  int permC = 0, permHW = 0;    // k = hw*C + c  ->  c*HW + hw   (0: identity)
  float beta = 0.f;
};

// Training statistics accumulate as fixed point (loss and mse per sample
// are >= 0): value * kStatScale rounded, added with 64-bit integer atomics.
constexpr double kStatScale = 4294967296.0;  // 2^32
// stats[kStatNaN] != 0: a non-finite / overflowing partial was seen since the
// last zero_stats (loss and MSE then read as NaN)
constexpr int kStatNaN = 3;
// stats[0..2] -> out[0..2] as floats (device side, for the drivers' logs)
void stats_to_f32(const unsigned long long* stats, float* out, hipStream_t s);

struct XentParams {
  int M = 0, N = 0;
  const float* logits = nullptr; int ldl = 0;
  const int32_t* labels_idx = nullptr;  // per-sample dataset index (nullable)
  const uint8_t* labels = nullptr;      // dataset labels (gathered by idx)
  void* dlogits = nullptr; int ldd = 0; // T
  float scale = 1.f;                    // dlogits = (p - y) * scale
  // [0]=loss sum [1]=mse sum (fixed point, kStatScale units) [2]=correct:
  // integer atomics, so the sums are deterministic and the count exact
  unsigned long long* stats = nullptr;
  float* probs = nullptr;               // optional fp32 probs [M][N] (eval)
  int32_t* pred = nullptr;              // optional argmax per sample
};

// Fused classifier head (bf16): softmax-CE forward+backward of XentParams
// plus the last FC layer's backward, so dlogits never leave the workgroup:
//   e      = (softmax(logits) - onehot) * scale         (bf16-rounded)
//   dh     = (e W) * act'(h)          -> bf16 [M][ldh], pad columns zeroed
//   slab_b = e^T [h | 1] over the workgroup's 128 rows: slab[b][n][ldp]
//            (n < N, k <= Kin, k == Kin the bias) for dw_reduce (S = nwg)
// Needs N <= 16, Kin < 128, ldh % 8 == 0.
struct XentHeadParams {
  XentParams x;
  const void* h = nullptr; int ldh = 0;     // last FC input activations, T [M][ldh]
  const float* w = nullptr;                // last FC weights, fp32 [N][Kin]
  int Kin = 0, act = 0;                    // act of h's producer (ACT_*)
  void* dh = nullptr;                      // T [M][ldh]
  float* slab = nullptr; int ldp = 0;      // [nwg][N][ldp]
  const float* bias = nullptr;             // non-null: the head computes the logits itself (its FC forward)
  // bf16 only, optional: the packed bf16 weights [N][ldw] (ldw % 8 == 0,
  // 16-byte aligned) select the MFMA head (xent_head_mfma_kernel)
  const void* wpk = nullptr; int ldw = 0;
};
bool xent_head_supported(int N, int Kin, int ldh);
int xent_head_slabs(int M);
// returns the number of slabs written (<= xent_head_slabs(M); dw_reduce's S)
int xent_head(DType t, const XentHeadParams& p, hipStream_t s);  // T = bf16 or fp32

// Explicit im2col for the large-image path: out[(n*OH+oy)*OW+ox][k], k =
// (kh*KS+kw)*SC + c (zero for k >= KS*KS*SC), source through `s` (tile
// coordinate oy*cs+kh maps to source (.. - off)/up).
struct Im2colParams {
  int N = 0, OH = 0, OW = 0, KS = 1, cs = 1;
  int ldk = 0;  // row stride of out (multiple of 8)
  StageSrc s;
  void* out = nullptr;
};
void im2col(DType t, const Im2colParams& p, hipStream_t s);
void maxpool2(DType t, const void* in, void* out, uint8_t* arg, int N, int H, int W, int C, hipStream_t s,
              bool post_relu = true);
// k x k / stride max-pool (floor mode, first max wins, argmax = dy * k + dx; k <= 15)
void maxpool(DType t, const void* in, void* out, uint8_t* arg, int N, int H, int W, int C, int k, int stride,
             hipStream_t s);
// dz[n][y][x][c] = transform(src) at the conv-output grid (SH x SW x SC)
void grad_xform(DType t, const StageSrc& src, void* dz, int N, hipStream_t s);

// ---------------------------------------------------------------------------
// Implicit-GEMM convolution for large images (igemm.hip, bf16 NHWC): no
// im2col matrix; 16-byte pieces of the implicit operand are DMA'd straight
// into LDS.  Forward / data gradient:
//   out[m][n] = epi(sum_k in(m, k) w[n][k]),  m = (b, oy, ox),
//   k = (ky*KS + kx)*C + c,  in(m, k) = in[b][oy*stride-pad+ky][ox*stride-pad+kx][c]
struct DivMagic { uint32_t mh = 0, ml = 0; };  // exact division by a constant (set at launch)
struct IgemmParams {
  int B = 0, H = 0, W = 0, C = 0;    // input NHWC
  int OH = 0, OW = 0, KS = 1, stride = 1, pad = 0;
  int M = 0, N = 0, K = 0;           // M = B*OH*OW, N = out channels, K = KS*KS*C
  const void* in = nullptr;          // bf16 [B][H][W][C]
  const void* w = nullptr;           // bf16 [N][ldw], k order as above
  int ldw = 0;
  const float* bias = nullptr;       // [N] (epi_bias_act)
  bool epi_bias_act = true;          // false: plain store (data gradient)
  int act = ACT_RELU;
  void* out = nullptr;               // bf16 [M][ldo]   (pool: [M/4][N] pooled)
  int ldo = 0;
  bool pool = false;                 // fused 2x2/2 max-pool (+ argmax bytes [M/4][N])
  uint8_t* out_arg = nullptr;
  bool u8 = false;                   // input = u8 image set (first layer), scaled 1/255
  const int32_t* idx = nullptr;      // u8: optional per-sample image index
  bool u8_runs = false;              // set at launch: u8 C=3 3x3 pad-1 im2col rows from dword runs
  const void* relu_mask = nullptr;   // bf16; data gradient only: out = dX * (relu_mask > 0), same layout as out
                                     // (writes the next-lower ReLU layer's dZ directly: no grad_xform pass)
  int tile = -1;                     // -1 auto, 0: 128x128 kernel,
                                     // 128 / 256: 256-pixel x 128 / 256-channel kernel where legal
  DivMagic div_ohw, div_ow;
  int c_shift = -1;                  // set at launch: log2(C) when C is a power of two (K-step tap by shift)
};
bool igemm_conv_supported(int C, int N, int KS);
void igemm_conv(const IgemmParams& p, hipStream_t s);

// Tall-skinny FC GEMM (fc_tall.hip): out[m][n] = act(sum_k A[m][k] W[n][k] + b[n])
// (bias null: plain store, the data gradient through a W^T copy), bf16 in /
// out, fp32 accumulate; large M, K % 8 == 0, N % 4 == 0.
struct FcTallParams {
  int M = 0, N = 0, K = 0;
  bool f32 = false;         // fp32 operands / output (exact f32 MFMA)
  const void* A = nullptr;  // bf16 [M][lda]
  int lda = 0;
  const void* W = nullptr;  // bf16 [N][ldw]
  int ldw = 0;
  const float* bias = nullptr;
  int act = ACT_NONE;
  void* out = nullptr;      // bf16 [M][ldo]
  int ldo = 0;
};
bool fc_tall_supported(int M, int N, int K);
void fc_tall(const FcTallParams& p, hipStream_t s);
// FC data gradient with W resident in LDS (fc_wres.hip): out = (A W^T) x act'(aux)
// for a short reduction (K <= 224 bf16 / 208 fp32); p.bias unused, p.act = the
// previous layer's activation whose gradient multiplies the result (aux = its output)
bool fc_wres_supported(bool f32, int M, int N, int K, int act);
void fc_wres(const FcTallParams& p, const void* aux, int ldaux, hipStream_t s);

// fp32 FC weight gradient for skinny outputs (fc_dw32.hip): split-K partials
// part[s][m][ldp] of dW[m][n] = sum_k dz[k][m] x[k][n] (m < M <= 208, n < N)
// and db[m] in column N; reduced by dw_reduce.
struct FcDw32Params {
  int M = 0, N = 0, K = 0;
  const float* dz = nullptr; int ldz = 0;  // [K][ldz]
  const float* x = nullptr; int ldx = 0;   // [K][ldx]
  float* slab = nullptr; int ldp = 0;      // [splitk][M][ldp]
  int64_t slab_stride = 0;
  int splitk = 1;
};
bool fc_dw32_supported(int M, int N, int ldz, int ldx);
int fc_dw32_splitk(int M, int N, int64_t K);
void fc_dw32(const FcDw32Params& p, hipStream_t s);

// Weight gradient: dW[co][k] = sum_m dz[m][co] in(m, k), db[co] = sum_m dz[m][co],
// split-K over m into fp32 slabs [splitk][kf+1][Cout], then reduced into the
// canonical gw[Cout][C][KS][KS], gb[Cout] (grad = beta*grad + sum).
struct IgemmDwParams {
  int B = 0, H = 0, W = 0, C = 0;
  int OH = 0, OW = 0, KS = 1, stride = 1, pad = 0;
  int M = 0, Cout = 0, kf = 0;       // kf = KS*KS*C
  const void* dz = nullptr;          // bf16 [M][ldz]
  int ldz = 0;
  const void* in = nullptr;          // bf16 [B][H][W][C]
  float* slab = nullptr;
  int64_t slab_stride = 0;           // >= (kf+1)*Cout
  int splitk = 1;
  int perm_c = 0, perm_hw = 0;       // KS == 1 only: feature k = hw*perm_c + c -> c*perm_hw + hw
  int kreal = 0;                     // KS == 1 only: features >= kreal (< kf) are padding, dropped (0: kf)
  bool direct = false;               // set at launch: one split, write gw/gb in place (no slab pass)
  float* gw = nullptr;               // set at launch
  float* gb = nullptr;
  DivMagic div_ohw, div_ow;
  int adv_x = 0, adv_y = 0, adv_b = 0;  // set at launch: +BK pixels as (ox, oy, b) increments
  int tile = -1;                     // -1 auto (MCC_AB=igemm_tile=), 0: 128x128 kernel, 128 / 256: BA x 256
                                     // phase-pipelined kernel (igemm_dw_splitk must see the same value)
};
int igemm_dw_splitk(int M, int Cout, int kf, int tile = -1);
size_t igemm_dw_slab_bytes(int Cout, int kf, int splitk);
void igemm_dw(const IgemmDwParams& p, float* gw, float* gb, float beta, hipStream_t s);

void conv_forward(DType t, const ConvParams& p, hipStream_t s);
size_t conv_forward_lds_bytes(DType t, const ConvParams& p);
void conv_dw(DType t, const ConvDwParams& p, hipStream_t s);
size_t conv_dw_lds_bytes(DType t, const ConvDwParams& p);
void conv_dw_reduce(const ConvDwReduceParams& p, hipStream_t s);

void gemm(DType t, const GemmParams& p, hipStream_t s);
// Split-K forward GEMM for skinny-M / long-K problems (large FC heads at a
// small batch): fp32 partials in `scratch` ([splitk][M][ldc]), then a pass
// applying the forward epilogue (bias + act -> T, or fp32 logits).
int gemm_fwd_splitk(int M, int N, int K);
void gemm_splitk_fwd(DType t, const GemmParams& p, float* scratch, int splitk, hipStream_t s);
void dw_reduce(const DwReduceParams& p, hipStream_t s);

void softmax_xent(DType t, const XentParams& p, hipStream_t s);

// params -= lr * (grad + wd * params) [momentum: v = mu*v + g; p -= lr*v]
void sgd_update(float* params, const float* grads, float* mom, int64_t n, float lr, float mu, float wd,
                hipStream_t s);
// dst[i] = idx[i] >= 0 ? T(src[idx[i]]) : 0
void pack_gather(DType t, void* dst, const float* src, const int32_t* idx, int64_t n, hipStream_t s);

// Fused SGD (+momentum, weight decay) and packed-copy refresh in ONE pass over
// the flat parameter buffer (reference Layer_update, cnn.c:303-314, followed
// by the re-cast of every compute copy).  A weight stage's parameter j, in
// canonical order (n, c, kh, kw) = OIHW or (n, k) for FC (KS = 1), lands in
// each of its packed copies at
//   base + n*sn + c*sc + kh'*skh + kw'*skw,   kh' = flip ? KS-1-kh : kh (same for kw)
// so the copies are written straight from the updated value: no index table,
// no second pass re-reading the parameters.
struct PackMap {
  int64_t base = 0;
  int sn = 0, sc = 0, skh = 0, skw = 0, flip = 0;
};
struct PackStage {
  int64_t w_off = 0, nw = 0;
  int inC = 1, KS = 1, nmaps = 0;
  uint64_t m_ckk = 0, m_kk = 0, m_ks = 0;  // division magic (set by sgd_pack)
  int tile0 = -1;  // set by sgd_pack: first tile of a tiled (transposing) stage, -1 elementwise
  PackMap map[3];
};
constexpr int kMaxPackStages = 14;
struct SgdPackParams {
  float* params = nullptr;
  const float* grads = nullptr;
  float* mom = nullptr;
  int64_t n = 0;
  int64_t lo = 0;      // parameters [lo, n) only (a stage boundary: sgd_range); 0 = all
  float lr = 0.f, mu = 0.f, wd = 0.f;
  bool update = true;  // false: refresh the packed copies only
  void* packed = nullptr;
  int nstages = 0;     // stages sorted by w_off
  int ntiles = 0;      // set by sgd_pack: workgroups of the tiled stages (the rest run elementwise)
  PackStage st[kMaxPackStages];
};
void sgd_pack(DType t, const SgdPackParams& p, hipStream_t s);
void fill_f32(float* dst, float v, int64_t n, hipStream_t s);
// Sampling with replacement (the reference draws rand() % N per sample,
// cnn.c:455): idx[b] = lo + hash(seed, *step, b) % (hi - lo).  `step` lives in
// device memory so a captured hipGraph replays with fresh indices; call
// advance_counter once per step (after the last consumer of idx).
void sample_indices(int32_t* idx, int B, int64_t lo, int64_t hi, uint64_t seed, const uint64_t* step,
                    hipStream_t s);
// idx[b] = ((*step) * stride + offset + b) mod n: rank slices of sequential global batches
void seq_sample_indices(int32_t* idx, int B, int64_t offset, int64_t stride, int64_t n, const uint64_t* step,
                        hipStream_t s);
void advance_counter(uint64_t* step, hipStream_t s);
// sample_indices at *step, then ++*step, in ONE launch; step -> uint64[2]
// (counter, ticket = 0): the same index stream as sample + advance
void sample_indices_advance(int32_t* idx, int B, int64_t lo, int64_t hi, uint64_t seed, uint64_t* step,
                            hipStream_t s);
// contention probe: nwg workgroups holding lds_bytes of LDS each, spinning usec
void cu_hold(int nwg, int lds_bytes, double usec, hipStream_t s);
// idx[b] = start + b (sequential evaluation windows)
void iota_i32(int32_t* idx, int B, int64_t start, hipStream_t s);
void cast_f32(DType t, void* dst, const float* src, int64_t n, hipStream_t s);
void to_f32(DType t, float* dst, const void* src, int64_t n, hipStream_t s);

// ---- fp64 executor (f64.hip; GpuNet64, the reference's precision) ----
// C[m][n] (+)= act(sum_k A(m,k) B(k,n) + bias_m[m] + bias_n[n]) with
// A(m,k) = A[m*sam + k*sak], B(k,n) = B[k*sbk + n*sbn] (v_mfma_f64_16x16x4).
// P > 0 stores C in the conv activation layout: n = b*P + p -> C[b][m][p].
// `accumulate` adds to C after the activation (weight gradients: act none).
struct Gemm64Params {
  int M = 0, N = 0;
  int64_t K = 0;
  const double* A = nullptr;
  int64_t sam = 0, sak = 0;
  const double* B = nullptr;
  int64_t sbk = 0, sbn = 0;
  double* C = nullptr;
  int64_t ldc = 0;
  int P = 0;
  const double* bias_m = nullptr;
  const double* bias_n = nullptr;
  int act = ACT_NONE;
  bool accumulate = false;
  double* part = nullptr;  // set by gemm64
  int64_t kchunk = 0;      // set by gemm64
};
// split-K slab count for an (M, N, K) product (shape-only: deterministic)
int gemm64_slabs(int M, int N, int64_t K);
// `part` (>= gemm64_slabs * M * N doubles) enables fixed-order split-K; nullptr: one slab
void gemm64(const Gemm64Params& p, double* part, hipStream_t s);
struct Conv64Geom { int Ci, H, W, k, s, pad, OH, OW; };
struct Pool64Geom { int C, H, W, k, s, OH, OW; };
void im2col64(const Conv64Geom& g, const double* x, double* col, int B, hipStream_t s);
void col2im64(const Conv64Geom& g, const double* dcol, double* dx, int B, hipStream_t s);
void weff64(const double* w, double* weff, int C, int Ci, int kk, hipStream_t s);
void fold64(const double* full, double* gw, int C, int Ci, int kk, hipStream_t s);
void dz64(const double* err, const double* y, double* dzT, int B, int C, int P, int act, hipStream_t s);
void rowsum64(const double* dzT, double* gb, int rows, int64_t n, double* part, hipStream_t s);
void pool64_fwd(const Pool64Geom& g, const double* x, double* y, int32_t* arg, int B, hipStream_t s);
void pool64_bwd(const Pool64Geom& g, const double* er, const int32_t* arg, double* dx, int B, hipStream_t s);
void softmax64(double* z, int B, int C, bool ref_compat, hipStream_t s);
void out_err64(const double* p, const int32_t* labels, double* err, double* stats, int B, int C, double scale,
               hipStream_t s);
void sgd64(double* w, double* g, double lr, int64_t n, hipStream_t s);
// x[b] = data[idx[b]] / 255 (doubles), labels[b] = lab[idx[b]] (idx nullable)
void u8_batch64(const uint8_t* data, const uint8_t* lab, const int32_t* idx, double* x, int32_t* labels, int B,
                int npix, hipStream_t s);

// CIFAR-3conv conv2 (cifar_c2.hip): conv 32 -> 64, 3x3, stride 1, pad 1 on
// 16x16 NHWC bf16, ReLU + 2x2/2 max-pool, one persistent workgroup image at a
// time with the input tile swizzled in LDS and the weights in registers.
// Layouts are the ones the small-image path uses: x [B][16][16][32], packed
// weights [64][ldw] with k = tap*32 + c, y / arg [B][8][8][64] (argmax
// position 0..3 = TL TR BL BR, 4 = ReLU-inactive window).
struct CifarC2Params {
  int B = 0;
  const void* x = nullptr;
  const void* w = nullptr;
  int ldw = 0;
  const float* bias = nullptr;
  void* y = nullptr;
  uint8_t* arg = nullptr;
  int H = 8, W = 8;  // cifar_c3: conv grid (multiples of 8; 8 x 8 output tiles)
};
bool cifar_c2_supported(int inC, int H, int W, int C, int KS, int stride, int pad, int act_relu, int pooled);
void cifar_c2_forward(const CifarC2Params& p, hipStream_t s);
// Backward of the same layer from the pooled output gradient dy [B][8][8][64]
// and the forward's argmax codes: data gradient dx [B][16][16][32] (plain
// store; flipped packed weights wd [32][ldw], k = tap*64 + co) and the weight
// / bias gradient (per-workgroup partials in slab, then dw_slab_reduce into the
// canonical OIHW gw and gb).
struct CifarC2BwdParams {
  int B = 0;
  const void* dy = nullptr;
  const uint8_t* arg = nullptr;
  const void* x = nullptr;   // dW: the layer input [B][16][16][32]
  const void* wd = nullptr;  // dX
  int ldw = 0;
  void* dx = nullptr;
  float* slab = nullptr;     // dW: cifar_c2_dw_scratch_bytes()
  int H = 8, W = 8;          // cifar_c3: conv grid (multiples of 8)
};
void cifar_c2_dx(const CifarC2BwdParams& p, hipStream_t s);
size_t cifar_c2_dw_scratch_bytes();
void cifar_c2_dw(const CifarC2BwdParams& p, float* gw, float* gb, hipStream_t s);
// conv 64 -> 128, 3x3, pad 1, ReLU + 2x2/2 max-pool on an H x W NHWC bf16 grid
// (H, W multiples of 8: CIFAR-3conv conv3 at 8 x 8, VGG-11 conv2 at 112 x 112)
// in 8 x 8 output tiles (cifar_c3.hip); same parameter blocks.  x
// [B][H][W][64], weights [128][ldw] with k = tap*64 + c (the implicit-GEMM
// packing), y / arg [B][H/2][W/2][128]; wd [64][ldw] with k = tap*128 + co
// (flipped taps), dx [B][H][W][64]; slab cifar_c3_dw_scratch_bytes().
using CifarC3Params = CifarC2Params;
using CifarC3BwdParams = CifarC2BwdParams;
bool cifar_c3_supported(int inC, int H, int W, int C, int KS, int stride, int pad, int act_relu, int pooled);
void cifar_c3_forward(const CifarC3Params& p, hipStream_t s);
void cifar_c3_dx(const CifarC3BwdParams& p, hipStream_t s);
size_t cifar_c3_dw_scratch_bytes();
void cifar_c3_dw(const CifarC3BwdParams& p, float* gw, float* gb, hipStream_t s);

}  // namespace gpu
}  // namespace mcc
