// LeNet-5 classifier chain on gfx950: FC 400 -> 120 (ReLU) -> 84 (ReLU) ->
// 10, softmax-cross-entropy and the whole backward of the three layers, as
// ONE persistent kernel per step (plus a fixed-order slab reduce), instead of
// the 11 launches of the per-layer path (3 forward FC kernels, the fused head,
// split-K / implicit-GEMM weight gradients and their reduces, 2 data-gradient
// FC kernels: ~324 us per step at B = 163,840).
//
// Reference semantics: Layer_feedForw_full / Layer_feedBack_full
// (/root/reference/cnn.c:113-173), the softmax + output error of
// Layer_learnOutputs (cnn.c:125-143, 284-286) and the logged MSE metric
// (cnn.c:275-282), with the LeNet-5 shapes of BASELINE.json; numerics and
// rounding points as the unfused bf16 path (bf16 activations, fp32 logits,
// bf16 dlogits scaled by 1 / global batch, fp32 accumulation everywhere).
//
// Design (one 512-thread workgroup per CU, persistent over 32-image tiles):
//  * All three weight matrices live in LDS as bf16 (118 KB) for the whole
//    kernel; one row-major copy serves both directions: the forward reads
//    weight rows with ds_read_b128, the data gradients read them transposed
//    with ds_read_b64_tr_b16.
//  * Per tile, every intermediate (the 32 x 400 input tile, H1 / dH1, H2 /
//    dH2, the dlogits E) stays in LDS: HBM traffic per image is the FC input
//    once (800 B) and its gradient once (800 B).  The per-layer path moved
//    the input three times plus H1, H2, logits and their gradients.
//  * GEMMs are written transposed (MFMA rows = output features, columns =
//    images), so each lane's four accumulator values are four CONSECUTIVE
//    features of one image: 8-byte LDS stores for the activations and 8-byte
//    global stores for the FC input gradient.
//  * Weight gradients sum over the images (the MFMA K = the 32 images of the
//    tile) into registers held across all tiles of the workgroup: dW1 (120 x
//    400) as 25 accumulator tiles per wave, dW2 as 6, dW3 as 1; bias
//    gradients are one extra MFMA against a ones fragment.  Each workgroup
//    writes one canonical-layout slab at the end; lenet_fc_reduce sums the
//    slabs in a fixed order (deterministic, no atomics).
//  * LDS layout from the bank model (tools/lds_banks.py): image rows are
//    stored in the permuted order pa(m) (bits 2 and 3 swapped) with row
//    strides = 32 B mod 256, which makes both the b128 row reads and the
//    8-row transposed reads conflict-free; W1 rows likewise (pw1).
#include "kernels.h"
#include "mfma.h"
#include "stats.h"

namespace mcc {
namespace gpu {
namespace {

typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) void gvoid;
typedef __attribute__((address_space(3))) void lvoid;

constexpr int TM = 32;  // images per tile (the weight-gradient MFMA K)
constexpr int K0 = 400, N1 = 120, N2 = 84, N3 = 10;
constexpr int kThreads = 512;

// LDS (bytes).  Row strides: 32 B mod 256 where a transposed 8-row read
// touches the buffer (conflict-free with the row permutations below); W2 and
// W3 are read a handful of times per tile and stay unpadded / lightly padded.
constexpr int SW1 = 800, SW2 = 240, SW3 = 224, SY = 800, SH1 = 288, SH2 = 224, SE = 32;
constexpr int OW1 = 0;                   // W1 [120][400]
constexpr int OW2 = OW1 + N1 * SW1;      // W2 [84][120]
constexpr int OW3 = OW2 + N2 * SW2;      // W3 [10][96] (cols 84..95 zero)
constexpr int OH1 = OW3 + N3 * SW3;      // H1 [32][128] (cols 120..127 zero), later dH1 (the FC input tile
                                         // [32][400]: its own LDS object, ysm)
constexpr int OH2 = OH1 + TM * SH1;      // H2 [32][96] (cols 84..95 zero), later dH2
constexpr int OE = OH2 + TM * SH2;       // E = dlogits [32][16] (cols 10..15 zero)
constexpr int OLAB = OE + TM * SE;       // labels of the tile (int)
constexpr int ORED = OLAB + TM * 4;      // statistics of the 8 waves
constexpr int OBIAS = ORED + 3 * 8 * 4;  // fp32 biases b1 [128] b2 [128] b3 [16] (zero padded)
constexpr int kLds = OBIAS + (128 + 128 + 16) * 4;
static_assert(kLds + TM * SY <= 163840, "lenet_fc: LDS budget");
static_assert(OW2 % 16 == 0 && OW3 % 16 == 0 && OH1 % 16 == 0 && OH2 % 16 == 0 && OE % 16 == 0,
              "16-byte aligned LDS buffers");

// canonical slab layout = the flat parameter range of the three FC layers
constexpr int kSlabW1 = 0, kSlabB1 = N1 * K0, kSlabW2 = kSlabB1 + N1, kSlabB2 = kSlabW2 + N2 * N1,
              kSlabW3 = kSlabB2 + N2, kSlabB3 = kSlabW3 + N3 * N2, kSlab = kSlabB3 + N3;  // 59,134
constexpr int kSlabP = (kSlab + 3) & ~3;  // slab stride (16-byte rows for the float4 reduce)

// image row m of a tile -> LDS row (bits 2 and 3 swapped: the 8 rows of a
// transposed read {0..3, 8..11} land in 8 different 32-byte bank slots)
__device__ __forceinline__ int pa(int m) { return (m & ~12) | ((m & 4) << 1) | ((m & 8) >> 1); }
// W1 row n (n >= 120: padding rows of the last 16-row tile, read only where
// the other operand is zero or the result is discarded: aliased 8 rows down,
// so the lanes broadcast instead of conflicting)
__device__ __forceinline__ int pw1(int n) {
  n = n >= N1 ? n - 8 : n;
  return n < 112 ? pa(n) : n;
}

// workgroup barrier for LDS hand-offs only: __syncthreads() also drains
// vmcnt (its release fence) -- the logits / prediction stores; the phases
// exchange nothing through global memory.  (An L2 warm-up DMA of the next
// input tile issued at P4, one 4-byte load per line, measured neutral:
// 140.6 / 142.2 vs 144.4 / 140.1 us, and dropped.)
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

__device__ __forceinline__ bf16x8 ld128(const char* p) { return *reinterpret_cast<const bf16x8*>(p); }
__device__ __forceinline__ bf16x4 ld64(const char* p) { return *reinterpret_cast<const bf16x4*>(p); }
// transposed K = 32 fragment: rows (8g + q) and (8g + 4 + q), 4 columns at 4p
__device__ __forceinline__ bf16x8 tr8(const char* p0, const char* p1) {
  const bf16x4 a = tr4(reinterpret_cast<const bf16*>(p0));
  const bf16x4 b = tr4(reinterpret_cast<const bf16*>(p1));
  return __builtin_shufflevector(a, b, 0, 1, 2, 3, 4, 5, 6, 7);
}
// v_mfma_f32_16x16x16_bf16: A[r][4g+j], B[4g+j][r], j = 0..3
__device__ __forceinline__ f32x4 mma16(f32x4 acc, bf16x4 a, bf16x4 b) {
  return __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(__builtin_bit_cast(v4s, a), __builtin_bit_cast(v4s, b), acc, 0, 0,
                                                   0);
}
__device__ __forceinline__ uint32_t bf16_bits(float v) { return (uint32_t)__builtin_bit_cast(unsigned short, (bf16)v); }
__device__ __forceinline__ u32x2 pack4(float a, float b, float c, float d) {
  return u32x2{bf16_bits(a) | (bf16_bits(b) << 16), bf16_bits(c) | (bf16_bits(d) << 16)};
}

// (sum4lanes / argmax4lanes: mfma.h)

__global__ void __launch_bounds__(kThreads, 1) lenet_fc_kernel(LenetFcParams P) {
  // the input tile is its own LDS object: the compiler then knows the
  // tile's DMA cannot alias the other buffers and does not drain it
  // (s_waitcnt vmcnt(0)) in front of the data gradient's LDS reads
  __shared__ __attribute__((aligned(16))) char smem[kLds];
  __shared__ __attribute__((aligned(16))) char ysm[TM * SY];
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave index in an SGPR: w-derived addresses are scalar
  const int r = lane & 15, g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  const int B = P.B;
  const int ntiles = (B + TM - 1) / TM;

  // ---- the three weight matrices (packed bf16 compute copies) into LDS ----
  {
    const char* w1 = static_cast<const char*>(P.w1);
    for (int i = tid; i < N1 * 50; i += kThreads) {
      const int n = i / 50, j = i - 50 * (i / 50);
      *reinterpret_cast<u32x4*>(smem + OW1 + pw1(n) * SW1 + 16 * j) =
          *reinterpret_cast<const u32x4*>(w1 + (size_t)n * P.ldw1 * 2 + 16 * j);
    }
    const char* w2 = static_cast<const char*>(P.w2);
    for (int i = tid; i < N2 * 15; i += kThreads) {
      const int n = i / 15, j = i - 15 * (i / 15);
      *reinterpret_cast<u32x4*>(smem + OW2 + n * SW2 + 16 * j) =
          *reinterpret_cast<const u32x4*>(w2 + (size_t)n * P.ldw2 * 2 + 16 * j);
    }
    const char* w3 = static_cast<const char*>(P.w3);
    for (int i = tid; i < N3 * 12; i += kThreads) {
      const int n = i / 12, j = i - 12 * (i / 12);
      u32x4 v = {0u, 0u, 0u, 0u};
      if (j <= 10) v = *reinterpret_cast<const u32x4*>(w3 + (size_t)n * P.ldw3 * 2 + 16 * j);
      if (j == 10) v[2] = v[3] = 0u;  // columns 84..87
      *reinterpret_cast<u32x4*>(smem + OW3 + n * SW3 + 16 * j) = v;
    }
  }
  // fp32 master biases, zero padded (read per tile: registers are the
  // weight-gradient accumulators' -- 140 of the 256 a lane has at 2 waves/SIMD)
  {
    float* bs = reinterpret_cast<float*>(smem + OBIAS);
    for (int i = tid; i < 128 + 128 + 16; i += kThreads) {
      float v = 0.f;
      if (i < 128) v = i < N1 ? P.b1[i] : 0.f;
      else if (i < 256) v = i - 128 < N2 ? P.b2[i - 128] : 0.f;
      else v = i - 256 < N3 ? P.b3[i - 256] : 0.f;
      bs[i] = v;
    }
  }
  const f32x4* bias = reinterpret_cast<const f32x4*>(smem + OBIAS);
  bf16x8 ones;
#pragma unroll
  for (int j = 0; j < 8; ++j) ones[j] = (bf16)1.f;

  // ---- per-lane LDS offsets (tile invariant) ----
  // transposed reads of the activation buffers: rows 8g + q and 8g + 4 + q
  const int tra0 = pa(8 * g + q), tra1 = pa(8 * g + 4 + q);
  // image-row reads (b128 / b64): rows r and 16 + r
  const int rm0 = pa(r), rm1 = pa(16 + r);

  // ---- the FC input tile moves HBM -> LDS by DMA (global_load_lds, 16 B per
  // lane, no registers): the LDS image of the tile is contiguous (row pa(m)
  // at pa(m) * 800), so 16-byte piece k of it comes from image row pa(k / 50)
  // (pa is an involution), chunk k % 50.  Issued while the previous tile's
  // data gradient runs (P6b); the label of the tile's row tid rides along in
  // a register. ----
  const char* ybase = static_cast<const char*>(P.y);
  // the tile's dataset rows ride along with the DMA; the labels behind them
  // (a dependent load) are fetched at the top of the tile and land in LDS
  // after P1: a dependent load here would put an s_waitcnt vmcnt(0) -- the
  // whole DMA -- right behind the DMA issue
  int labrow = 0, labpre = 0;
  auto load_tile = [&](int t) {
    const int row0 = t * TM;
    for (int k = tid; k < TM * 50; k += kThreads) {
      const int prow = k / 50, j = k - 50 * (k / 50);
      const char* src = ybase + (size_t)min(row0 + pa(prow), B - 1) * P.ldy * 2 + 16 * j;
      // wave-uniform LDS base of this 64-lane piece; lane l lands at + 16 l
      __builtin_amdgcn_global_load_lds((gvoid*)src, (lvoid*)(ysm + 16 * (k - lane)), 16, 0, 0);
    }
    if (tid < TM) {
      const int gr = min(row0 + tid, B - 1);
      labrow = P.idx ? P.idx[gr] : gr;
    }
  };

  // weight-gradient accumulators, held across all tiles.  The bias gradients
  // of FC2 and FC3 come out of these tiles too: H1 column 120 and H2 column 84
  // are ones (padding columns; zero weights in the forward, masked in the data
  // gradients), so dW2 column 120 = db2 and dW3 column 84 = db3.
  f32x4 dw1[25], dw2[6], dw3, db1;
  const f32x4 z4 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int b = 0; b < 25; ++b) dw1[b] = z4;
#pragma unroll
  for (int a = 0; a < 6; ++a) dw2[a] = z4;
  dw3 = db1 = z4;
  float st_loss = 0.f, st_mse = 0.f, st_cor = 0.f;

  int t = blockIdx.x;
  if (t < ntiles) load_tile(t);
  for (; t < ntiles; t += gridDim.x) {
    const int row0 = t * TM;
    const int nvalid = min(TM, B - row0);
    // this wave's input-tile DMAs (and last tile's gradient stores) are done;
    // the barrier makes every wave's pieces visible
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (tid < TM) labpre = P.labels[labrow];
    __syncthreads();

    // ---- P1: H1^T = relu(W1 Y^T + b1), wave w: features 16w .. 16w+15 ----
    uint32_t mask1 = 0, mask2 = 0;
    {
      f32x4 acc0 = bias[4 * w + g], acc1 = acc0;
      const char* aw = smem + OW1 + pw1(16 * w + r) * SW1;
      const char* y0 = ysm + rm0 * SY;
      const char* y1 = ysm + rm1 * SY;
      // operands of chunk c + 2 are read while chunk c multiplies (a ring of
      // three: the compiler would otherwise hoist all 36 reads -- 144
      // registers on top of the 140 accumulator registers)
      bf16x8 fa[3], f0[3], f1[3];
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        fa[c] = ld128(aw + 64 * c + 16 * g);
        f0[c] = ld128(y0 + 64 * c + 16 * g);
        f1[c] = ld128(y1 + 64 * c + 16 * g);
      }
#pragma unroll
      for (int c = 0; c < 12; ++c) {
        if (c + 2 < 12) {
          fa[(c + 2) % 3] = ld128(aw + 64 * (c + 2) + 16 * g);
          f0[(c + 2) % 3] = ld128(y0 + 64 * (c + 2) + 16 * g);
          f1[(c + 2) % 3] = ld128(y1 + 64 * (c + 2) + 16 * g);
        }
        __builtin_amdgcn_sched_barrier(0);
        acc0 = mma(acc0, fa[c % 3], f0[c % 3]);
        acc1 = mma(acc1, fa[c % 3], f1[c % 3]);
        __builtin_amdgcn_sched_barrier(0);
      }
      {  // k = 384 .. 399
        const bf16x4 a = ld64(aw + 768 + 8 * g);
        acc0 = mma16(acc0, a, ld64(y0 + 768 + 8 * g));
        acc1 = mma16(acc1, a, ld64(y1 + 768 + 8 * g));
      }
#pragma unroll
      for (int mt = 0; mt < 2; ++mt) {
        const f32x4 acc = mt ? acc1 : acc0;
        float h[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int n1 = 16 * w + 4 * g + i;
          const float v = n1 < N1 ? fmaxf(acc[i], 0.f) : 0.f;
          h[i] = n1 == N1 ? 1.f : v;  // the ones column of dW2 (-> db2)
          mask1 |= (bf16_bits(v) & 0x7fffu) ? 1u << (4 * mt + i) : 0u;
        }
        *reinterpret_cast<u32x2*>(smem + OH1 + (mt ? rm1 : rm0) * SH1 + (16 * w + 4 * g) * 2) =
            pack4(h[0], h[1], h[2], h[3]);
      }
    }
    if (tid < TM) reinterpret_cast<int*>(smem + OLAB)[tid] = labpre;  // read in P3, two barriers on
    lds_barrier();

    // ---- P2: H2^T = relu(W2 H1^T + b2), waves 0..5 ----
    if (w < 6) {
      f32x4 acc0 = bias[32 + 4 * w + g], acc1 = acc0;
      // rows >= 84 read row 83 (outputs discarded); k 120..127 of the last
      // chunk (past the row; H1 column 120 is the ones column) is zeroed
      const char* aw = smem + OW2 + min(16 * w + r, N2 - 1) * SW2 + 16 * g;
      const char* h0 = smem + OH1 + rm0 * SH1 + 16 * g;
      const char* h1 = smem + OH1 + rm1 * SH1 + 16 * g;
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        bf16x8 a = ld128(aw + 64 * c);
        if (c == 3 && g == 3) a = bf16x8{};
        acc0 = mma(acc0, a, ld128(h0 + 64 * c));
        acc1 = mma(acc1, a, ld128(h1 + 64 * c));
      }
#pragma unroll
      for (int mt = 0; mt < 2; ++mt) {
        const f32x4 acc = mt ? acc1 : acc0;
        float h[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int n2 = 16 * w + 4 * g + i;
          const float v = n2 < N2 ? fmaxf(acc[i], 0.f) : 0.f;
          h[i] = n2 == N2 ? 1.f : v;  // the ones column of dW3 (-> db3)
          mask2 |= (bf16_bits(v) & 0x7fffu) ? 1u << (4 * mt + i) : 0u;
        }
        *reinterpret_cast<u32x2*>(smem + OH2 + (mt ? rm1 : rm0) * SH2 + (16 * w + 4 * g) * 2) =
            pack4(h[0], h[1], h[2], h[3]);
      }
    }
    lds_barrier();

    // ---- P3: logits^T = W3 H2^T + b3 and softmax-CE, wave mt = m-tile ----
    if (w < 2) {
      f32x4 acc = bias[64 + g];
      const char* aw = smem + OW3 + min(r, N3 - 1) * SW3 + 16 * g;
      const char* hb = smem + OH2 + (w ? rm1 : rm0) * SH2 + 16 * g;
#pragma unroll
      for (int c = 0; c < 3; ++c) acc = mma(acc, ld128(aw + 64 * c), ld128(hb + 64 * c));
      // lane (image m, g) holds classes 4g .. 4g+3 of image m; the image's
      // 16 classes are spread over lanes r, r+16, r+32, r+48
      const int m = 16 * w + r;
      const bool valid = m < nvalid;
      const int label = reinterpret_cast<const int*>(smem + OLAB)[m];
      float v[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) v[i] = 4 * g + i < N3 ? acc[i] : -__builtin_inff();
      float mx = v[0];
      int am = 4 * g;
#pragma unroll
      for (int i = 1; i < 4; ++i)
        if (v[i] > mx) { mx = v[i]; am = 4 * g + i; }
      argmax4lanes(mx, am);
      float sum = 0.f;
#pragma unroll
      for (int i = 0; i < 4; ++i)
        if (4 * g + i < N3) sum += __expf(v[i] - mx);
      sum = sum4lanes(sum);
      const float inv = 1.f / sum;
      float e[4], mse = 0.f, vl = 0.f;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int j = 4 * g + i;
        e[i] = 0.f;
        if (j < N3) {
          const float d = __expf(v[i] - mx) * inv - (j == label ? 1.f : 0.f);
          mse += d * d;
          if (valid) e[i] = (float)(bf16)(d * P.scale);  // the bf16 dlogits of the unfused path
          if (j == label) vl = v[i];
        }
      }
      mse = sum4lanes(mse);
      vl = sum4lanes(vl);
      *reinterpret_cast<u32x2*>(smem + OE + (w ? rm1 : rm0) * SE + 8 * g) = pack4(e[0], e[1], e[2], e[3]);
      if (valid) {
        const int row = row0 + m;
        if (P.logits && g < 3) {
          float* lg = P.logits + (size_t)row * P.ldl + 4 * g;
          if (g < 2) *reinterpret_cast<f32x4*>(lg) = acc;
          else *reinterpret_cast<float2*>(lg) = float2{acc[0], acc[1]};
        }
        if (g == 0) {
          if (P.pred) P.pred[row] = am;
          st_loss += __logf(sum) - (vl - mx);
          st_mse += mse / (float)N3;
          st_cor += am == label ? 1.f : 0.f;
        }
      }
    }
    lds_barrier();

    // ---- P4: dH2^T = (W3^T E^T) * relu'(H2) (waves 0..5), dW3 += E^T H2, db3 ----
    u32x2 dh2v[2] = {u32x2{0u, 0u}, u32x2{0u, 0u}};
    if (w < 6) {
      const bf16x4 a = tr4(reinterpret_cast<const bf16*>(smem + OW3 + min(4 * g + q, N3 - 1) * SW3 + (16 * w + 4 * p) * 2));
#pragma unroll
      for (int mt = 0; mt < 2; ++mt) {
        const f32x4 acc = mma16(z4, a, ld64(smem + OE + (mt ? rm1 : rm0) * SE + 8 * g));
        float d[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) d[i] = (mask2 >> (4 * mt + i)) & 1u ? acc[i] : 0.f;
        dh2v[mt] = pack4(d[0], d[1], d[2], d[3]);
      }
      const bf16x8 ae = tr8(smem + OE + tra0 * SE + 8 * p, smem + OE + tra1 * SE + 8 * p);
      const bf16x8 bh = tr8(smem + OH2 + tra0 * SH2 + (16 * w + 4 * p) * 2, smem + OH2 + tra1 * SH2 + (16 * w + 4 * p) * 2);
      dw3 = mma(dw3, ae, bh);
    }
    lds_barrier();  // H2 reads done
    if (w < 6) {
      *reinterpret_cast<u32x2*>(smem + OH2 + rm0 * SH2 + (16 * w + 4 * g) * 2) = dh2v[0];
      *reinterpret_cast<u32x2*>(smem + OH2 + rm1 * SH2 + (16 * w + 4 * g) * 2) = dh2v[1];
    }
    lds_barrier();

    // ---- P5: dW2 += dH2^T H1, db2; dH1^T = (W2^T dH2^T) * relu'(H1) ----
    u32x2 dh1v[2];
    {
      const bf16x8 bh = tr8(smem + OH1 + tra0 * SH1 + (16 * w + 4 * p) * 2, smem + OH1 + tra1 * SH1 + (16 * w + 4 * p) * 2);
#pragma unroll
      for (int a = 0; a < 6; ++a) {
        const bf16x8 ad =
            tr8(smem + OH2 + tra0 * SH2 + (16 * a + 4 * p) * 2, smem + OH2 + tra1 * SH2 + (16 * a + 4 * p) * 2);
        dw2[a] = mma(dw2[a], ad, bh);
      }
      f32x4 x0 = z4, x1 = z4;
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        // rows >= 84 read row 83 against dH2's zero columns; wave 7's columns
        // 120..127 read past the row (finite LDS), discarded by the mask
        const bf16x8 a = tr8(smem + OW2 + min(32 * c + 8 * g + q, N2 - 1) * SW2 + (16 * w + 4 * p) * 2,
                             smem + OW2 + min(32 * c + 8 * g + 4 + q, N2 - 1) * SW2 + (16 * w + 4 * p) * 2);
        x0 = mma(x0, a, ld128(smem + OH2 + rm0 * SH2 + 64 * c + 16 * g));
        x1 = mma(x1, a, ld128(smem + OH2 + rm1 * SH2 + 64 * c + 16 * g));
      }
#pragma unroll
      for (int mt = 0; mt < 2; ++mt) {
        const f32x4 acc = mt ? x1 : x0;
        float d[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) d[i] = (mask1 >> (4 * mt + i)) & 1u ? acc[i] : 0.f;
        dh1v[mt] = pack4(d[0], d[1], d[2], d[3]);
      }
    }
    lds_barrier();  // H1 and dH2 reads done
    *reinterpret_cast<u32x2*>(smem + OH1 + rm0 * SH1 + (16 * w + 4 * g) * 2) = dh1v[0];
    *reinterpret_cast<u32x2*>(smem + OH1 + rm1 * SH1 + (16 * w + 4 * g) * 2) = dh1v[1];
    lds_barrier();

    // ---- P6: dW1 += dH1^T Y, db1; dY^T = W1^T dH1^T -> global ----
    {
      const bf16x8 ad = tr8(smem + OH1 + tra0 * SH1 + (16 * w + 4 * p) * 2, smem + OH1 + tra1 * SH1 + (16 * w + 4 * p) * 2);
      db1 = mma(db1, ad, ones);
      const char* ya = ysm + tra0 * SY + 8 * p;
      const char* yb = ysm + tra1 * SY + 8 * p;
      bf16x8 fy[4];
#pragma unroll
      for (int b = 0; b < 3; ++b) fy[b] = tr8(ya + 32 * b, yb + 32 * b);
#pragma unroll
      for (int b = 0; b < 25; ++b) {
        if (b + 3 < 25) fy[(b + 3) & 3] = tr8(ya + 32 * (b + 3), yb + 32 * (b + 3));
        __builtin_amdgcn_sched_barrier(0);
        dw1[b] = mma(dw1[b], ad, fy[b & 3]);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    // every wave is done with the input tile: the next one streams into LDS
    // while the data gradient below runs
    lds_barrier();
#ifndef MCC_FC_ABL_NOLOAD  // timing ablation (tools/build_variant.sh): reuse the first tile's input
    if (t + (int)gridDim.x < ntiles) load_tile(t + gridDim.x);
#endif
    {      // data gradient: unit (k-tile b, image tile mt); wave w takes b = w,
      // w + 8, w + 16 of both image tiles and b = 24 of image tile w (w < 2)
      int wrow[8];  // W1 LDS rows of this lane's transposed reads, chunk c, half h
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        wrow[2 * c] = OW1 + pw1(32 * c + 8 * g + q) * SW1;
        wrow[2 * c + 1] = OW1 + pw1(32 * c + 8 * g + 4 + q) * SW1;
      }
      char* dyb = static_cast<char*>(P.dy);
      const bool st0 = r < nvalid, st1 = 16 + r < nvalid;
      char* drow0 = dyb + (size_t)(row0 + (st0 ? r : 0)) * P.ldd * 2 + 8 * g;
      char* drow1 = dyb + (size_t)(row0 + (st1 ? 16 + r : 0)) * P.ldd * 2 + 8 * g;
      const char* hrow0 = smem + OH1 + rm0 * SH1 + 16 * g;
      const char* hrow1 = smem + OH1 + rm1 * SH1 + 16 * g;
      // k-tiles b = w, w + 8, w + 16 for BOTH image tiles: one W1 fragment
      // read feeds two independent MFMA chains
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        const int b = w + 8 * k;
        bf16x8 fw[2], f0[2], f1[2];
        fw[0] = tr8(smem + wrow[0] + (16 * b + 4 * p) * 2, smem + wrow[1] + (16 * b + 4 * p) * 2);
        f0[0] = ld128(hrow0);
        f1[0] = ld128(hrow1);
        f32x4 acc0 = z4, acc1 = z4;
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          if (c + 1 < 4) {
            fw[(c + 1) & 1] = tr8(smem + wrow[2 * c + 2] + (16 * b + 4 * p) * 2, smem + wrow[2 * c + 3] + (16 * b + 4 * p) * 2);
            f0[(c + 1) & 1] = ld128(hrow0 + 64 * (c + 1));
            f1[(c + 1) & 1] = ld128(hrow1 + 64 * (c + 1));
          }
          __builtin_amdgcn_sched_barrier(0);
          acc0 = mma(acc0, fw[c & 1], f0[c & 1]);
          acc1 = mma(acc1, fw[c & 1], f1[c & 1]);
          __builtin_amdgcn_sched_barrier(0);
        }
        if (st0) *reinterpret_cast<u32x2*>(drow0 + 32 * b) = pack4(acc0[0], acc0[1], acc0[2], acc0[3]);
        if (st1) *reinterpret_cast<u32x2*>(drow1 + 32 * b) = pack4(acc1[0], acc1[1], acc1[2], acc1[3]);
      }
      if (w < 2) {  // k-tile 24 of image tile w
        const int b = 24;
        const char* hrow = w ? hrow1 : hrow0;
        bf16x8 fw[2], fh[2];
        fw[0] = tr8(smem + wrow[0] + (16 * b + 4 * p) * 2, smem + wrow[1] + (16 * b + 4 * p) * 2);
        fh[0] = ld128(hrow);
        f32x4 acc = z4;
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          if (c + 1 < 4) {
            fw[(c + 1) & 1] = tr8(smem + wrow[2 * c + 2] + (16 * b + 4 * p) * 2, smem + wrow[2 * c + 3] + (16 * b + 4 * p) * 2);
            fh[(c + 1) & 1] = ld128(hrow + 64 * (c + 1));
          }
          __builtin_amdgcn_sched_barrier(0);
          acc = mma(acc, fw[c & 1], fh[c & 1]);
          __builtin_amdgcn_sched_barrier(0);
        }
        if (w ? st1 : st0) *reinterpret_cast<u32x2*>((w ? drow1 : drow0) + 32 * b) = pack4(acc[0], acc[1], acc[2], acc[3]);
      }
    }
  }

  // ---- this workgroup's weight-gradient slab (canonical layout) ----
  float* slab = P.slab + (size_t)blockIdx.x * kSlabP;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int n1 = 16 * w + 4 * g + i;
    if (n1 < N1) {
#pragma unroll
      for (int b = 0; b < 25; ++b) slab[kSlabW1 + n1 * K0 + 16 * b + r] = dw1[b][i];
      if (r == 0) slab[kSlabB1 + n1] = db1[i];
    }
#pragma unroll
    for (int a = 0; a < 6; ++a) {
      const int n2 = 16 * a + 4 * g + i, c1 = 16 * w + r;
      if (n2 < N2 && c1 < N1) slab[kSlabW2 + n2 * N1 + c1] = dw2[a][i];
    }
    if (w == 7 && r == 8) {  // column 120 of dW2: the bias gradient
#pragma unroll
      for (int a = 0; a < 6; ++a) {
        const int n2 = 16 * a + 4 * g + i;
        if (n2 < N2) slab[kSlabB2 + n2] = dw2[a][i];
      }
    }
    const int n3 = 4 * g + i, c2 = 16 * w + r;
    if (w < 6 && n3 < N3 && c2 < N2) slab[kSlabW3 + n3 * N2 + c2] = dw3[i];
    if (w == 5 && r == 4 && n3 < N3) slab[kSlabB3 + n3] = dw3[i];  // column 84 of dW3
  }

  // ---- statistics: lanes, then the 8 waves in a fixed order ----
  for (int o = 32; o > 0; o >>= 1) {
    st_loss += __shfl_xor(st_loss, o);
    st_mse += __shfl_xor(st_mse, o);
    st_cor += __shfl_xor(st_cor, o);
  }
  float* red = reinterpret_cast<float*>(smem + ORED);
  if (lane == 0) {
    red[w] = st_loss;
    red[8 + w] = st_mse;
    red[16 + w] = st_cor;
  }
  __syncthreads();
  if (tid < 3 && P.stats) {
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < 8; ++k) s += red[8 * tid + k];
    stat_add(P.stats, tid, s);
  }
}

// out[i] = sum over the workgroup slabs in order; 16 waves per 64 positions
constexpr int kRedWaves = 16;
__global__ void __launch_bounds__(64 * kRedWaves) lenet_fc_reduce_kernel(const float* slab, int nslabs, float* out) {
  // float4 per lane (1 KB per wave load): wave w sums slabs w, w + 16, ... of
  // positions 4 (blk * 64 + lane) .. + 3, then wave 0 adds the 16 partials in order
  __shared__ float4 part[kRedWaves][64];
  const int l = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int p4 = blockIdx.x * 64 + l;
  float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
  if (4 * p4 < kSlab) {
#pragma unroll 8
    for (int k = wv; k < nslabs; k += kRedWaves) {
      const float4 v = *reinterpret_cast<const float4*>(slab + (size_t)k * kSlabP + 4 * p4);
      s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
    }
  }
  part[wv][l] = s;
  __syncthreads();
  if (wv != 0 || 4 * p4 >= kSlab) return;
  float4 v = part[0][l];
#pragma unroll
  for (int i = 1; i < kRedWaves; ++i) {
    const float4 t = part[i][l];
    v.x += t.x; v.y += t.y; v.z += t.z; v.w += t.w;
  }
  const float r[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int i = 0; i < 4; ++i)
    if (4 * p4 + i < kSlab) out[4 * p4 + i] = r[i];
}

int fc_grid(int B) { return std::min((B + TM - 1) / TM, 256); }

}  // namespace

bool lenet_fc_supported(int kin, int n1, int n2, int n3) { return kin == K0 && n1 == N1 && n2 == N2 && n3 == N3; }
size_t lenet_fc_slab_bytes(int max_batch) { return (size_t)fc_grid(max_batch) * kSlabP * 4; }
int lenet_fc_grad_count() { return kSlab; }

void lenet_fc(const LenetFcParams& p, float* grads, hipStream_t s) {
  if (p.B <= 0) return;
  MCC_CHECK(p.y && p.dy && p.labels && p.slab && p.w1 && p.w2 && p.w3 && p.b1 && p.b2 && p.b3 && grads,
            "lenet_fc: missing buffer");
  MCC_CHECK(p.ldy % 8 == 0 && p.ldd % 4 == 0 && p.ldw1 % 8 == 0 && p.ldw2 % 8 == 0 && p.ldw3 % 8 == 0 &&
                p.ldw1 >= K0 && p.ldw2 >= N1 && p.ldw3 >= N2 && p.ldy >= K0 && p.ldd >= K0 && (!p.logits || p.ldl >= N3),
            "lenet_fc: leading dimensions");
  const int grid = fc_grid(p.B);
  hipLaunchKernelGGL(lenet_fc_kernel, dim3(grid), dim3(kThreads), 0, s, p);
  hipLaunchKernelGGL(lenet_fc_reduce_kernel, dim3((kSlab + 255) / 256), dim3(64 * kRedWaves), 0, s, p.slab, grid, grads);
}

}  // namespace gpu
}  // namespace mcc
