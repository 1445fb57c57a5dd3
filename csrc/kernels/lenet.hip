// LeNet-5 conv block on gfx950: conv1 (1->6, 5x5, pad 2) + ReLU + 2x2 pool
// and conv2 (6->16, 5x5) + ReLU + 2x2 pool on 28x28 u8 images, forward and
// backward, as two kernels instead of the five generic small-image conv
// launches (plus their slab reduces) the engine used for these layers.
//
// Reference semantics: Layer_feedForw_conv / Layer_feedBack_conv
// (/root/reference/cnn.c:175-247, with the D1 index bug fixed as in
// CUDAcnn.cu:167-195); the pool and the LeNet-5 topology are BASELINE.json
// additions.  Everything here is shaped for one 64-lane wave per image:
//
//  * Wave-private LDS, 64-thread workgroups, persistent grids.  A wave stages
//    one image, computes, and moves on; no workgroup barrier ever waits on
//    another wave, so LDS and MFMA latency are hidden by the other waves of
//    the CU instead of by lock-step phases.
//  * All geometry is compile-time, so every LDS operand read is a base VGPR
//    plus an immediate offset.
//  * Forward (lenet_fwd): conv1 as an MFMA GEMM whose columns are (channel,
//    pixel pair) -- 12 of 16 columns useful, vs 6 -- with the bias in the
//    accumulator's initial value; the 2x2 max-pool and its argmax take one
//    integer max tree over keys (bits & ~3 | 3 - pos): positive floats order
//    as integers, the low two bits break ties toward the first position and
//    a window whose max is <= 0 is ReLU-inactive anyway.  The pooled conv1
//    output stays in LDS for conv2 (register-resident weights).
//  * Backward (lenet_bwd): one pass per image computes
//      conv2 dW (dZ2^T x im2col(Y1), transposed LDS reads, bias as a ones
//        column),
//      conv2 dX (dZ2 padded x flipped W2, rows = output pixels, columns =
//        (input channel, vertical pixel pair); 10 of each tile's 15 A
//        fragments are the previous tile's, reused from registers),
//      and the unpool of dY1 straight into LDS rows of dZ1, then
//      conv1 dW (rows = (channel, kernel-row half), columns = 15 taps + a
//        ones column: one MFMA per 32-pixel output row),
//    accumulating dW2/dW1 in registers across the wave's images; one slab
//    per wave, reduced in a fixed order (deterministic).
//
// Layouts produced by lenet_fwd and consumed by lenet_bwd:
//   Y1 [B][14][14][8] bf16 (HWC, channels 6..7 zero), A1 [B][6][14][16] u8
//   (planar, argmax position 0..3 or 4 = ReLU-inactive), Y2 [B][25][16] bf16
//   (the FC input, NHWC flatten), A2 [B][25][16] u8.
#include "kernels.h"
#include "mfma.h"
#include "mcc/ab.h"

#include <algorithm>

#ifndef MCC_LENET_STAMP
#define MCC_LENET_STAMP 0  // per-phase s_memtime stamps of lenet_bwd4 (diagnostic builds only)
#endif
#ifndef MCC_BWD4_SPLIT
#define MCC_BWD4_SPLIT 1  // conv2 dX tiles: 0 = w1 0-2 / w2 3-5 / w3 6 (+ dW1); 1 = w1 0-3 / w2 4-6 / w3 dW1 only
#endif
#ifndef MCC_BWD4_STAGE
#define MCC_BWD4_STAGE 1  // 1: w1 stages Y1 and w2 dZ2 (swapped); X0 row groups [0, MCC_BWD4_XW0) on w0, the rest on w3
#endif
#ifndef MCC_BWD4_XW0
#define MCC_BWD4_XW0 3
#endif
#ifndef MCC_DW1_D
#define MCC_DW1_D 8  // conv1 dW operand read lookahead (MFMAs)
#endif
#ifndef MCC_LENET_ABL
#define MCC_LENET_ABL 0  // phase ablations for timing studies only (tools/build_variant.sh); 0 in every build
#endif

namespace mcc {
namespace gpu {
namespace {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

// ---- geometry ----
constexpr int kImgPix = 784;          // 28 x 28 u8
constexpr int kY1Elems = 14 * 14 * 8; // HWC-8
constexpr int kA1Bytes = 6 * 14 * 16;
constexpr int kY2Elems = 25 * 16;

// forward LDS per wave (bytes): two copies of the zero-padded input (shifts
// 0 and 2 elements; 36-element rows: 18 dwords, so the five kernel rows a
// fragment group reads sit on different banks), the pooled conv1 output
// (HWC-8) and its argmax codes (planar), both copied out in bulk, and the
// image-invariant index tables of the tile loops.
// Bank-model choices (LDS table of MI355X_MICROARCH.md; measured forward
// LDS-bound at 84 % busy, 44 % of it conflict cycles): the conv1 A fragments
// are read as two ds_read_b64 (2 x 2 cycles, 64 banks) instead of the fused
// ds_read2_b64 (8 cycles, 32 banks), with the second copy offset by 8 B so the
// two copies' lanes do not share banks (extra cycles per image 400 -> 80);
// A1 planes are 240 B apart (224 B put channels c and c+4 on one bank).
// Round 4 (tools/lds_banks.py lenet_fwd, conflict cycles per image 308 -> 95):
// the conv1 tiles take their four 2x4 pixel blocks in the order kC1Blk (not
// four consecutive blocks) and the second copy sits 80 B past its 2304-byte
// image, so the 24 distinct 8-byte A-fragment addresses of each half-wave
// (4 blocks x 2 copies x 3 kernel rows) land in 24 different bank pairs.
constexpr int kFxPitch = 36, kFxRows = 32;
constexpr int kFxCopy = kFxPitch * kFxRows * 2 + 80;  // 2384
constexpr int kFY1 = 2 * kFxCopy;                // 4768: Y1 HWC-8, 196 x 16 B
constexpr int kFJunk = kFY1 + 196 * 16;          // 7904: 32 B sink for the two padding blocks' Y1
constexpr int kFA1 = kFJunk + 32;                // 7936: A1 [7][14][16] u8, planes 240 B apart (plane 6:
                                                 // sink of the idle columns 6, 7's codes, never copied out)
constexpr int kFA1Plane = 240;
constexpr int kFTabA = kFA1 + 7 * kFA1Plane;     // 9616: u16 [100] conv1 A offset of tile slot b
constexpr int kFTabE = kFTabA + 200;             // 9816: u16 [100] epilogue: pixel (lo byte), A1 offset (hi)
constexpr int kFTab2 = kFTabE + 200;             // 10016: u16 [112] conv2 row -> Y1 byte offset
constexpr int kFLds = kFTab2 + 224;              // 10240 (16 waves per CU: exactly the 160 KB)
static_assert(16 * kFLds <= 163840, "lenet_fwd: 16 waves per CU");
// conv1 tile slot -> 2x4 pixel block (98, 99: padding)
__device__ constexpr unsigned char kC1Blk[100] = {55, 85, 91, 90, 5, 41, 3, 60, 45, 43, 81, 28, 25, 71, 44, 19, 93, 88, 12, 68, 63, 14, 89, 29, 35, 61, 13, 8, 97, 31, 33, 48, 83, 6, 73, 58, 15, 10, 46, 30, 27, 82, 79, 22, 87, 42, 78, 84, 18, 37, 24, 94, 86, 9, 40, 34, 26, 21, 92, 56, 7, 23, 49, 54, 76, 50, 59, 95, 62, 2, 36, 17, 65, 53, 38, 80, 0, 47, 32, 16, 11, 1, 57, 77, 51, 70, 75, 66, 4, 20, 39, 96, 72, 74, 98, 99, 64, 69, 52, 67};

// conv2 tile order (bank-model search: b128 conflict cycles per image 202 ->
// 34): tile T's four pool windows are kC2Win[4T..4T+3] (-1: padding row
// quad), and K slot 4c + g of chunk c holds tap kC2Tap[4c + g] (>= 25: zero).
__device__ constexpr int kC2Win[28] = {13, 18, 8, 3, 20, 5, 15, 10, 1, -1, -1, 23, 7, 2,
                                       12, 17, 11, 6, 16, 21, 9, 4, 0, 19, -1, 14, 22, 24};
__device__ constexpr int kC2Tap[28] = {12, 19, 7, 0, 17, 10, 8, 1, 2, 9, 26, 14, 20, 5,
                                       13, 6, 21, 16, 15, 22, 27, 25, 18, 11, 3, 23, 24, 4};

// backward LDS per wave (bytes)
constexpr int kBDz2 = 0;                 // dZ2 padded by 4: 18 rows x 20 px x 16 ch bf16 (640 B rows)
constexpr int kBY1 = 11520;              // Y1 HWC-8: 196 x 16 B
constexpr int kBOne2 = kBY1 + 3136;      // 16 B of bf16 ones (dW2 bias column)
// The copy and plane strides are padded off multiples of 256 B (the 64-bank
// period): with 2560 / 2048 B strides every copy / plane mapped to the same
// banks and the dW1 operand reads and the dZ1 row writes ran 4-6-way
// conflicted (measured: 258M conflict cycles of 376M LDS-active cycles per
// step).  +24 B / +32 B leave the dW1 reads at 8 extra cycles per MFMA pair
// of fragments and the dZ1 writes conflict-free (LDS bank model).
constexpr int kBXs = 14720;              // X0 padded by 2, 4 copies shifted by 0..3: 32 rows x 40
constexpr int kBxCopy = 32 * 80 + 24;    // 2584
constexpr int kBOne1 = kBXs + 4 * kBxCopy;  // 25056: 30 rows x 80 B of ones (dW1 bias column)
constexpr int kBDz1 = kBOne1 + 30 * 80;  // 27456: dZ1 planar, 6 x 32 rows (zy + 2) x 32 px
constexpr int kBDz1Plane = 32 * 64 + 32; // 2080
constexpr int kBLds = kBDz1 + 6 * kBDz1Plane;  // 39936
// dZ1 rows are stored with their four 16-byte pixel chunks XOR-swizzled by
// row bit 1 (chunk c of row r at c ^ ((r >> 1) & 1)), and the conv1
// weight-gradient MFMA rows m hold (channel, kernel-row half) pairs in the
// order below (rows 12..15 repeat rows 0..3: broadcast reads).  With the
// 2080-byte plane stride this makes both the dZ1 row writes of the conv2
// data gradient and the dW1 operand reads conflict-free (bank model,
// tools/lds_banks.py: 112 + 120 -> 0 extra LDS cycles per image).
__device__ constexpr int kDw1Co[12] = {0, 1, 4, 5, 2, 3, 4, 5, 0, 1, 2, 3};
// conv2 weight gradient: MFMA K position (32c + 8g + 4hf + q) -> dZ2 pixel z
// (< 100), or padding (>= 128: the A operand reads a zero row, the B operand
// repeats pixel v - 128 of the same half-wave, a broadcast).  Annealed in the
// bank model so each half-wave's 8 pixels x 2 taps hit 16 different Y1 bank
// slots: transposed-read conflict cycles per image 150 -> 15.
__device__ constexpr unsigned char kZPos[128] = {90, 91, 32, 31, 97, 225, 225, 45, 84, 83, 92, 75, 0, 225, 2, 9, 190, 62, 81, 88, 185, 57, 26, 185, 66, 190, 190, 39, 48, 55, 4, 63, 43, 33, 50, 37, 87, 215, 54, 86, 34, 38, 41, 35, 11, 93, 94, 10, 3, 5, 1, 131, 96, 74, 70, 65, 8, 131, 30, 6, 80, 67, 69, 64, 68, 196, 71, 17, 53, 18, 19, 47, 46, 196, 49, 42, 16, 181, 181, 181, 36, 20, 164, 72, 79, 22, 78, 15, 164, 51, 77, 73, 98, 14, 23, 99, 13, 58, 89, 7, 59, 187, 187, 60, 44, 12, 85, 95, 52, 187, 187, 56, 149, 21, 28, 24, 189, 61, 189, 189, 29, 149, 76, 82, 25, 27, 40, 189};
__device__ constexpr int kDw1S[12] = {0, 0, 1, 1, 0, 0, 0, 0, 1, 1, 1, 1};

// per-wave slab of the weight gradients, in MFMA accumulator order
constexpr int kSlabW2 = 13 * 4 * 64;     // 3328
constexpr int kSlab = kSlabW2 + 4 * 64;  // 3584

__device__ __forceinline__ uint32_t bf16_bits(float v) {
  return (uint32_t)__builtin_bit_cast(unsigned short, (bf16)v);
}
// four u8 pixels -> two dwords of bf16 holding the exact integers 0..255
__device__ __forceinline__ void u8x4_ints(uint32_t w, uint32_t& lo, uint32_t& hi) {
  const uint32_t f0 = __builtin_bit_cast(uint32_t, (float)(w & 0xffu));
  const uint32_t f1 = __builtin_bit_cast(uint32_t, (float)((w >> 8) & 0xffu));
  const uint32_t f2 = __builtin_bit_cast(uint32_t, (float)((w >> 16) & 0xffu));
  const uint32_t f3 = __builtin_bit_cast(uint32_t, (float)(w >> 24));
  lo = __builtin_amdgcn_perm(f1, f0, 0x07060302u);
  hi = __builtin_amdgcn_perm(f3, f2, 0x07060302u);
}
// DPP: lane i <- lane i-1 / i+1 within each 16-lane row (0 at the row edge)
__device__ __forceinline__ uint32_t from_left(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, true);
}
__device__ __forceinline__ uint32_t from_right(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x101, 0xf, 0xf, true);
}
// DPP quad_perm [1,0,3,2]: swap with the neighbouring lane
__device__ __forceinline__ int swap1(int v) { return __builtin_amdgcn_mov_dpp(v, 0xB1, 0xf, 0xf, false); }
// (a.hi, b.lo) as a bf16 pair
__device__ __forceinline__ uint32_t mid16(uint32_t a, uint32_t b) { return __builtin_amdgcn_alignbit(b, a, 16); }

__device__ __forceinline__ int imax(int a, int b) { return a > b ? a : b; }
// one v_max3_i32 (the compiler reassociates nested maxes into max + max3 + max)
__device__ __forceinline__ int max3i(int a, int b, int c) {
  int r;
  asm("v_max3_i32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}
// NB: never __builtin_bit_cast an ext_vector element (acc[i]): this clang
// (ROCm 7.2) lowers it to a bitcast of the whole vector and extracts lane 0,
// silently reading acc[0] for every i.  __float_as_int on the scalar is fine.

template <int OFF>
__device__ __forceinline__ bf16x8 lds16(const char* base) {
  return *reinterpret_cast<const bf16x8*>(base + OFF);
}
// 8 elements at 8-byte alignment as two separate ds_read_b64 (2 x 2 LDS
// cycles, 64-bank service; fused, they would issue as one ds_read2_b64: 8
// cycles at 32 banks)
__device__ __forceinline__ bf16x8 lds8(const char* p) {
  int hb = 8;
  asm volatile("" : "+v"(hb));
  const bf16x4 lo = *reinterpret_cast<const bf16x4*>(p);
  const bf16x4 hi = *reinterpret_cast<const bf16x4*>(p + hb);
  return __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
}
// 8 elements at 8-byte alignment; the compiler fuses the pair into one
// ds_read2_b64 (fewer instructions, 8 LDS cycles): for the VALU-bound forward
// two ds_read_b64 at p and p2 (= p + 8 through an opaque register, so the
// pair is not fused into a ds_read2_b64)
__device__ __forceinline__ bf16x8 lds8p(const char* p, const char* p2) {
  const bf16x4 lo = *reinterpret_cast<const bf16x4*>(p);
  const bf16x4 hi = *reinterpret_cast<const bf16x4*>(p2);
  return __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
}
__device__ __forceinline__ bf16x8 tr8(const char* p0, const char* p1) {
  const bf16x4 a = tr4(reinterpret_cast<const bf16*>(p0));
  const bf16x4 b = tr4(reinterpret_cast<const bf16*>(p1));
  return __builtin_shufflevector(a, b, 0, 1, 2, 3, 4, 5, 6, 7);
}

// LDS hand-off between the lanes of the (single-wave) workgroup: a wave's LDS
// operations execute in issue order, so the compiler only must not move LDS
// accesses across this point -- a compiler fence, no s_waitcnt: the wave
// keeps issuing (reads of the next phase queue behind the writes of this one
// instead of the wave idling until every outstanding LDS operation returned).
// (__syncthreads would also drain vmcnt: the in-flight prefetch loads and
// epilogue stores.)
__device__ __forceinline__ void wave_lds_sync() { asm volatile("" ::: "memory"); }

// Dataset index of the k-th image of this wave (images blockIdx.x + k*stride):
// the indices of 64 consecutive iterations come in one vector load (lane k),
// so an image's pixel loads never wait on a dependent scalar index load.
struct WaveIdx {
  int v = 0;
  __device__ __forceinline__ void load(const int32_t* idx, int first, int stride, int B, int k0) {
    const int i = first + (k0 + (int)(threadIdx.x & 63)) * stride;
    v = idx ? idx[min(i, B - 1)] : min(i, B - 1);
  }
  __device__ __forceinline__ int get(int k) const { return __builtin_amdgcn_readlane(v, k & 63); }
};

__device__ __forceinline__ void zero_wave_lds(char* p, int bytes) {
  const u32x4 z = {0u, 0u, 0u, 0u};
  for (int i = threadIdx.x * 16; i < bytes; i += 64 * 16) *reinterpret_cast<u32x4*>(p + i) = z;
}

// ============================================================================
// Forward
// ============================================================================
//
// conv1 GEMM, per tile of 16 rows x 16 columns, two K chunks of 32:
//   row m (of the A operand) = the left pixel of a horizontal output pair;
//     the 16 rows are four 2x4 pixel blocks b = 4T + m/4, block b = (row pair
//     yp, column quad x4) = divmod(b, 7); row m%4 -> (y + (m&1), x + 2(m>>1)).
//   column n = 2*co + j (co < 6): output pixel (y, x + j) of channel co.
//   k = 8*kh + kw' (chunk 0: kh 0..3; chunk 1: kh 4), kw' = 0..7:
//     A[m][k] = Xpad[y + kh][x + kw'],  B[k][n] = W1[co][kh][kw' - j].
// The accumulator of lane (n, g) holds rows 4g..4g+3 = (y,x) (y+1,x)
// (y,x+2) (y+1,x+2) of block 4T+g: window A = cols x..x+1 is split over the
// lane pair (j = 0, 1), window B = cols x+2..x+3 likewise; one DPP swap
// finishes both (lane j = 0 keeps A, j = 1 keeps B).
//
// conv2 GEMM: rows = output pixels ordered by pool window (R = 4w + pos),
// columns = 16 output channels, k = 8*tap + ci over the HWC-8 LDS copy of the
// pooled conv1 output (7 chunks, taps >= 25 carry zero weights).
__global__ void __launch_bounds__(64) lenet_fwd_kernel(LenetFwdParams p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = threadIdx.x;
  const int n16 = lane & 15, g = lane >> 4;

  // ---- weights into registers (bf16 of the fp32 master, as the packer) ----
  bf16x8 w1[2];
  float bias1;
  {
    const int co = n16 >> 1, j = n16 & 1;
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      const int kh = c == 0 ? g : 4;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int kw = e - j;
        float v = 0.f;
        // unconditional loads of a clamped index, then a select: a load under
        // a lane condition is a branch + load + vmcnt(0) each (serialised)
        const bool ok = n16 < 12 && (c == 0 || g == 0) && kw >= 0 && kw < 5;
        v = p.w1[ok ? co * 25 + kh * 5 + kw : 0];
        w1[c][e] = (bf16)(ok ? v : 0.f);
      }
    }
    bias1 = n16 < 12 ? 255.f * p.b1[co] : 0.f;  // the tile holds raw integer pixels
  }
  bf16x8 w2[7];
  int koff2[7];  // A-fragment byte offset of this lane's tap per chunk (HWC-8 copy)
#pragma unroll
  for (int c = 0; c < 7; ++c) {
    const int t = kC2Tap[4 * c + g], kh = t < 25 ? t / 5 : 0, kw = t < 25 ? t % 5 : 0;
    koff2[c] = (kh * 14 + kw) * 16;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      float v = 0.f;
      const bool ok = t < 25 && e < 6;
      v = p.w2[ok ? (n16 * 6 + e) * 25 + t : 0];
      v = ok ? v : 0.f;
      w2[c][e] = (bf16)v;
    }
  }
  const float bias2 = p.b2[n16];

  char* xf = smem;
  char* y1s = smem + kFY1;
  char* a1s = smem + kFA1;
  zero_wave_lds(smem, kFLds);
  wave_lds_sync();
  // index tables (image invariant): block b = (row pair yp, column quad x4)
  for (int b = lane; b < 100; b += 64) {
    const int blk = kC1Blk[b];
    const int bb = blk < 98 ? blk : 97;
    const int yp = bb / 7, x4 = bb % 7;
    reinterpret_cast<unsigned short*>(smem + kFTabA)[b] = (unsigned short)(yp * 4 * kFxPitch + x4 * 8);
    // low byte: Y1 pixel of the block's left window (x16 = byte offset); high
    // byte: A1 offset of that window.  The two padding blocks write Y1 into
    // the sink (pixel index (kFJunk - kFY1) / 16) and A1 into the unused
    // columns 14, 15 of row 13.
    const uint32_t e = blk < 98 ? (uint32_t)(yp * 14 + 2 * x4) | ((uint32_t)(yp * 16 + 2 * x4) << 8)
                              : (uint32_t)((kFJunk - kFY1) / 16) | ((uint32_t)(13 * 16 + 14) << 8);
    reinterpret_cast<unsigned short*>(smem + kFTabE)[b] = (unsigned short)e;
  }
  // conv2: Y1 byte offset of A row (T, n) (table), and the window this lane's
  // accumulator rows pool, per tile (bytes of two registers, window + 1)
  for (int r = lane; r < 112; r += 64) {
    const int wr = kC2Win[4 * (r >> 4) + ((r & 15) >> 2)], w = wr < 0 ? 24 : wr, pos = r & 3;
    reinterpret_cast<unsigned short*>(smem + kFTab2)[r] =
        (unsigned short)(((2 * (w / 5) + (pos >> 1)) * 14 + 2 * (w % 5) + (pos & 1)) * 16);
  }
  uint32_t c2win[2] = {0u, 0u};
#pragma unroll
  for (int T = 0; T < 7; ++T) c2win[T >> 2] |= (uint32_t)(kC2Win[4 * T + g] + 1) << (8 * (T & 3));

  // conv1 A-fragment address of this lane: copy (m>>1)&1, row (m&1) + kh
  const int msub = n16 & 3, mblk = n16 >> 2;
  const int a1base = ((msub >> 1) * kFxCopy) + ((msub & 1) * kFxPitch + g * kFxPitch) * 2;
  const int a1base_c1 = a1base + (4 - g) * kFxPitch * 2;
  const int stride_w = (int)gridDim.x;

  // staging items: 8 lanes per image row (k = lane & 7 -> pixel quad)
  const int sk = lane & 7, srow = lane >> 3;

  // the u8 image of the next iteration is loaded while this one computes
  uint32_t xw[4];
  WaveIdx widx;
  widx.load(p.idx, blockIdx.x, stride_w, p.B, 0);
  auto load_img = [&](int k) {  // k-th image of this wave
    if ((k & 63) == 0 && k > 0) widx.load(p.idx, blockIdx.x, stride_w, p.B, k);
    const uint8_t* xin = p.x + (size_t)widx.get(k) * kImgPix;
#pragma unroll
    for (int it = 0; it < 4; ++it) {
      const int yy = it * 8 + srow;
      xw[it] = (yy < 28 && sk < 7) ? *reinterpret_cast<const uint32_t*>(xin + yy * 28 + sk * 4) : 0u;
    }
  };
  if ((int)blockIdx.x < p.B) load_img(0);
  const int co1 = n16 >> 1, j1 = n16 & 1;
  const int cA = 3 - j1, cB = 1 - j1;  // 3 - position in the window, rows (y) and (y+1)
  const int ey1 = j1 * 16 + co1 * 2;   // lane part of the epilogue's Y1 / A1 offsets
  const int ea1 = min(co1, 6) * kFA1Plane + j1;
  const unsigned short* tabA = reinterpret_cast<const unsigned short*>(smem + kFTabA);
  const unsigned short* tabE = reinterpret_cast<const unsigned short*>(smem + kFTabE);
  const unsigned short* tab2 = reinterpret_cast<const unsigned short*>(smem + kFTab2);
  // second halves of the conv1 A fragments: +8 B through an opaque register
  int hb8 = 8;
  asm volatile("" : "+v"(hb8));
  const int a1base2 = a1base + hb8, a1base_c12 = a1base_c1 + hb8;
  // A1 bulk copy: 16-B chunk i = (plane i / 14, row i % 14)
  const int a1src0 = (lane / 14) * kFA1Plane + (lane % 14) * 16;
  const int a1src1 = ((lane + 64) / 14) * kFA1Plane + ((lane + 64) % 14) * 16;

  for (int img = blockIdx.x, kimg = 0; img < p.B; img += stride_w, ++kimg) {
    wave_lds_sync();  // the previous image's LDS reads are done
#pragma unroll
    for (int it = 0; it < 4; ++it) {
      const int yy = it * 8 + srow;
      uint32_t lo, hi;
      u8x4_ints(xw[it], lo, hi);
      const uint32_t phi = from_left(hi);
      if (yy < 28) {
        char* d = xf + ((yy + 2) * kFxPitch + 4 * sk) * 2;
        *reinterpret_cast<u32x2*>(d) = u32x2{phi, lo};            // Xpad cols 4k .. 4k+3
        *reinterpret_cast<u32x2*>(d + kFxCopy) = u32x2{lo, hi};   // Xpad cols 4k+2 .. 4k+5
      }
    }
    wave_lds_sync();
    if (img + stride_w < p.B) load_img(kimg + 1);

    // ---- conv1 + ReLU + pool: the next tile's A fragments are read before this tile's epilogue ----
    if constexpr (!(MCC_LENET_ABL & 16)) {
    bf16x8 fa, fb;
    {
      const int off = tabA[mblk];
      fa = lds8p(xf + a1base + off, xf + a1base2 + off);
      fb = lds8p(xf + a1base_c1 + off, xf + a1base_c12 + off);
    }
    for (int T = 0; T < 25; ++T) {
      f32x4 acc = {bias1, bias1, bias1, bias1};
      acc = mma(acc, fa, w1[0]);
      acc = mma(acc, fb, w1[1]);
      const uint32_t e = tabE[4 * T + g];
      if (T + 1 < 25) {
        const int off = tabA[4 * T + 4 + mblk];
        fa = lds8p(xf + a1base + off, xf + a1base2 + off);
        fb = lds8p(xf + a1base_c1 + off, xf + a1base_c12 + off);
      }
      const int k0 = (__float_as_int(acc[0]) & ~3) | cA;
      const int k1 = (__float_as_int(acc[1]) & ~3) | cB;
      const int k2 = (__float_as_int(acc[2]) & ~3) | cA;
      const int k3 = (__float_as_int(acc[3]) & ~3) | cB;
      const int vA = imax(k0, k1), vB = imax(k2, k3);
      const int keep = j1 ? vB : vA, send = j1 ? vA : vB;
      const int best = imax(keep, swap1(send));
      // the two code bits left in the value perturb it by < 2^-21: below the bf16 rounding
      const bf16 yb = (bf16)(__int_as_float(imax(best, 0)) * (1.f / 255.f));
      *reinterpret_cast<bf16*>(y1s + (e & 0xffu) * 16 + ey1) = yb;
      a1s[(e >> 8) + ea1] = (uint8_t)((float)yb > 0.f ? ((best & 3) ^ 3) : 4);
    }
    wave_lds_sync();  // pooled conv1 output and codes complete in LDS
    if constexpr (!(MCC_LENET_ABL & 512)) {  // bulk copies to HBM: Y1 (196 x 16 B), A1 (84 x 16 B)
      u32x4* y1g = reinterpret_cast<u32x4*>(static_cast<bf16*>(p.y1) + (size_t)img * kY1Elems);
      u32x4* a1g = reinterpret_cast<u32x4*>(p.a1 + (size_t)img * kA1Bytes);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int i = lane + 64 * r;
        if (i < 196) y1g[i] = *reinterpret_cast<const u32x4*>(y1s + i * 16);
      }
      a1g[lane] = *reinterpret_cast<const u32x4*>(a1s + a1src0);
      if (lane < 20) a1g[lane + 64] = *reinterpret_cast<const u32x4*>(a1s + a1src1);
    }

    }
    // ---- conv2 + ReLU + pool: all seven A fragments in flight before the MFMA chain ----
    if constexpr (!(MCC_LENET_ABL & 32)) {
    bf16* y2g = static_cast<bf16*>(p.y2) + (size_t)img * kY2Elems;
    uint8_t* a2g = p.a2 + (size_t)img * kY2Elems;
#pragma unroll 1
    for (int T = 0; T < 7; ++T) {
      const char* pa = y1s + tab2[16 * T + n16];
      bf16x8 af[7];
#pragma unroll
      for (int c = 0; c < 7; ++c) af[c] = *reinterpret_cast<const bf16x8*>(pa + koff2[c]);
      __builtin_amdgcn_sched_barrier(0);
      f32x4 acc = {bias2, bias2, bias2, bias2};
#pragma unroll
      for (int c = 0; c < 7; ++c) acc = mma(acc, af[c], w2[c]);
      const int wo = (int)(((T < 4 ? c2win[0] : c2win[1]) >> (8 * (T & 3))) & 0xffu) - 1;
      const int k0 = __float_as_int(acc[0]) | 3;
      const int k1 = (__float_as_int(acc[1]) & ~3) | 2;
      const int k2 = (__float_as_int(acc[2]) & ~3) | 1;
      const int k3 = __float_as_int(acc[3]) & ~3;
      const int best = imax(imax(k0, k1), imax(k2, k3));
      const bf16 yb = (bf16)__int_as_float(imax(best, 0));
      if (wo >= 0) {
        y2g[wo * 16 + n16] = yb;
        a2g[wo * 16 + n16] = (uint8_t)((float)yb > 0.f ? ((best & 3) ^ 3) : 4);
      }
    }
    }
  }
}

// ---------------------------------------------------------------------------
// Forward, round 5: conv1 with whole pooling windows in a lane.
//
// The kernel above spends ~60 % of its time in the conv1 epilogue (phase
// ablation: conv1 266 of 433 us): its MFMA rows are pixel pairs, so a 2x2
// window is split over two lanes (DPP swap + selects), and every tile reads
// three index tables (A offsets, Y1 / A1 epilogue offsets) whose values feed
// the next tile's address math (26 VALU + 2 dependent LDS table reads per
// tile).  Here:
//   * MFMA row m = 4w + i is POSITION i = (dy, dx) = (i >> 1, i & 1) of window
//     slot w, so lane (n, g) holds the four positions of window slot g in its
//     accumulator: the pool is two v_max3 (keys with the position in the low
//     bits, as before, and the ReLU clamp folded in);
//   * column n = 2 co + s computes channel co of the window s = 0 / 1 pooled
//     columns to the right (taps shifted by two inside the 8-wide K window):
//     12 of 16 columns useful, as before;
//   * a tile's four window slots are the 2x2 block of even-column windows
//     (py0 + (w >> 1), px0 + 2 (w & 1)), so with the s shift a tile covers
//     2 pooled rows x 4 pooled columns and every operand / result address is
//     a per-lane constant plus a per-tile immediate: no tables, no address
//     VALU.  28 tiles (7 row pairs x 4 column blocks; the last block's
//     columns 14, 15 land in junk columns of the LDS Y1 / A1 rows) vs 25;
//   * the odd-position rows read a second copy of the padded input shifted by
//     ONE element (copies: shift 0 and 1), so every A fragment is two aligned
//     ds_read_b64;
//   * conv2's pooled outputs are staged in LDS (in the dead input copies) and
//     leave as 16-byte rows instead of 2-byte / 1-byte scattered stores.
constexpr int kGxPitch = 36;                      // elements (72 B: rows on distinct bank pairs)
constexpr int kGxCopy = kGxPitch * 32 * 2 + 16;   // 2320 (copy 1 on banks 4 dwords off copy 0)
// Y1 keeps the compact HWC-8 layout of the global tensor (14-pixel rows: the
// conv2 operand reads were bank-annealed for it; 16-pixel rows measured 701
// conflict cycles per image, tools/lds_banks.py lenet_fwd2), so the windows of
// the last column block that fall past column 13 are masked at the Y1 store.
constexpr int kGY1 = 2 * kGxCopy;                 // 4640: Y1 HWC-8, 196 x 16 B
constexpr int kGA1 = kGY1 + 196 * 16;             // 7776: A1 [7][14][16] u8 (plane 6: columns co 6, 7)
constexpr int kGA1Plane = 240;
constexpr int kGTab2 = kGA1 + 7 * kGA1Plane;      // 9456: u16 [112] conv2 row -> Y1 byte offset
constexpr int kGLds = kGTab2 + 224;               // 9680
static_assert(16 * kGLds <= 163840, "lenet_fwd2: 16 waves per CU");
static_assert(kGY1 % 16 == 0 && kGY1 >= 2 * kGxCopy, "lenet_fwd2 layout");
// conv2 pooled outputs staged over A1 (copied out before conv2; the next
// image's conv1 rewrites every byte of A1 that is copied out).  Not over the
// input copies: their zero padding rows / columns are written only once.
constexpr int kGY2 = kGA1;                        // Y2 [25][16] bf16 = 800 B
constexpr int kGA2 = kGA1 + 800;                  // A2 [25][16] u8 = 400 B
static_assert(kGA2 + 400 <= kGA1 + 7 * kGA1Plane, "Y2 / A2 staging fits in A1");

// 8 bf16 from two 8-byte LDS reads that the compiler must not fuse into one
// ds_read2_b64 (8 cycles at 32 banks vs 2 x 2 cycles)
typedef __attribute__((address_space(3))) const volatile bf16x4 lds_vbf16x4;
__device__ __forceinline__ bf16x8 lds8v(const char* p) {
  const auto* q = (const __attribute__((address_space(3))) char*)(p);
  const bf16x4 lo = *reinterpret_cast<lds_vbf16x4*>(q);
  const bf16x4 hi = *reinterpret_cast<lds_vbf16x4*>(q + 8);
  return __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
}

__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(4))) lenet_fwd2_kernel(LenetFwdParams p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = threadIdx.x;
  const int n16 = lane & 15, g = lane >> 4;
  const int co = n16 >> 1, sh = n16 & 1;

  // ---- weights: conv1 B[k][n = 2 co + s] = W1[co][kh][kw' - 2 s] ----
  bf16x8 w1[2];
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    const int kh = c == 0 ? g : 4;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int kw = e - 2 * sh;
      const bool ok = n16 < 12 && (c == 0 || g == 0) && kw >= 0 && kw < 5;
      const float v = p.w1[ok ? co * 25 + kh * 5 + kw : 0];
      w1[c][e] = (bf16)(ok ? v : 0.f);
    }
  }
  const float bias1 = n16 < 12 ? 255.f * p.b1[co] : 0.f;  // the tile holds raw integer pixels
  bf16x8 w2[7];
  int koff2[7];
#pragma unroll
  for (int c = 0; c < 7; ++c) {
    const int t = kC2Tap[4 * c + g], kh = t < 25 ? t / 5 : 0, kw = t < 25 ? t % 5 : 0;
    koff2[c] = (kh * 14 + kw) * 16;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const bool ok = t < 25 && e < 6;
      const float v = p.w2[ok ? (n16 * 6 + e) * 25 + t : 0];
      w2[c][e] = (bf16)(ok ? v : 0.f);
    }
  }
  const float bias2 = p.b2[n16];

  char* xf = smem;
  char* y1s = smem + kGY1;
  char* a1s = smem + kGA1;
  zero_wave_lds(smem, kGLds);
  wave_lds_sync();
  for (int r = lane; r < 112; r += 64) {
    const int wr = kC2Win[4 * (r >> 4) + ((r & 15) >> 2)], w = wr < 0 ? 24 : wr, pos = r & 3;
    reinterpret_cast<unsigned short*>(smem + kGTab2)[r] =
        (unsigned short)(((2 * (w / 5) + (pos >> 1)) * 14 + 2 * (w % 5) + (pos & 1)) * 16);
  }
  uint32_t c2win[2] = {0u, 0u};
#pragma unroll
  for (int T = 0; T < 7; ++T) c2win[T >> 2] |= (uint32_t)(kC2Win[4 * T + g] + 1) << (8 * (T & 3));
  const unsigned short* tab2 = reinterpret_cast<const unsigned short*>(smem + kGTab2);

  // conv1 A operand of this lane: row m = n16 = 4 wa + ia, k-group g (kernel row g; chunk 1: row 4)
  const int wa = n16 >> 2, ia = n16 & 3;
  const int abase = (ia & 1) * kGxCopy + (2 * (wa >> 1) + (ia >> 1) + g) * kGxPitch * 2 + 8 * (wa & 1);
  // epilogue of this lane: window slot g, column shift sh, channel co
  const int ey1 = ((g >> 1) * 14 + 2 * (g & 1) + sh) * 16 + co * 2;
  const bool y1last = (g & 1) == 0;  // in the last column block (px0 = 12) only slots 0, 2 are columns < 14
  const int ea1 = min(co, 6) * kGA1Plane + (g >> 1) * 16 + 2 * (g & 1) + sh;

  const int sk = lane & 7, srow = lane >> 3;
  const int stride_w = (int)gridDim.x;
  uint32_t xw[4];
  WaveIdx widx;
  widx.load(p.idx, blockIdx.x, stride_w, p.B, 0);
  auto load_img = [&](int k) {
    if ((k & 63) == 0 && k > 0) widx.load(p.idx, blockIdx.x, stride_w, p.B, k);
    const uint8_t* xin = p.x + (size_t)widx.get(k) * kImgPix;
#pragma unroll
    for (int it = 0; it < 4; ++it) {
      const int yy = it * 8 + srow;
      xw[it] = (yy < 28 && sk < 7) ? *reinterpret_cast<const uint32_t*>(xin + yy * 28 + sk * 4) : 0u;
    }
  };
  if ((int)blockIdx.x < p.B) load_img(0);
  // A1 bulk copy: chunk i = (plane i / 14, row i % 14)
  const int a1src0 = (lane / 14) * kGA1Plane + (lane % 14) * 16;
  const int a1src1 = ((lane + 64) / 14) * kGA1Plane + ((lane + 64) % 14) * 16;

  for (int img = blockIdx.x, kimg = 0; img < p.B; img += stride_w, ++kimg) {
    wave_lds_sync();  // the previous image's LDS reads (incl. the Y2 / A2 copy-out) are done
#pragma unroll
    for (int it = 0; it < 4; ++it) {
      const int yy = it * 8 + srow;
      uint32_t lo, hi;
      u8x4_ints(xw[it], lo, hi);
      const uint32_t phi = from_left(hi);
      if (yy < 28) {
        char* d = xf + ((yy + 2) * kGxPitch + 4 * sk) * 2;
        *reinterpret_cast<u32x2*>(d) = u32x2{phi, lo};                                    // Xpad cols 4k .. 4k+3
        *reinterpret_cast<u32x2*>(d + kGxCopy) = u32x2{mid16(phi, lo), mid16(lo, hi)};    // Xpad cols 4k+1 .. 4k+4
      }
    }
    wave_lds_sync();
    if (img + stride_w < p.B) load_img(kimg + 1);

    // ---- conv1 + ReLU + pool: 28 tiles, operand reads of tile T+1 before tile T's epilogue ----
    if constexpr (!(MCC_LENET_ABL & 16)) {
      auto tile_a = [](int T) { return (2 * (T >> 2)) * 2 * kGxPitch * 2 + 4 * (4 * (T & 3)); };  // py0 = 2 (T/4), px0 = 4 (T%4)
      auto tile_y = [](int T) { return ((2 * (T >> 2)) * 14 + 4 * (T & 3)) * 16; };               // Y1 (py0, px0)
      auto tile_c = [](int T) { return (2 * (T >> 2)) * 16 + 4 * (T & 3); };                      // A1 (py0, px0)
      // software-pipelined: tile T + 1's MFMAs are issued before tile T's
      // epilogue (which then needs no wait states for its accumulator), and
      // tile T + 2's operands are read meanwhile (two operand sets)
      const f32x4 b4 = {bias1, bias1, bias1, bias1};
      bf16x8 fa[2], fb[2];
      fa[0] = lds8v(xf + abase + tile_a(0));
      fb[0] = lds8v(xf + abase + tile_a(0) + 4 * kGxPitch * 2);
      fa[1] = lds8v(xf + abase + tile_a(1));
      fb[1] = lds8v(xf + abase + tile_a(1) + 4 * kGxPitch * 2);
      f32x4 acc = mma(mma(b4, fa[0], w1[0]), fb[0], w1[1]);
      float kprev = 0.f;
#pragma unroll
      for (int T = 0; T < 28; ++T) {
        f32x4 accn = acc;
        if (T + 1 < 28) accn = mma(mma(b4, fa[(T + 1) & 1], w1[0]), fb[(T + 1) & 1], w1[1]);
        if (T + 2 < 28) {
          fa[T & 1] = lds8v(xf + abase + tile_a(T + 2));
          fb[T & 1] = lds8v(xf + abase + tile_a(T + 2) + 4 * kGxPitch * 2);
        }
        __builtin_amdgcn_sched_barrier(0);
        const int k0 = __float_as_int(acc[0]) | 3;
        const int k1 = (__float_as_int(acc[1]) & ~3) | 2;
        const int k2 = (__float_as_int(acc[2]) & ~3) | 1;
        const int k3 = __float_as_int(acc[3]) & ~3;
        // ReLU folded into the pool max: the key is >= 0, and > 3 iff the
        // window's maximum is positive (position code ~key & 3)
        const int key = max3i(max3i(k0, k1, k2), k3, 0);
        a1s[ea1 + tile_c(T)] = (uint8_t)(key > 3 ? (~key & 3) : 4);
        // the two code bits left in the value perturb it by < 2^-21: below the
        // bf16 rounding.  Scale and convert two tiles at a time (v_pk_mul_f32,
        // one v_cvt_pk_bf16_f32)
        if (T & 1) {
          typedef float f2 __attribute__((ext_vector_type(2)));
          typedef bf16 b2 __attribute__((ext_vector_type(2)));
          const f2 v = f2{kprev, __int_as_float(key)} * f2{1.f / 255.f, 1.f / 255.f};
          const b2 y = __builtin_convertvector(v, b2);
          *reinterpret_cast<bf16*>(y1s + ey1 + tile_y(T - 1)) = y[0];
          if ((T & 3) != 3 || y1last) *reinterpret_cast<bf16*>(y1s + ey1 + tile_y(T)) = y[1];
        } else {
          kprev = __int_as_float(key);
        }
        acc = accn;
      }
    }
    wave_lds_sync();  // pooled conv1 output and codes complete in LDS
    if constexpr (!(MCC_LENET_ABL & 512)) {  // bulk copies to HBM: Y1 (196 x 16 B), A1 (84 x 16 B)
      u32x4* y1g = reinterpret_cast<u32x4*>(static_cast<bf16*>(p.y1) + (size_t)img * kY1Elems);
      u32x4* a1g = reinterpret_cast<u32x4*>(p.a1 + (size_t)img * kA1Bytes);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int i = lane + 64 * r;
        if (i < 196) y1g[i] = *reinterpret_cast<const u32x4*>(y1s + i * 16);
      }
      a1g[lane] = *reinterpret_cast<const u32x4*>(a1s + a1src0);
      if (lane < 20) a1g[lane + 64] = *reinterpret_cast<const u32x4*>(a1s + a1src1);
    }

    // ---- conv2 + ReLU + pool -> Y2 / A2 staged in LDS (over A1) ----
    if constexpr (!(MCC_LENET_ABL & 32)) {
#pragma unroll 1
      for (int T = 0; T < 7; ++T) {
        const char* pa = y1s + tab2[16 * T + n16];
        bf16x8 af[7];
#pragma unroll
        for (int c = 0; c < 7; ++c) af[c] = *reinterpret_cast<const bf16x8*>(pa + koff2[c]);
        __builtin_amdgcn_sched_barrier(0);
        f32x4 acc = {bias2, bias2, bias2, bias2};
#pragma unroll
        for (int c = 0; c < 7; ++c) acc = mma(acc, af[c], w2[c]);
        const int wo = (int)(((T < 4 ? c2win[0] : c2win[1]) >> (8 * (T & 3))) & 0xffu) - 1;
        const int k0 = __float_as_int(acc[0]) | 3;
        const int k1 = (__float_as_int(acc[1]) & ~3) | 2;
        const int k2 = (__float_as_int(acc[2]) & ~3) | 1;
        const int k3 = __float_as_int(acc[3]) & ~3;
        const int best = imax(imax(imax(k0, k1), imax(k2, k3)), 0);
        const bf16 yb = (bf16)__int_as_float(best);
        if (wo >= 0) {
          *reinterpret_cast<bf16*>(smem + kGY2 + (wo * 16 + n16) * 2) = yb;
          smem[kGA2 + wo * 16 + n16] = (uint8_t)(best > 3 ? (~best & 3) : 4);
        }
      }
    }
    wave_lds_sync();
    if constexpr (!(MCC_LENET_ABL & 1024)) {  // Y2: 50 x 16 B, A2: 25 x 16 B
      u32x4* y2g = reinterpret_cast<u32x4*>(static_cast<bf16*>(p.y2) + (size_t)img * kY2Elems);
      u32x4* a2g = reinterpret_cast<u32x4*>(p.a2 + (size_t)img * kY2Elems);
      // chunks 0..74 = Y2 0..49, A2 0..24 over lanes 0..63, then 64..74
      if (lane < 50) y2g[lane] = *reinterpret_cast<const u32x4*>(smem + kGY2 + lane * 16);
      else a2g[lane - 50] = *reinterpret_cast<const u32x4*>(smem + kGA2 + (lane - 50) * 16);
      if (lane < 11) a2g[lane + 14] = *reinterpret_cast<const u32x4*>(smem + kGA2 + (lane + 14) * 16);
    }
  }
}

// ============================================================================
// Backward
// ============================================================================
//
// tapoff2(t): byte offset of conv2 tap t in the HWC-8 Y1 copy
__host__ __device__ constexpr int tapoff2(int t) { return ((t / 5) * 14 + t % 5) * 16; }
// dX2 chunk c covers taps (u', v) = divmod(2c, 5) and the next one; byte
// offset of the first in the padded dZ2 copy (20-pixel rows, 32 B pixels)
__host__ __device__ constexpr int dxoff(int c) { return (((2 * c) / 5) * 20 + (2 * c) % 5) * 32; }
__host__ __device__ constexpr bool dxwrap(int c) { return (2 * c) % 5 == 4; }

// Two waves per image (a 128-thread workgroup, four per CU: two waves per
// SIMD, where the single-wave version ran one and exposed every LDS / VALU
// latency of its phases):
//   wave 0 (weight gradients): conv2 dW (reads dZ2, Y1), then conv1 dW
//     (reads dZ1, X0); owns the dW accumulators and the slab;
//   wave 1 (data gradient + staging): conv2 dX -> dZ1 (reads dZ2), then the
//     NEXT image's dZ2 and Y1 (their last readers are done) while wave 0
//     runs conv1 dW.
// Both stage their half of X0.  Three barriers per image: B1 (X0, dZ2, Y1
// staged), B2 (dZ1 complete, dZ2 / Y1 free), B3 (conv1 dW done: X0 and dZ1
// free).  Barriers are explicit s_barrier after lgkmcnt(0) (the LDS writes),
// never __syncthreads(), which would also drain the in-flight prefetch loads.
__device__ __forceinline__ void wg_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

__global__ void __launch_bounds__(128) __attribute__((amdgpu_waves_per_eu(2, 2))) lenet_bwd_kernel(LenetBwdParams p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int n16 = lane & 15, g = lane >> 4;
  const int tq = (lane >> 2) & 3, tp = lane & 3;  // transposed-read roles (row q, column quad p)
  const int sk = lane & 7, srow = lane >> 3;      // X0 staging items

  {
    const u32x4 z = {0u, 0u, 0u, 0u};
    for (int i = threadIdx.x * 16; i < kBLds; i += 128 * 16) *reinterpret_cast<u32x4*>(smem + i) = z;
  }
  wg_barrier();
  if (wv == 0) {  // bf16 ones: the dW2 bias pixel and the dW1 bias rows (cols 0..31 of 30 rows)
    const uint32_t one2 = 0x3f803f80u;
    if (lane < 4) *reinterpret_cast<uint32_t*>(smem + kBOne2 + 4 * lane) = one2;
    for (int i = lane; i < 30 * 16; i += 64)
      *reinterpret_cast<uint32_t*>(smem + kBOne1 + (i >> 4) * 80 + (i & 15) * 4) = one2;
  }

  // X0 staging of rows it*8 + srow (it = 2 wv, 2 wv + 1): copy c holds Xpad[r][p + c] at position p
  uint32_t xw[2];
  auto load_x = [&](const uint8_t* xin) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int yy = (2 * wv + h) * 8 + srow;
      xw[h] = (yy < 28 && sk < 7) ? *reinterpret_cast<const uint32_t*>(xin + yy * 28 + sk * 4) : 0u;
    }
  };
  auto stage_x = [&]() {
#pragma unroll
    for (int h = 0; h < ((MCC_LENET_ABL & 128) ? 0 : 2); ++h) {
      const int yy = (2 * wv + h) * 8 + srow;
      uint32_t lo, hi;
      u8x4_ints(xw[h], lo, hi);
      const uint32_t phi = from_left(hi);
      const uint32_t rlo = from_right(lo);
      const uint32_t nlo = sk == 7 ? 0u : rlo;
      if (yy < 28) {
        char* d = smem + kBXs + ((yy + 2) * 40 + 4 * sk) * 2;
        *reinterpret_cast<u32x2*>(d) = u32x2{phi, lo};
        *reinterpret_cast<u32x2*>(d + kBxCopy) = u32x2{mid16(phi, lo), mid16(lo, hi)};
        *reinterpret_cast<u32x2*>(d + 2 * kBxCopy) = u32x2{lo, hi};
        *reinterpret_cast<u32x2*>(d + 3 * kBxCopy) = u32x2{mid16(lo, hi), mid16(hi, nlo)};
      }
    }
  };
  WaveIdx widx;
  widx.load(p.idx, blockIdx.x, (int)gridDim.x, p.B, 0);
  auto image_x = [&](int k) {  // dataset image of this workgroup's k-th image
    if ((k & 63) == 0 && k > 0) widx.load(p.idx, blockIdx.x, (int)gridDim.x, p.B, k);
    return p.x + (size_t)widx.get(k) * kImgPix;
  };

  // conv1 dW (wave 0, all 30 output rows: splitting the rows between the two
  // waves measured no faster and costs a second slab half): A row m = (kDw1Co[m], kDw1S[m]) (rows 12..15 repeat 0..3), B column n =
  // 5*kh' + kw (15 = ones).  Row zy + 2 - 2s of the swizzled dZ1 plane: its
  // chunk bit is (zy >> 1) ^ 1 ^ s, so two bases by the parity of zy >> 1.
  int a1b[2];
  {
    const int m = n16 < 12 ? n16 : n16 - 12, co = kDw1Co[m], s2 = kDw1S[m];
    const int base = kBDz1 + co * kBDz1Plane + (2 - 2 * s2) * 64;
    a1b[0] = base + 16 * (g ^ 1 ^ s2);
    a1b[1] = base + 16 * (g ^ s2);
  }
  int b1b;
  {
    if (n16 == 15) b1b = kBOne1 + 16 * g;
    else {
      const int kh = n16 / 5, kw = n16 % 5, c = kw & 3;
      b1b = kBXs + c * kBxCopy + (kh * 40 + 8 * g + kw - c) * 2;
    }
  }
  f32x4 acc1 = {0.f, 0.f, 0.f, 0.f};
  auto dw1 = [&]() {  // one MFMA per output row (32 pixels), 4 rows of reads in flight
    if constexpr (!(MCC_LENET_ABL & 4)) {
      constexpr int D = 4, NR = 30;
      const int z0 = 0;
      bf16x8 a[D], b[D];
#pragma unroll
      for (int i = 0; i < D; ++i) {
        const int zy = z0 + i;
        a[i] = *reinterpret_cast<const bf16x8*>(smem + a1b[(zy >> 1) & 1] + zy * 64);
        b[i] = lds8(smem + b1b + zy * 80);
      }
#pragma unroll
      for (int i = 0; i < NR; ++i) {
        const bf16x8 ca = a[i % D], cb = b[i % D];
        if (i + D < NR) {
          const int zy = z0 + i + D;
          a[i % D] = *reinterpret_cast<const bf16x8*>(smem + a1b[(zy >> 1) & 1] + zy * 64);
          b[i % D] = lds8(smem + b1b + zy * 80);
        }
        __builtin_amdgcn_sched_barrier(0);
        acc1 = mma(acc1, ca, cb);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
  };

  if (wv == 0) {
    // ======================= wave 0: conv2 dW, conv1 dW =======================
    // dW2: transposed reads, K position 32c + 8g + 4hf + tq holds pixel kZPos[.]
    int aw2[4][2], bw2a[4][2], bw2b[4][2], bw2c[4][2];
#pragma unroll
    for (int c = 0; c < 4; ++c)
#pragma unroll
      for (int hf = 0; hf < 2; ++hf) {
        const int v = kZPos[32 * c + 8 * g + 4 * hf + tq];
        const bool ok = v < 100;
        const int z = ok ? v : v - 128;
        const int zy = z / 10, zx = z % 10;
        aw2[c][hf] = ok ? kBDz2 + ((zy + 4) * 20 + zx + 4) * 32 + 8 * tp : kBDz2 + 8 * tp;
        const int yb = kBY1 + (zy * 14 + zx) * 16 + 8 * (tp & 1);
        bw2a[c][hf] = yb + (tp >> 1) * 16;
        bw2b[c][hf] = yb + (tp >> 1) * 160;
        bw2c[c][hf] = (tp >> 1) ? kBOne2 + 8 * (tp & 1) - tapoff2(24) : yb;
      }
    f32x4 acc2[13];
#pragma unroll
    for (int t = 0; t < 13; ++t) acc2[t] = f32x4{0.f, 0.f, 0.f, 0.f};

    if ((int)blockIdx.x < p.B) load_x(image_x(0));
    for (int img = blockIdx.x, kimg = 0; img < p.B; img += (int)gridDim.x, ++kimg) {
      stage_x();
      wg_barrier();  // B1
      if (img + (int)gridDim.x < p.B && !(MCC_LENET_ABL & 256)) load_x(image_x(kimg + 1));

      // ---- conv2 weight gradient (operands of chunk c+1 read during chunk c) ----
      if constexpr (!(MCC_LENET_ABL & 1)) {
        bf16x8 af[2], bfr[2][13];
        auto load_chunk = [&](int c, int buf) {
          af[buf] = tr8(smem + aw2[c][0], smem + aw2[c][1]);
#pragma unroll
          for (int t = 0; t < 13; ++t) {
            const int o = tapoff2(2 * t);
            const int* base = t == 12 ? bw2c[c] : ((2 * t) % 5 == 4 ? bw2b[c] : bw2a[c]);
            bfr[buf][t] = tr8(smem + base[0] + o, smem + base[1] + o);
          }
        };
        load_chunk(0, 0);
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          if (c + 1 < 4) load_chunk(c + 1, (c + 1) & 1);
          __builtin_amdgcn_sched_barrier(0);  // keep the reads of chunk c+1 ahead of chunk c's MFMAs
#pragma unroll
          for (int t = 0; t < 13; ++t) acc2[t] = mma(acc2[t], af[c & 1], bfr[c & 1][t]);
          __builtin_amdgcn_sched_barrier(0);
        }
      }
      wg_barrier();  // B2: dZ1 complete
      dw1();
      wg_barrier();  // B3: X0 and dZ1 free
    }

    // ---- per-workgroup slab (accumulator order) ----
    float* slab = p.slab + (size_t)blockIdx.x * kSlab;
#pragma unroll
    for (int t = 0; t < 13; ++t)
#pragma unroll
      for (int i = 0; i < 4; ++i) slab[(t * 4 + i) * 64 + lane] = acc2[t][i];
#pragma unroll
    for (int i = 0; i < 4; ++i) slab[kSlabW2 + i * 64 + lane] = acc1[i];
  } else {
    // ================ wave 1: conv2 dX -> dZ1, dZ2 / Y1 staging ================
    // conv2 data-gradient weights in registers: lane (n, kgroup g): k = 32c +
    // 8g + e -> tap t = 2c + (g>>1) = (u', v), output channel co = 8(g&1) + e;
    // column n = 2*ci + j (ci < 6): B = W2[co][ci][4 + j - u'][4 - v] where the
    // row is in range.
    bf16x8 wdx[15];
    {
      const int ci = n16 >> 1, j = n16 & 1;
#pragma unroll
      for (int c = 0; c < 15; ++c) {
        const int t = 2 * c + (g >> 1), u = t / 5, v = t % 5;
        const int kh = 4 + j - u, kw = 4 - v;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const int co = 8 * (g & 1) + e;
          const bool ok = n16 < 12 && kh >= 0 && kh < 5;
          float w = p.w2[ok ? ((co * 6 + ci) * 5 + kh) * 5 + kw : 0];
          w = ok ? w : 0.f;
          wdx[c][e] = (bf16)w;
        }
      }
    }
    // A rows px = n16, k-group g: chunk tap parity (g>>1), channel half (g&1)
    const int hxa = kBDz2 + n16 * 32 + 16 * (g & 1) + (g >> 1) * 32;
    const int hxb = kBDz2 + n16 * 32 + 16 * (g & 1) + (g >> 1) * 512;
    const int zq = lane >> 1, zh = lane & 1;  // dZ2 staging items (lane < 50)
    const int zqy = (zq * 205) >> 10, zqx = zq - 5 * zqy;
    const int zbase = kBDz2 + ((2 * zqy + 4) * 20 + 2 * zqx + 4) * 32 + 16 * zh;
    const int dxci = n16 < 12 ? n16 >> 1 : 5, dxj = n16 & 1;

    // per-image loads, issued one image ahead: dY2 + argmax codes of conv2
    // (lanes < 50), Y1 (196 x 16 B), the u8 image rows of this wave, conv1
    // codes per dX tile
    u32x4 dy = {0u, 0u, 0u, 0u}, yv[4];
    u32x2 cw = {0u, 0u};
    uint32_t a1n[7], a1w[7];
    auto load_img = [&](int k) {
      const int img = blockIdx.x + k * (int)gridDim.x;
      load_x(image_x(k));  // first: the address needs the index vector
      if (lane < 50) {
        dy = *reinterpret_cast<const u32x4*>(static_cast<const bf16*>(p.dy2) + (size_t)img * kY2Elems + zq * 16 + 8 * zh);
        cw = *reinterpret_cast<const u32x2*>(p.a2 + (size_t)img * kY2Elems + zq * 16 + 8 * zh);
      }
      const bf16* y1g = static_cast<const bf16*>(p.y1) + (size_t)img * kY1Elems;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int px = min(lane + 64 * r, 195);
        yv[r] = *reinterpret_cast<const u32x4*>(y1g + px * 8);
      }
      const uint8_t* a1g = p.a1 + (size_t)img * kA1Bytes + dxci * 224 + 4 * g;
#pragma unroll
      for (int t = 0; t < 7; ++t) a1n[t] = *reinterpret_cast<const uint32_t*>(a1g + (2 * t + dxj) * 16);
    };
    auto stage_dz2_y1 = [&]() {
      if (lane < 50 && !(MCC_LENET_ABL & 8)) {  // dZ2 = unpool of dY2 by the argmax codes
        const u32x4 z = {0u, 0u, 0u, 0u};
        *reinterpret_cast<u32x4*>(smem + zbase) = z;
        *reinterpret_cast<u32x4*>(smem + zbase + 32) = z;
        *reinterpret_cast<u32x4*>(smem + zbase + 640) = z;
        *reinterpret_cast<u32x4*>(smem + zbase + 672) = z;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const uint32_t code = (cw[i >> 2] >> (8 * (i & 3))) & 0xffu;
          const uint32_t v = (dy[i >> 1] >> (16 * (i & 1))) & 0xffffu;
          const int off = ((code & 2u) ? 640 : 0) + ((code & 1u) ? 32 : 0);  // code 4: value 0 at TL
          *reinterpret_cast<unsigned short*>(smem + zbase + off + 2 * i) = (unsigned short)(code < 4u ? v : 0u);
        }
      }
#pragma unroll
      for (int r = 0; r < ((MCC_LENET_ABL & 64) ? 0 : 4); ++r) {
        const int px = lane + 64 * r;
        if (px < 196) *reinterpret_cast<u32x4*>(smem + kBY1 + px * 16) = yv[r];
      }
    };
    if ((int)blockIdx.x < p.B) {
      load_img(0);
      stage_dz2_y1();
    }
    for (int img = blockIdx.x, kimg = 0; img < p.B; img += (int)gridDim.x, ++kimg) {
      stage_x();
#pragma unroll
      for (int t = 0; t < 7; ++t) a1w[t] = a1n[t];
      wg_barrier();  // B1
      const bool more = img + (int)gridDim.x < p.B;
      if (more && !(MCC_LENET_ABL & 256)) load_img(kimg + 1);

      // ---- conv2 data gradient -> dZ1 rows (unpool by the conv1 argmax) ----
      if constexpr (!(MCC_LENET_ABL & 2)) {
        bf16x8 fr[15], nx[5];
#pragma unroll
        for (int c = 0; c < 15; ++c)
          fr[c] = *reinterpret_cast<const bf16x8*>(smem + (dxwrap(c) ? hxb : hxa) + dxoff(c));
        // software pipelined: tile T's 15 chained MFMAs are issued together with
        // tile T-1's epilogue (unpool by the conv1 argmax, dZ1 row stores)
        f32x4 accp = {0.f, 0.f, 0.f, 0.f};
        auto epilogue = [&](int T, const f32x4& acc) {
          // lane (n = 2ci + j, g): rows px = 4g + i of dY1 row py = 2T + j
          uint32_t top[4], bot[4];
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const uint32_t code = (a1w[T] >> (8 * i)) & 0xffu;
            const uint64_t h = code < 4u ? (uint64_t)bf16_bits(acc[i]) : 0ull;
            const uint64_t w = h << (16u * (code & 3u));
            top[i] = (uint32_t)w;
            bot[i] = (uint32_t)(w >> 32);
          }
          if (n16 < 12) {
            // rows 4T + 2dxj + 2 and + 3: swizzle bit (2T + dxj + 1) & 1 = 1 - dxj
            char* d = smem + kBDz1 + dxci * kBDz1Plane + (4 * T + 2 * dxj + 2) * 64 + 16 * (g ^ (1 - dxj));
            *reinterpret_cast<u32x4*>(d) = u32x4{top[0], top[1], top[2], top[3]};
            *reinterpret_cast<u32x4*>(d + 64) = u32x4{bot[0], bot[1], bot[2], bot[3]};
          }
        };
#pragma unroll
        for (int T = 0; T < 7; ++T) {
          if (T + 1 < 7) {  // tile T+1 reuses fr[5..14] as its chunks 0..9; read its chunks 10..14 now
#pragma unroll
            for (int c = 10; c < 15; ++c)
              nx[c - 10] = *reinterpret_cast<const bf16x8*>(smem + (dxwrap(c) ? hxb : hxa) + dxoff(c) + (T + 1) * 1280);
          }
          f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int c = 0; c < 15; ++c) acc = mma(acc, fr[c], wdx[c]);
          if (T > 0) epilogue(T - 1, accp);
          accp = acc;
#pragma unroll
          for (int c = 0; c < 10; ++c) fr[c] = fr[c + 5];
#pragma unroll
          for (int c = 10; c < 15; ++c) fr[c] = nx[c - 10];
        }
        epilogue(6, accp);
      }
      wg_barrier();  // B2: dZ1 complete; dZ2 and Y1 free
      if (more) stage_dz2_y1();  // the next image's, while wave 0 runs conv1 dW
      wg_barrier();  // B3
    }
  }
}

// ---------------------------------------------------------------------------
// Four waves per image (round 5).  The two-wave kernel above serialises each
// image as [dW2 | dX2 (105 MFMAs)] -> [dW1 (30)] -> staging, so wave 1's 105
// MFMAs + wave 0's 30 are its critical path and the staging loads / LDS
// writes sit between barriers.  Here a 256-thread workgroup (two per CU: two
// waves per SIMD) gives every wave ~1/4 of an image's 187 MFMAs:
//   w0: conv2 dW (52)
//   w1: conv2 dX tiles 0..2 (45)      w2: conv2 dX tiles 3..5 (45)
//   w3: conv1 dW of the PREVIOUS image (30) + conv2 dX tile 6 (15)
// conv1 dW lags one image, so dZ1 and X0 are double-buffered; per image two
// barriers: A (image k's dZ2 / Y1 / X0 staged) and B (everything that reads
// dZ2 / Y1 done: stage image k+1; dZ1[(k-1)&1] and X0[(k-1)&1] free).  The
// staging is split over w0 (X0 rows 0..15), w1 (dZ2), w2 (Y1), w3 (X0 rows
// 16..27); every wave's global loads for image k+1 are issued at the start of
// phase A and land during its MFMAs.  Buffer strides are multiples of 256 B,
// so both buffers keep the bank-model layout of the single-buffer version.
constexpr int kQXs = kBXs;                   // 14720: X0 [2][4 copies]
constexpr int kQXbuf = 41 * 256;             // 10496 (>= 4 * kBxCopy = 10336)
constexpr int kQOne1 = kQXs + kQXbuf + 4 * kBxCopy;  // 35552 (== 224 mod 256, as kBOne1)
constexpr int kQDz1 = kQOne1 + 30 * 80;      // dZ1 [2][6 planes]  (== 64 mod 256, as kBDz1)
constexpr int kQDz1buf = 49 * 256;           // 12544 (>= 6 * kBDz1Plane = 12480)
constexpr int kQLds = kQDz1 + 2 * kQDz1buf;
static_assert(kQOne1 % 256 == kBOne1 % 256 && kQDz1 % 256 == kBDz1 % 256, "bank-model offsets");
static_assert(kQXs % 256 == kBXs % 256, "bank-model offsets");
static_assert(2 * kQLds <= 163840, "lenet_bwd4: two workgroups per CU");
// One-barrier schedule (round 6): dZ2 / Y1 (+ the dW2 ones pixel) double-
// buffered -- region 1 after the two-barrier layout, at a multiple of 256 B so
// it keeps region 0's bank mapping -- so image k+1's dZ2 / Y1 are staged right
// after a wave's compute(k), and X0 of image k is staged after barrier A(k)
// (its buffer's last reader, conv1 dW of image k-2, ran in compute(k-1)).
constexpr int kQR1 = (kQLds + 255) / 256 * 256;      // 63232
constexpr int kQLds1 = kQR1 + kQXs;                   // + dZ2 / Y1 / ones: 77952
static_assert(kQXs >= kBOne2 + 16, "region 0 = [0, kQXs)");
static_assert(2 * kQLds1 <= 163840, "lenet_bwd4 one-barrier: two workgroups per CU");
constexpr int kXw0 = MCC_BWD4_XW0;  // X0 row groups (of 8 rows) staged by w0; the rest by w3
static_assert(kXw0 >= 1 && kXw0 <= 3, "X0 staging split");

template <int T0, int T1>
__device__ __forceinline__ void lenet_dx2_tiles(char* smem, const bf16x8 (&wdx)[15], const uint32_t* a1w, int hxa,
                                                int hxb, int n16, int g, int dxci, int dxj, int dz1, int roff = 0) {
  bf16x8 fr[15], nx[5];
  const char* rs = smem + roff;  // dZ2 region of this image
#pragma unroll
  for (int c = 0; c < 15; ++c)
    fr[c] = *reinterpret_cast<const bf16x8*>(rs + (dxwrap(c) ? hxb : hxa) + dxoff(c) + T0 * 1280);
  f32x4 accp = {0.f, 0.f, 0.f, 0.f};
  auto epilogue = [&](int T, const f32x4& acc) {
    uint32_t top[4], bot[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const uint32_t code = (a1w[T - T0] >> (8 * i)) & 0xffu;
      const uint64_t h = code < 4u ? (uint64_t)bf16_bits(acc[i]) : 0ull;
      const uint64_t w = h << (16u * (code & 3u));
      top[i] = (uint32_t)w;
      bot[i] = (uint32_t)(w >> 32);
    }
    if (n16 < 12) {
      char* d = smem + dz1 + dxci * kBDz1Plane + (4 * T + 2 * dxj + 2) * 64 + 16 * (g ^ (1 - dxj));
      *reinterpret_cast<u32x4*>(d) = u32x4{top[0], top[1], top[2], top[3]};
      *reinterpret_cast<u32x4*>(d + 64) = u32x4{bot[0], bot[1], bot[2], bot[3]};
    }
  };
#pragma unroll
  for (int T = T0; T < T1; ++T) {
    if (T + 1 < T1) {
#pragma unroll
      for (int c = 10; c < 15; ++c)
        nx[c - 10] = *reinterpret_cast<const bf16x8*>(rs + (dxwrap(c) ? hxb : hxa) + dxoff(c) + (T + 1) * 1280);
    }
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int c = 0; c < 15; ++c) acc = mma(acc, fr[c], wdx[c]);
    if (T > T0) epilogue(T - 1, accp);
    accp = acc;
#pragma unroll
    for (int c = 0; c < 10; ++c) fr[c] = fr[c + 5];
#pragma unroll
    for (int c = 10; c < 15; ++c) fr[c] = nx[c - 10];
  }
  epilogue(T1 - 1, accp);
}

// X0 staging shared by the w0 / w3 roles of lenet_bwd4_kernel (NH row groups
// of 8 rows from group XG): loads into xw[], LDS copies c = 0..3 of buffer buf.
#define LENET_LOAD_X(XG, NH)                                                                       \
  if ((k & 63) == 0 && k > 0) widx.load(p.idx, blockIdx.x, grid, p.B, k);                         \
  {                                                                                                \
    const uint8_t* xin = p.x + (size_t)widx.get(k) * kImgPix;                                      \
    _Pragma("unroll") for (int h = 0; h < (NH); ++h) {                                             \
      const int yy = ((XG) + h) * 8 + srow;                                                        \
      xw[h] = (yy < 28 && sk < 7) ? *reinterpret_cast<const uint32_t*>(xin + yy * 28 + sk * 4) : 0u; \
    }                                                                                              \
  }
#define LENET_STAGE_X(XG, NH)                                                                      \
  _Pragma("unroll") for (int h = 0; h < ((MCC_LENET_ABL & 128) ? 0 : (NH)); ++h) {                 \
    const int yy = ((XG) + h) * 8 + srow;                                                          \
    uint32_t lo, hi;                                                                               \
    u8x4_ints(xw[h], lo, hi);                                                                      \
    const uint32_t phi = from_left(hi);                                                            \
    const uint32_t rlo = from_right(lo);                                                           \
    const uint32_t nlo = sk == 7 ? 0u : rlo;                                                       \
    if (yy < 28) {                                                                                 \
      char* d = smem + kQXs + buf * kQXbuf + ((yy + 2) * 40 + 4 * sk) * 2;                         \
      *reinterpret_cast<u32x2*>(d) = u32x2{phi, lo};                                               \
      *reinterpret_cast<u32x2*>(d + kBxCopy) = u32x2{mid16(phi, lo), mid16(lo, hi)};               \
      *reinterpret_cast<u32x2*>(d + 2 * kBxCopy) = u32x2{lo, hi};                                  \
      *reinterpret_cast<u32x2*>(d + 3 * kBxCopy) = u32x2{mid16(lo, hi), mid16(hi, nlo)};           \
    }                                                                                              \
  }

// One role's per-image loop: every wave runs the same barrier sequence, but
// each role is its own inlined loop, so its registers (w0's 52 dW2
// accumulators, w1..w3's 60 dX2 weight registers) are not live in the others.
// pre(k): staging of image k that must follow barrier A(k) in the
// one-barrier schedule (X0); post(k): staging of image k's dZ2 / Y1 into
// region k & 1.  Two-barrier schedule (kOne = false): both after barrier B.
template <bool kOne, typename Load, typename Begin, typename Compute, typename Pre, typename Post>
__device__ __forceinline__ int lenet_bwd4_loop(const LenetBwdParams& p, Load&& load, Begin&& begin, Compute&& compute,
                                               Pre&& pre, Post&& post) {
  const int grid = (int)gridDim.x;
  if ((int)blockIdx.x < p.B) {
    load(0);
    if constexpr (!kOne) pre(0);
    post(0);
  }
  int k = 0;
#if MCC_LENET_STAMP
  // diagnostic build only: per-phase s_memtime sums (wave-uniform, in SGPRs),
  // written once at the end into the unused second half of the slab buffer
  // (tools/probes/lenet_stamp_probe.py); no memory traffic inside the loop
  unsigned long long tprev = 0, tsum[4] = {0, 0, 0, 0};
  auto stamp = [&](int, int e) {
    const unsigned long long t = __builtin_amdgcn_s_memtime();
    if (e > 0) tsum[e - 1] += t - tprev;
    tprev = t;
  };
#else
  auto stamp = [](int, int) {};
#endif
  for (int img = blockIdx.x; img < p.B; img += grid, ++k) {
    stamp(k, 0);
    wg_barrier();  // A: image k staged (dZ2, Y1; two-barrier: X0[k & 1] too)
    stamp(k, 1);
    begin();
    if constexpr (kOne) pre(k);
    const bool more = img + grid < p.B;
    if (more && !(MCC_LENET_ABL & 256)) load(k + 1);
    compute(k);
    stamp(k, 2);
    if constexpr (!kOne) wg_barrier();  // B: dZ2 / Y1 / X0[(k - 1) & 1] / dZ1[(k - 1) & 1] free
    stamp(k, 3);
    if (more) {
      if constexpr (!kOne) pre(k + 1);
      post(k + 1);
    }
    stamp(k, 4);
  }
  // one-barrier: the last image's dZ1 / X0 complete before w3's trailing conv1 dW
  if constexpr (kOne) wg_barrier();
#if MCC_LENET_STAMP
  if ((threadIdx.x & 63) == 0) {
    unsigned long long* st = reinterpret_cast<unsigned long long*>(p.slab + (size_t)512 * kSlab) +
                             (size_t)(blockIdx.x * 4 + (threadIdx.x >> 6)) * 5;
    for (int e = 0; e < 4; ++e) st[e] = tsum[e];
    st[4] = (unsigned long long)k;
  }
#endif
  return k;
}

template <bool kOne>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2, 2))) lenet_bwd4_kernel(LenetBwdParams p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int kLds = kOne ? kQLds1 : kQLds;
  auto roff = [](int k) { return kOne ? (k & 1) * kQR1 : 0; };  // dZ2 / Y1 region of image k
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int n16 = lane & 15, g = lane >> 4;
  const int sk = lane & 7, srow = lane >> 3;
  const int grid = (int)gridDim.x;

  {
    const u32x4 z = {0u, 0u, 0u, 0u};
    for (int i = threadIdx.x * 16; i < kLds; i += 256 * 16) *reinterpret_cast<u32x4*>(smem + i) = z;
  }
  wg_barrier();
  if (wv == 0) {  // bf16 ones: the dW2 bias pixel (each region) and the dW1 bias rows
    const uint32_t one2 = 0x3f803f80u;
    if (lane < 4) *reinterpret_cast<uint32_t*>(smem + kBOne2 + 4 * lane) = one2;
    if (kOne && lane < 4) *reinterpret_cast<uint32_t*>(smem + kQR1 + kBOne2 + 4 * lane) = one2;
    for (int i = lane; i < 30 * 16; i += 64)
      *reinterpret_cast<uint32_t*>(smem + kQOne1 + (i >> 4) * 80 + (i & 15) * 4) = one2;
  }
  float* slab = p.slab + (size_t)blockIdx.x * kSlab;
  auto nothing = [] {};


  if (wv == 0) {
    // ======================= w0: conv2 dW; X0 rows 0..15 =======================
    const int tq = (lane >> 2) & 3, tp = lane & 3;
    int aw2[4][2], bw2a[4][2], bw2b[4][2], bw2c[4][2];
#pragma unroll
    for (int c = 0; c < 4; ++c)
#pragma unroll
      for (int hf = 0; hf < 2; ++hf) {
        const int v = kZPos[32 * c + 8 * g + 4 * hf + tq];
        const bool ok = v < 100;
        const int z = ok ? v : v - 128;
        const int zy = z / 10, zx = z % 10;
        aw2[c][hf] = ok ? kBDz2 + ((zy + 4) * 20 + zx + 4) * 32 + 8 * tp : kBDz2 + 8 * tp;
        const int yb = kBY1 + (zy * 14 + zx) * 16 + 8 * (tp & 1);
        bw2a[c][hf] = yb + (tp >> 1) * 16;
        bw2b[c][hf] = yb + (tp >> 1) * 160;
        bw2c[c][hf] = (tp >> 1) ? kBOne2 + 8 * (tp & 1) - tapoff2(24) : yb;
      }
    f32x4 acc2[13];
#pragma unroll
    for (int t = 0; t < 13; ++t) acc2[t] = f32x4{0.f, 0.f, 0.f, 0.f};
    uint32_t xw[kXw0] = {};
    WaveIdx widx;
    widx.load(p.idx, blockIdx.x, grid, p.B, 0);
    auto load = [&](int k) { LENET_LOAD_X(0, kXw0) };
    auto pre = [&](int k) { const int buf = k & 1; LENET_STAGE_X(0, kXw0) };
    auto compute = [&](int k) {
      if constexpr (!(MCC_LENET_ABL & 1)) {
        bf16x8 af[2], bfr[2][13];
        char* rs = smem + roff(k);
        auto load_chunk = [&](int c, int buf) {
          af[buf] = tr8(rs + aw2[c][0], rs + aw2[c][1]);
#pragma unroll
          for (int t = 0; t < 13; ++t) {
            const int o = tapoff2(2 * t);
            const int* base = t == 12 ? bw2c[c] : ((2 * t) % 5 == 4 ? bw2b[c] : bw2a[c]);
            bfr[buf][t] = tr8(rs + base[0] + o, rs + base[1] + o);
          }
        };
        load_chunk(0, 0);
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          if (c + 1 < 4) load_chunk(c + 1, (c + 1) & 1);
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (int t = 0; t < 13; ++t) acc2[t] = mma(acc2[t], af[c & 1], bfr[c & 1][t]);
          __builtin_amdgcn_sched_barrier(0);
        }
      }
    };
    lenet_bwd4_loop<kOne>(p, load, nothing, compute, pre, [](int) {});
#pragma unroll
    for (int t = 0; t < 13; ++t)
#pragma unroll
      for (int i = 0; i < 4; ++i) slab[(t * 4 + i) * 64 + lane] = acc2[t][i];
    return;
  }

  // ================= w1..w3: conv2 dX (w1 tiles 0-2, w2 3-5, w3 6) =================
  bf16x8 wdx[15];
  {
    const int ci = n16 >> 1, j = n16 & 1;
#pragma unroll
    for (int c = 0; c < 15; ++c) {
      const int t = 2 * c + (g >> 1), u = t / 5, v = t % 5;
      const int kh = 4 + j - u, kw = 4 - v;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int co = 8 * (g & 1) + e;
        const bool ok = n16 < 12 && kh >= 0 && kh < 5;
        float w = p.w2[ok ? ((co * 6 + ci) * 5 + kh) * 5 + kw : 0];
        wdx[c][e] = (bf16)(ok ? w : 0.f);
      }
    }
  }
  const int hxa = kBDz2 + n16 * 32 + 16 * (g & 1) + (g >> 1) * 32;
  const int hxb = kBDz2 + n16 * 32 + 16 * (g & 1) + (g >> 1) * 512;
  const int dxci = n16 < 12 ? n16 >> 1 : 5, dxj = n16 & 1;
  constexpr int kT1 = MCC_BWD4_SPLIT ? 4 : 3, kT2 = MCC_BWD4_SPLIT ? 7 : 6;  // w1: [0, kT1), w2: [kT1, kT2), w3: [kT2, 7)
  const int t_lo = wv == 1 ? 0 : wv == 2 ? kT1 : kT2;
  uint32_t a1n[4] = {0u, 0u, 0u, 0u}, a1w[4] = {0u, 0u, 0u, 0u};
  auto load_codes = [&](int k, int nt) {
    const int img = blockIdx.x + k * grid;
    const uint8_t* a1g = p.a1 + (size_t)img * kA1Bytes + dxci * 224 + 4 * g;
#pragma unroll
    for (int t = 0; t < 4; ++t)
      if (t < nt) a1n[t] = *reinterpret_cast<const uint32_t*>(a1g + (2 * (t_lo + t) + dxj) * 16);
  };
  auto begin = [&] {
#pragma unroll
    for (int t = 0; t < 4; ++t) a1w[t] = a1n[t];
  };
  auto dz1_of = [](int k) { return kQDz1 + (k & 1) * kQDz1buf; };

  // dZ2 = unpool of dY2 (lanes < 50) and Y1: staged by w1 / w2, or swapped
  // (MCC_BWD4_STAGE: the wave with more dX tiles takes the cheaper Y1 copy)
  const int zq = lane >> 1, zh = lane & 1;
  const int zqy = (zq * 205) >> 10, zqx = zq - 5 * zqy;
  const int zbase = kBDz2 + ((2 * zqy + 4) * 20 + 2 * zqx + 4) * 32 + 16 * zh;
  u32x4 dy = {0u, 0u, 0u, 0u};
  u32x2 cw = {0u, 0u};
  auto load_dz2 = [&](int k) {
    const int img = blockIdx.x + k * grid;
    if (lane < 50) {
      dy = *reinterpret_cast<const u32x4*>(static_cast<const bf16*>(p.dy2) + (size_t)img * kY2Elems + zq * 16 + 8 * zh);
      cw = *reinterpret_cast<const u32x2*>(p.a2 + (size_t)img * kY2Elems + zq * 16 + 8 * zh);
    }
  };
  auto stage_dz2 = [&](int k) {
    char* smem_r = smem + roff(k);
    if (lane < 50 && !(MCC_LENET_ABL & 8)) {
      const u32x4 z = {0u, 0u, 0u, 0u};
      *reinterpret_cast<u32x4*>(smem_r + zbase) = z;
      *reinterpret_cast<u32x4*>(smem_r + zbase + 32) = z;
      *reinterpret_cast<u32x4*>(smem_r + zbase + 640) = z;
      *reinterpret_cast<u32x4*>(smem_r + zbase + 672) = z;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const uint32_t code = (cw[i >> 2] >> (8 * (i & 3))) & 0xffu;
        const uint32_t v = (dy[i >> 1] >> (16 * (i & 1))) & 0xffffu;
        const int off = ((code & 2u) ? 640 : 0) + ((code & 1u) ? 32 : 0);  // code 4: value 0 at TL
        *reinterpret_cast<unsigned short*>(smem_r + zbase + off + 2 * i) = (unsigned short)(code < 4u ? v : 0u);
      }
    }
  };
  u32x4 yv[4];
  auto load_y1 = [&](int k) {
    const int img = blockIdx.x + k * grid;
    const bf16* y1g = static_cast<const bf16*>(p.y1) + (size_t)img * kY1Elems;
#pragma unroll
    for (int r = 0; r < 4; ++r) yv[r] = *reinterpret_cast<const u32x4*>(y1g + min(lane + 64 * r, 195) * 8);
  };
  auto stage_y1 = [&](int k) {
    if constexpr (!(MCC_LENET_ABL & 64)) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int px = lane + 64 * r;
        if (px < 196) *reinterpret_cast<u32x4*>(smem + roff(k) + kBY1 + px * 16) = yv[r];
      }
    }
  };

  if (wv == 1) {
    // ---- w1: dX tiles [0, kT1); stages dZ2 (or Y1) ----
    auto load = [&](int k) {
      if constexpr (MCC_BWD4_STAGE) load_y1(k); else load_dz2(k);
      load_codes(k, kT1);
    };
    auto post = [&](int k) {
      if constexpr (MCC_BWD4_STAGE) stage_y1(k); else stage_dz2(k);
    };
    auto compute = [&](int k) {
      if constexpr (!(MCC_LENET_ABL & 2))
        lenet_dx2_tiles<0, kT1>(smem, wdx, a1w, hxa, hxb, n16, g, dxci, dxj, dz1_of(k), roff(k));
    };
    lenet_bwd4_loop<kOne>(p, load, begin, compute, [](int) {}, post);
  } else if (wv == 2) {
    // ---- w2: dX tiles [kT1, kT2); stages Y1 (or dZ2) ----
    auto load = [&](int k) {
      if constexpr (MCC_BWD4_STAGE) load_dz2(k); else load_y1(k);
      load_codes(k, kT2 - kT1);
    };
    auto post = [&](int k) {
      if constexpr (MCC_BWD4_STAGE) stage_dz2(k); else stage_y1(k);
    };
    auto compute = [&](int k) {
      if constexpr (!(MCC_LENET_ABL & 2))
        lenet_dx2_tiles<kT1, kT2>(smem, wdx, a1w, hxa, hxb, n16, g, dxci, dxj, dz1_of(k), roff(k));
    };
    lenet_bwd4_loop<kOne>(p, load, begin, compute, [](int) {}, post);
  } else {
    // ---- w3: conv1 dW of the previous image + dX tile 6; X0 rows 16..27 ----
    int a1b[2], b1b;
    {
      const int m = n16 < 12 ? n16 : n16 - 12, co = kDw1Co[m], s2 = kDw1S[m];
      const int base = kQDz1 + co * kBDz1Plane + (2 - 2 * s2) * 64;
      a1b[0] = base + 16 * (g ^ 1 ^ s2);
      a1b[1] = base + 16 * (g ^ s2);
      if (n16 == 15) b1b = kQOne1 + 16 * g;
      else {
        const int kh = n16 / 5, kw = n16 % 5, c = kw & 3;
        b1b = kQXs + c * kBxCopy + (kh * 40 + 8 * g + kw - c) * 2;
      }
    }
    f32x4 acc1 = {0.f, 0.f, 0.f, 0.f};
    auto dw1 = [&](int buf) {  // conv1 dW of the image staged in buffer `buf`
      if constexpr (!(MCC_LENET_ABL & 4)) {
        constexpr int D = MCC_DW1_D, NR = 30;
        const int ao = buf * kQDz1buf, bo = n16 == 15 ? 0 : buf * kQXbuf;
        bf16x8 a[D], b[D];
#pragma unroll
        for (int i = 0; i < D; ++i) {
          a[i] = *reinterpret_cast<const bf16x8*>(smem + a1b[(i >> 1) & 1] + ao + i * 64);
          b[i] = lds8(smem + b1b + bo + i * 80);
        }
#pragma unroll
        for (int i = 0; i < NR; ++i) {
          const bf16x8 ca = a[i % D], cb = b[i % D];
          if (i + D < NR) {
            const int zy = i + D;
            a[i % D] = *reinterpret_cast<const bf16x8*>(smem + a1b[(zy >> 1) & 1] + ao + zy * 64);
            b[i % D] = lds8(smem + b1b + bo + zy * 80);
          }
          __builtin_amdgcn_sched_barrier(0);
          acc1 = mma(acc1, ca, cb);
          __builtin_amdgcn_sched_barrier(0);
        }
      }
    };
    uint32_t xw[4 - kXw0] = {};
    WaveIdx widx;
    widx.load(p.idx, blockIdx.x, grid, p.B, 0);
    auto load = [&](int k) {
      LENET_LOAD_X(kXw0, 4 - kXw0)
      if constexpr (kT2 < 7) load_codes(k, 7 - kT2);
    };
    auto pre = [&](int k) { const int buf = k & 1; LENET_STAGE_X(kXw0, 4 - kXw0) };
    auto compute = [&](int k) {
      if (k > 0) dw1((k - 1) & 1);
      if constexpr (!(MCC_LENET_ABL & 2) && kT2 < 7)
        lenet_dx2_tiles<kT2, 7>(smem, wdx, a1w, hxa, hxb, n16, g, dxci, dxj, dz1_of(k), roff(k));
    };
    const int n = lenet_bwd4_loop<kOne>(p, load, begin, compute, pre, [](int) {});
    if (n > 0) dw1((n - 1) & 1);  // the last image's conv1 dW
#pragma unroll
    for (int i = 0; i < 4; ++i) slab[kSlabW2 + i * 64 + lane] = acc1[i];
  }
}

// Fixed-order sum of the per-wave slabs, mapped to the canonical gradients.
// Block = 1024 threads over 64 slab positions: wave w sums slabs w, w+16, ...
// of position blk*64 + lane (16 loads in flight per lane), then wave 0 adds
// the sixteen partials in order.
constexpr int kRedWaves = 16;
__global__ void __launch_bounds__(64 * kRedWaves) lenet_bwd_reduce_kernel(LenetBwdParams p, int nslabs) {
  __shared__ float part[kRedWaves][64];
  const int l = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int pos = blockIdx.x * 64 + l;
  float s = 0.f;
#pragma unroll 8
  for (int k = w; k < nslabs; k += kRedWaves) s += p.slab[(size_t)k * kSlab + pos];
  part[w][l] = s;
  __syncthreads();
  if (w != 0) return;
  float v = part[0][l];
#pragma unroll
  for (int i = 1; i < kRedWaves; ++i) v += part[i][l];
  if (pos < kSlabW2) {
    const int t = pos / 256, i = (pos / 64) & 3, ln = pos & 63;
    const int co = 4 * (ln >> 4) + i, n = 16 * t + (ln & 15);
    const int tap = n >> 3, ci = n & 7;
    if (n == 200) p.gb2[co] = v;
    else if (tap < 25 && ci < 6) p.gw2[(co * 6 + ci) * 25 + tap] = v;
  } else {
    const int q = pos - kSlabW2, i = q >> 6, ln = q & 63;
    const int m = 4 * (ln >> 4) + i, n = ln & 15;
    if (m >= 12) return;
    const int co = kDw1Co[m], s2 = kDw1S[m];
    if (n == 15) {
      if (s2 == 0) p.gb1[co] = v;
      return;
    }
    const int khp = n / 5, kw = n % 5;
    if (s2 == 1 && khp == 0) return;  // tap row 2 comes from s = 0
    p.gw1[co * 25 + (khp + 2 * s2) * 5 + kw] = v * (1.f / 255.f);
  }
}

}  // namespace

// two-wave kernel: 4 workgroups per CU; four-wave kernel: 2
// MCC_AB=bwd_reserve_cus=k leaves k CUs without a backward workgroup, for an
// RCCL kernel that overlaps it (profiles/cu_contention_r5.txt)
int lenet_bwd_grid() {
  const int k = std::max(0, std::min(ab_int("bwd_reserve_cus", 0), 128));
  return ab_flag("lenet_bwd2") ? 4 * (256 - k) : 2 * (256 - k);
}
size_t lenet_slab_bytes() { return (size_t)1024 * kSlab * 4; }  // the larger of the two grids
int lenet_y1_elems() { return kY1Elems; }
int lenet_a1_bytes() { return kA1Bytes; }

void lenet_forward(const LenetFwdParams& p, hipStream_t s) {
  if (p.B <= 0) return;
  const int grid = std::min(p.B, 256 * 16);
  if (ab_flag("lenet_fwd1")) hipLaunchKernelGGL(lenet_fwd_kernel, dim3(grid), dim3(64), kFLds, s, p);
  else hipLaunchKernelGGL(lenet_fwd2_kernel, dim3(grid), dim3(64), kGLds, s, p);
}

void lenet_backward(const LenetBwdParams& p, hipStream_t s) {
  if (p.B <= 0) return;
  const int grid = lenet_bwd_grid();
  if (ab_flag("lenet_bwd2")) hipLaunchKernelGGL(lenet_bwd_kernel, dim3(grid), dim3(128), kBLds, s, p);
  else if (ab_flag("bwd4_twobar")) hipLaunchKernelGGL(lenet_bwd4_kernel<false>, dim3(grid), dim3(256), kQLds, s, p);
  else hipLaunchKernelGGL(lenet_bwd4_kernel<true>, dim3(grid), dim3(256), kQLds1, s, p);
  hipLaunchKernelGGL(lenet_bwd_reduce_kernel, dim3(kSlab / 64), dim3(64 * kRedWaves), 0, s, p, grid);
}

}  // namespace gpu
}  // namespace mcc
