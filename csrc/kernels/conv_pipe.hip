// Persistent, pipelined implicit-GEMM convolution for small images (bf16).
//
// Replaces, for the layers it covers, the per-workgroup conv_small kernels
// of conv.hip (same math: reference Layer_feedForw_conv cnn.c:175-210 and
// Layer_feedBack_conv cnn.c:212-247, done correctly as in CUDAcnn.cu:167-195).
// What is different is the execution structure, shaped for gfx950:
//
//  * Persistent workgroups.  A workgroup stages its packed weights, bias and
//    index tables into LDS and zeroes its image tiles ONCE, then walks image
//    groups blockIdx.x, blockIdx.x + gridDim.x, ...  Every group rewrites the
//    same tile positions (halo and channel padding stay zero), so there is no
//    per-group zero fill.
//  * Register prefetch across the compute phase (the "issue early / write
//    late" staging split): the global loads of group g+1 are issued right
//    after group g is in LDS and land while the MFMA loop runs; they are
//    written to LDS after the next barrier.
//  * Stage-invariant staging geometry: each thread's items (image, source
//    offset, LDS destination) are computed once; a group costs one or two
//    loads and one to four 8/16-byte LDS writes per item, no divisions.
//  * Single-channel inputs (the MNIST conv) use four shifted copies of the
//    tile so every 4-tap run is one aligned 8-byte read: a K fragment of
//    (kernel row, 8 taps) is two ds_read_b64 instead of eight 2-byte gathers.
//  * Results are written to an LDS output tile and leave as coalesced 16-byte
//    stores (the C fragment holds 16 channels of 4 rows: direct stores would
//    be 2-byte scatters).
//  * Weight gradient: dY^T x im2col(X) with the pixel axis as K, both
//    operands read with ds_read_b64_tr_b16 from their staged layouts; slabs
//    per workgroup, reduced by a two-level deterministic sum.
#include <algorithm>

#include "kernels.h"
#include "mfma.h"

namespace mcc {
namespace gpu {

namespace {

constexpr int kT = 256;  // threads per workgroup (4 waves)
enum { FE_POOL = 0, FE_ACT = 1, FE_PLAIN = 2 };

typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));

template <int MODE> struct ModeInfo;
template <> struct ModeInfo<PM_U8S1> { static constexpr int W = 2, NI = 4; };
template <> struct ModeInfo<PM_PLAIN> { static constexpr int W = 4, NI = 8; };
template <> struct ModeInfo<PM_RELU> { static constexpr int W = 8, NI = 4; };
template <> struct ModeInfo<PM_UNPOOL> { static constexpr int W = 10, NI = 4; };

constexpr int mode_ni(int mode) { return mode == PM_PLAIN ? 8 : 4; }

__device__ __forceinline__ uint32_t pack2(float lo, float hi) {
  const bf16x2 v = {(bf16)lo, (bf16)hi};
  return __builtin_bit_cast(uint32_t, v);
}
// four u8 pixels -> four bf16 (x / 255, as the reference normalises, cnn.c:457)
__device__ __forceinline__ void u8x4_bf16(uint32_t w, uint32_t& h0, uint32_t& h1) {
  const float s = 1.0f / 255.0f;
  h0 = pack2((float)(w & 0xffu) * s, (float)((w >> 8) & 0xffu) * s);
  h1 = pack2((float)((w >> 16) & 0xffu) * s, (float)(w >> 24) * s);
}
// (a.hi, b.lo) as a bf16 pair
__device__ __forceinline__ uint32_t mid(uint32_t a, uint32_t b) { return __builtin_amdgcn_alignbit(b, a, 16); }

__device__ __forceinline__ void st8(bf16* p, uint32_t a, uint32_t b) { *reinterpret_cast<uint2*>(p) = make_uint2(a, b); }
__device__ __forceinline__ void st16(bf16* p, const uint32_t* w) {
  *reinterpret_cast<uint4*>(p) = make_uint4(w[0], w[1], w[2], w[3]);
}

// RW bf16 channels -> words (zero beyond RW).  Alignment: RW=8 16 B, 4 8 B, 6/2 4 B.
__device__ __forceinline__ void ld_chan(const bf16* p, int RW, uint32_t* r) {
  if (RW == 8) {
    const uint4 v = *reinterpret_cast<const uint4*>(p);
    r[0] = v.x; r[1] = v.y; r[2] = v.z; r[3] = v.w;
  } else if (RW == 6) {
    const uint32_t* q = reinterpret_cast<const uint32_t*>(p);
    r[0] = q[0]; r[1] = q[1]; r[2] = q[2]; r[3] = 0;
  } else if (RW == 4) {
    const uint2 v = *reinterpret_cast<const uint2*>(p);
    r[0] = v.x; r[1] = v.y; r[2] = 0; r[3] = 0;
  } else {
    r[0] = *reinterpret_cast<const uint32_t*>(p); r[1] = 0; r[2] = 0; r[3] = 0;
  }
}
// RW argmax bytes -> two words (channel j in byte j&3 of word j>>2)
__device__ __forceinline__ void ld_arg(const uint8_t* p, int RW, uint32_t* r) {
  if (RW == 8) {
    const uint2 v = *reinterpret_cast<const uint2*>(p);
    r[0] = v.x; r[1] = v.y;
  } else if (RW == 6) {
    const unsigned short* q = reinterpret_cast<const unsigned short*>(p);
    r[0] = (uint32_t)q[0] | ((uint32_t)q[1] << 16); r[1] = q[2];
  } else if (RW == 4) {
    r[0] = *reinterpret_cast<const uint32_t*>(p); r[1] = 0;
  } else {
    r[0] = *reinterpret_cast<const unsigned short*>(p); r[1] = 0;
  }
}
// keep the bf16 halves of d whose y half is > 0 (positive non-zero bf16 <=> int16 > 0)
__device__ __forceinline__ uint32_t relu_mask(uint32_t d, uint32_t y) {
  const uint32_t lo = ((int)(short)(y & 0xffffu) > 0) ? 0x0000ffffu : 0u;
  const uint32_t hi = ((int)(short)(y >> 16) > 0) ? 0xffff0000u : 0u;
  return d & (lo | hi);
}

// Per-thread staging of one image group: items e = tid + i*kT (i < NI).
template <int MODE>
struct Loader {
  static constexpr int W = ModeInfo<MODE>::W, NI = ModeInfo<MODE>::NI;
  int im[NI];     // image within the group, -1: no item
  int soff[NI];   // source offset within an image (bytes for u8, elements otherwise)
  int dst[NI];    // LDS destination (elements)
  uint32_t fl[NI];  // U8S1: bit0 first word of a row, bit1 last word of a row
  uint32_t r[NI][W];

  __device__ __forceinline__ void init(const PipeSrc& s, int imgs) {
    const int total = imgs * s.per_img;
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int e = threadIdx.x + i * kT;
      im[i] = -1; soff[i] = 0; dst[i] = 0; fl[i] = 0;
#pragma unroll
      for (int k = 0; k < W; ++k) r[i][k] = 0;
      if (e >= total) continue;
      const int m = e / s.per_img, rem = e - m * s.per_img;
      im[i] = m;
      if constexpr (MODE == PM_U8S1) {
        const int wpr = s.SW >> 2;
        const int y = rem / wpr, w = rem - y * wpr;
        soff[i] = y * s.SW + 4 * w;
        dst[i] = m * s.IMG + (y + s.offy) * s.LWp + 4 * w + s.offx;
        fl[i] = (w == 0 ? 1u : 0u) | (w == wpr - 1 ? 2u : 0u);
      } else {
        const int runs = s.SC / s.RW;
        const int pix = rem / runs, run = rem - pix * runs;
        const int sy = pix / s.SW, sx = pix - sy * s.SW;
        soff[i] = pix * s.SC + run * s.RW;
        const int ty = (MODE == PM_UNPOOL ? 2 * sy : sy) * s.up + s.offy;
        const int tx = (MODE == PM_UNPOOL ? 2 * sx : sx) * s.up + s.offx;
        dst[i] = m * s.IMG + (ty * s.LWp + tx) * s.CL + run * s.RW;
      }
    }
  }

  // Issue the group's global loads (no waits here).
  __device__ __forceinline__ void load(const PipeSrc& s, int img0, int N) {
    const size_t img_src = (size_t)s.SH * s.SW * s.SC;
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      if (im[i] < 0) continue;
      const int n = img0 + im[i];
      if (n >= N) continue;
      if constexpr (MODE == PM_U8S1) {
        const int gim = s.idx ? s.idx[n] : n;
        const uint8_t* p = static_cast<const uint8_t*>(s.src) + (size_t)gim * img_src + soff[i];
        r[i][0] = *reinterpret_cast<const uint32_t*>(p);
        r[i][1] = (fl[i] & 2u) ? 0u : *reinterpret_cast<const uint32_t*>(p + 4);
      } else {
        const size_t g = (size_t)n * img_src + soff[i];
        ld_chan(static_cast<const bf16*>(s.src) + g, s.RW, r[i]);
        if constexpr (MODE == PM_RELU || MODE == PM_UNPOOL) ld_chan(static_cast<const bf16*>(s.aux_y) + g, s.RW, r[i] + 4);
        if constexpr (MODE == PM_UNPOOL) ld_arg(s.aux_arg + g, s.RW, r[i] + 8);
      }
    }
  }

  // Write the loaded group into LDS (valid images only).
  __device__ __forceinline__ void store(const PipeSrc& s, bf16* lds, int nimg) {
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      if (im[i] < 0 || im[i] >= nimg) continue;
      if constexpr (MODE == PM_U8S1) {
        uint32_t h0, h1, h2, h3;
        u8x4_bf16(r[i][0], h0, h1);
        u8x4_bf16(r[i][1], h2, h3);
        bf16* b = lds + dst[i];
        st8(b, h0, h1);
        st8(b + s.CS, mid(h0, h1), mid(h1, h2));
        st8(b + 2 * s.CS, h1, h2);
        st8(b + 3 * s.CS, mid(h1, h2), mid(h2, h3));
        if (fl[i] & 1u) {  // the quad left of the row: (halo zeros, first pixels)
          st8(b - 4 + s.CS, 0u, mid(0u, h0));
          st8(b - 4 + 2 * s.CS, 0u, h0);
          st8(b - 4 + 3 * s.CS, mid(0u, h0), mid(h0, h1));
        }
      } else if constexpr (MODE == PM_PLAIN) {
        st16(lds + dst[i], r[i]);
      } else if constexpr (MODE == PM_RELU) {
        uint32_t v[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) v[k] = relu_mask(r[i][k], r[i][4 + k]);
        st16(lds + dst[i], v);
      } else {  // PM_UNPOOL: dense write of the four window positions
        uint32_t d[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) d[k] = relu_mask(r[i][k], r[i][4 + k]);
        const int dxo = s.up * s.CL, dyo = s.up * s.LWp * s.CL;
#pragma unroll
        for (int pos = 0; pos < 4; ++pos) {
          uint32_t v[4];
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            const uint32_t a = r[i][8 + (k >> 1)] >> (16 * (k & 1));  // bytes of channels 2k, 2k+1
            const uint32_t lo = ((a & 0xffu) == (uint32_t)pos) ? 0x0000ffffu : 0u;
            const uint32_t hi = (((a >> 8) & 0xffu) == (uint32_t)pos) ? 0xffff0000u : 0u;
            v[k] = d[k] & (lo | hi);
          }
          st16(lds + dst[i] + (pos & 1) * dxo + (pos >> 1) * dyo, v);
        }
      }
    }
  }
};

// XL_S1 fragment read: 8 consecutive tile elements starting at flat index e.
__device__ __forceinline__ bf16x8 read_s1(const bf16* xs, int CS, int e) {
  const int c = e & 3;
  const bf16* a = xs + c * CS + (e - c);
  const bf16x4 lo = *reinterpret_cast<const bf16x4*>(a);
  const bf16x4 hi = *reinterpret_cast<const bf16x4*>(a + 4);
  return __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
}
// XL_S1 transpose read (4 consecutive tile elements per lane)
__device__ __forceinline__ bf16x4 tr4_s1(const bf16* xs, int CS, int e) {
  const int c = e & 3;
  return tr4(xs + c * CS + (e - c));
}

// Output-pixel (row) -> tile offset of its first tap.  Pool: rows ordered by
// 2x2 window so a 16-row tile holds four whole windows.
__device__ void row_table(int* tab, int rows, bool pool, int OW, int cs, int ty0, int tx0, int LWp, int CL,
                          bool pair = false) {
  const int PW = OW >> 1;
  for (int r = threadIdx.x; r < rows; r += blockDim.x) {
    int oy, ox;
    if (pair && pool) {  // row = (window, top/bottom pixel pair)
      const int win = r >> 1;
      const int ph = win / PW, pw = win - ph * PW;
      oy = 2 * ph + (r & 1);
      ox = 2 * pw;
    } else if (pair) {   // row = horizontal pixel pair
      const int oy_ = r / PW;
      oy = oy_;
      ox = 2 * (r - oy_ * PW);
    } else if (pool) {
      const int win = r >> 2, pos = r & 3;
      const int ph = win / PW, pw = win - ph * PW;
      oy = 2 * ph + (pos >> 1);
      ox = 2 * pw + (pos & 1);
    } else {
      oy = r / OW;
      ox = r - oy * OW;
    }
    tab[r] = ((oy * cs + ty0) * LWp + ox * cs + tx0) * CL;
  }
}

__device__ __forceinline__ void zero_lds(bf16* p, int n) {  // n multiple of 8, p 16-byte aligned
  const uint4 z = make_uint4(0, 0, 0, 0);
  for (int i = threadIdx.x * 8; i < n; i += blockDim.x * 8) *reinterpret_cast<uint4*>(p + i) = z;
}

// LDS -> global copy of `bytes` bytes with the widest access both sides allow.
__device__ __forceinline__ void copy_out(char* g, const char* l, int bytes, int align) {
  if (align >= 16) {
    for (int i = threadIdx.x * 16; i < bytes; i += blockDim.x * 16)
      *reinterpret_cast<uint4*>(g + i) = *reinterpret_cast<const uint4*>(l + i);
  } else if (align >= 8) {
    for (int i = threadIdx.x * 8; i < bytes; i += blockDim.x * 8)
      *reinterpret_cast<uint2*>(g + i) = *reinterpret_cast<const uint2*>(l + i);
  } else if (align >= 4) {
    for (int i = threadIdx.x * 4; i < bytes; i += blockDim.x * 4)
      *reinterpret_cast<uint32_t*>(g + i) = *reinterpret_cast<const uint32_t*>(l + i);
  } else if (align >= 2) {
    for (int i = threadIdx.x * 2; i < bytes; i += blockDim.x * 2)
      *reinterpret_cast<unsigned short*>(g + i) = *reinterpret_cast<const unsigned short*>(l + i);
  } else {
    for (int i = threadIdx.x; i < bytes; i += blockDim.x) g[i] = l[i];
  }
}

__host__ __device__ constexpr int pow2_align(int bytes) {
  return (bytes & 15) == 0 ? 16 : ((bytes & 7) == 0 ? 8 : ((bytes & 3) == 0 ? 4 : ((bytes & 1) == 0 ? 2 : 1)));
}

struct FwdLayout {  // LDS carve-up shared by the planner and the kernel
  int xs_elems, ws_off, bias_off, ktab_off, ptab_off, outs_off, args_off, total;
};
__host__ __device__ inline FwdLayout fwd_layout(const ConvPipeParams& p) {
  FwdLayout L;
  const int ntiles = (p.Cout + 15) / 16;
  const bool pool = p.epi == FE_POOL;
  const int rows_img = (pool ? (p.OH / 2) * (p.OW / 2) * 4 : p.OH * p.OW) / (p.pair ? 2 : 1);
  const int out_img = (pool ? (p.OH / 2) * (p.OW / 2) : p.OH * p.OW) * p.Cout;
  L.xs_elems = p.layout == XL_S1 ? 4 * p.in.CS : ((p.imgs * p.in.IMG + 8 + 7) & ~7);
  int o = align16(L.xs_elems * 2);
  L.ws_off = o; o += align16(ntiles * 16 * (p.kpad + 8) * 2);
  L.bias_off = o; o += ntiles * 16 * 4;
  L.ktab_off = o; o += align16(p.nchunks * 4 * 4);
  L.ptab_off = o; o += align16(rows_img * 4);
  L.outs_off = o; o += align16(p.imgs * out_img * 2);
  L.args_off = o; o += pool ? align16(p.imgs * out_img) : 0;
  L.total = o;
  return L;
}

// DPP row_ror:8 — lane i <- lane i^8 within each 16-lane row
__device__ __forceinline__ float swap8(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x128, 0xf, 0xf, false));
}

template <int MODE, int EPI, int ACT, bool PAIR = false>
__global__ void __launch_bounds__(kT) conv_pipe_fwd_kernel(ConvPipeParams p) {
  constexpr int MT = 4;
  constexpr bool S1 = MODE == PM_U8S1;
  constexpr bool pool = EPI == FE_POOL;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const PipeSrc& s = p.in;
  const FwdLayout L = fwd_layout(p);
  bf16* xs = reinterpret_cast<bf16*>(smem);
  bf16* ws = reinterpret_cast<bf16*>(smem + L.ws_off);
  float* bias_s = reinterpret_cast<float*>(smem + L.bias_off);
  int* ktab = reinterpret_cast<int*>(smem + L.ktab_off);
  int* ptab = reinterpret_cast<int*>(smem + L.ptab_off);
  bf16* outs = reinterpret_cast<bf16*>(smem + L.outs_off);
  uint8_t* args = reinterpret_cast<uint8_t*>(smem + L.args_off);

  const int tid = threadIdx.x;
  const int ntiles = cdiv(p.Cout, 16);
  const int wld = p.kpad + 8;
  const int PH = p.OH >> 1, PW = p.OW >> 1;
  const int rows_img = (pool ? PH * PW * 4 : p.OH * p.OW) / (PAIR ? 2 : 1);
  const int out_img = (pool ? PH * PW : p.OH * p.OW) * p.Cout;
  const int KK = p.KS * p.KS;

  // ---- one-time setup ----
  zero_lds(xs, L.xs_elems);
  {
    const bf16* wpk = static_cast<const bf16*>(p.wpk);
    const int vpr = p.kpad >> 3, nv = ntiles * 16 * vpr;
    for (int v = tid; v < nv; v += kT) {
      const int r = v / vpr, c = (v - r * vpr) * 8;
      store8(ws + r * wld + c, load8(wpk + (size_t)r * p.kpad + c));
    }
  }
  for (int n = tid; n < ntiles * 16; n += kT) {
    const int c = PAIR ? (n & 7) : n;
    bias_s[n] = (EPI != FE_PLAIN && c < p.Cout) ? p.bias[c] : 0.f;
  }
  for (int gi = tid; gi < p.nchunks * 4; gi += kT) {
    int off = 0;
    if (S1) {
      if (gi < p.KS) off = gi * s.LWp;
    } else {
      const int CG = s.CL >> 3;
      const int kp = gi / CG, cg = gi - kp * CG;
      if (kp < KK) {
        const int kh = kp / p.KS, kw = kp - kh * p.KS;
        off = (kh * s.LWp + kw) * s.CL + cg * 8;
      }
    }
    ktab[gi] = off;  // padding groups point at tap 0 (zero weights)
  }
  row_table(ptab, rows_img, pool, p.OW, p.cs, p.ty0, p.tx0, s.LWp, S1 ? 1 : s.CL, PAIR);

  Loader<MODE> ld;
  ld.init(s, p.imgs);
  int grp = blockIdx.x;
  if (grp < p.ngroups) ld.load(s, grp * p.imgs, p.N);

  const int lane = tid & 63, wave = tid >> 6;
  const int r16 = lane & 15, g = lane >> 4;
  const Div drpi(rows_img);

  for (; grp < p.ngroups; grp += gridDim.x) {
    const int img0 = grp * p.imgs;
    const int nimg = min(p.imgs, p.N - img0);
    __syncthreads();  // tiles free: previous compute and copy-out done (and setup, first time)
    ld.store(s, xs, nimg);
    __syncthreads();
    if (grp + (int)gridDim.x < p.ngroups) ld.load(s, (grp + gridDim.x) * p.imgs, p.N);

    const int M = nimg * rows_img;
    const int mtiles = cdiv(M, 16), mgroups = cdiv(mtiles, MT);
    for (int item = wave; item < ntiles * mgroups; item += kT / 64) {
      const int nt = item / mgroups, mg = item - nt * mgroups;
      int base[MT];
#pragma unroll
      for (int t = 0; t < MT; ++t) {
        const int r = (mg * MT + t) * 16 + r16;
        const int img = drpi.div(r);
        int b = r < M ? img * s.IMG + ptab[r - img * rows_img] : 0;  // past M: finite, discarded
        if (S1) {  // K-group offsets are multiples of 4: the copy depends on the row only
          const int c = b & 3;
          b = c * s.CS + b - c;
        }
        base[t] = b;
      }
      f32x4 acc[MT];
#pragma unroll
      for (int t = 0; t < MT; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
      const bf16* wrow = ws + (nt * 16 + r16) * wld + 8 * g;
      for (int q = 0; q < p.nchunks; ++q) {
        const bf16x8 b = load8(wrow + q * 32);
        const int ko = ktab[q * 4 + g];
#pragma unroll
        for (int t = 0; t < MT; ++t) {
          bf16x8 a;
          if (S1) {
            const bf16* ap = xs + base[t] + ko;
            const bf16x4 lo = *reinterpret_cast<const bf16x4*>(ap);
            const bf16x4 hi = *reinterpret_cast<const bf16x4*>(ap + 4);
            a = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
          } else {
            a = load8(xs + base[t] + ko);
          }
          acc[t] = mma(acc[t], a, b);
        }
      }
      // epilogue into the LDS output tile: lane holds rows 4g..4g+3, column n
      if constexpr (PAIR) {
        // column r16 = channel (r16 & 7) of the left (r16 < 8) or right pixel
        const int c = r16 & 7;
        const float bv = bias_s[r16];
#pragma unroll
        for (int t = 0; t < MT; ++t) {
          const int rb = (mg * MT + t) * 16 + 4 * g;
          float v[4];
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const float x = acc[t][i] + bv;
            v[i] = ACT == ACT_RELU ? fmaxf(x, 0.f) : (ACT == ACT_TANH ? tanhf(x) : x);
          }
          if (pool) {
            // rows (4g, 4g+1) and (4g+2, 4g+3): top/bottom pairs of two windows
#pragma unroll
            for (int w2 = 0; w2 < 2; ++w2) {
              const float lt = v[2 * w2], lb = v[2 * w2 + 1];
              const float rt = swap8(lt), rbv = swap8(lb);
              // first max in window order TL, TR, BL, BR (cnn-style argmax)
              float best = lt;
              int arg = 0;
              if (rt > best) { best = rt; arg = 1; }
              if (lb > best) { best = lb; arg = 2; }
              if (rbv > best) { best = rbv; arg = 3; }
              if (r16 < 8 && c < p.Cout && rb + 2 * w2 < M) {
                const int o = ((rb >> 1) + w2) * p.Cout + c;
                outs[o] = (bf16)best;
                args[o] = (uint8_t)arg;
              }
            }
          } else if (c < p.Cout) {
#pragma unroll
            for (int i = 0; i < 4; ++i)
              if (rb + i < M) outs[(2 * (rb + i) + (r16 >> 3)) * p.Cout + c] = (bf16)v[i];
          }
        }
        continue;
      }
      const int n = nt * 16 + r16;
      if (n >= p.Cout) continue;
      const float bv = bias_s[n];
#pragma unroll
      for (int t = 0; t < MT; ++t) {
        const int rb = (mg * MT + t) * 16 + 4 * g;
        if (rb >= M) continue;
        float v[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float x = acc[t][i] + bv;
          v[i] = ACT == ACT_RELU ? fmaxf(x, 0.f) : (ACT == ACT_TANH ? tanhf(x) : x);
        }
        if (pool) {
          float best = v[0];
          int arg = 0;
#pragma unroll
          for (int i = 1; i < 4; ++i) {
            const bool gt = v[i] > best;
            best = gt ? v[i] : best;
            arg = gt ? i : arg;
          }
          const int o = (rb >> 2) * p.Cout + n;
          outs[o] = (bf16)best;
          args[o] = (uint8_t)arg;
        } else {
#pragma unroll
          for (int i = 0; i < 4; ++i)
            if (rb + i < M) outs[(rb + i) * p.Cout + n] = (bf16)v[i];
        }
      }
    }
    __syncthreads();
    char* gout = static_cast<char*>(p.out) + (size_t)img0 * out_img * 2;
    copy_out(gout, reinterpret_cast<const char*>(outs), nimg * out_img * 2, pow2_align(out_img * 2));
    if (pool) {
      char* garg = reinterpret_cast<char*>(p.out_arg) + (size_t)img0 * out_img;
      copy_out(garg, reinterpret_cast<const char*>(args), nimg * out_img, pow2_align(out_img));
    }
  }
}

// ---------------------------------------------------------------------------
// Weight gradient.

struct DwLayout {
  int xs_elems, dys_off, pixbase_off, ptab_off, stage, red, total;
};
__host__ __device__ inline int dw_ntw(int mtw, int ncol_tiles) {
  if (mtw <= 1)
    return ncol_tiles <= 2 ? 2 : ncol_tiles <= 3 ? 3 : ncol_tiles <= 4 ? 4 : ncol_tiles <= 8 ? 8 : ncol_tiles <= 13 ? 13 : 16;
  return mtw <= 2 ? 8 : (mtw <= 4 ? 4 : 2);
}
__host__ __device__ inline DwLayout dw_layout(const ConvDwPipeParams& p) {
  DwLayout L;
  L.xs_elems = p.layout == XL_S1 ? 4 * p.x.CS : ((p.imgs * p.x.IMG + 8 + 7) & ~7);
  int o = align16(L.xs_elems * 2);
  L.dys_off = o; o += align16((p.ppad * p.drow + 8) * 2);  // +8: the Cout<=8 over-read of the last row
  L.pixbase_off = o; o += align16(p.ppad * 4);
  L.ptab_off = o; o += align16(p.OH * p.OW * 4);
  L.stage = o;
  const int ntw = dw_ntw(p.cout_pad / 16, p.kbias / 16);
  L.red = p.cout_pad * (ntw * 16 + 1) * 4;
  L.total = L.stage > L.red ? L.stage : L.red;
  return L;
}

template <int XM, int DM, int MTW, int NTW>
__global__ void __launch_bounds__(kT) conv_dw_pipe_kernel(ConvDwPipeParams p) {
  constexpr bool S1 = XM == PM_U8S1;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const DwLayout L = dw_layout(p);
  bf16* xs = reinterpret_cast<bf16*>(smem);
  bf16* dys = reinterpret_cast<bf16*>(smem + L.dys_off);
  int* pixbase = reinterpret_cast<int*>(smem + L.pixbase_off);
  int* ptab = reinterpret_cast<int*>(smem + L.ptab_off);
  float* red = reinterpret_cast<float*>(smem);  // reused after the main loop

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int r16 = lane & 15, g = lane >> 4;
  const int q = r16 >> 2, pp = r16 & 3;  // transpose-read address role
  const int KK = p.KS * p.KS;
  const int opix = p.OH * p.OW;
  const int drow = p.drow;
  const PipeSrc& sx = p.x;
  const PipeSrc& sd = p.dy;

  int koff[NTW];
#pragma unroll
  for (int t = 0; t < NTW; ++t) {
    const int c4 = (blockIdx.y * NTW + t) * 16 + 4 * pp;  // first of this lane's 4 columns
    koff[t] = 0;
    if (S1) {
      const int kh = c4 >> 3;
      if (kh < p.KS) koff[t] = kh * sx.LWp + (c4 & 7);
    } else {
      const int kp = c4 / sx.CL, c0 = c4 - kp * sx.CL;
      if (kp < KK) {
        const int kh = kp / p.KS, kw = kp - kh * p.KS;
        koff[t] = (kh * sx.LWp + kw) * sx.CL + c0;
      }
    }
  }

  zero_lds(xs, L.xs_elems);
  zero_lds(dys, p.ppad * drow + 8);
  row_table(ptab, opix, false, p.OW, p.cs, p.ty0, p.tx0, sx.LWp, S1 ? 1 : sx.CL);
  Loader<XM> lx;
  Loader<DM> ld;
  lx.init(sx, p.imgs);
  ld.init(sd, p.imgs);
  int grp = blockIdx.x;
  if (grp < p.ngroups) {
    lx.load(sx, grp * p.imgs, p.N);
    ld.load(sd, grp * p.imgs, p.N);
  }
  __syncthreads();  // ptab
  {
    // stage-invariant pixel -> tile base; rows past the last image of a tail
    // group read stale (finite) pixels against zeroed dY rows
    const int full = p.imgs * opix;
    for (int pix = tid; pix < p.ppad; pix += kT) {
      const int img = pix / opix;
      pixbase[pix] = pix < full ? img * sx.IMG + ptab[pix - img * opix] : 0;
    }
  }

  f32x4 acc[MTW][NTW];
  float bsum[MTW];
#pragma unroll
  for (int m = 0; m < MTW; ++m) {
    bsum[m] = 0.f;
#pragma unroll
    for (int t = 0; t < NTW; ++t) acc[m][t] = f32x4{0.f, 0.f, 0.f, 0.f};
  }

  for (; grp < p.ngroups; grp += gridDim.x) {
    const int img0 = grp * p.imgs;
    const int nimg = min(p.imgs, p.N - img0);
    const int npix = nimg * opix;
    __syncthreads();  // previous group consumed
    lx.store(sx, xs, nimg);
    ld.store(sd, dys, nimg);
    if (nimg < p.imgs) zero_lds(dys + npix * drow, (p.ppad - npix) * drow);  // stale rows of a tail group
    __syncthreads();
    if (grp + (int)gridDim.x < p.ngroups) {
      lx.load(sx, (grp + gridDim.x) * p.imgs, p.N);
      ld.load(sd, (grp + gridDim.x) * p.imgs, p.N);
    }
    const int nq = cdiv(npix, 32);
    for (int qc = wave; qc < nq; qc += kT / 64) {
      // fragment k -> pixel: lane group g reads rows 4g..4g+3 (and +16)
      const int pix1 = qc * 32 + 4 * g + q, pix2 = pix1 + 16;
      const int pb1 = pixbase[pix1], pb2 = pixbase[pix2];
      bf16x8 a[MTW];
#pragma unroll
      for (int m = 0; m < MTW; ++m) {
        const bf16x4 lo = tr4(dys + pix1 * drow + m * 16 + 4 * pp);
        const bf16x4 hi = tr4(dys + pix2 * drow + m * 16 + 4 * pp);
        a[m] = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
#pragma unroll
        for (int j = 0; j < 8; ++j) bsum[m] += (float)a[m][j];
      }
#pragma unroll
      for (int t = 0; t < NTW; ++t) {
        const bf16x4 lo = S1 ? tr4_s1(xs, sx.CS, pb1 + koff[t]) : tr4(xs + pb1 + koff[t]);
        const bf16x4 hi = S1 ? tr4_s1(xs, sx.CS, pb2 + koff[t]) : tr4(xs + pb2 + koff[t]);
        const bf16x8 b = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
#pragma unroll
        for (int m = 0; m < MTW; ++m) acc[m][t] = mma(acc[m][t], a[m], b);
      }
    }
  }
  // bias: lanes r16 hold channel m*16+r16; sum the 4 lane groups
#pragma unroll
  for (int m = 0; m < MTW; ++m) {
    bsum[m] += __shfl_xor(bsum[m], 16);
    bsum[m] += __shfl_xor(bsum[m], 32);
  }
  // combine the waves in a fixed order: red[MTW*16 rows][NTW*16 + 1 cols]
  const int rcols = NTW * 16 + 1;
  for (int w = 0; w < kT / 64; ++w) {
    __syncthreads();
    if (wave == w) {
#pragma unroll
      for (int m = 0; m < MTW; ++m) {
#pragma unroll
        for (int t = 0; t < NTW; ++t)
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            float* d = red + (m * 16 + 4 * g + i) * rcols + t * 16 + r16;
            *d = (w == 0 ? 0.f : *d) + acc[m][t][i];
          }
        if (g == 0) {
          float* d = red + (m * 16 + r16) * rcols + NTW * 16;
          *d = (w == 0 ? 0.f : *d) + bsum[m];
        }
      }
    }
  }
  __syncthreads();
  for (int e = tid; e < p.cout_pad * rcols; e += kT) {
    const int row = e / rcols, c = e - row * rcols;
    float* srow = p.slab + ((size_t)blockIdx.x * p.cout_pad + row) * p.ncols_pad;
    if (c < NTW * 16) {
      const int col = blockIdx.y * NTW * 16 + c;
      if (col < p.kbias) srow[col] = red[row * rcols + c];
    } else if (blockIdx.y == 0) {
      srow[p.kbias] = red[row * rcols + c];
    }
  }
}

// Level 1: part[xc][v] = sum of slabs x in chunk xc (v over the whole slab).
__global__ void __launch_bounds__(256) dw_slab_sum_kernel(const float* slab, int nx, int nv, int xs_per,
                                                          float* part) {
  __shared__ float red[4][65];
  const int tv = threadIdx.x & 63, tx = threadIdx.x >> 6;
  const int v = blockIdx.x * 64 + tv;
  const int x0 = blockIdx.y * xs_per, x1 = min(nx, x0 + xs_per);
  float acc = 0.f;
  if (v < nv)
    for (int x = x0 + tx; x < x1; x += 4) acc += slab[(size_t)x * nv + v];
  red[tx][tv] = acc;
  __syncthreads();
  if (tx == 0 && v < nv) part[(size_t)blockIdx.y * nv + v] = (red[0][tv] + red[1][tv]) + (red[2][tv] + red[3][tv]);
}

// Level 2: canonical gradient from the chunk partials.
__global__ void __launch_bounds__(256) dw_slab_final_kernel(const float* part, int nxc, int nv, int ncols_pad,
                                                            int kbias, int Cout, int Cin, int KS, int layout,
                                                            int CL, float* gw, float* gb) {
  const int KK = KS * KS;
  const int nW = Cout * Cin * KK;
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= nW + Cout) return;
  int row, col;
  if (j < nW) {
    row = j / (Cin * KK);
    const int rem = j - row * Cin * KK;
    const int ci = rem / KK, kp = rem - ci * KK;
    const int kh = kp / KS, kw = kp - kh * KS;
    col = layout == XL_S1 ? kh * 8 + kw : kp * CL + ci;
  } else {
    row = j - nW;
    col = kbias;
  }
  const int v = row * ncols_pad + col;
  float s = 0.f;
  for (int xc = 0; xc < nxc; ++xc) s += part[(size_t)xc * nv + v];
  if (j < nW) gw[j] = s;
  else gb[row] = s;
}

inline int r8h(int x) { return (x + 7) & ~7; }
inline int r16h(int x) { return (x + 15) & ~15; }
inline int r32h(int x) { return (x + 31) & ~31; }

constexpr int kCUs = 256;
constexpr size_t kLdsPerCU = 160 * 1024;

// Destination geometry of a staged source; returns false if unsupported.
bool plan_src(PipeSrc& s, int layout, int CLdst, int LH, int LWp, int IMGextra) {
  (void)LH; (void)IMGextra;
  if (s.mode == PM_U8S1) {
    if (s.SC != 1 || (s.SW & 3) != 0 || s.up != 1 || (s.offx & 3) != 0 || s.offx < 4) return false;
    s.RW = 4;
    s.per_img = s.SH * (s.SW >> 2);
    s.CL = 1;
    (void)layout;
    return true;
  }
  if (s.SC <= 0 || (s.SC & 1)) return false;
  s.RW = (s.SC & 7) == 0 ? 8 : s.SC;
  if (s.RW > 8) return false;
  s.per_img = s.SH * s.SW * (s.SC / s.RW);
  s.CL = CLdst;
  s.LWp = LWp;
  return true;
}

int wgs_per_cu(size_t lds, int cap) {
  int w = (int)(kLdsPerCU / (lds + 512));
  return w < 1 ? 1 : (w > cap ? cap : w);
}

}  // namespace

bool conv_pipe_plan(ConvPipeParams& p) {
  PipeSrc& s = p.in;
  const bool s1 = s.mode == PM_U8S1;
  if (s1 && (p.KS > 8 || p.Cin != 1)) return false;
  if (!s1 && s.SC != p.Cin) return false;
  if (p.Cout > 128) return false;
  p.layout = s1 ? XL_S1 : XL_C8;
  p.pair = s1 && p.Cout <= 8 && p.KS <= 7 && p.cs == 1 && (p.OW & 1) == 0 &&
           (p.epi == FE_POOL || (p.epi == FE_ACT && (p.act == ACT_RELU || p.act == ACT_NONE)));
  if (s1) {  // align the source columns to 4 (shift the conv origin accordingly)
    const int ox = s.offx < 4 ? 4 : (s.offx + 3) & ~3;
    p.tx0 += ox - s.offx;
    s.offx = ox;
  }
  const int grid_h = (s.mode == PM_UNPOOL ? 2 * s.SH : s.SH);
  const int grid_w = (s.mode == PM_UNPOOL ? 2 * s.SW : s.SW);
  const int LH = std::max(p.ty0 + (p.OH - 1) * p.cs + p.KS, s.offy + (grid_h - 1) * s.up + 1);
  int LWp;
  if (s1) LWp = (std::max(p.tx0 + (p.OW - 1) * p.cs + 8, s.offx + grid_w + 4) + 3) & ~3;
  else LWp = std::max(p.tx0 + (p.OW - 1) * p.cs + p.KS, s.offx + (grid_w - 1) * s.up + 1);
  const int CL = s1 ? 1 : r8h(p.Cin);
  if (!plan_src(s, p.layout, CL, LH, LWp, 0)) return false;
  s.LWp = LWp;
  p.LH = LH;
  s.IMG = LH * LWp * CL;
  const int KK = p.KS * p.KS;
  p.nchunks = s1 ? (p.KS + 3) / 4 : (KK * (CL / 8) + 3) / 4;
  p.kpad = p.nchunks * 32;
  // images per group: prefetch items within the thread budget, LDS ~64 KB
  const int ni = mode_ni(s.mode);
  if (s.per_img > ni * kT) return false;
  int imgs = std::max(1, std::min(16, ni * kT / std::max(1, s.per_img)));
  for (; imgs >= 1; --imgs) {
    p.imgs = imgs;
    if (s1) s.CS = r8h(imgs * s.IMG + 8);
    if ((size_t)fwd_layout(p).total <= 64 * 1024 || imgs == 1) break;
  }
  if (imgs < 1) return false;
  const FwdLayout L = fwd_layout(p);
  if ((size_t)L.total > kLdsPerCU) return false;
  p.lds = (size_t)L.total;
  p.ngroups = cdiv(p.N, p.imgs);
  p.grid = std::min(p.ngroups, kCUs * wgs_per_cu(p.lds, 4));
  return true;
}

void conv_pipe_forward(const ConvPipeParams& pin, hipStream_t st) {
  ConvPipeParams p = pin;
  p.ngroups = cdiv(p.N, p.imgs);
  p.grid = std::min(p.ngroups, kCUs * wgs_per_cu(p.lds, 4));
  if (p.grid <= 0) return;
  const dim3 grid((unsigned)p.grid), block(kT);
  auto go = [&](auto kern) { hipLaunchKernelGGL(kern, grid, block, p.lds, st, p); };
#define MCC_PIPE_EPI(MODE)                                                                      \
  if (p.epi == FE_POOL) go(conv_pipe_fwd_kernel<MODE, FE_POOL, ACT_RELU>);                      \
  else if (p.epi == FE_PLAIN) go(conv_pipe_fwd_kernel<MODE, FE_PLAIN, ACT_NONE>);               \
  else if (p.act == ACT_RELU) go(conv_pipe_fwd_kernel<MODE, FE_ACT, ACT_RELU>);                 \
  else if (p.act == ACT_TANH) go(conv_pipe_fwd_kernel<MODE, FE_ACT, ACT_TANH>);                 \
  else go(conv_pipe_fwd_kernel<MODE, FE_ACT, ACT_NONE>);
  if (p.pair) {
    if (p.epi == FE_POOL) go(conv_pipe_fwd_kernel<PM_U8S1, FE_POOL, ACT_RELU, true>);
    else if (p.act == ACT_RELU) go(conv_pipe_fwd_kernel<PM_U8S1, FE_ACT, ACT_RELU, true>);
    else go(conv_pipe_fwd_kernel<PM_U8S1, FE_ACT, ACT_NONE, true>);
    return;
  }
  switch (p.in.mode) {
    case PM_U8S1: MCC_PIPE_EPI(PM_U8S1) break;
    case PM_PLAIN: MCC_PIPE_EPI(PM_PLAIN) break;
    case PM_RELU: MCC_PIPE_EPI(PM_RELU) break;
    default: MCC_PIPE_EPI(PM_UNPOOL) break;
  }
#undef MCC_PIPE_EPI
}

bool conv_dw_pipe_plan(ConvDwPipeParams& p) {
  PipeSrc& x = p.x;
  PipeSrc& d = p.dy;
  const bool s1 = x.mode == PM_U8S1;
  if (s1 && (p.KS > 8 || p.Cin != 1)) return false;
  if (!s1 && (x.mode != PM_PLAIN || x.SC != p.Cin)) return false;
  if (d.mode == PM_U8S1 || d.SC != p.Cout || p.Cout > 128) return false;
  p.layout = s1 ? XL_S1 : XL_C8;
  if (s1) {
    const int ox = x.offx < 4 ? 4 : (x.offx + 3) & ~3;
    p.tx0 += ox - x.offx;
    x.offx = ox;
  }
  const int LH = std::max(p.ty0 + (p.OH - 1) * p.cs + p.KS, x.offy + (x.SH - 1) * x.up + 1);
  int LWp;
  if (s1) LWp = (std::max(p.tx0 + (p.OW - 1) * p.cs + 8, x.offx + x.SW + 4) + 3) & ~3;
  else LWp = std::max(p.tx0 + (p.OW - 1) * p.cs + p.KS, x.offx + (x.SW - 1) * x.up + 1);
  const int CL = s1 ? 1 : r8h(p.Cin);  // C8 staging writes whole 16-byte pixels
  if (!plan_src(x, p.layout, CL, LH, LWp, 0)) return false;
  x.LWp = LWp;
  x.IMG = LH * LWp * CL;
  p.LH = LH;
  p.cout_pad = r16h(p.Cout);
  // Cout <= 8: 16-byte dY rows; the A fragment's channels 8..15 then read the
  // next row (rows 8..15 of the product are garbage and never reduced)
  p.drow = p.Cout <= 8 ? 8 : conv_dw_tr_drow(p.cout_pad);
  d.up = 1; d.offy = 0; d.offx = 0;
  if (!plan_src(d, XL_C8, p.drow, p.OH, p.OW, 0)) return false;
  d.LWp = p.OW;
  d.IMG = p.OH * p.OW * p.drow;
  const int KK = p.KS * p.KS;
  p.kbias = s1 ? r16h(p.KS * 8) : r16h(KK * CL);
  p.ncols_pad = p.kbias + 16;
  const int nix = mode_ni(x.mode) * kT / std::max(1, x.per_img);
  const int nid = mode_ni(d.mode) * kT / std::max(1, d.per_img);
  int imgs = std::max(1, std::min(16, std::min(nix, nid)));
  for (; imgs >= 1; --imgs) {
    p.imgs = imgs;
    p.ppad = r32h(imgs * p.OH * p.OW);
    if (s1) x.CS = r8h(imgs * x.IMG + 8);
    if ((size_t)dw_layout(p).total <= 64 * 1024 || imgs == 1) break;
  }
  if (nix < 1 || nid < 1) return false;
  const DwLayout L = dw_layout(p);
  if ((size_t)L.total > kLdsPerCU) return false;
  p.lds = (size_t)L.total;
  p.ngroups = cdiv(p.N, p.imgs);
  p.grid = std::min(p.ngroups, kCUs * wgs_per_cu(p.lds, 2));
  return true;
}

void conv_dw_pipe(const ConvDwPipeParams& pin, hipStream_t st) {
  ConvDwPipeParams p = pin;
  p.ngroups = cdiv(p.N, p.imgs);
  p.grid = std::min(p.ngroups, std::min(pin.grid, kCUs * wgs_per_cu(p.lds, 2)));
  if (p.grid <= 0) return;
  const int mtw = p.cout_pad / 16;
  const int ncol_tiles = p.kbias / 16;
  const int ntw = dw_ntw(mtw, ncol_tiles);
  const dim3 grid((unsigned)p.grid, (unsigned)cdiv(ncol_tiles, ntw)), block(kT);
  auto go = [&](auto kern) { hipLaunchKernelGGL(kern, grid, block, p.lds, st, p); };
#define MCC_DW_TILES(XM, DM)                                     \
  if (mtw <= 1) {                                                \
    if (ntw == 2) go(conv_dw_pipe_kernel<XM, DM, 1, 2>);         \
    else if (ntw == 3) go(conv_dw_pipe_kernel<XM, DM, 1, 3>);    \
    else if (ntw == 4) go(conv_dw_pipe_kernel<XM, DM, 1, 4>);    \
    else if (ntw == 8) go(conv_dw_pipe_kernel<XM, DM, 1, 8>);    \
    else if (ntw == 13) go(conv_dw_pipe_kernel<XM, DM, 1, 13>);  \
    else go(conv_dw_pipe_kernel<XM, DM, 1, 16>);                 \
  } else if (mtw <= 2) go(conv_dw_pipe_kernel<XM, DM, 2, 8>);   \
  else if (mtw <= 4) go(conv_dw_pipe_kernel<XM, DM, 4, 4>);     \
  else go(conv_dw_pipe_kernel<XM, DM, 8, 2>);
#define MCC_DW_DM(XM)                                            \
  if (p.dy.mode == PM_UNPOOL) { MCC_DW_TILES(XM, PM_UNPOOL) }    \
  else if (p.dy.mode == PM_RELU) { MCC_DW_TILES(XM, PM_RELU) }   \
  else { MCC_DW_TILES(XM, PM_PLAIN) }
  if (p.x.mode == PM_U8S1) { MCC_DW_DM(PM_U8S1) }
  else { MCC_DW_DM(PM_PLAIN) }
#undef MCC_DW_DM
#undef MCC_DW_TILES
}

void conv_dw_pipe_reduce(const ConvDwPipeParams& pin, float* gw, float* gb, hipStream_t st) {
  ConvDwPipeParams p = pin;
  const int ngroups = cdiv(p.N, p.imgs);
  const int nx = std::min(ngroups, std::min(pin.grid, kCUs * wgs_per_cu(p.lds, 2)));
  if (nx <= 0) return;
  const int nv = p.cout_pad * p.ncols_pad;
  const int xs_per = 16;
  const int nxc = cdiv(nx, xs_per);
  float* part = p.slab + (size_t)pin.grid * nv;  // after the slabs (scratch sized by the planner's grid)
  hipLaunchKernelGGL(dw_slab_sum_kernel, dim3((unsigned)cdiv(nv, 64), (unsigned)nxc), dim3(256), 0, st, p.slab, nx,
                     nv, xs_per, part);
  const int nout = p.Cout * p.Cin * p.KS * p.KS + p.Cout;
  hipLaunchKernelGGL(dw_slab_final_kernel, dim3((unsigned)cdiv(nout, 256)), dim3(256), 0, st, part, nxc, nv,
                     p.ncols_pad, p.kbias, p.Cout, p.Cin, p.KS, p.layout, p.x.CL, gw, gb);
}

}  // namespace gpu
}  // namespace mcc
