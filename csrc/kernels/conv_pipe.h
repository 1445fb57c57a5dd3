// Device/host helpers shared by the pipelined conv kernels (conv_pipe_*.hip).
// See conv_pipe_fwd.hip for the design notes.
#pragma once

#include "mcc/ab.h"
#include <cstdlib>

#include <algorithm>

#include "kernels.h"
#include "mfma.h"

// Device-side bounds checks, compiled in with
// `make checked` (-DMCC_DEVICE_CHECKS).  A failed check prints and the
// kernel carries on: it never traps, so a bad index is reported without
// faulting the GPU.  Compiles to nothing in the default build.
#ifdef MCC_DEVICE_CHECKS
#define MCC_DCHECK(cond)                                                                         \
  do {                                                                                           \
    if (!(cond)) printf("MCC_DCHECK failed %s:%d: %s (block %d thread %d)\n", __FILE__, __LINE__, \
                        #cond, (int)blockIdx.x, (int)threadIdx.x);                               \
  } while (0)
#else
#define MCC_DCHECK(cond) \
  do {                   \
  } while (0)
#endif

namespace mcc {
namespace gpu {
namespace {


constexpr int kT = 256;  // default threads per workgroup (4 waves); kernels take NT
enum { FE_POOL = 0, FE_ACT = 1, FE_PLAIN = 2 };

typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));

template <int MODE> struct ModeInfo;
template <> struct ModeInfo<PM_U8S1> { static constexpr int W = 2, NI = 4; };
template <> struct ModeInfo<PM_PLAIN> { static constexpr int W = 4, NI = 8; };
template <> struct ModeInfo<PM_RELU> { static constexpr int W = 8, NI = 4; };
template <> struct ModeInfo<PM_UNPOOL> { static constexpr int W = 6, NI = 4; };  // 4 dY + 2 argmax words

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
// four u8 pixels -> four bf16 holding the exact integers 0..255 (the f32 of
// an integer below 256 has zero low half-word, so its high half IS the bf16)
__device__ __forceinline__ void u8x4_int_bf16(uint32_t w, uint32_t& h0, uint32_t& h1) {
  const uint32_t f0 = __builtin_bit_cast(uint32_t, (float)(w & 0xffu));
  const uint32_t f1 = __builtin_bit_cast(uint32_t, (float)((w >> 8) & 0xffu));
  const uint32_t f2 = __builtin_bit_cast(uint32_t, (float)((w >> 16) & 0xffu));
  const uint32_t f3 = __builtin_bit_cast(uint32_t, (float)(w >> 24));
  h0 = __builtin_amdgcn_perm(f1, f0, 0x07060302u);
  h1 = __builtin_amdgcn_perm(f3, f2, 0x07060302u);
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

// Per-thread staging of one image group: items e = tid + i*NT (i < NI).
// INTU8 (PM_U8S1): the tile holds the exact integers 0..255 (the consumer
// applies 1/255 in fp32), and the dataset indices of a group are gathered one
// group ahead (load_idx) so the pixel loads never wait on the index gather.
template <int MODE, int NT = kT, bool INTU8 = false>
struct Loader {
  static constexpr int W = ModeInfo<MODE>::W, NI = ModeInfo<MODE>::NI;
  int im[NI];     // image within the group, -1: no item
  int soff[NI];   // source offset within an image (bytes for u8, elements otherwise);
                  // U8S1: | bit0 first word of a row, bit1 last word of a row
  int dst[NI];    // LDS destination (elements)
  int gim[NI];    // INTU8: dataset index of the item's image (next group to load)
  uint32_t r[NI][W];

  __device__ __forceinline__ void load_idx(const PipeSrc& s, int img0, int N) {
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int n = min(img0 + max(im[i], 0), N - 1);
      gim[i] = s.idx ? s.idx[n] : n;
    }
  }

  __device__ __forceinline__ void init(const PipeSrc& s, int imgs) {
    const int total = imgs * s.per_img;
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int e = threadIdx.x + i * NT;
      im[i] = -1; soff[i] = 0; dst[i] = 0;
#pragma unroll
      for (int k = 0; k < W; ++k) r[i][k] = 0;
      if (e >= total) continue;
      const int m = e / s.per_img, rem = e - m * s.per_img;
      im[i] = m;
      if constexpr (MODE == PM_U8S1) {
        const int wpr = s.SW >> 2;
        const int y = rem / wpr, w = rem - y * wpr;
        soff[i] = y * s.SW + 4 * w + (w == 0 ? 1 : 0) + (w == wpr - 1 ? 2 : 0);
        dst[i] = m * s.IMG + (y + s.offy) * s.LWp + 4 * w + s.offx;
      } else {
        const int runs = s.SC / s.RW;
        const int pix = rem / runs, run = rem - pix * runs;
        const int sy = pix / s.SW, sx = pix - sy * s.SW;
        soff[i] = pix * s.SC + run * s.RW;
        const int ty = (MODE == PM_UNPOOL ? 2 * sy : sy) * s.up + s.offy;
        const int tx = (MODE == PM_UNPOOL ? 2 * sx : sx) * s.up + s.offx;
        dst[i] = m * s.IMG + (ty * s.LWp + tx) * s.CL + run * s.RW;
        MCC_DCHECK(dst[i] >= 0 && dst[i] + s.RW <= imgs * s.IMG);
      }
    }
  }

  // Issue the group's global loads (no waits here).  INTU8: unconditional
  // loads of the prefetched indices, then the indices of group next_img0.
  __device__ __forceinline__ void load(const PipeSrc& s, int img0, int N, int next_img0 = 0) {
    const size_t img_src = (size_t)s.SH * s.SW * s.SC;
    if constexpr (INTU8) {
#pragma unroll
      for (int i = 0; i < NI; ++i) {
        const uint8_t* p = static_cast<const uint8_t*>(s.src) + (size_t)gim[i] * img_src + (soff[i] & ~3);
        r[i][0] = *reinterpret_cast<const uint32_t*>(p);
        r[i][1] = *reinterpret_cast<const uint32_t*>(p + 4 - 2 * (soff[i] & 2));  // masked at the store
      }
      if (next_img0 < N) load_idx(s, next_img0, N);
      return;
    }
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      if (im[i] < 0) continue;
      const int n = img0 + im[i];
      if (n >= N) continue;
      if constexpr (MODE == PM_U8S1) {
        const int gim = s.idx ? s.idx[n] : n;
        const uint8_t* p = static_cast<const uint8_t*>(s.src) + (size_t)gim * img_src + (soff[i] & ~3);
        r[i][0] = *reinterpret_cast<const uint32_t*>(p);
        r[i][1] = (soff[i] & 2) ? 0u : *reinterpret_cast<const uint32_t*>(p + 4);
      } else {
        const size_t g = (size_t)n * img_src + soff[i];
        ld_chan(static_cast<const bf16*>(s.src) + g, s.RW, r[i]);
        if constexpr (MODE == PM_RELU) ld_chan(static_cast<const bf16*>(s.aux_y) + g, s.RW, r[i] + 4);
        // PM_UNPOOL: the argmax byte is 4 for ReLU-inactive windows, so it
        // carries the ReLU mask too and the layer output is not read
        if constexpr (MODE == PM_UNPOOL) ld_arg(s.aux_arg + g, s.RW, r[i] + 4);
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
        if constexpr (INTU8) {
          u8x4_int_bf16(r[i][0], h0, h1);
          u8x4_int_bf16((soff[i] & 2) ? 0u : r[i][1], h2, h3);
        } else {
          u8x4_bf16(r[i][0], h0, h1);
          u8x4_bf16(r[i][1], h2, h3);
        }
        bf16* b = lds + dst[i];
        st8(b, h0, h1);
        st8(b + s.CS, mid(h0, h1), mid(h1, h2));
        st8(b + 2 * s.CS, h1, h2);
        st8(b + 3 * s.CS, mid(h1, h2), mid(h2, h3));
        if (soff[i] & 1) {  // the quad left of the row: (halo zeros, first pixels)
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
        const uint32_t* d = r[i];
        const int dxo = s.up * s.CL, dyo = s.up * s.LWp * s.CL;
#pragma unroll
        for (int pos = 0; pos < 4; ++pos) {
          uint32_t v[4];
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            const uint32_t a = r[i][4 + (k >> 1)] >> (16 * (k & 1));  // bytes of channels 2k, 2k+1
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
// XL_S1 fragment read at an 8-byte aligned element offset (shifted copy
// already chosen): two 8-byte reads kept apart (fused, they would issue as
// one ds_read2_b64: 8 LDS cycles and 32-bank instead of 64-bank service)
__device__ __forceinline__ bf16x8 read_s1_pair(const bf16* xs, int e) {
  int hb = 2 * e + 8;  // byte offset of the high half
  asm volatile("" : "+v"(hb));
  const bf16x4 lo = *reinterpret_cast<const bf16x4*>(xs + e);
  const bf16x4 hi = *reinterpret_cast<const bf16x4*>(reinterpret_cast<const char*>(xs) + hb);
  return __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
}
// max of four floats without the NaN canonicalisation fmaxf adds (v_max3 + v_max)
__device__ __forceinline__ float max4(float a, float b, float c, float d) {
  float m;
  asm("v_max3_f32 %0, %1, %2, %3\n\tv_max_f32 %0, %0, %4" : "=&v"(m) : "v"(a), "v"(b), "v"(c), "v"(d));
  return m;
}
// XL_S1 transpose read (4 consecutive tile elements per lane)
__device__ __forceinline__ bf16x4 tr4_s1(const bf16* xs, int CS, int e) {
  const int c = e & 3;
  return tr4(xs + c * CS + (e - c));
}

// Output-pixel (row) -> tile offset of its first tap.  Pool: rows ordered by
// 2x2 window so a 16-row tile holds four whole windows.
// (host copy for the planners' LDS bank model: row_offset)
__host__ __device__ inline int row_offset(int r, bool pool, int OW, int cs, int ty0, int tx0, int LWp, int CL,
                                          int pair) {
  const int PW = OW >> 1;
  {
    int oy, ox;
    if (pair == 2) {  // row = (base window (even column), position TL/TR/BL/BR)
      const int bw = r >> 2, pos = r & 3, PB = PW >> 1;
      const int ph = bw / PB, pm = bw - ph * PB;
      oy = 2 * ph + (pos >> 1);
      ox = 4 * pm + (pos & 1);
    } else if (pair && pool) {  // row = (window, top/bottom pixel pair)
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
    return ((oy * cs + ty0) * LWp + ox * cs + tx0) * CL;
  }
}
// Entries rows..rows_pad-1 (tile padding) repeat row 0.
[[maybe_unused]] __device__ void row_table(int* tab, int rows, bool pool, int OW, int cs, int ty0, int tx0, int LWp, int CL,
                          int pair = 0, int rows_pad = 0) {
  for (int rr = threadIdx.x; rr < max(rows, rows_pad); rr += blockDim.x)
    tab[rr] = row_offset(rr < rows ? rr : 0, pool, OW, cs, ty0, tx0, LWp, CL, pair);
}

// LDS bank model (MI355X_MICROARCH.md, LDS table): extra cycles of one wave
// instruction whose lane l touches the `dw` consecutive dwords from dword
// address a[l].  Lane groups are serviced one per cycle; in a group each
// additional distinct dword on a bank costs one cycle.
enum { LDS_B64 = 0, LDS_B128 = 1 };
inline int lds_conflicts(const int* a, int kind) {
  static const int g128[4][16] = {{0, 1, 2, 3, 12, 13, 14, 15, 20, 21, 22, 23, 24, 25, 26, 27},
                                  {4, 5, 6, 7, 8, 9, 10, 11, 16, 17, 18, 19, 28, 29, 30, 31},
                                  {32, 33, 34, 35, 44, 45, 46, 47, 52, 53, 54, 55, 56, 57, 58, 59},
                                  {36, 37, 38, 39, 40, 41, 42, 43, 48, 49, 50, 51, 60, 61, 62, 63}};
  const int ngroups = kind == LDS_B128 ? 4 : 2, glanes = kind == LDS_B128 ? 16 : 32;
  const int dw = kind == LDS_B128 ? 4 : 2;
  int extra = 0;
  for (int gi = 0; gi < ngroups; ++gi) {
    int cnt[64] = {0};
    int seen[64 * 4];
    int nseen = 0;
    for (int j = 0; j < glanes; ++j) {
      const int l = kind == LDS_B128 ? g128[gi][j] : gi * 32 + j;
      for (int d = 0; d < dw; ++d) {
        const int addr = a[l] + d;
        bool dup = false;
        for (int k = 0; k < nseen && !dup; ++k) dup = seen[k] == addr;
        if (dup) continue;
        seen[nseen++] = addr;
        ++cnt[addr & 63];
      }
    }
    int mx = 0;
    for (int b = 0; b < 64; ++b) mx = cnt[b] > mx ? cnt[b] : mx;
    extra += mx > 1 ? mx - 1 : 0;
  }
  return extra;
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
  L.ws_off = o; o += align16((ntiles * 16 * (p.kpad + 8) + 32) * 2);  // +32: look-ahead read past the last row
  L.bias_off = o; o += ntiles * 16 * 4;
  L.ktab_off = o; o += align16((p.nchunks + 2) * 4 * 4);                 // +2 chunks of look-ahead (offset 0)
  L.ptab_off = o; o += align16(((rows_img + 15) & ~15) * 4);  // tile padding (pair 2)
  L.outs_off = o; o += align16(p.imgs * out_img * 2);
  L.args_off = o; o += pool ? align16(p.imgs * out_img) : 0;
  L.total = o;
  return L;
}

struct DwLayout {
  int xs_elems, dys_off, pixbase_off, ptab_off, ones_off, stage, red, total;
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
  L.pixbase_off = o; o += align16((p.ppad + 32) * 4);  // +32: look-ahead chunk
  L.ptab_off = o; o += align16(p.OH * p.OW * 4);
  L.ones_off = o; o += 16;
  L.stage = o;
  const int ntw = dw_ntw(p.cout_pad / 16, p.ncols_pad / 16);
  L.red = p.cout_pad * ntw * 16 * 4 * (p.wsplit ? 4 : 1);
  L.total = L.stage > L.red ? L.stage : L.red;
  return L;
}

inline int r8h(int x) { return (x + 7) & ~7; }
inline int r16h(int x) { return (x + 15) & ~15; }
inline int r32h(int x) { return (x + 31) & ~31; }

constexpr int kCUs = 256;
constexpr size_t kLdsPerCU = 160 * 1024;

// Destination geometry of a staged source; returns false if unsupported.
[[maybe_unused]] bool plan_src(PipeSrc& s, int layout, int CLdst, int LH, int LWp, int IMGextra) {
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

// Occupancy / group-size choices of the pipelined conv planners (measured:
// workgroups per CU and the LDS footprint a group of images may grow to).
constexpr int dw_wgs_cap() { return 2; }
constexpr int fwd_wgs_cap() { return 4; }
constexpr size_t dw_lds_target() { return (size_t)64 * 1024; }
constexpr size_t fwd_lds_target() { return (size_t)64 * 1024; }

int wgs_per_cu(size_t lds, int cap) {
  int w = (int)(kLdsPerCU / (lds + 512));
  return w < 1 ? 1 : (w > cap ? cap : w);
}

}  // namespace
}  // namespace gpu
}  // namespace mcc
