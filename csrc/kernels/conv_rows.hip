// Row-chunked weight gradient of a single-channel first conv layer (bf16).
//
// Reference: the dW part of Layer_feedBack_conv (cnn.c:212-247) for the
// input layer, whose Cin = 1 / K = KS*KS = 25 shape wastes most of a
// pixel-major MFMA formulation (conv_dw_pipe: 16 x 48 tiles of which 6 x 26
// are real, ~20 VALU per MFMA of transpose-read and address work).
//
// Formulation (per workgroup, persistent over image groups):
//   dW[c][tap] = sum_pixels dZ[c][pix] X[pix + off(tap)],  db[c] = sum dZ[c]
// as v_mfma_f32_16x16x32_bf16 with
//   rows (M)  = output channels c                              (A = dZ)
//   cols (N)  = tap-packed kernel positions kh*KS + kw, then a ones column
//               for the bias: ceil((KK+1)/16) tiles, e.g. 26 of 32 for 5x5
//   K (32)    = ONE output row of 32 pixels (OW <= 32; pixels >= OW carry
//               dZ = 0), lane group g holding pixels 8g..8g+7.
// Both operands are then plain contiguous LDS reads, no transposes:
//   A: dZ staged channel-planar ([c][oy][32] per image): lane (c, g) reads
//      the 8 pixels of its row chunk as one 16-byte read;
//   B: the input staged as four copies shifted by 0..3 elements, so the 8
//      inputs X[oy+kh][8g+kw-pad ..+7] of lane (tap, g) are two aligned
//      8-byte reads from copy (kw - pad + A) & 3; a fifth copy holds ones
//      (the bias column reads it at the same chunk offset, no select).  The
//      u8 pixels are staged as exact bf16 integers 0..255; the 1/255 input
//      scale (cnn.c:457) is applied to the weight columns in the reduce.
// Per chunk and wave: 1 + 2*NT LDS reads, NT MFMAs and 1 + 2*NT address adds
// (every lane base is precomputed, the chunk offset is wave-uniform); the
// chunk loop is unrolled by two with ping-pong fragment registers.  The dZ staging applies the
// max-pool backward (the pooled gradient routed to its argmax, masked by
// ReLU) while writing the planes, so dZ never exists in HBM.  Plane and copy
// strides are chosen by a host-side search over the LDS bank map.
// Per-workgroup fp32 slabs are reduced by the deterministic two-level sum of
// conv_pipe_dw.hip.
#include "conv_pipe.h"

namespace mcc {
namespace gpu {

namespace {

struct RowsDwLayout {
  int xs_off, dz_off, ones_off, total;
};
__host__ __device__ inline RowsDwLayout rows_dw_layout(const ConvDwRowsParams& p) {
  RowsDwLayout L;
  L.xs_off = 0;
  int o = align16(p.imgs * p.ximg * 2);
  L.dz_off = o;
  o += align16(p.imgs * p.dzimg * 2);
  L.ones_off = o;
  o += 16;
  L.total = o;
  return L;
}

// dY items per thread (prefetched in registers across the compute phase)
constexpr int kNiX = 4, kNiD = 3;

// Raw buffer loads (one VGPR each): the compiler neither fuses them into
// multi-dword tuples nor re-homes their results with register moves, either
// of which would force a wait on the load right after issuing it.
typedef __amdgpu_buffer_rsrc_t rsrc_t;
__device__ __forceinline__ rsrc_t make_rsrc(const void* base, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes, 0x00020000);
}
__device__ __forceinline__ uint32_t bload32(rsrc_t r, int off) { return __builtin_amdgcn_raw_buffer_load_b32(r, off, 0, 0); }
__device__ __forceinline__ uint32_t bload16(rsrc_t r, int off) {
  return (uint32_t)__builtin_amdgcn_raw_buffer_load_b16(r, off, 0, 0);
}

template <int DM, int NT, int CW>  // DM: PM_UNPOOL / PM_RELU; CW: u32 words of dY per pixel (Cout/2)
__global__ void __launch_bounds__(kT) conv_dw_rows_kernel(ConvDwRowsParams p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const RowsDwLayout L = rows_dw_layout(p);
  bf16* xs = reinterpret_cast<bf16*>(smem + L.xs_off);
  bf16* dz = reinterpret_cast<bf16*>(smem + L.dz_off);
  float* red = reinterpret_cast<float*>(smem);  // reused after the main loop

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform: scalar loop control
  const int r16 = lane & 15, g = lane >> 4;

  zero_lds(reinterpret_cast<bf16*>(smem), L.ones_off / 2);
  __syncthreads();
  // the ones copy (copy 4) of every image slot: rows [0, OH), columns [0, 32)
  for (int e = tid; e < p.imgs * p.OH * 4; e += kT) {
    const int m = e / (p.OH * 4), r = e - m * p.OH * 4, y = r >> 2, c8 = (r & 3) * 8;
    const uint32_t one2 = 0x3f803f80u;  // two bf16 1.0
    bf16* d = xs + m * p.ximg + 4 * p.CS + y * p.Pw + c8;  // 8-byte aligned (Pw % 4 == 0)
    st8(d, one2, one2);
    st8(d + 4, one2, one2);
  }

  // ---- per-lane operand byte offsets (kernel-invariant) ----
  const int c_l = r16 < p.Cout ? r16 : r16 % p.Cout;  // rows >= Cout: duplicate rows, discarded
  const int a_lane = 2 * (L.dz_off / 2 + c_l * p.dplane + 8 * g);
  int b_lo[NT], b_hi[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    const int n = t * 16 + r16;
    const int kh = n / p.KS, kw = n - kh * p.KS;
    const int sh = kw - p.pad + p.A, s = sh & 3;
    // taps: shifted copy s; bias and padding columns: the ones copy
    const int e = n < p.KK ? s * p.CS + kh * p.Pw + (sh - s) + 8 * g : 4 * p.CS + 8 * g;
    b_lo[t] = 2 * e;
    b_hi[t] = 2 * (e + 4);
    // opaque to the optimiser: two ds_read_b64 (2 + 2 LDS cycles) instead
    // of one fused ds_read2_b64 (8 cycles, MI355X_MICROARCH.md §LDS)
    asm volatile("" : "+v"(b_hi[t]));
  }

  // ---- staging geometry (per thread, group-invariant) ----
  const int xper = p.SH * p.nblk;
  const int dper = p.DH * p.DW;
  // Loads are issued unconditionally from clamped (always valid) addresses
  // and masked at store time: a conditional load would merge with the old
  // register value and make the compiler wait for it on the spot, which
  // serialises the prefetch against HBM latency.
  int xim[kNiX], xsrc0[kNiX], xsrc1[kNiX], xdst[kNiX];
  uint32_t xw[kNiX][2];
  uint32_t xfl[kNiX];  // bit0: word w0 valid, bit1: word w1 valid
#pragma unroll
  for (int i = 0; i < kNiX; ++i) {
    const int e = tid + i * kT;
    xim[i] = -1; xsrc0[i] = 0; xsrc1[i] = 0; xdst[i] = 0; xfl[i] = 0; xw[i][0] = xw[i][1] = 0;
    if (e >= p.imgs * xper) continue;
    const int m = e / xper, rem = e - m * xper;
    const int y = rem / p.nblk, b = rem - y * p.nblk;
    const int mb = p.m0 + b;
    const int w0 = mb - p.A / 4;
    xim[i] = m;
    xfl[i] = (w0 >= 0 && w0 < p.SW / 4 ? 1u : 0u) | (w0 + 1 >= 0 && w0 + 1 < p.SW / 4 ? 2u : 0u);
    xsrc0[i] = (xfl[i] & 1u) ? y * p.SW + 4 * w0 : 0;
    xsrc1[i] = (xfl[i] & 2u) ? y * p.SW + 4 * (w0 + 1) : 0;
    xdst[i] = m * p.ximg + (y + p.pad) * p.Pw + 4 * mb;
  }
  int dim_[kNiD], dsrc[kNiD], ddst[kNiD];
  uint32_t dv[kNiD][CW], dyv[kNiD][CW], darg[kNiD][CW];  // darg[k]: argmax bytes of channels 2k, 2k+1
#pragma unroll
  for (int i = 0; i < kNiD; ++i) {
    const int e = tid + i * kT;
    dim_[i] = -1; dsrc[i] = 0; ddst[i] = 0;
#pragma unroll
    for (int k = 0; k < CW; ++k) dv[i][k] = dyv[i][k] = 0;
#pragma unroll
    for (int k = 0; k < CW; ++k) darg[i][k] = 0;
    if (e >= p.imgs * dper) continue;
    const int m = e / dper, rem = e - m * dper;
    const int wy = rem / p.DW, wx = rem - wy * p.DW;
    dim_[i] = m;
    dsrc[i] = rem;  // pixel within the image of the dY grid
    ddst[i] = m * p.dzimg + (DM == PM_UNPOOL ? (2 * wy) * 32 + 2 * wx : wy * 32 + wx);
  }

  const rsrc_t r_dy = make_rsrc(p.dy, (uint32_t)p.N * dper * p.Cout * 2);
  const rsrc_t r_arg = make_rsrc(p.aux_arg, (uint32_t)p.N * dper * p.Cout);
  const rsrc_t r_y = make_rsrc(p.aux_y, DM == PM_RELU ? (uint32_t)p.N * dper * p.Cout * 2 : 0u);
  // dataset indices of the group to load, fetched one group ahead so the
  // pixel loads never wait on the index gather
  int gim[kNiX];
  auto load_idx = [&](int img0) {
#pragma unroll
    for (int i = 0; i < kNiX; ++i) {
      const int n = min(img0 + max(xim[i], 0), p.N - 1);
      gim[i] = p.idx ? p.idx[n] : n;
    }
  };
  auto load_group = [&](int img0, int next_img0) {
#pragma unroll
    for (int i = 0; i < kNiX; ++i) {
      const uint8_t* img = p.x + (size_t)gim[i] * p.SH * p.SW;
      xw[i][0] = *reinterpret_cast<const uint32_t*>(img + xsrc0[i]);
      xw[i][1] = *reinterpret_cast<const uint32_t*>(img + xsrc1[i]);
    }
#pragma unroll
    for (int i = 0; i < kNiD; ++i) {
      const int n = min(img0 + max(dim_[i], 0), p.N - 1);
      const int pix = n * dper + dsrc[i];  // < 2^31 / (2 Cout): planner
#pragma unroll
      for (int k = 0; k < CW; ++k) dv[i][k] = bload32(r_dy, pix * p.Cout * 2 + 4 * k);
      if (DM == PM_RELU) {
#pragma unroll
        for (int k = 0; k < CW; ++k) dyv[i][k] = bload32(r_y, pix * p.Cout * 2 + 4 * k);
      }
      if (DM == PM_UNPOOL) {
#pragma unroll
        for (int k = 0; k < CW; ++k) darg[i][k] = bload16(r_arg, pix * p.Cout + 2 * k);
      }
    }
    if (next_img0 < p.N) load_idx(next_img0);
  };

  auto store_group = [&](int nimg) {
#pragma unroll
    for (int i = 0; i < kNiX; ++i) {
      if (xim[i] < 0 || xim[i] >= nimg) continue;
      uint32_t h0, h1, h2, h3;
      u8x4_int_bf16((xfl[i] & 1u) ? xw[i][0] : 0u, h0, h1);
      u8x4_int_bf16((xfl[i] & 2u) ? xw[i][1] : 0u, h2, h3);
      bf16* b = xs + xdst[i];
      st8(b, h0, h1);
      st8(b + p.CS, mid(h0, h1), mid(h1, h2));
      st8(b + 2 * p.CS, h1, h2);
      st8(b + 3 * p.CS, mid(h1, h2), mid(h2, h3));
    }
#pragma unroll
    for (int i = 0; i < kNiD; ++i) {
      if (dim_[i] < 0 || dim_[i] >= nimg) continue;
      bf16* d = dz + ddst[i];
#pragma unroll
      for (int k = 0; k < CW; ++k) {
        // channels 2k, 2k+1; PM_UNPOOL: the argmax byte (4 = ReLU-inactive) is the mask
        const uint32_t v = DM == PM_UNPOOL ? dv[i][k] : relu_mask(dv[i][k], dyv[i][k]);
        if (DM == PM_UNPOOL) {
          const uint32_t a = darg[i][k];  // bytes: arg of 2k, 2k+1
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            const uint32_t vh = (v >> (16 * h)) & 0xffffu;
            const uint32_t ah = (a >> (8 * h)) & 0xffu;
            // rows 2wy / 2wy+1 of plane 2k+h: (left, right) pairs of the window
            const uint32_t top = ah == 0 ? vh : (ah == 1 ? vh << 16 : 0u);
            const uint32_t bot = ah == 2 ? vh : (ah == 3 ? vh << 16 : 0u);
            uint32_t* q = reinterpret_cast<uint32_t*>(d + (2 * k + h) * p.dplane);
            q[0] = top;
            q[16] = bot;  // next row: +32 elements
          }
        } else {
          d[(2 * k) * p.dplane] = __builtin_bit_cast(bf16, (unsigned short)(v & 0xffffu));
          d[(2 * k + 1) * p.dplane] = __builtin_bit_cast(bf16, (unsigned short)(v >> 16));
        }
      }
    }
  };

  f32x4 acc[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};

  // Iteration k prefetches group blockIdx.x + k*gridDim.x and computes the
  // one before it.  ONE load site: the prefetched values stay in the load
  // destination registers until the store after the next barrier (two sites
  // would merge through register moves, each of which waits on its load).
  if ((int)blockIdx.x < p.ngroups) load_idx(blockIdx.x * p.imgs);
  for (int k = 0;; ++k) {
    const int lgrp = blockIdx.x + k * gridDim.x, grp = lgrp - gridDim.x;
    if (grp >= p.ngroups) break;
    if (k > 0) {
      __syncthreads();  // previous group consumed (and the zero fill, first time)
      store_group(min(p.imgs, p.N - grp * p.imgs));
      __syncthreads();
    }
    if (lgrp < p.ngroups) load_group(lgrp * p.imgs, (lgrp + gridDim.x) * p.imgs);
    if (k == 0) continue;
    const int nimg = min(p.imgs, p.N - grp * p.imgs);

    // chunks q = (image, output row), wave-strided; offsets are wave-uniform
    const int nq = nimg * p.OH;
    const char* lds = smem;
    auto frag = [&](int im, int y, bf16x8& a, bf16x8 (&b)[NT]) {
      a = *reinterpret_cast<const bf16x8*>(lds + a_lane + 2 * (im * p.dzimg + y * 32));
      const int xo = 2 * (im * p.ximg + y * p.Pw);
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        const bf16x4 lo = *reinterpret_cast<const bf16x4*>(lds + b_lo[t] + xo);
        const bf16x4 hi = *reinterpret_cast<const bf16x4*>(lds + b_hi[t] + xo);
        b[t] = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
      }
    };
    // chunks wave, wave + 4, ...: (image, row) advanced incrementally
    // (scalar, OH >= 4); unrolled by two with ping-pong fragments so no
    // fragment is copied between registers
    constexpr int NW = kT / 64;
    const int cnt = nq > wave ? (nq - wave + NW - 1) / NW : 0;
    int im = 0, y = wave;
    auto step = [&](int& i, int& r) {
      r += NW;
      if (r >= p.OH) { r -= p.OH; ++i; }
    };
    bf16x8 a0, b0[NT], a1, b1[NT];
    if (cnt > 0) frag(im, y, a0, b0);
    int i = 0;
    for (; i + 2 <= cnt; i += 2) {
      int im1 = im, y1 = y;
      step(im1, y1);
      frag(im1, y1, a1, b1);
#pragma unroll
      for (int t = 0; t < NT; ++t) acc[t] = mma(acc[t], a0, b0[t]);
      im = im1; y = y1;
      step(im, y);
      if (i + 2 < cnt) frag(im, y, a0, b0);
#pragma unroll
      for (int t = 0; t < NT; ++t) acc[t] = mma(acc[t], a1, b1[t]);
    }
    if (i < cnt) {
#pragma unroll
      for (int t = 0; t < NT; ++t) acc[t] = mma(acc[t], a0, b0[t]);
    }
  }

  // combine the waves in a fixed order into red[16][NT*16], then the slab
  constexpr int RC = NT * 16;
  for (int w = 0; w < kT / 64; ++w) {
    __syncthreads();
    if (wave == w) {
#pragma unroll
      for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          float* d = red + (4 * g + i) * RC + t * 16 + r16;
          *d = (w == 0 ? 0.f : *d) + acc[t][i];
        }
    }
  }
  __syncthreads();
  for (int e = tid; e < 16 * RC; e += kT) p.slab[(size_t)blockIdx.x * 16 * RC + e] = red[e];
}

// bank conflict cycles of the B-operand reads (ds_read_b64, two 32-lane groups)
int rows_b_conflicts(const ConvDwRowsParams& p, int Pw, int CS) {
  int total = 0;
  for (int t = 0; t < p.ntiles; ++t)
    for (int half = 0; half < 2; ++half)
      for (int grp = 0; grp < 2; ++grp) {
        int cnt[64] = {0};
        int seen[64][64];
        int ns[64] = {0};
        for (int lane = 32 * grp; lane < 32 * grp + 32; ++lane) {
          const int r16 = lane & 15, g = lane >> 4, n = t * 16 + r16;
          long e;
          if (n >= p.KK) e = 1 << 24;
          else {
            const int kh = n / p.KS, kw = n % p.KS, sh = kw - p.pad + p.A, s = sh & 3;
            e = (long)s * CS + kh * Pw + (sh - s) + 8 * g + 4 * half;
          }
          for (int d = 0; d < 2; ++d) {
            const int dw = (int)(e / 2 + d), bk = dw & 63;
            bool dup = false;
            for (int j = 0; j < ns[bk]; ++j) dup |= seen[bk][j] == dw;
            if (!dup) { seen[bk][ns[bk]++] = dw; cnt[bk]++; }
          }
        }
        int mx = 1;
        for (int bk = 0; bk < 64; ++bk) mx = std::max(mx, cnt[bk]);
        total += mx;
      }
  return total;
}

}  // namespace

bool conv_dw_rows_plan(ConvDwRowsParams& p) {
  if (ab_flag("no_rows")) return false;  // A/B: the pixel-major conv_dw_pipe kernel (tested)
  const int cw = p.Cout / 2;
  if ((p.Cout & 1) || !(cw == 1 || cw == 2 || cw == 3 || cw == 4 || cw == 8) || p.OW > 32 || p.OW < 1 || p.OH < 4)
    return false;
  if (p.dmode != PM_UNPOOL && p.dmode != PM_RELU) return false;
  if ((p.SW & 3) || p.SW > 64) return false;
  if (p.OH != p.SH + 2 * p.pad - p.KS + 1 || p.OW != p.SW + 2 * p.pad - p.KS + 1) return false;  // stride 1
  p.KK = p.KS * p.KS;
  p.ntiles = cdiv(p.KK + 1, 16);
  if (p.ntiles > 3) return false;
  if (p.dmode == PM_UNPOOL && (p.DH != p.OH / 2 || p.DW != p.OW / 2)) return false;
  if ((int64_t)p.N * p.DH * p.DW * p.Cout * 2 >= (1ll << 31)) return false;  // 32-bit buffer offsets
  if (p.dmode == PM_RELU && (p.DH != p.OH || p.DW != p.OW)) return false;
  p.A = (p.pad + 3) & ~3;
  p.LH = p.OH + p.KS - 1;
  // LDS columns read: up to 31 + KS - 1 - pad + A (+3 for the copy offset)
  const int maxcol = 31 + p.KS - 1 - p.pad + p.A + 4;
  const int Pmin = ((std::max(maxcol, p.A + p.SW + 4)) + 3) & ~3;
  // blocks of 4 copy columns that can hold real pixels (the rest stay zero)
  p.m0 = 0;
  while (4 * p.m0 - p.A + 6 < 0) ++p.m0;
  int mend = p.m0;
  while (4 * mend - p.A < p.SW) ++mend;
  p.nblk = mend - p.m0;
  // copy pitch / copy stride with the fewest B-read bank conflicts
  int best = 1 << 30;
  for (int Pw = Pmin; Pw < Pmin + 32; Pw += 4)
    for (int skew = 0; skew < 128; skew += 4) {
      const int CS = p.LH * Pw + skew;
      const int c = rows_b_conflicts(p, Pw, CS);
      if (c < best) { best = c; p.Pw = Pw; p.CS = CS; }
    }
  p.ximg = (5 * p.CS + 7) & ~7;  // four shifted copies + the ones copy
  p.dplane = p.OH * 32 + 16;  // 16-element skew: conflict-free 16-byte A reads (host search, r2)
  p.dzimg = p.Cout * p.dplane;
  const int xper = p.SH * p.nblk, dper = p.DH * p.DW;
  int imgs = std::min(16, std::min(kNiX * kT / std::max(1, xper), kNiD * kT / std::max(1, dper)));
  if (imgs < 1) return false;
  for (; imgs > 1; --imgs) {
    p.imgs = imgs;
    if ((size_t)rows_dw_layout(p).total <= dw_lds_target()) break;
  }
  p.imgs = imgs;
  const RowsDwLayout L = rows_dw_layout(p);
  if ((size_t)L.total > kLdsPerCU || (size_t)(16 * p.ntiles * 16 * 4) > (size_t)L.total) return false;
  p.lds = (size_t)L.total;
  p.ngroups = cdiv(p.N, p.imgs);
  p.grid = std::min(p.ngroups, kCUs * wgs_per_cu(p.lds, 3));
  return true;
}

size_t conv_dw_rows_scratch_bytes(const ConvDwRowsParams& p) {
  const size_t nv = (size_t)16 * p.ntiles * 16;
  return ((size_t)p.grid + cdiv(p.grid, 64)) * nv * 4;
}

void conv_dw_rows(const ConvDwRowsParams& pin, float* gw, float* gb, hipStream_t st) {
  ConvDwRowsParams p = pin;
  p.ngroups = cdiv(p.N, p.imgs);
  p.grid = std::min(p.ngroups, pin.grid);
  if (p.grid <= 0) return;
  const dim3 grid((unsigned)p.grid), block(kT);
  auto go = [&](auto kern) { hipLaunchKernelGGL(kern, grid, block, p.lds, st, p); };
  const int cw = p.Cout / 2;
#define MCC_ROWS_CW(DM, NT)                                          \
  if (cw <= 1) go(conv_dw_rows_kernel<DM, NT, 1>);                   \
  else if (cw <= 2) go(conv_dw_rows_kernel<DM, NT, 2>);              \
  else if (cw <= 3) go(conv_dw_rows_kernel<DM, NT, 3>);              \
  else if (cw <= 4) go(conv_dw_rows_kernel<DM, NT, 4>);              \
  else go(conv_dw_rows_kernel<DM, NT, 8>);  /* planner: cw in {1,2,3,4,8} */
#define MCC_ROWS_NT(DM)                 \
  if (p.ntiles == 1) { MCC_ROWS_CW(DM, 1) } \
  else if (p.ntiles == 2) { MCC_ROWS_CW(DM, 2) } \
  else { MCC_ROWS_CW(DM, 3) }
  if (p.dmode == PM_UNPOOL) { MCC_ROWS_NT(PM_UNPOOL) }
  else { MCC_ROWS_NT(PM_RELU) }
#undef MCC_ROWS_NT
#undef MCC_ROWS_CW
  // deterministic two-level reduce of the per-workgroup slabs
  const int ncols = p.ntiles * 16;
  dw_slab_reduce(p.slab, p.grid, 16, ncols, p.slab + (size_t)pin.grid * 16 * ncols, p.Cout, 1, p.KS, XL_ROWS, 1,
                 p.KK, gw, gb, st, 1.0f / 255.0f);  // the input was staged unscaled
}

}  // namespace gpu
}  // namespace mcc
