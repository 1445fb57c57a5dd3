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
#include "conv_pipe.h"

#include <cstdio>
#include <utility>
#include <vector>

namespace mcc {
namespace gpu {

namespace {

// DPP row_ror:8 — lane i <- lane i^8 within each 16-lane row
__device__ __forceinline__ float swap8(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x128, 0xf, 0xf, false));
}

// WR > 0 (one column tile, exactly WR K chunks): every lane keeps its B
// fragments and K-group offsets in registers for the whole launch, so the
// K loop reads only the A operand from LDS (half the LDS traffic and none of
// the weight-row bank conflicts); two row tiles per item keep the register
// budget at four waves per SIMD.
// (waves_per_eu(4): two 512-thread or four 256-thread workgroups per CU need
// <= 128 VGPRs; at 129+ the CU holds half the waves)
template <int MODE, int EPI, int ACT, int PAIR, int NT, int WR = 0>
__global__ void __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(WR > 0 ? 1 : 4))) conv_pipe_fwd_kernel(ConvPipeParams p) {
  constexpr int MT = WR > 8 ? 2 : 4;
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
    for (int v = tid; v < nv; v += NT) {
      const int r = v / vpr, c = (v - r * vpr) * 8;
      store8(ws + r * wld + c, load8(wpk + (size_t)r * p.kpad + c));
    }
  }
  for (int n = tid; n < ntiles * 16; n += NT) {
    const int c = PAIR ? (n & 7) : n;
    bias_s[n] = (EPI != FE_PLAIN && c < p.Cout) ? p.bias[c] : 0.f;
  }
  for (int gi = tid; gi < (p.nchunks + 2) * 4; gi += NT) {
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
  const int rows_pad = PAIR == 2 ? (rows_img + 15) & ~15 : rows_img;
  row_table(ptab, rows_img, pool, p.OW, p.cs, p.ty0, p.tx0, s.LWp, S1 ? 1 : s.CL, PAIR, rows_pad);  // PAIR 2: window pairs
  if (S1) {  // bake the shifted-copy choice into the table (IMG and K offsets are multiples of 4)
    for (int r = tid; r < rows_pad; r += NT) {
      const int b = ptab[r], c = b & 3;
      ptab[r] = c * s.CS + b - c;
    }
  }

  // S1 (the dataset input): exact-integer tile, 1/255 applied in the epilogue
  constexpr float xsc = S1 ? 1.f / 255.f : 1.f;
  Loader<MODE, NT, S1> ld;
  ld.init(s, p.imgs);
  if (S1) ld.load_idx(s, blockIdx.x * p.imgs, p.N);

  const int lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r16 = lane & 15, g = lane >> 4;
  constexpr int NW = WR > 0 ? WR : (PAIR == 2 ? 2 : 1);
  bf16x8 wreg[NW];
  int kreg[NW];
  if constexpr (WR > 0 || PAIR == 2) {
    __syncthreads();  // weights and K table staged
#pragma unroll
    for (int q = 0; q < NW; ++q) {  // PAIR 2: nchunks <= 2 (the ws padding covers q = 1)
      wreg[q] = load8(ws + r16 * wld + 8 * g + q * 32);
      kreg[q] = ktab[q * 4 + g];
    }
  }
  Div drpi;
  drpi.mh = p.rows_mh;
  drpi.ml = p.rows_ml;

  // Iteration k loads group blockIdx.x + k*gridDim.x and computes the one
  // before it: ONE load site, so the prefetched registers stay in place until
  // the store after the next barrier (a second site would merge the values
  // through register moves that wait on the loads).
  for (int k = 0;; ++k) {
    const int lgrp = blockIdx.x + k * (int)gridDim.x, grp = lgrp - (int)gridDim.x;
    if (grp >= p.ngroups) break;
    const int img0 = grp * p.imgs;
    const int nimg = min(p.imgs, p.N - img0);
    if (k > 0) {
      __syncthreads();  // tiles free: previous compute and copy-out done (and setup, first time)
      ld.store(s, xs, nimg);
      __syncthreads();
    }
    if (lgrp < p.ngroups) ld.load(s, lgrp * p.imgs, p.N, (lgrp + (int)gridDim.x) * p.imgs);
    if (k == 0) continue;

    if constexpr (PAIR == 2) {
      // Window pairs on the single-channel input.  Tiles never straddle an
      // image (rows padded to 16 per image), so a tile's image, its tile
      // index and every bound are wave-uniform scalars; the lane's row offset
      // is one table read.  Weights are register-resident (<= 2 K chunks).
      const int tpi = rows_pad >> 4, ntl = nimg * tpi, nbw = rows_img >> 2;
      for (int item = wave; item < cdiv(ntl, MT); item += NT / 64) {
        int img[MT], ti[MT], base[MT];
#pragma unroll
        for (int t = 0; t < MT; ++t) {
          const int T = min(item * MT + t, ntl - 1);
          img[t] = drpi.div(T);
          ti[t] = T - img[t] * tpi;
          base[t] = img[t] * s.IMG + ptab[ti[t] * 16 + r16];
        }
        bf16x8 a0[MT], a1[MT];
        f32x4 acc[MT];
#pragma unroll
        for (int t = 0; t < MT; ++t) {
          a0[t] = read_s1_pair(xs, base[t] + kreg[0]);
          acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
        }
        if (p.nchunks > 1) {
#pragma unroll
          for (int t = 0; t < MT; ++t) a1[t] = read_s1_pair(xs, base[t] + kreg[1]);
#pragma unroll
          for (int t = 0; t < MT; ++t) acc[t] = mma(acc[t], a0[t], wreg[0]);
#pragma unroll
          for (int t = 0; t < MT; ++t) acc[t] = mma(acc[t], a1[t], wreg[1]);
        } else {
#pragma unroll
          for (int t = 0; t < MT; ++t) acc[t] = mma(acc[t], a0[t], wreg[0]);
        }
        // rows 4g..4g+3 = positions (TL, TR, BL, BR) of window pair bw;
        // column r16 = channel (r16 & 7) of its left (r16 < 8) or right
        // window: the 2x2 max-pool and its argmax are in-lane
        const int c = r16 & 7, sft = r16 >> 3;
        const float bv = bias_s[r16];
        const int olane = (2 * g + sft) * p.Cout + c;  // + img*out_img + ti*8*Cout (scalar)
#pragma unroll
        for (int t = 0; t < MT; ++t) {
          if (item * MT + t < ntl && c < p.Cout && g < nbw - ti[t] * 4) {
            const float best = max4(acc[t][0], acc[t][1], acc[t][2], acc[t][3]);
            // first maximum wins (as the reference's strict > scan)
            int arg = 3;
            arg = acc[t][2] == best ? 2 : arg;
            arg = acc[t][1] == best ? 1 : arg;
            arg = acc[t][0] == best ? 0 : arg;
            const bf16 yb = (bf16)fmaxf(fmaf(best, xsc, bv), 0.f);
            const int o = img[t] * out_img + ti[t] * 8 * p.Cout + olane;
            MCC_DCHECK(o < p.imgs * out_img);
            outs[o] = yb;
            args[o] = (uint8_t)((float)yb > 0.f ? arg : 4);  // 4: ReLU-inactive window
          }
        }
      }
    } else {
    const int M = nimg * rows_img;
    const int mtiles = cdiv(M, 16), mgroups = cdiv(mtiles, MT);
    const int ko_s0 = ktab[g], ko_s1 = ktab[4 + g];  // XL_S1: at most two chunks, item-invariant
    for (int item = wave; item < ntiles * mgroups; item += NT / 64) {
      const int nt = ntiles == 1 ? 0 : item / mgroups, mg = item - nt * mgroups;
      // rows past M (last tile of a partial group) re-read row M-1: finite, discarded
      int base[MT], ti[MT];
#pragma unroll
      for (int t = 0; t < MT; ++t) {
        const int r = min((mg * MT + t) * 16 + r16, M - 1);
        const int img = drpi.div(r);
        ti[t] = r - img * rows_img;
        base[t] = img * s.IMG;
      }
#pragma unroll
      for (int t = 0; t < MT; ++t) {
        base[t] += ptab[ti[t]];
        MCC_DCHECK(base[t] >= 0 && base[t] < L.xs_elems);
      }
      f32x4 acc[MT];
#pragma unroll
      for (int t = 0; t < MT; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
      // K loop, software-pipelined one chunk deep: chunk q+1's fragments (and
      // chunk q+2's K-group offset) are read while chunk q's MFMAs issue.
      // ktab and ws carry padding so the look-ahead reads stay in bounds.
      const bf16* wrow = ws + (nt * 16 + r16) * wld + 8 * g;
      auto read_a = [&](bf16x8 (&a)[MT], int ko) {
#pragma unroll
        for (int t = 0; t < MT; ++t) {
          if (S1) {
            const bf16* ap = xs + base[t] + ko;
            const bf16x4 lo = *reinterpret_cast<const bf16x4*>(ap);
            const bf16x4 hi = *reinterpret_cast<const bf16x4*>(ap + 4);
            a[t] = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
          } else {
            a[t] = load8(xs + base[t] + ko);
          }
        }
      };
      if (S1) {
        // at most two chunks (KS <= 8): issue every fragment read, then the MFMAs
        bf16x8 a0[MT], a1[MT];
        const bf16x8 b0 = load8(wrow);
        read_a(a0, ko_s0);
        if (p.nchunks > 1) {
          const bf16x8 b1 = load8(wrow + 32);
          read_a(a1, ko_s1);
#pragma unroll
          for (int t = 0; t < MT; ++t) acc[t] = mma(acc[t], a0[t], b0);
#pragma unroll
          for (int t = 0; t < MT; ++t) acc[t] = mma(acc[t], a1[t], b1);
        } else {
#pragma unroll
          for (int t = 0; t < MT; ++t) acc[t] = mma(acc[t], a0[t], b0);
        }
      } else if constexpr (WR > 0) {
        // fully unrolled K loop on register-resident weights; chunk q+1's A
        // fragments are read while chunk q's MFMAs issue
        bf16x8 a[MT], an[MT];
        read_a(a, kreg[0]);
#pragma unroll
        for (int q = 0; q < WR; ++q) {
          if (q + 1 < WR) read_a(an, kreg[q + 1]);
#pragma unroll
          for (int t = 0; t < MT; ++t) acc[t] = mma(acc[t], a[t], wreg[q]);
          if (q + 1 < WR) {
#pragma unroll
            for (int t = 0; t < MT; ++t) a[t] = an[t];
          }
        }
      } else {
        // one chunk of look-ahead: chunk q+1's fragments (and chunk q+2's
        // K-group offset) are read while chunk q's MFMAs issue (ktab/ws
        // padding keeps the look-ahead in bounds)
        bf16x8 a[MT], an[MT];
        bf16x8 b = load8(wrow);
        read_a(a, ktab[g]);
        int ko_next = ktab[4 + g];
        for (int q = 0; q < p.nchunks; ++q) {
          const bf16x8 bn = load8(wrow + (q + 1) * 32);
          read_a(an, ko_next);
          ko_next = ktab[(q + 2) * 4 + g];
#pragma unroll
          for (int t = 0; t < MT; ++t) acc[t] = mma(acc[t], a[t], b);
          b = bn;
#pragma unroll
          for (int t = 0; t < MT; ++t) a[t] = an[t];
        }
      }
      // epilogue into the LDS output tile: lane holds rows 4g..4g+3, column n
      if constexpr (PAIR == 1) {
        // column r16 = channel (r16 & 7) of the left (r16 < 8) or right pixel
        const int c = r16 & 7;
        const bool right = r16 >= 8;
        const float bv = bias_s[r16];
#pragma unroll
        for (int t = 0; t < MT; ++t) {
          const int rb = (mg * MT + t) * 16 + 4 * g;
          if (pool) {
            // rows 4g..4g+3 = (top, bottom) pairs of windows w0 = rb/2 and w0+1.
            // The left lane finishes w0, the right lane w0+1: each sends its
            // partner the two values of the partner's window (DPP row_ror:8).
            // Max/argmax on raw sums (bias and ReLU are monotone; where ReLU
            // ties, the pooled value is 0 and its gradient is masked anyway).
            // (selects are always between an accumulator and a DPP result, so
            // they stay v_cndmask instead of a dynamically indexed extract)
            const float p0 = swap8(acc[t][0]), p1 = swap8(acc[t][1]);
            const float p2 = swap8(acc[t][2]), p3 = swap8(acc[t][3]);
            // window order TL, TR, BL, BR; first maximum wins
            const float tl = right ? p2 : acc[t][0];
            const float bl = right ? p3 : acc[t][1];
            const float tr = right ? acc[t][2] : p0;
            const float br = right ? acc[t][3] : p1;
            float best = tl;
            int arg = 0;
            if (tr > best) { best = tr; arg = 1; }
            if (bl > best) { best = bl; arg = 2; }
            if (br > best) { best = br; arg = 3; }
            const float y = ACT == ACT_RELU ? fmaxf(fmaf(best, xsc, bias_s[c]), 0.f) : fmaf(best, xsc, bias_s[c]);
            const int win = (rb >> 1) + (right ? 1 : 0);
            if (c < p.Cout && 2 * win < M) {
              const int o = win * p.Cout + c;
              MCC_DCHECK(o < p.imgs * out_img);
              outs[o] = (bf16)y;
              // ReLU-inactive window: argmax byte 4 (the backward routes nothing, no y read)
              args[o] = (uint8_t)(ACT == ACT_RELU && !((float)(bf16)y > 0.f) ? 4 : arg);
            }
          } else if (c < p.Cout) {
#pragma unroll
            for (int i = 0; i < 4; ++i) {
              const float x = fmaf(acc[t][i], xsc, bv);
              const float v = ACT == ACT_RELU ? fmaxf(x, 0.f) : (ACT == ACT_TANH ? tanhf(x) : x);
              if (rb + i < M) outs[(2 * (rb + i) + (r16 >> 3)) * p.Cout + c] = (bf16)v;
            }
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
        if (pool) {
          // max/argmax on the raw sums, then bias + ReLU once (monotone)
          float best = acc[t][0];
          int arg = 0;
#pragma unroll
          for (int i = 1; i < 4; ++i) {
            const bool gt = acc[t][i] > best;
            best = gt ? acc[t][i] : best;
            arg = gt ? i : arg;
          }
          const int o = (rb >> 2) * p.Cout + n;
          MCC_DCHECK(o < p.imgs * out_img);
          const bf16 yb = (bf16)fmaxf(fmaf(best, xsc, bv), 0.f);
          outs[o] = yb;
          args[o] = (uint8_t)((float)yb > 0.f ? arg : 4);  // 4: ReLU-inactive window
        } else {
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const float x = fmaf(acc[t][i], xsc, bv);
            const float v = ACT == ACT_RELU ? fmaxf(x, 0.f) : (ACT == ACT_TANH ? tanhf(x) : x);
            if (rb + i < M) outs[(rb + i) * p.Cout + n] = (bf16)v;
          }
        }
      }
    }
    }  // PAIR != 2
    __syncthreads();
    char* gout = static_cast<char*>(p.out) + (size_t)img0 * out_img * 2;
    copy_out(gout, reinterpret_cast<const char*>(outs), nimg * out_img * 2, pow2_align(out_img * 2));
    if (pool) {
      char* garg = reinterpret_cast<char*>(p.out_arg) + (size_t)img0 * out_img;
      copy_out(garg, reinterpret_cast<const char*>(args), nimg * out_img, pow2_align(out_img));
    }
  }
}

// register-resident weights for the LeNet-class shapes (one column tile, 7
// or 13 K chunks): conv2 forward and conv2 data gradient
int fwd_wreg(const ConvPipeParams& p) {
  if (p.layout != XL_C8 || cdiv(p.Cout, 16) != 1) return 0;
  if (p.nchunks == 7 && p.in.mode == PM_PLAIN && p.epi == FE_POOL) return 7;
  if (p.nchunks == 13 && p.in.mode == PM_UNPOOL && p.epi == FE_PLAIN) return 13;
  return 0;
}

// Bank-conflict cycles of the K-loop A-fragment reads over one full group
// (the kernel's own row table, K table and tile walk, fed to the LDS bank
// model), and the number of read instructions they belong to.
std::pair<long, long> fwd_a_conflicts(const ConvPipeParams& p) {
  const PipeSrc& s = p.in;
  const bool S1 = p.layout == XL_S1, pool = p.epi == FE_POOL;
  const int rows_img = (pool ? (p.OH / 2) * (p.OW / 2) * 4 : p.OH * p.OW) / (p.pair ? 2 : 1);
  const int rows_pad = p.pair == 2 ? (rows_img + 15) & ~15 : rows_img;
  std::vector<int> ptab(rows_pad);
  for (int r = 0; r < rows_pad; ++r) {
    const int b = row_offset(r < rows_img ? r : 0, pool, p.OW, p.cs, p.ty0, p.tx0, s.LWp, S1 ? 1 : s.CL, p.pair);
    ptab[r] = S1 ? (b & 3) * s.CS + b - (b & 3) : b;
  }
  const int KK = p.KS * p.KS;
  std::vector<int> ktab(p.nchunks * 4);
  for (int gi = 0; gi < p.nchunks * 4; ++gi) {
    int off = 0;
    if (S1) {
      if (gi < p.KS) off = gi * s.LWp;
    } else {
      const int CG = s.CL >> 3, kp = gi / CG, cg = gi - kp * CG;
      if (kp < KK) off = ((kp / p.KS) * s.LWp + kp % p.KS) * s.CL + cg * 8;
    }
    ktab[gi] = off;
  }
  const int M = p.imgs * rows_img, tiles = p.pair == 2 ? p.imgs * (rows_pad / 16) : (M + 15) / 16;
  long extra = 0, instrs = 0;
  int a[64];
  for (int T = 0; T < tiles; ++T) {
    int base[16];
    for (int r16 = 0; r16 < 16; ++r16) {
      if (p.pair == 2) {
        const int tpi = rows_pad / 16, img = T / tpi;
        base[r16] = img * s.IMG + ptab[(T - img * tpi) * 16 + r16];
      } else {
        const int r = std::min(T * 16 + r16, M - 1), img = r / rows_img;
        base[r16] = img * s.IMG + ptab[r - img * rows_img];
      }
    }
    for (int q = 0; q < p.nchunks; ++q) {
      for (int half = 0; half < (S1 ? 2 : 1); ++half) {  // S1: two 8-byte reads
        for (int l = 0; l < 64; ++l) a[l] = (base[l & 15] + ktab[q * 4 + (l >> 4)]) / 2 + 2 * half;
        extra += lds_conflicts(a, S1 ? LDS_B64 : LDS_B128);
        ++instrs;
      }
    }
  }
  return {extra, instrs};
}

}  // namespace

// Swizzle by padding: pick the tile row stride (and for XL_S1 the stride
// between the shifted copies) with the fewest modelled bank conflicts per
// A-fragment read, keeping the workgroups per CU (LDS budget) -- if need be
// with up to a third fewer images per group.
static void fwd_pick_strides(ConvPipeParams& p) {
  PipeSrc& s = p.in;
  const bool s1 = p.layout == XL_S1;
  const int LW0 = s.LWp, CL = s1 ? 1 : s.CL, imgs0 = p.imgs;
  // the register-resident-weight kernels (fwd_wreg) hold 3 workgroups per CU
  // on VGPRs whatever the LDS allows
  const int cap = fwd_wreg(p) ? std::min(3, fwd_wgs_cap()) : fwd_wgs_cap();
  const int wgs = wgs_per_cu((size_t)fwd_layout(p).total, cap);
  const auto e0 = fwd_a_conflicts(p);
  double best = (double)e0.first / std::max(1L, e0.second);
  ConvPipeParams bp = p;
  const int step = s1 ? 4 : 1;
  for (int im = imgs0; im >= std::max(1, (2 * imgs0 + 2) / 3); --im) {
    for (int j = 0; j < 12; ++j) {
      for (int m = 0; m < (s1 ? 8 : 1); ++m) {
        ConvPipeParams q = p;
        q.imgs = im;
        q.in.LWp = LW0 + j * step;
        q.in.IMG = p.LH * q.in.LWp * CL;
        if (s1) q.in.CS = r8h(q.imgs * q.in.IMG + 8) + 8 * m;
        const FwdLayout L = fwd_layout(q);
        if ((size_t)L.total > kLdsPerCU || wgs_per_cu((size_t)L.total, cap) < wgs) continue;
        const auto e = fwd_a_conflicts(q);
        const double c = (double)e.first / std::max(1L, e.second);
        // fewer images per group (more barriers) only for a clear gain
        if (c < best - 1e-9 && (im == imgs0 || c < 0.5 * e0.first / std::max(1L, e0.second))) { best = c; bp = q; }
      }
    }
  }
  p = bp;
}

bool conv_pipe_plan(ConvPipeParams& p) {
  PipeSrc& s = p.in;
  const bool s1 = s.mode == PM_U8S1;
  if (s1 && (p.KS > 8 || p.Cin != 1)) return false;
  if (!s1 && s.SC != p.Cin) return false;
  if (p.Cout > 128) return false;
  p.layout = s1 ? XL_S1 : XL_C8;
  p.pair = s1 && p.Cout <= 8 && p.KS <= 7 && p.cs == 1 && (p.OW & 1) == 0 &&
           (p.epi == FE_POOL || (p.epi == FE_ACT && (p.act == ACT_RELU || p.act == ACT_NONE)));
  // window pairs (the second column half computes the next 2x2 window, taps
  // shifted by two): the pool is in-lane, no DPP exchange
  if (p.pair && p.epi == FE_POOL && p.KS <= 6 && (p.OW & 3) == 0 && (p.OH & 1) == 0)
    p.pair = 2;
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
  const int nt = p.pair ? 512 : 256;
  if (s.per_img > ni * nt) return false;
  int imgs = std::max(1, std::min(16, ni * nt / std::max(1, s.per_img)));
  for (; imgs >= 1; --imgs) {
    p.imgs = imgs;
    if (s1) s.CS = r8h(imgs * s.IMG + 8);
    if ((size_t)fwd_layout(p).total <= fwd_lds_target() || imgs == 1) break;
  }
  if (imgs < 1) return false;
  if ((size_t)fwd_layout(p).total > kLdsPerCU) return false;
  fwd_pick_strides(p);
  const FwdLayout L = fwd_layout(p);
  p.lds = (size_t)L.total;
  p.ngroups = cdiv(p.N, p.imgs);
  p.grid = std::min(p.ngroups, kCUs * wgs_per_cu(p.lds, fwd_wgs_cap()));
  return true;
}

void conv_pipe_forward(const ConvPipeParams& pin, hipStream_t st) {
  ConvPipeParams p = pin;
  {
    const bool pool = p.epi == FE_POOL;
    const int rows_img = (pool ? (p.OH / 2) * (p.OW / 2) * 4 : p.OH * p.OW) / (p.pair ? 2 : 1);
    // PAIR 2: the kernel divides tile indices by the (16-padded) tiles per image
    const Div d = Div::host(p.pair == 2 ? (rows_img + 15) / 16 : rows_img);
    p.rows_mh = d.mh;
    p.rows_ml = d.ml;
  }
  p.ngroups = cdiv(p.N, p.imgs);
  p.grid = std::min(p.ngroups, kCUs * wgs_per_cu(p.lds, fwd_wgs_cap()));
  if (p.grid <= 0) return;
  // the single-channel pair kernel has long per-group MFMA phases: 8 waves
  // hide more LDS latency; the others are barrier-bound at 4 waves
  const int nt = p.pair ? 512 : 256;
  const dim3 grid((unsigned)p.grid), block((unsigned)nt);
  auto go = [&](auto kern) { hipLaunchKernelGGL(kern, grid, block, p.lds, st, p); };
  switch (fwd_wreg(p)) {
    case 7: go(conv_pipe_fwd_kernel<PM_PLAIN, FE_POOL, ACT_RELU, 0, 256, 7>); return;
    case 13: go(conv_pipe_fwd_kernel<PM_UNPOOL, FE_PLAIN, ACT_NONE, 0, 256, 13>); return;
    default: break;
  }
#define MCC_PIPE_EPI(MODE)                                                                      \
  if (p.epi == FE_POOL) go(conv_pipe_fwd_kernel<MODE, FE_POOL, ACT_RELU, 0, 256>);                      \
  else if (p.epi == FE_PLAIN) go(conv_pipe_fwd_kernel<MODE, FE_PLAIN, ACT_NONE, 0, 256>);               \
  else if (p.act == ACT_RELU) go(conv_pipe_fwd_kernel<MODE, FE_ACT, ACT_RELU, 0, 256>);                 \
  else if (p.act == ACT_TANH) go(conv_pipe_fwd_kernel<MODE, FE_ACT, ACT_TANH, 0, 256>);                 \
  else go(conv_pipe_fwd_kernel<MODE, FE_ACT, ACT_NONE, 0, 256>);
  if (p.pair == 2) {
    go(conv_pipe_fwd_kernel<PM_U8S1, FE_POOL, ACT_RELU, 2, 512>);
    return;
  }
  if (p.pair) {
    if (p.epi == FE_POOL) go(conv_pipe_fwd_kernel<PM_U8S1, FE_POOL, ACT_RELU, 1, 512>);
    else if (p.act == ACT_RELU) go(conv_pipe_fwd_kernel<PM_U8S1, FE_ACT, ACT_RELU, 1, 512>);
    else go(conv_pipe_fwd_kernel<PM_U8S1, FE_ACT, ACT_NONE, 1, 512>);
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

}  // namespace gpu
}  // namespace mcc
