// fp32 weight gradient of a fully-connected layer with a skinny output:
//   dW[m][n] = sum_k dZ[k][m] X[k][n],  db[m] = sum_k dZ[k][m]
// (Layer_feedBack_full's dW / db loops, /root/reference/cnn.c:154-173), for
// Nout <= 208 outputs and K = the batch (163,840 at the bench): the ref
// model's FC1 (200 x 1568) and LeNet-5's FC1 (120 x 400).
//
// The generic 64 x 64 split-K GEMM spent 1.86 ms on the ref FC1 shape: 200
// rows in 64-row tiles compute 256 (22 % padding), and each of the 4 row
// tiles re-streams the 1 GB activation X. Here one workgroup owns ALL
// output rows (13 or 8 blocks of 16) for a 16 * NW column slice:
//  * NW waves, wave w: columns 16 w .. 16 w + 15 x every row block, so X is
//    read once per split and dZ once per column slice (7 / 5 slices);
//  * v_mfma_f32_16x16x4_f32 (exact fp32), lane (r, g) supplying
//    A[16 b + r][k g] = dZ[k][16 b + r] and B[k g][n] = X[k][n];
//  * K chunks of 16 rows, double-buffered in LDS (16-byte copies as the rows
//    sit in memory: no transposes), register prefetch of chunk c + 1;
//  * db on the VALU from the staged dZ chunk (column slice 0, thread m);
//  * split-K partials [S][Nout][ldp] (bias in column N), summed in a fixed
//    order by dw_reduce (deterministic).
#include "kernels.h"
#include "mfma.h"

#include <algorithm>

namespace mcc {
namespace gpu {
namespace {

constexpr int kKc = 16;  // K rows per LDS chunk (4 MFMA k-steps)

template <int MB, int NW>
__global__ void __launch_bounds__(64 * NW) fc_dw32_kernel(FcDw32Params p) {
  // A chunk pitch (floats): rows k and k + 1 of a fragment read 16 banks apart
  constexpr int MP = 16 * MB + (MB % 2 == 0 ? 16 : 0);
  constexpr int NT = 16 * NW;  // columns per workgroup (B chunk pitch)
  constexpr int NTH = 64 * NW;
  constexpr int AV = kKc * MP / 4;  // float4 slots of an A chunk (padding included)
  constexpr int APER = (AV + NTH - 1) / NTH;
  static_assert(kKc * NT / 4 == NTH, "one B float4 per thread");
  __shared__ __attribute__((aligned(16))) float As[2][kKc * MP];
  __shared__ __attribute__((aligned(16))) float Bs[2][kKc * NT];

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int r = lane & 15, g = lane >> 4;
  const int n0 = blockIdx.x * NT;
  const int chunks = (p.K + kKc - 1) / kKc;
  const int per = (chunks + (int)gridDim.y - 1) / (int)gridDim.y;
  const int c0 = blockIdx.y * per, c1 = min(chunks, c0 + per);
  const bool dbw = blockIdx.x == 0 && tid < p.M;  // column slice 0: thread m sums dZ[.][m]

  f32x4 acc[MB];
#pragma unroll
  for (int b = 0; b < MB; ++b) acc[b] = f32x4{0.f, 0.f, 0.f, 0.f};
  float dbs = 0.f;

  // global -> register staging of one chunk
  f32x4 ra[APER], rb;
  auto load = [&](int c) {
    const int k0 = c * kKc;
#pragma unroll
    for (int j = 0; j < APER; ++j) {
      const int v = tid + j * NTH;
      const int kr = v / (MP / 4), m4 = (v - kr * (MP / 4)) * 4;
      ra[j] = (v < AV && k0 + kr < p.K && m4 < p.M)
                  ? *reinterpret_cast<const f32x4*>(p.dz + (size_t)(k0 + kr) * p.ldz + m4)
                  : f32x4{0.f, 0.f, 0.f, 0.f};
    }
    const int kr = tid / (NT / 4), n4 = (tid - kr * (NT / 4)) * 4;
    rb = (k0 + kr < p.K && n0 + n4 < p.N) ? *reinterpret_cast<const f32x4*>(p.x + (size_t)(k0 + kr) * p.ldx + n0 + n4)
                                          : f32x4{0.f, 0.f, 0.f, 0.f};
  };
  auto store = [&](int buf) {
#pragma unroll
    for (int j = 0; j < APER; ++j) {
      const int v = tid + j * NTH;
      if (v < AV) *reinterpret_cast<f32x4*>(&As[buf][v * 4]) = ra[j];
    }
    *reinterpret_cast<f32x4*>(&Bs[buf][tid * 4]) = rb;
  };

  if (c0 < c1) {
    load(c0);
    store(0);
  }
  __syncthreads();
  int buf = 0;
  for (int c = c0; c < c1; ++c) {
    const bool more = c + 1 < c1;
    if (more) load(c + 1);
    const float* A = As[buf];
    const float* Bm = Bs[buf];
#pragma unroll
    for (int ks = 0; ks < kKc / 4; ++ks) {
      const int kk = 4 * ks + g;
      const float bv = Bm[kk * NT + 16 * w + r];
      float av[MB];
#pragma unroll
      for (int b = 0; b < MB; ++b) av[b] = A[kk * MP + 16 * b + r];
#pragma unroll
      for (int b = 0; b < MB; ++b) acc[b] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[b], bv, acc[b], 0, 0, 0);
    }
    if (dbw) {
#pragma unroll
      for (int k = 0; k < kKc; ++k) dbs += A[k * MP + tid];
    }
    if (more) store(buf ^ 1);
    __syncthreads();
    buf ^= 1;
  }

  // partial slab of split blockIdx.y: rows m = 16 b + 4 g + i, column n0 + 16 w + r
  float* part = p.slab + (size_t)blockIdx.y * p.slab_stride;
  const int n = n0 + 16 * w + r;
  if (n < p.N) {
#pragma unroll
    for (int b = 0; b < MB; ++b)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int m = 16 * b + 4 * g + i;
        if (m < p.M) part[(size_t)m * p.ldp + n] = acc[b][i];
      }
  }
  if (dbw) part[(size_t)tid * p.ldp + p.N] = dbs;
}

template <int MB, int NW>
void launch(const FcDw32Params& p, hipStream_t s) {
  const dim3 grid((unsigned)((p.N + 16 * NW - 1) / (16 * NW)), (unsigned)p.splitk);
  hipLaunchKernelGGL((fc_dw32_kernel<MB, NW>), grid, dim3(64 * NW), 0, s, p);
}

// column-slice width: the widest of 7 / 5 / 4 waves that tiles N exactly
int pick_nw(int N) {
  for (int nw : {7, 5, 4})
    if (N % (16 * nw) == 0) return nw;
  return 7;
}

}  // namespace

// N >= 192: narrower inputs leave most of a 16 * NW column slice idle (LeNet's
// FC2, 84 x 120: 116 us here vs 74 us on the generic GEMM)
bool fc_dw32_supported(int M, int N, int ldz, int ldx) {
  return M > 0 && M <= 208 && N >= 192 && M % 4 == 0 && N % 4 == 0 && ldz % 4 == 0 && ldx % 4 == 0;
}

int fc_dw32_splitk(int M, int N, int64_t K) {
  const int slices = (N + 16 * pick_nw(N) - 1) / (16 * pick_nw(N));
  // ~3 workgroups per CU, and at least 32 chunks (512 rows) per split
  const int64_t chunks = (K + kKc - 1) / kKc;
  int sk = (int)std::max<int64_t>(1, 768 / slices);
  sk = (int)std::min<int64_t>(sk, std::max<int64_t>(1, chunks / 32));
  (void)M;
  return std::max(1, sk);
}

void fc_dw32(const FcDw32Params& p, hipStream_t s) {
  MCC_CHECK(fc_dw32_supported(p.M, p.N, p.ldz, p.ldx), "fc_dw32: unsupported shape");
  MCC_CHECK(p.splitk >= 1 && p.ldp >= p.N + 1, "fc_dw32: bad split / partial pitch");
  const int nw = pick_nw(p.N);
  if (p.M <= 128) {
    if (nw == 7) launch<8, 7>(p, s);
    else if (nw == 5) launch<8, 5>(p, s);
    else launch<8, 4>(p, s);
  } else {
    if (nw == 7) launch<13, 7>(p, s);
    else if (nw == 5) launch<13, 5>(p, s);
    else launch<13, 4>(p, s);
  }
}

}  // namespace gpu
}  // namespace mcc
