// Kernel table of the CPU executor's default (batched) mode: one baseline
// x86-64 build and one AVX2/FMA build of the same source
// (csrc/core/cpu_kernels.inc), chosen once at run time.
#pragma once

#include <cstdint>

namespace mcc {

template <typename T>
struct CpuKernels {
  // C[M][N] += A[M][K] B[K][N] (row-major, leading dimensions lda / ldb / ldc)
  void (*gemm_acc)(int64_t M, int64_t N, int64_t K, const T* A, int64_t lda, const T* B, int64_t ldb, T* C,
                   int64_t ldc) = nullptr;
  // dst[c][r] = src[r][c]
  void (*transpose)(const T* src, int64_t rows, int64_t cols, T* dst) = nullptr;
};

namespace cpu_base {
template <typename T> CpuKernels<T> kernels();
}
namespace cpu_v3 {
template <typename T> CpuKernels<T> kernels();
}

// The table for this CPU (AVX2+FMA when available).  MCC_AB=cpu_baseline forces
// the baseline build.
template <typename T> const CpuKernels<T>& cpu_kernels();

}  // namespace mcc
