// AVX2 + FMA build of the CPU kernels (see cpu_kernels.inc); compiled
// with -mavx2 -mfma and only called when the CPU supports both.
#define MCC_CPU_NS cpu_v3
#include "cpu_kernels.inc"
