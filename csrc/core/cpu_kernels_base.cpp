// Baseline x86-64 build of the CPU kernels (see cpu_kernels.inc).
#define MCC_CPU_NS cpu_base
#include "cpu_kernels.inc"
