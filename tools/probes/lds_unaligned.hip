// Probe: cost of misaligned ds_read_b128 / ds_read_b64 on gfx950 (unaligned
// DS access mode).  Each lane reads 16 (8) bytes at element offset
// lane*STRIDE + OFF (bf16 elements) in a loop; prints us per launch.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));

template <int BYTES>
__global__ void __launch_bounds__(256) probe(unsigned* out, int off_el, int stride_el, int iters) {
  __shared__ __attribute__((aligned(16))) unsigned short s[32768];
  for (int i = threadIdx.x; i < 32768; i += 256) s[i] = (unsigned short)(i * 2654435761u >> 16);
  __syncthreads();
  unsigned acc = 0;
  int base = (threadIdx.x & 63) * stride_el + off_el + (threadIdx.x >> 6) * 4096;
  for (int it = 0; it < iters; ++it) {
    const char* p = reinterpret_cast<const char*>(s + base + ((it & 7) << 9));
    if constexpr (BYTES == 16) {
      u32x4 v;
      __builtin_memcpy(&v, p, 16);
      acc ^= v.x + v.y + v.z + v.w;
    } else {
      u32x2 v;
      __builtin_memcpy(&v, p, 8);
      acc ^= v.x + v.y;
    }
    asm volatile("" : "+v"(acc));
  }
  out[blockIdx.x * 256 + threadIdx.x] = acc;
}

int main() {
  unsigned* d;
  hipMalloc(&d, 1024 * 256 * 4);
  hipEvent_t a, b;
  hipEventCreate(&a); hipEventCreate(&b);
  const int iters = 4096;
  for (int bytes : {16, 8}) {
    for (int stride : {8, 12}) {
      for (int off : {0, 1, 2, 3, 4}) {
        float best = 1e9;
        for (int rep = 0; rep < 5; ++rep) {
          hipEventRecord(a);
          if (bytes == 16) hipLaunchKernelGGL(probe<16>, dim3(1024), dim3(256), 0, 0, d, off, stride, iters);
          else hipLaunchKernelGGL(probe<8>, dim3(1024), dim3(256), 0, 0, d, off, stride, iters);
          hipEventRecord(b);
          hipEventSynchronize(b);
          float ms; hipEventElapsedTime(&ms, a, b);
          if (ms < best) best = ms;
        }
        // reads per CU: 4 blocks/CU x 4 waves x iters
        const double rd = 1024.0 * 4 * iters;
        printf("b%d stride_el %2d off_el %d: %.3f ms  %.2f cycles/wave-read/CU @2.1GHz\n", bytes * 8, stride, off, best,
               best * 1e-3 * 2.1e9 / (rd / 256));
      }
    }
  }
  return 0;
}
