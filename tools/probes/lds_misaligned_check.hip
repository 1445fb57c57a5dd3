// Probe: do misaligned ds_read_b128 / ds_read_b64 return the right bytes on
// gfx950 (unaligned DS access mode), and at what cost?  Each lane reads 16 (8)
// bytes at byte offset lane*STRIDE + OFF from a pattern buffer in LDS; the
// result is compared with the expected bytes on the host.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));

template <int BYTES>
__global__ void __launch_bounds__(256) check(unsigned* out, int off, int stride) {
  __shared__ __attribute__((aligned(16))) unsigned char s[16384];
  for (int i = threadIdx.x; i < 16384; i += 256) s[i] = (unsigned char)(i * 7 + (i >> 8));
  __syncthreads();
  int o = off;
  asm volatile("" : "+v"(o));
  const unsigned char* p = s + (threadIdx.x & 63) * stride + o;
  if constexpr (BYTES == 16) {
    const u32x4 v = *reinterpret_cast<const u32x4*>(p);
    for (int k = 0; k < 4; ++k) out[threadIdx.x * 4 + k] = v[k];
  } else {
    const u32x2 v = *reinterpret_cast<const u32x2*>(p);
    for (int k = 0; k < 2; ++k) out[threadIdx.x * 4 + k] = v[k];
  }
}

template <int BYTES>
__global__ void __launch_bounds__(256) timing(unsigned* out, int off, int stride, int iters) {
  __shared__ __attribute__((aligned(16))) unsigned char s[32768];
  for (int i = threadIdx.x; i < 32768; i += 256) s[i] = (unsigned char)i;
  __syncthreads();
  unsigned acc = 0;
  int o = off + (threadIdx.x & 63) * stride + (threadIdx.x >> 6) * 4096;
  asm volatile("" : "+v"(o));
  for (int it = 0; it < iters; ++it) {
    const unsigned char* p = s + o + ((it & 3) << 10);
    if constexpr (BYTES == 16) {
      const u32x4 v = *reinterpret_cast<const u32x4*>(p);
      acc ^= v.x + v.y + v.z + v.w;
    } else {
      const u32x2 v = *reinterpret_cast<const u32x2*>(p);
      acc ^= v.x + v.y;
    }
    asm volatile("" : "+v"(acc));
  }
  out[blockIdx.x * 256 + threadIdx.x] = acc;
}

int main() {
  unsigned *d, h[1024];
  hipMalloc(&d, 1024 * 256 * 4);
  for (int bytes : {16, 8})
    for (int off : {0, 2, 4, 6, 8, 10, 12, 14}) {
      const int stride = 36;  // bytes between lanes (a 18-element row pitch)
      if (bytes == 16) hipLaunchKernelGGL(check<16>, dim3(1), dim3(256), 0, 0, d, off, stride);
      else hipLaunchKernelGGL(check<8>, dim3(1), dim3(256), 0, 0, d, off, stride);
      hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
      int bad = 0;
      for (int t = 0; t < 256; ++t)
        for (int k = 0; k < bytes / 4; ++k) {
          unsigned e = 0;
          for (int b = 0; b < 4; ++b) {
            const int i = (t & 63) * stride + off + 4 * k + b;
            e |= (unsigned)(unsigned char)(i * 7 + (i >> 8)) << (8 * b);
          }
          bad += h[t * 4 + k] != e;
        }
      printf("b%d off %2d: %s (%d bad words)\n", bytes * 8, off, bad ? "WRONG" : "ok", bad);
    }
  hipEvent_t a, b;
  hipEventCreate(&a); hipEventCreate(&b);
  const int iters = 4096;
  for (int bytes : {16, 8})
    for (int stride : {16, 36, 72})
      for (int off : {0, 2, 4, 8}) {
        float best = 1e9;
        for (int rep = 0; rep < 3; ++rep) {
          hipEventRecord(a);
          if (bytes == 16) hipLaunchKernelGGL(timing<16>, dim3(1024), dim3(256), 0, 0, d, off, stride, iters);
          else hipLaunchKernelGGL(timing<8>, dim3(1024), dim3(256), 0, 0, d, off, stride, iters);
          hipEventRecord(b);
          hipEventSynchronize(b);
          float ms; hipEventElapsedTime(&ms, a, b);
          if (ms < best) best = ms;
        }
        const double rd = 1024.0 * 4 * iters;  // wave-reads over the chip
        printf("time b%d stride %2d off %d: %.3f ms  %.2f cycles/wave-read/CU @2.1GHz\n", bytes * 8, stride, off,
               best, best * 1e-3 * 2.1e9 / (rd / 256));
      }
  return 0;
}
