// Probe of ds_read_b64_tr_b16 lane semantics (diagnostic, not part of the build).
#include <hip/hip_runtime.h>
#include <cstdio>
typedef short v4s __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) v4s lds_v4s;
__global__ void probe(short* out) {
  __shared__ short lds[16 * 64];
  for (int i = threadIdx.x; i < 16 * 64; i += 64) lds[i] = (short)((i / 64) * 100 + (i % 64));
  __syncthreads();
  const int l = threadIdx.x, g = l >> 4, i16 = l & 15, q = i16 >> 2, p = i16 & 3;
  short* a = lds + (4 * g + q) * 64 + 4 * p;
  v4s v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)a);
  for (int e = 0; e < 4; ++e) out[l * 4 + e] = v[e];
}
int main() {
  short* d; hipMalloc(&d, 64 * 4 * 2);
  hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, d);
  short h[256]; hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  for (int l = 0; l < 64; ++l) printf("lane %2d: %5d %5d %5d %5d\n", l, h[l*4], h[l*4+1], h[l*4+2], h[l*4+3]);
  return 0;
}
