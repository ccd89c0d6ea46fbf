// Probe of ds_read_b64_tr_b16 lane semantics: LDS [16 rows][16 cols] bf16 bits = row*16+col.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef short s16x4 __attribute__((ext_vector_type(4)));
__global__ void k(short* out) {
  __shared__ short lds[16 * 16];
  for (int i = threadIdx.x; i < 256; i += 64) lds[i] = (short)i;
  __syncthreads();
  const int l = threadIdx.x, g = l >> 4, q = (l & 15) >> 2, p = l & 3;
  const int row = 4 * g + q, col = 4 * p;
  typedef __attribute__((address_space(3))) s16x4 L;
  s16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((L*)(lds + row * 16 + col));
  for (int j = 0; j < 4; ++j) out[l * 4 + j] = v[j];
}
int main() {
  short* d; hipMalloc(&d, 64 * 4 * 2);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
  short h[256]; hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  for (int l = 0; l < 64; ++l) {
    printf("lane %2d:", l);
    for (int j = 0; j < 4; ++j) printf(" (r%d,c%d)", h[l * 4 + j] / 16, h[l * 4 + j] % 16);
    printf("\n");
  }
  return 0;
}
