// Probe: semantics of ds_read_b64_tr_b16 (__builtin_amdgcn_ds_read_tr16_b64_v4i16) on gfx950.
// LDS holds a 32 x 64 matrix of 16-bit values v = row*64 + col; lane 4q+p of each 16-lane group
// g supplies the address of row (4g + q), columns 4p..4p+3.  Prints what each lane receives.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef short v4s __attribute__((ext_vector_type(4)));
__global__ void k(short* out) {
  __shared__ short lds[32 * 64];
  for (int i = threadIdx.x; i < 32 * 64; i += 64) lds[i] = (short)i;
  __syncthreads();
  const int l = threadIdx.x, g = l >> 4, q = (l & 15) >> 2, p = l & 3;
  const int row = 4 * g + q, col = 4 * p;
  v4s r = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (__attribute__((address_space(3))) v4s*)(lds + row * 64 + col));
  for (int j = 0; j < 4; ++j) out[l * 4 + j] = r[j];
}
int main() {
  short* d; hipMalloc(&d, 64 * 4 * 2);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
  short h[256]; hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  for (int l = 0; l < 64; ++l) {
    printf("lane %2d:", l);
    for (int j = 0; j < 4; ++j) printf(" (r%2d,c%2d)", h[l * 4 + j] / 64, h[l * 4 + j] % 64);
    printf("\n");
  }
  return 0;
}
