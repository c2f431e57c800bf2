// Probe of cross-lane primitive semantics on gfx950: permlane16/32 swap pairs and DPP row_ror.
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(int* o) {
  const int l = threadIdx.x;
  const unsigned u = (unsigned)l;
  auto a = __builtin_amdgcn_permlane32_swap(u, u, false, false);
  auto b = __builtin_amdgcn_permlane16_swap(u, u, false, false);
  const int r = __builtin_amdgcn_mov_dpp(l, 0x120 + 15, 0xF, 0xF, false);
  o[l * 5 + 0] = a[0];
  o[l * 5 + 1] = a[1];
  o[l * 5 + 2] = b[0];
  o[l * 5 + 3] = b[1];
  o[l * 5 + 4] = r;
}
int main() {
  int* d;
  hipMalloc(&d, 64 * 5 * 4);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
  int h[320];
  hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  printf("lane: p32[0] p32[1] p16[0] p16[1] ror15\n");
  for (int l = 0; l < 64; ++l)
    printf("%2d: %2d %2d %2d %2d %2d\n", l, h[l * 5], h[l * 5 + 1], h[l * 5 + 2], h[l * 5 + 3], h[l * 5 + 4]);
  return 0;
}
