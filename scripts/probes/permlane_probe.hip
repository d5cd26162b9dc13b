// Prints the lane mapping of gfx950's v_permlane16_swap / v_permlane32_swap
// (the 4x4 cross-row transpose of xconv's pixel-shuffle epilogue relies on it).
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(int *o) {
  const int l = threadIdx.x;
  const int a = l, b = 100 + l;
  const auto r = __builtin_amdgcn_permlane16_swap(a, b, false, false);
  const auto q = __builtin_amdgcn_permlane32_swap(a, b, false, false);
  o[l] = r[0];
  o[64 + l] = r[1];
  o[128 + l] = q[0];
  o[192 + l] = q[1];
}
int main() {
  int *d, h[256];
  if (hipMalloc(&d, sizeof(h)) != hipSuccess) return 1;
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
  if (hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost) != hipSuccess) return 2;
  const char *nm[4] = {"p16 first", "p16 second", "p32 first", "p32 second"};
  for (int i = 0; i < 4; ++i) {
    printf("%s:", nm[i]);
    for (int l = 0; l < 64; l += 4) printf(" %d", h[i * 64 + l]);
    printf("\n");
  }
  hipFree(d);
  return 0;
}
