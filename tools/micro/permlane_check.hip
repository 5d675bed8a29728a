// Prints what v_permlane32_swap / v_permlane16_swap do on gfx950 (dev check).
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(unsigned* out) {
  const unsigned l = threadIdx.x;
  unsigned x = 1000 + l, y = 2000 + l;
  auto r = __builtin_amdgcn_permlane32_swap(x, y, false, false);
  auto s = __builtin_amdgcn_permlane16_swap(x, y, false, false);
  out[l] = r[0];
  out[64 + l] = r[1];
  out[128 + l] = s[0];
  out[192 + l] = s[1];
}
int main() {
  unsigned* d;
  (void)hipMalloc(&d, 256 * 4);
  k<<<1, 64>>>(d);
  unsigned h[256];
  (void)hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost);
  const char* nm[4] = {"p32[0]", "p32[1]", "p16[0]", "p16[1]"};
  for (int i = 0; i < 4; ++i) {
    printf("%s:", nm[i]);
    for (int l = 0; l < 64; ++l) printf(" %u", h[64 * i + l]);
    printf("\n");
  }
  return 0;
}
