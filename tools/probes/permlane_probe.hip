// v_permlane16_swap_b32 semantics probe: a = lane, b = 100 + lane; prints both results per lane.
#include <hip/hip_runtime.h>
#include <stdio.h>
__global__ void k(unsigned *o) {
  unsigned l = threadIdx.x;
  auto r = __builtin_amdgcn_permlane16_swap(l, 100u + l, false, false);
  o[l] = r[0]; o[64 + l] = r[1];
}
int main() {
  unsigned *d, h[128];
  hipMalloc(&d, 512);
  k<<<1, 64>>>(d);
  hipMemcpy(h, d, 512, hipMemcpyDeviceToHost);
  for (int l = 0; l < 64; l += 4) printf("lane %2d: r0 %3u r1 %3u\n", l, h[l], h[64 + l]);
  return 0;
}
