// Semantics probe for v_permlane32_swap_b32 / v_permlane16_swap_b32 on gfx950 (diagnostic).
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(unsigned *o) {
    const unsigned l = threadIdx.x;
    auto r = __builtin_amdgcn_permlane32_swap(100 + l, 200 + l, false, false);
    o[l] = r[0]; o[64 + l] = r[1];
    auto s = __builtin_amdgcn_permlane16_swap(100 + l, 200 + l, false, false);
    o[128 + l] = s[0]; o[192 + l] = s[1];
}
int main() {
    unsigned *d, h[256];
    hipMalloc(&d, sizeof h);
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
    hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost);
    const char *nm[4] = {"p32 vdst(100+l)", "p32 src(200+l)", "p16 vdst(100+l)", "p16 src(200+l)"};
    for (int t = 0; t < 4; t++) {
        printf("%s:", nm[t]);
        for (int l = 0; l < 64; l += 4) printf(" %u", h[t * 64 + l]);
        printf("\n");
    }
    return 0;
}
