// membench.hip -- memory-pattern ceilings for the block-transform kernel (not product code).
// Measures, on 8 x 4K frames (597 MB moved), the HBM rate of:
//   rd      : the transform's input pattern only (lane = block, 8 rows x 24 B)
//   wr_lane : output pattern of the transform (lane writes its own 128-B block, 8 x 16 B)
//   wr_coal : coalesced output (consecutive lanes write consecutive 16 B)
//   rw_lane : input pattern + per-lane output pattern, trivial compute
//   rw_coal : input pattern + coalesced output (data exchanged through LDS)
//   copy    : float4 copy of the same byte count (reference point)
// Build: hipcc --offload-arch=gfx950 -O3 tools/membench.hip -o tools/membench
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

struct Geo { const uint8_t *in; uint8_t *out; int bpr, nb, nframes; long long pitch, fstride; };

__device__ __forceinline__ void load_rows(const Geo &g, unsigned b, uint32_t (&raw)[8][6])
{
    const unsigned f = b / g.nb, bi = b - f * g.nb, r = bi / g.bpr, c = bi - r * g.bpr;
    const uint8_t *base = g.in + (long long)f * g.fstride + 8ll * r * g.pitch + 24ll * c;
#pragma unroll
    for (int y = 0; y < 8; y++) {
        const uint8_t *p = (const uint8_t *)__builtin_assume_aligned(base + y * g.pitch, 8);
        u32x4 a; u32x2 bb;
        __builtin_memcpy(&a, p, 16); __builtin_memcpy(&bb, p + 16, 8);
        raw[y][0] = a.x; raw[y][1] = a.y; raw[y][2] = a.z; raw[y][3] = a.w; raw[y][4] = bb.x; raw[y][5] = bb.y;
    }
}

template <int MODE>  // 1 = read, 2 = write per-lane, 4 = write coalesced
__global__ __launch_bounds__(256) void k_pattern(Geo g)
{
    __shared__ u32x4 stage[4][64 * 8 + 8];
    const unsigned total = g.nb * g.nframes;
    const unsigned b = blockIdx.x * 256 + threadIdx.x;
    if (b >= total) return;
    uint32_t acc = b * 2654435761u;
    uint32_t raw[8][6];
    if (MODE & 1) {
        load_rows(g, b, raw);
#pragma unroll
        for (int y = 0; y < 8; y++)
#pragma unroll
            for (int k = 0; k < 6; k++) acc = acc * 31u + raw[y][k];
        if (!(MODE & 6) && acc == 0x12345u) g.out[b] = 1;   /* keep the loads alive */
    }
    const unsigned f = b / g.nb, bi = b - f * g.nb;
    for (int ch = 0; ch < 3; ch++) {
        u32x4 *o = (u32x4 *)(g.out + ((long long)f * 3 * g.nb + (long long)ch * g.nb + bi) * 128);
        if (MODE & 2) {
#pragma unroll
            for (int j = 0; j < 8; j++) o[j] = u32x4{acc + j, acc ^ j, acc + ch, acc};
        }
        if (MODE & 4) {
            const unsigned w = threadIdx.x >> 6, l = threadIdx.x & 63;
#pragma unroll
            for (int j = 0; j < 8; j++) stage[w][l * 8 + j + (l >> 3)] = u32x4{acc + j, acc ^ j, acc + ch, acc};
            __builtin_amdgcn_s_barrier();
            // wave writes its 64 blocks x 128 B = 8 KB contiguous: instruction j covers 1 KB
            const unsigned b0 = b - l;  // first block of this wave (same frame assumed)
            u32x4 *ow = (u32x4 *)(g.out + ((long long)f * 3 * g.nb + (long long)ch * g.nb + (bi - l)) * 128);
            (void)b0;
#pragma unroll
            for (int j = 0; j < 8; j++) {
                const unsigned e = j * 64 + l;             // 16-B element of the 8 KB span
                const unsigned blk = e >> 3, part = e & 7;
                ow[e] = stage[w][blk * 8 + part + (blk >> 3)];
            }
            __builtin_amdgcn_s_barrier();
        }
    }
}

__global__ void k_copy(const u32x4 *in, u32x4 *out, size_t n)
{
    for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) out[i] = in[i];
}

int main()
{
    const int W = 3840, H = 2160, F = 8;
    Geo g;
    g.bpr = W / 8; g.nb = (W / 8) * (H / 8); g.nframes = F; g.pitch = W * 3; g.fstride = (long long)W * H * 3;
    const size_t in_bytes = (size_t)F * g.fstride, out_bytes = (size_t)F * g.nb * 3 * 128;
    uint8_t *din, *dout;
    CK(hipMalloc(&din, in_bytes)); CK(hipMalloc(&dout, out_bytes));
    CK(hipMemset(din, 7, in_bytes)); CK(hipMemset(dout, 0, out_bytes));
    g.in = din; g.out = dout;
    const unsigned total = g.nb * F, grid = (total + 255) / 256;
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    auto run = [&](const char *name, auto launch, double bytes) {
        for (int i = 0; i < 3; i++) launch();
        CK(hipDeviceSynchronize());
        const int it = 20;
        CK(hipEventRecord(e0));
        for (int i = 0; i < it; i++) launch();
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms; CK(hipEventElapsedTime(&ms, e0, e1));
        ms /= it;
        printf("%-8s %8.1f us  %7.1f GB/s\n", name, ms * 1e3, bytes / (ms * 1e-3) / 1e9);
    };
    run("rd", [&] { hipLaunchKernelGGL(k_pattern<1>, dim3(grid), dim3(256), 0, 0, g); }, (double)in_bytes);
    run("wr_lane", [&] { hipLaunchKernelGGL(k_pattern<2>, dim3(grid), dim3(256), 0, 0, g); }, (double)out_bytes);
    run("wr_coal", [&] { hipLaunchKernelGGL(k_pattern<4>, dim3(grid), dim3(256), 0, 0, g); }, (double)out_bytes);
    run("rw_lane", [&] { hipLaunchKernelGGL(k_pattern<3>, dim3(grid), dim3(256), 0, 0, g); }, (double)(in_bytes + out_bytes));
    run("rw_coal", [&] { hipLaunchKernelGGL(k_pattern<5>, dim3(grid), dim3(256), 0, 0, g); }, (double)(in_bytes + out_bytes));
    const size_t n16 = out_bytes / 2 / 16;   /* copy half of the output buffer onto its other half */
    run("copy", [&] { hipLaunchKernelGGL(k_copy, dim3(4096), dim3(256), 0, 0, (const u32x4 *)dout, (u32x4 *)dout + n16, n16); }, (double)n16 * 32);
    return 0;
}
