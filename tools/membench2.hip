// membench2.hip -- streaming ceilings for a 1:2 read:write byte mix (not product code).
// F x 4K frames (argv[1], default 8): 3 B/px read (RGB) + 6 B/px written, like the kernels.
//   ideal     : every lane reads 16 B and writes 2 x 16 B, all perfectly coalesced, persistent
//   ideal_nt  : same with nontemporal stores
//   ideal_np  : same, one element per thread (non-persistent grid)
//   rd_only   : the 199 MB read alone (coalesced)
//   wr_only   : the 398 MB write alone (coalesced)
//   copy      : float4 copy of 199 MB -> 199 MB
// Build: hipcc --offload-arch=gfx950 -O3 tools/membench2.hip -o tools/membench2
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <int NT>
__global__ __launch_bounds__(256) void k_ideal(const u32x4 *__restrict__ in, u32x4 *__restrict__ out,
                                               size_t n)
{
    for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
        const u32x4 v = in[i];
        const u32x4 a = v * 3u, b = v ^ 0x5a5a5a5au;
        if (NT) {
            __builtin_nontemporal_store(a, out + i);
            __builtin_nontemporal_store(b, out + n + i);
        } else {
            out[i] = a;
            out[n + i] = b;
        }
    }
}

__global__ __launch_bounds__(256) void k_rd(const u32x4 *__restrict__ in, u32x4 *__restrict__ out, size_t n)
{
    u32x4 acc = {0, 0, 0, 0};
    for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) acc ^= in[i];
    if (acc.x == 0x12345u && acc.y == 7u) out[0] = acc;
}

template <int NT>
__global__ __launch_bounds__(256) void k_wr(u32x4 *__restrict__ out, size_t n)
{
    for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
        const u32x4 v = {(uint32_t)i, 1u, 2u, 3u};
        if (NT) __builtin_nontemporal_store(v, out + i);
        else out[i] = v;
    }
}

__global__ void k_copy(const u32x4 *in, u32x4 *out, size_t n)
{
    for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) out[i] = in[i];
}

int main(int argc, char **argv)
{
    /* argv[1]: 4K frames of input (default 8 = 199 MB, under the 256 MiB Infinity Cache; 16+
     * streams from HBM) */
    const size_t frames = argc > 1 ? (size_t)atoi(argv[1]) : 8;
    const size_t in_bytes = frames * 3840 * 2160 * 3, out_bytes = 2 * in_bytes;
    const size_t n = in_bytes / 16;
    u32x4 *din, *dout;
    CK(hipMalloc(&din, in_bytes));
    CK(hipMalloc(&dout, out_bytes));
    CK(hipMemset(din, 7, in_bytes));
    CK(hipMemset(dout, 0, out_bytes));
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto run = [&](const char *name, auto launch, double bytes) {
        for (int i = 0; i < 200; i++) launch();      /* settle: the GPU's ramp out of idle */
        CK(hipDeviceSynchronize());
        const int it = 20;
        CK(hipEventRecord(e0));
        for (int i = 0; i < it; i++) launch();
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        ms /= it;
        printf("%-10s %8.1f us  %7.1f GB/s\n", name, ms * 1e3, bytes / (ms * 1e-3) / 1e9);
    };
    const double all = (double)(in_bytes + out_bytes);
    for (int per_cu : {4, 8, 16}) {
        const unsigned grid = cus * per_cu;
        printf("-- persistent grid %u (%d WG/CU)\n", grid, per_cu);
        run("ideal", [&] { hipLaunchKernelGGL(k_ideal<0>, dim3(grid), dim3(256), 0, 0, din, dout, n); }, all);
        run("ideal_nt", [&] { hipLaunchKernelGGL(k_ideal<1>, dim3(grid), dim3(256), 0, 0, din, dout, n); }, all);
        run("rd_only", [&] { hipLaunchKernelGGL(k_rd, dim3(grid), dim3(256), 0, 0, din, dout, n); }, (double)in_bytes);
        run("wr_only", [&] { hipLaunchKernelGGL(k_wr<0>, dim3(grid), dim3(256), 0, 0, dout, 2 * n); }, (double)out_bytes);
        run("wr_nt", [&] { hipLaunchKernelGGL(k_wr<1>, dim3(grid), dim3(256), 0, 0, dout, 2 * n); }, (double)out_bytes);
        run("copy", [&] { hipLaunchKernelGGL(k_copy, dim3(grid), dim3(256), 0, 0, din, dout, n); }, 2.0 * in_bytes);
    }
    const unsigned gnp = (unsigned)((n + 255) / 256);
    run("ideal_np", [&] { hipLaunchKernelGGL(k_ideal<0>, dim3(gnp), dim3(256), 0, 0, din, dout, n); }, all);
    run("ideal_np_nt", [&] { hipLaunchKernelGGL(k_ideal<1>, dim3(gnp), dim3(256), 0, 0, din, dout, n); }, all);
    return 0;
}
