/*
 * pk_hazard4.hip -- round-5 probe of the rows-12..15 fault: packed-fp32 VALU (jx_fdct8_pk's
 * v_pk_*_f32, as k_mxs's column pass) on one wave while OTHER waves of the same SIMD have memory
 * data returning into their VGPRs.  Workgroups alternate roles: even blocks compute (per iteration
 * optionally four + eight v_mfma_f32_16x16x32_f16 products, then the packed 8-point DCT of per-lane
 * pseudo-random rows, checked bit for bit against the same arithmetic in scalar fp32), odd blocks
 * load (LOAD: 0 none, 1 global_load_dwordx4 streams into VGPRs, 2 ds_read_b128 into VGPRs,
 * 3 global_load_lds_dwordx4, i.e. LDS-DMA: no VGPR data).  Wrong packed results are counted per
 * 16-lane group.  Usage: ./pk_hazard4 [blocks] [iters] [0: loader modes | 1: fence modes]
 * Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -fno-slp-vectorize
 *        -I jpeg-encoder-and-decoder_amd/csrc -o tools/probes/pk_hazard4 tools/probes/pk_hazard4.hip
 */
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include "xform_math.h"

#pragma clang fp contract(off)

typedef float f2 __attribute__((ext_vector_type(2)));
typedef float f4 __attribute__((ext_vector_type(4)));
typedef uint32_t u4 __attribute__((ext_vector_type(4)));
typedef _Float16 h8 __attribute__((ext_vector_type(8)));

#define CK(x)                                                                              \
    do {                                                                                   \
        hipError_t e_ = (x);                                                               \
        if (e_ != hipSuccess) {                                                            \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                        \
            exit(1);                                                                       \
        }                                                                                  \
    } while (0)

struct Pair {
    typedef f2 V;
    static __device__ __forceinline__ V mk(float a, float b) { return V{a, b}; }
    static __device__ __forceinline__ float lo(V a) { return a.x; }
    static __device__ __forceinline__ float hi(V a) { return a.y; }
    static __device__ __forceinline__ V add(V a, V b) { return a + b; }
    static __device__ __forceinline__ V sub(V a, V b) { return a - b; }
    static __device__ __forceinline__ V mul(V a, V b) { return a * b; }
    static __device__ __forceinline__ V fma(V a, V b, V c) { return __builtin_elementwise_fma(a, b, c); }
};

__device__ __forceinline__ uint32_t hash(uint32_t x)
{
    x ^= x >> 16;
    x *= 0x7feb352du;
    x ^= x >> 15;
    x *= 0x846ca68bu;
    return x ^ (x >> 16);
}

/* FENCE (compute waves): 0 none; 1 every product read by a VALU instruction before the packed
 * DCT (hipcc pads the XDL-write -> VALU-read wait states: the products are done); 2 no products in
 * the compute waves, but the loader blocks issue products in a loop instead of loading (other waves'
 * MFMAs only) */
template <int LOAD, bool MFMA, int FENCE = 0>
__global__ __launch_bounds__(256) void k_mix(const u4 *stream, size_t nstream, unsigned *bad, int iters)
{
    __shared__ u4 lds[1024];
    const unsigned lane = threadIdx.x & 63u;
    if (FENCE == 2 && (blockIdx.x & 1u)) {                   /* MFMA-only waves */
        h8 a, b;
        for (int i = 0; i < 8; i++) {
            a[i] = (_Float16)(float)((hash(threadIdx.x * 8 + i) & 255u) * (1.0f / 64.0f) - 2.0f);
            b[i] = (_Float16)(float)((hash(lane * 8 + i + 5) & 255u) * (1.0f / 64.0f) - 2.0f);
        }
        f4 acc[8] = {};
        for (int it = 0; it < iters; it++) {
#pragma unroll
            for (int k = 0; k < 8; k++) acc[k] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, acc[k], 0, 0, 0);
        }
        uint32_t v = 0;
        for (int k = 0; k < 8; k++) v += __float_as_uint(acc[k].w);
        if (v == 0x12345678u) bad[10] = 1u;
        return;
    }
    if (blockIdx.x & 1u) {                                   /* loader */
        if (LOAD == 0) return;
        u4 x = {};
        size_t i = ((size_t)(blockIdx.x >> 1) * 256u + threadIdx.x) % nstream;
        const size_t step = (size_t)(gridDim.x >> 1) * 256u;
        for (int it = 0; it < iters * 8; it++) {
            if (LOAD == 1) {
                u4 v[4];
#pragma unroll
                for (int k = 0; k < 4; k++) v[k] = __builtin_nontemporal_load(&stream[(i + k * step) % nstream]);
#pragma unroll
                for (int k = 0; k < 4; k++) x ^= v[k];
            } else if (LOAD == 2) {
                u4 v[4];
#pragma unroll
                for (int k = 0; k < 4; k++) v[k] = lds[(threadIdx.x + 64u * k + (unsigned)it) & 1023u];
#pragma unroll
                for (int k = 0; k < 4; k++) x ^= v[k];
            } else {
#pragma unroll
                for (int k = 0; k < 4; k++)
                    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *)&stream[(i + k * step) % nstream],
                                                     (__attribute__((address_space(3))) void *)&lds[256u * k + 64u * (threadIdx.x >> 6)],
                                                     16, 0, 0);
            }
            i = (i + 4 * step) % nstream;
        }
        if (x.x == 0x12345678u && x.y == 0x9abcdef0u) bad[8] = 1u;
        return;
    }
    /* compute */
    const unsigned gid = (blockIdx.x >> 1) * 256u + threadIdx.x;
    h8 a0, a1, b0, b1;
    for (int i = 0; i < 8; i++) {
        a0[i] = (_Float16)(float)((hash(gid * 8 + i) & 255u) * (1.0f / 64.0f) - 2.0f);
        a1[i] = (_Float16)(float)((hash(gid * 8 + i + 99) & 255u) * (1.0f / 64.0f) - 2.0f);
        b0[i] = (_Float16)(float)((hash(lane * 8 + i + 7) & 255u) * (1.0f / 64.0f) - 2.0f);
        b1[i] = (_Float16)(float)((hash(lane * 8 + i + 77) & 255u) * (1.0f / 64.0f) - 2.0f);
    }
    unsigned nbad = 0;
    uint32_t keep = 0, seed = gid * 0x9E3779B9u;
    for (int it = 0; it < iters; it++) {
        f4 cr[8];
        if (MFMA) {
#pragma unroll
            for (int k = 0; k < 8; k++) {
                cr[k] = __builtin_amdgcn_mfma_f32_16x16x32_f16((k & 1) ? a1 : a0, (k & 2) ? b1 : b0, f4{}, 0, 0, 0);
                a0[k] = (_Float16)((float)a0[k] + 0.0625f);
            }
        }
        __builtin_amdgcn_sched_barrier(0);
        if (FENCE == 1 && MFMA) {
            uint32_t v = 0;
#pragma unroll
            for (int k = 0; k < 8; k++) v += __float_as_uint(cr[k].w);
            asm volatile("" ::"v"(v) : "memory");
            __builtin_amdgcn_sched_barrier(0);
        }
        f2 R[4], F[4];
        float in[8];
#pragma unroll
        for (int k = 0; k < 8; k++) {
            seed = hash(seed + (uint32_t)k);
            in[k] = (float)(int)(seed & 0xffffu) * (1.0f / 4096.0f) - 8.0f;
        }
#pragma unroll
        for (int p = 0; p < 4; p++) R[p] = f2{in[2 * p], in[2 * p + 1]};
        jx_fdct8_pk<Pair>(R, F);
        __builtin_amdgcn_sched_barrier(0);
        float out[8];
        jx_fdct8<FOps>(in, out);
        bool ok = true;
#pragma unroll
        for (int p = 0; p < 4; p++)
            ok = ok && __float_as_uint(F[p].x) == __float_as_uint(out[jx_pk_k(p, 0)]) &&
                 __float_as_uint(F[p].y) == __float_as_uint(out[jx_pk_k(p, 1)]);
        nbad += ok ? 0u : 1u;
        if (MFMA)
            for (int k = 0; k < 8; k++) keep += __float_as_uint(cr[k].w);
    }
    if (nbad) atomicAdd(&bad[lane >> 4], nbad);
    if (keep == 0x12345678u) bad[9] = 1u;
}

template <int LOAD, bool MFMA, int FENCE = 0>
static void run(const u4 *d_stream, size_t n, unsigned *d_bad, int blocks, int iters)
{
    CK(hipMemset(d_bad, 0, 16 * sizeof(unsigned)));
    hipLaunchKernelGGL((k_mix<LOAD, MFMA, FENCE>), dim3(blocks), dim3(256), 0, 0, d_stream, n, d_bad, iters);
    CK(hipGetLastError());
    CK(hipDeviceSynchronize());
    unsigned h[16];
    CK(hipMemcpy(h, d_bad, sizeof h, hipMemcpyDeviceToHost));
    printf("loaders %d (0 none, 1 global->VGPR, 2 LDS->VGPR, 3 LDS-DMA), MFMA %d, fence %d: wrong packed DCTs per "
           "lane group [0-15, 16-31, 32-47, 48-63]: %u %u %u %u of %.0f\n",
           LOAD, (int)MFMA, FENCE, h[0], h[1], h[2], h[3], (double)(blocks / 2) * 256.0 * iters);
    fflush(stdout);
}

int main(int argc, char **argv)
{
    const int blocks = argc > 1 ? atoi(argv[1]) : 8192, iters = argc > 2 ? atoi(argv[2]) : 400;
    const size_t n = (size_t)64 << 20;                       /* 1 GiB stream */
    u4 *d_stream;
    unsigned *d_bad;
    CK(hipMalloc(&d_stream, n * sizeof(u4)));
    CK(hipMemset(d_stream, 0x5a, n * sizeof(u4)));
    CK(hipMalloc(&d_bad, 16 * sizeof(unsigned)));
    const int which = argc > 3 ? atoi(argv[3]) : 0;
    if (which == 0) {
        run<0, true>(d_stream, n, d_bad, blocks, iters);
        run<1, true>(d_stream, n, d_bad, blocks, iters);
        run<2, true>(d_stream, n, d_bad, blocks, iters);
        run<3, true>(d_stream, n, d_bad, blocks, iters);
        run<1, false>(d_stream, n, d_bad, blocks, iters);
        run<2, false>(d_stream, n, d_bad, blocks, iters);
        run<0, false>(d_stream, n, d_bad, blocks, iters);
    } else {
        run<0, true, 0>(d_stream, n, d_bad, blocks, iters);
        run<0, true, 1>(d_stream, n, d_bad, blocks, iters);
        run<0, false, 2>(d_stream, n, d_bad, blocks, iters);
        run<0, true, 0>(d_stream, n, d_bad, blocks, iters);
    }
    return 0;
}
