/*
 * pk_hazard3.hip -- round-5 probe of the rows-12..15 fault, k_mxs's step structure in isolation:
 * a Y|Cb-like group of four v_mfma_f32_16x16x32_f16 products, a Cr-like group of eight independent
 * products issued behind it, then the column pass of the first tile exactly as the kernel's source
 * writes it (mx_combine: v_pk_add_f32 of the hi / lo tiles; jx_fdct8_pk: v_pk_*_f32 with op_sel
 * swaps and SGPR constants) while the second group is in the matrix pipe.  Per iteration every lane
 * stores its R pairs (the column input) and F pairs (the column output); the host recomputes F from
 * R with the scalar code (jx_fdct8<FOps>, lane-wise identical) and counts wrong lanes per 16-lane
 * group.  Modes: 0 as above; 1 no Cr group; 2 the column in scalar fp32 (control);
 * 3 the Cr group fenced (results read) before the column.
 * Usage: ./pk_hazard3 [blocks] [iters]
 * Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -fno-slp-vectorize
 *        -I jpeg-encoder-and-decoder_amd/csrc -o tools/probes/pk_hazard3 tools/probes/pk_hazard3.hip
 */
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <vector>

#include "xform_math.h"

#pragma clang fp contract(off)

typedef float f2 __attribute__((ext_vector_type(2)));
typedef float f4 __attribute__((ext_vector_type(4)));
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

__device__ __forceinline__ f4 mma(h8 a, h8 b) { return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, f4{}, 0, 0, 0); }

template <int MODE>
__global__ __launch_bounds__(256, 4) void k_col(const _Float16 *src, float *dump, int iters)
{
    const unsigned gid = blockIdx.x * 256u + threadIdx.x, lane = threadIdx.x & 63u;
    h8 a0, a1, b0, b1, c[8];
    for (int i = 0; i < 8; i++) {
        a0[i] = src[(gid * 8 + i) & 65535];
        a1[i] = src[(gid * 8 + i + 777) & 65535];
        b0[i] = src[(lane * 8 + i + 1234) & 65535];
        b1[i] = src[(lane * 8 + i + 4321) & 65535];
        for (int k = 0; k < 8; k++) c[k][i] = src[(lane * 8 + i + 999 * (k + 1)) & 65535];
    }
    uint32_t keep = 0;
    for (int it = 0; it < iters; it++) {
        f4 acc[4];
        acc[0] = mma(a0, b0);
        acc[2] = mma(a1, b0);
        acc[1] = mma(a0, b1);
        acc[3] = mma(a1, b1);
        __builtin_amdgcn_sched_barrier(0);
        f4 cr[8];
        if (MODE != 1) {
#pragma unroll
            for (int k = 0; k < 8; k++) {
                cr[k] = mma((k & 1) ? a1 : a0, c[k]);
                __builtin_amdgcn_sched_barrier(0);
            }
        }
        if (MODE == 3) {
            uint32_t v = 0;
            for (int k = 0; k < 8; k++) v += __float_as_uint(cr[k].w);
            asm volatile("" ::"v"(v) : "memory");
            __builtin_amdgcn_sched_barrier(0);
        }
        f2 R[4], F[4];
        R[0] = f2{acc[1].x, acc[1].y} + f2{acc[0].x, acc[0].y};
        R[1] = f2{acc[1].z, acc[1].w} + f2{acc[0].z, acc[0].w};
        R[2] = f2{acc[3].x, acc[3].y} + f2{acc[2].x, acc[2].y};
        R[3] = f2{acc[3].z, acc[3].w} + f2{acc[2].z, acc[2].w};
        if (MODE == 2) {
            const float in[8] = {R[0].x, R[0].y, R[1].x, R[1].y, R[2].x, R[2].y, R[3].x, R[3].y};
            float out[8];
            jx_fdct8<FOps>(in, out);
            for (int p = 0; p < 4; p++) F[p] = f2{out[jx_pk_k(p, 0)], out[jx_pk_k(p, 1)]};
        } else {
            jx_fdct8_pk<Pair>(R, F);
        }
        __builtin_amdgcn_sched_barrier(0);
        float *d = dump + ((size_t)it * gridDim.x * 256u + gid) * 16u;
        *(f4 *)d = f4{R[0].x, R[0].y, R[1].x, R[1].y};
        *(f4 *)(d + 4) = f4{R[2].x, R[2].y, R[3].x, R[3].y};
        *(f4 *)(d + 8) = f4{F[0].x, F[0].y, F[1].x, F[1].y};
        *(f4 *)(d + 12) = f4{F[2].x, F[2].y, F[3].x, F[3].y};
        if (MODE != 1)
            for (int k = 0; k < 8; k++) keep += __float_as_uint(cr[k].w) + __float_as_uint(cr[k].x);
        /* next iteration's operands */
        a0 = __builtin_shufflevector(a0, a1, 1, 2, 3, 4, 5, 6, 7, 8);
        a1 = __builtin_shufflevector(a1, a0, 1, 2, 3, 4, 5, 6, 7, 8);
    }
    if (keep == 0x12345678u) dump[0] = 1.0f;
}

/* host: F from R with the scalar code, bit for bit */
static void host_f(const float *R, float *F)
{
    float out[8];
    jx_fdct8<FOps>(R, out);
    for (int p = 0; p < 4; p++) {
        F[2 * p] = out[jx_pk_k(p, 0)];
        F[2 * p + 1] = out[jx_pk_k(p, 1)];
    }
}

template <int MODE>
static void run(const _Float16 *d_src, float *d_dump, std::vector<float> &h, int blocks, int iters)
{
    hipLaunchKernelGGL(k_col<MODE>, dim3(blocks), dim3(256), 0, 0, d_src, d_dump, iters);
    CK(hipGetLastError());
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(h.data(), d_dump, h.size() * sizeof(float), hipMemcpyDeviceToHost));
    const size_t n = h.size() / 16;
    size_t bad[4] = {0, 0, 0, 0};
    int shown = 0;
    for (size_t i = 0; i < n; i++) {
        float F[8];
        host_f(&h[16 * i], F);
        if (memcmp(F, &h[16 * i + 8], sizeof F)) {
            const unsigned lane = (unsigned)(i % 256u) & 63u;
            bad[lane >> 4]++;
            if (shown++ < 3) {
                printf("   lane %u: R", lane);
                for (int k = 0; k < 8; k++) printf(" %.6g", h[16 * i + k]);
                printf("\n      F got");
                for (int k = 0; k < 8; k++) printf(" %.6g", h[16 * i + 8 + k]);
                printf("\n      F want");
                for (int k = 0; k < 8; k++) printf(" %.6g", F[k]);
                printf("\n");
            }
        }
    }
    printf("mode %d: wrong column passes per lane group [0-15, 16-31, 32-47, 48-63]: %zu %zu %zu %zu of %zu\n", MODE,
           bad[0], bad[1], bad[2], bad[3], n);
    fflush(stdout);
}

int main(int argc, char **argv)
{
    const int blocks = argc > 1 ? atoi(argv[1]) : 4096, iters = argc > 2 ? atoi(argv[2]) : 16;
    static _Float16 hs[65536];
    for (int i = 0; i < 65536; i++) {
        const unsigned r = (unsigned)i * 2654435761u;
        hs[i] = (_Float16)((float)(r >> 24) * (1.0f / 64.0f) - 2.0f);
    }
    _Float16 *d_src;
    float *d_dump;
    std::vector<float> h((size_t)blocks * 256u * iters * 16u);
    CK(hipMalloc(&d_src, sizeof hs));
    CK(hipMalloc(&d_dump, h.size() * sizeof(float)));
    CK(hipMemcpy(d_src, hs, sizeof hs, hipMemcpyHostToDevice));
    for (int rep = 0; rep < 2; rep++) {
        run<0>(d_src, d_dump, h, blocks, iters);
        run<1>(d_src, d_dump, h, blocks, iters);
        run<2>(d_src, d_dump, h, blocks, iters);
        run<3>(d_src, d_dump, h, blocks, iters);
    }
    return 0;
}
