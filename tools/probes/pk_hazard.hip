/*
 * pk_hazard.hip -- round-5 probe of the rows-12..15 fault: do packed-fp32 VALU chains
 * (v_pk_fma_f32 / v_pk_add_f32 / v_pk_mul_f32) give wrong lanes on gfx950 when MFMAs run on the
 * same SIMD?  Each wave runs, per iteration, an optional burst of eight independent
 * v_mfma_f32_16x16x32_f16 products (as k_mxs's Cr group) and then a dependent chain of 16 packed
 * ops written in inline asm (hipcc pads nothing inside it: the hardware alone orders it), and
 * compares the chain's result with the same arithmetic in scalar v_fma_f32 / v_add_f32 (lane-wise
 * identical by the ISA's definition of the packed ops).  Mismatches are counted per 16-lane group.
 *
 * Modes (template MODE):
 *   0  pk_fma chain, no MFMA            1  MFMA burst, then the pk_fma chain
 *   2  MFMA burst, then a scalar asm chain (v_fma_f32 x2 per step; control)
 *   3  MFMA burst, then the pk_fma chain with s_nop 0 between dependent ops
 *   4  MFMA burst, then a pk_add chain   5  MFMA burst, then two interleaved pk_fma chains
 *   6  MFMA burst, then a pk_mul chain   7  MFMA burst + s_nop 7 x 8 (bursts drain), pk_fma chain
 * Usage: ./pk_hazard [blocks] [iters]   (prints mode, wrong results per lane group)
 * Build: hipcc --offload-arch=gfx950 -O3 -fno-slp-vectorize -o tools/probes/pk_hazard tools/probes/pk_hazard.hip
 */
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

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

#define PK1(op) op " %0, %0, %1, %2\n"
#define PK4(op) PK1(op) PK1(op) PK1(op) PK1(op)
#define PKN1(op) op " %0, %0, %1, %2\n\ts_nop 0\n"
#define PKN4(op) PKN1(op) PKN1(op) PKN1(op) PKN1(op)
#define PA1 "v_pk_add_f32 %0, %0, %1\n"
#define PA4 PA1 PA1 PA1 PA1
#define PM1 "v_pk_mul_f32 %0, %0, %1\n"
#define PM4 PM1 PM1 PM1 PM1

template <int MODE>
__global__ __launch_bounds__(256, 4) void k_pk(const float *in, unsigned *bad, int iters)
{
    const unsigned gid = blockIdx.x * 256u + threadIdx.x, lane = threadIdx.x & 63u;
    f2 v = {in[(2 * gid) & 4095], in[(2 * gid + 1) & 4095]};
    const f2 c = {0.999f + 1e-4f * (float)(lane & 7), 1.0001f - 1e-4f * (float)(lane >> 3)};
    const f2 d = {0.125f * (float)lane, -0.0625f * (float)lane};
    h8 a, b;
    for (int i = 0; i < 8; i++) {
        a[i] = (_Float16)(0.01f * (float)((gid + i) % 97));
        b[i] = (_Float16)(0.02f * (float)((lane * 3 + i) % 89));
    }
    f4 acc[8] = {};
    unsigned nbad = 0;
    for (int it = 0; it < iters; it++) {
        if (MODE != 0) {
#pragma unroll
            for (int m = 0; m < 8; m++) acc[m] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, acc[m], 0, 0, 0);
        }
        __builtin_amdgcn_sched_barrier(0);
        if (MODE == 7) asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7");
        f2 p = v, p2 = v + d;
        if (MODE == 0 || MODE == 1 || MODE == 7)
            asm volatile(PK4("v_pk_fma_f32") PK4("v_pk_fma_f32") PK4("v_pk_fma_f32") PK4("v_pk_fma_f32")
                         : "+v"(p) : "v"(c), "v"(d));
        else if (MODE == 3)
            asm volatile(PKN4("v_pk_fma_f32") PKN4("v_pk_fma_f32") PKN4("v_pk_fma_f32") PKN4("v_pk_fma_f32")
                         : "+v"(p) : "v"(c), "v"(d));
        else if (MODE == 4)
            asm volatile(PA4 PA4 PA4 PA4 : "+v"(p) : "v"(d));
        else if (MODE == 6)
            asm volatile(PM4 PM4 PM4 PM4 : "+v"(p) : "v"(c));
        else if (MODE == 5)
            asm volatile(
#define PI "v_pk_fma_f32 %0, %0, %2, %3\n\tv_pk_fma_f32 %1, %1, %2, %3\n"
                PI PI PI PI PI PI PI PI PI PI PI PI PI PI PI PI
#undef PI
                : "+v"(p), "+v"(p2) : "v"(c), "v"(d));
        else if (MODE == 2) {
            float px = p.x, py = p.y;
            asm volatile(
#define SI "v_fma_f32 %0, %0, %2, %4\n\tv_fma_f32 %1, %1, %3, %5\n"
                SI SI SI SI SI SI SI SI SI SI SI SI SI SI SI SI
#undef SI
                : "+v"(px), "+v"(py) : "v"(c.x), "v"(c.y), "v"(d.x), "v"(d.y));
            p = f2{px, py};
        }
        __builtin_amdgcn_sched_barrier(0);
        /* the reference: the same operations one lane-half at a time (scalar fp32) */
        float rx = v.x, ry = v.y, r2x = v.x + d.x, r2y = v.y + d.y;
        for (int s = 0; s < 16; s++) {
            if (MODE == 4) {
                rx = rx + d.x;
                ry = ry + d.y;
            } else if (MODE == 6) {
                rx = rx * c.x;
                ry = ry * c.y;
            } else {
                rx = __builtin_fmaf(rx, c.x, d.x);
                ry = __builtin_fmaf(ry, c.y, d.y);
                r2x = __builtin_fmaf(r2x, c.x, d.x);
                r2y = __builtin_fmaf(r2y, c.y, d.y);
            }
        }
        bool ok = __float_as_uint(p.x) == __float_as_uint(rx) && __float_as_uint(p.y) == __float_as_uint(ry);
        if (MODE == 5)
            ok = ok && __float_as_uint(p2.x) == __float_as_uint(r2x) && __float_as_uint(p2.y) == __float_as_uint(r2y);
        nbad += ok ? 0u : 1u;
        v = f2{p.x * 0.5f + 1.0f, p.y * 0.25f - 1.0f};   /* next iteration's input */
    }
    float keep = 0.0f;
#pragma unroll
    for (int m = 0; m < 8; m++) keep += acc[m].x + acc[m].w;
    if (nbad) atomicAdd(&bad[lane >> 4], nbad);
    if (keep == 12345.678f) bad[4] = 1u;   /* keep the products */
}

template <int MODE>
static void run(const float *d_in, unsigned *d_bad, int blocks, int iters)
{
    CK(hipMemset(d_bad, 0, 8 * sizeof(unsigned)));
    hipLaunchKernelGGL(k_pk<MODE>, dim3(blocks), dim3(256), 0, 0, d_in, d_bad, iters);
    CK(hipGetLastError());
    CK(hipDeviceSynchronize());
    unsigned h[8];
    CK(hipMemcpy(h, d_bad, sizeof h, hipMemcpyDeviceToHost));
    const double total = (double)blocks * 256.0 * iters;
    printf("mode %d: wrong chain results per lane group [0-15, 16-31, 32-47, 48-63]: %u %u %u %u of %.0f\n", MODE,
           h[0], h[1], h[2], h[3], total);
    fflush(stdout);
}

int main(int argc, char **argv)
{
    const int blocks = argc > 1 ? atoi(argv[1]) : 4096, iters = argc > 2 ? atoi(argv[2]) : 200;
    float h_in[4096];
    for (int i = 0; i < 4096; i++) h_in[i] = (float)((i * 2654435761u) % 100000u) * 1e-3f - 50.0f;
    float *d_in;
    unsigned *d_bad;
    CK(hipMalloc(&d_in, sizeof h_in));
    CK(hipMalloc(&d_bad, 8 * sizeof(unsigned)));
    CK(hipMemcpy(d_in, h_in, sizeof h_in, hipMemcpyHostToDevice));
    run<0>(d_in, d_bad, blocks, iters);
    run<1>(d_in, d_bad, blocks, iters);
    run<2>(d_in, d_bad, blocks, iters);
    run<3>(d_in, d_bad, blocks, iters);
    run<4>(d_in, d_bad, blocks, iters);
    run<5>(d_in, d_bad, blocks, iters);
    run<6>(d_in, d_bad, blocks, iters);
    run<7>(d_in, d_bad, blocks, iters);
    return 0;
}
