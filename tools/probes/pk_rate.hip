// Issue-rate probe: v_fma_f32 vs v_pk_fma_f32 (2 FMAs per lane) vs v_pk_add_f32, with
// 1..4 waves per SIMD, 8 independent accumulator chains per lane (diagnostic).
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f2 __attribute__((ext_vector_type(2)));

template <int MODE>
__global__ __launch_bounds__(256) void k(float *o, int iters, float s)
{
    f2 a[8];
    for (int i = 0; i < 8; i++) a[i] = f2{(float)threadIdx.x + i, (float)i};
    const f2 m = f2{s, s * 0.5f};
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int r = 0; r < 16; r++)
#pragma unroll
            for (int i = 0; i < 8; i++) {
                if (MODE == 0) {        // 2 scalar FMAs (same flops as one packed)
                    asm volatile("v_fma_f32 %0, %0, %1, %1" : "+v"(a[i].x) : "v"(m.x));
                    asm volatile("v_fma_f32 %0, %0, %1, %1" : "+v"(a[i].y) : "v"(m.y));
                } else if (MODE == 1) { // one packed FMA
                    asm volatile("v_pk_fma_f32 %0, %0, %1, %1" : "+v"(a[i]) : "v"(m));
                } else if (MODE == 2) { // packed FMA, SGPR pair operand broadcast (op_sel_hi 0)
                    asm volatile("v_pk_fma_f32 %0, %0, %1, %0 op_sel_hi:[1,0,1]" : "+v"(a[i]) : "s"(m));
                } else {                // packed add
                    asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(a[i]) : "v"(m));
                }
            }
    }
    f2 t = a[0];
    for (int i = 1; i < 8; i++) t += a[i];
    o[blockIdx.x * blockDim.x + threadIdx.x] = t.x + t.y;
}

int main()
{
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    float *o;
    hipMalloc(&o, (size_t)cus * 16 * 256 * sizeof(float));
    const int iters = 2000;
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const char *nm[4] = {"2x v_fma_f32", "v_pk_fma_f32", "v_pk_fma_f32 sgpr", "v_pk_add_f32"};
    for (int wps = 1; wps <= 4; wps++) {
        const int grid = cus * wps;           // 4 waves per WG -> wps waves per SIMD
        for (int mode = 0; mode < 4; mode++) {
            auto fn = mode == 0 ? k<0> : mode == 1 ? k<1> : mode == 2 ? k<2> : k<3>;
            hipLaunchKernelGGL(fn, dim3(grid), dim3(256), 0, 0, o, 10, 1.0001f);
            hipEventRecord(e0);
            hipLaunchKernelGGL(fn, dim3(grid), dim3(256), 0, 0, o, iters, 1.0001f);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms = 0;
            hipEventElapsedTime(&ms, e0, e1);
            const double instr_per_simd = (double)iters * 128 * wps * (mode == 0 ? 2 : 1);
            // cycles per wave-instruction per SIMD at an assumed 2.4 GHz
            printf("waves/SIMD %d  %-20s %8.3f ms  %.2f ns/instr/SIMD  (%.2f cyc @2.4GHz)\n", wps,
                   nm[mode], ms, ms * 1e6 / instr_per_simd, ms * 1e6 / instr_per_simd * 2.4);
        }
    }
    return 0;
}
