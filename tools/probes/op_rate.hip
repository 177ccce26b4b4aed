// Issue-cost probe for the instruction kinds of k_xform's tile body (diagnostic): per SIMD,
// cycles per wave-instruction at 1..4 waves/SIMD, 8 independent streams per lane.
#include <hip/hip_runtime.h>
#include <cstdio>

template <int MODE>
__global__ __launch_bounds__(256) void k(float *o, int iters, float s)
{
    __shared__ unsigned short lds[256 * 66];
    float a[8];
    unsigned u[8];
    for (int i = 0; i < 8; i++) {
        a[i] = (float)threadIdx.x + i;
        u[i] = threadIdx.x * 0x01010101u + i;
    }
    unsigned long long seen = 0;
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int r = 0; r < 16; r++)
#pragma unroll
            for (int i = 0; i < 8; i++) {
                if (MODE == 0) {          // fma e64
                    asm volatile("v_fma_f32 %0, %0, %1, %1" : "+v"(a[i]) : "v"(s));
                } else if (MODE == 1) {   // fmac e32 with SGPR
                    asm volatile("v_fmac_f32_e32 %0, %1, %0" : "+v"(a[i]) : "s"(s));
                } else if (MODE == 2) {   // cvt ubyte
                    asm volatile("v_cvt_f32_ubyte1_e32 %0, %1" : "=v"(a[i]) : "v"(u[i]));
                } else if (MODE == 3) {   // compare to SGPR mask + scalar or
                    unsigned long long m;
                    asm volatile("v_cmp_ge_f32_e64 %[m], |%[d]|, %[l]\n\ts_or_b64 %[seen], %[seen], %[m]"
                                 : [m] "=&s"(m), [seen] "+s"(seen) : [d] "v"(a[i]), [l] "s"(s) : "scc");
                } else if (MODE == 4) {   // ds_write_b16
                    asm volatile("ds_write_b16 %0, %1 offset:%2" :: "v"((unsigned)(threadIdx.x * 132)), "v"(u[i]), "i"(i * 2) : "memory");
                } else if (MODE == 5) {   // max3
                    asm volatile("v_max3_f32 %0, %0, %1, %1" : "+v"(a[i]) : "v"(a[(i + 1) & 7]));
                } else if (MODE == 6) {   // v_cmp e64 into SGPR only (no scalar use)
                    unsigned long long m;
                    asm volatile("v_cmp_ge_f32_e64 %[m], |%[d]|, %[l]" : [m] "=s"(m) : [d] "v"(a[i]), [l] "s"(s));
                } else if (MODE == 7) {   // v_add_f32 e32
                    asm volatile("v_add_f32_e32 %0, %1, %0" : "+v"(a[i]) : "v"(s));
                } else if (MODE == 8) {   // v_perm_b32
                    asm volatile("v_perm_b32 %0, %0, %1, %2" : "+v"(u[i]) : "v"(u[(i + 1) & 7]), "s"(0x0c010c00u));
                } else if (MODE == 9) {   // v_fma_mix_f32 (f16 lo of src0, f32 src1/src2)
                    asm volatile("v_fma_mix_f32 %0, %1, %2, %0 op_sel_hi:[1,0,0]" : "+v"(a[i]) : "v"(u[i]), "s"(s));
                } else if (MODE == 10) {  // v_cvt_f32_u32
                    asm volatile("v_cvt_f32_u32_e32 %0, %1" : "=v"(a[i]) : "v"(u[i]));
                } else if (MODE == 11) {  // v_dot2_f32_f16
                    asm volatile("v_dot2_f32_f16 %0, %1, %2, %0" : "+v"(a[i]) : "v"(u[i]), "v"(u[(i + 1) & 7]));
                } else if (MODE == 12) {  // dependent fma chain (latency): one chain
                    asm volatile("v_fma_f32 %0, %0, %1, %1" : "+v"(a[0]) : "v"(s));
                } else if (MODE == 13) {  // dependent pk_fma chain (latency): one chain
                    typedef float f2 __attribute__((ext_vector_type(2)));
                    f2 t = f2{a[0], a[1]};
                    asm volatile("v_pk_fma_f32 %0, %0, %1, %1" : "+v"(t) : "v"(f2{s, s}));
                    a[0] = t.x; a[1] = t.y;
                } else if (MODE == 14) {  // v_bfe_u32
                    asm volatile("v_bfe_u32 %0, %0, 8, 8" : "+v"(u[i]));
                } else if (MODE == 15) {  // v_mul_f32 e32
                    asm volatile("v_mul_f32_e32 %0, %1, %0" : "+v"(a[i]) : "v"(s));
                }
            }
    }
    float t = a[0];
    for (int i = 1; i < 8; i++) t += a[i];
    o[blockIdx.x * blockDim.x + threadIdx.x] = t + (float)(seen & 1) + lds[threadIdx.x];
}

int main()
{
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    float *o;
    hipMalloc(&o, (size_t)cus * 16 * 256 * sizeof(float));
    const int iters = 1000;
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const char *nm[16] = {"v_fma_f32 e64", "v_fmac_f32 e32 sgpr", "v_cvt_f32_ubyte1", "v_cmp e64 + s_or",
                         "ds_write_b16", "v_max3_f32", "v_cmp e64 only", "v_add_f32 e32",
                         "v_perm_b32", "v_fma_mix_f32", "v_cvt_f32_u32", "v_dot2_f32_f16",
                         "fma dep chain", "pk_fma dep chain", "v_bfe_u32", "v_mul_f32 e32"};
    typedef void (*fn_t)(float *, int, float);
    fn_t fns[16] = {k<0>, k<1>, k<2>, k<3>, k<4>, k<5>, k<6>, k<7>, k<8>, k<9>, k<10>, k<11>, k<12>, k<13>, k<14>, k<15>};
    for (int wps = 1; wps <= 3; wps += 2) {
        const int grid = cus * wps;
        for (int mode = 0; mode < 16; mode++) {
            hipLaunchKernelGGL(fns[mode], dim3(grid), dim3(256), 0, 0, o, 10, 1.0001f);
            hipEventRecord(e0);
            hipLaunchKernelGGL(fns[mode], dim3(grid), dim3(256), 0, 0, o, iters, 1.0001f);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms = 0;
            hipEventElapsedTime(&ms, e0, e1);
            const double instr_per_simd = (double)iters * 128 * wps;
            printf("waves/SIMD %d  %-22s %8.3f ms  %.2f cyc/instr/SIMD @2.4GHz\n", wps, nm[mode], ms,
                   ms * 1e6 / instr_per_simd * 2.4);
        }
    }
    return 0;
}
