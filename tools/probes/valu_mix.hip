// Issue-cost probe (diagnostic, not product): cycles per wave-instruction per SIMD, measured
// in-kernel with s_memtime (shader clock), for the instruction kinds an MFMA row pass + VALU
// column pass would use, alone and beside a co-resident MFMA stream on the same SIMD.
//   workgroup = 4*W waves; wave w sits on SIMD (w % 4) (one wave per SIMD per group of 4).
//   role A (waves 0..4*WA-1): stream MODE_A; role B (the rest): stream MODE_B (or idle).
// Output per config: median over waves of (end - start) cycles, per role, and the derived
// cycles per instruction per SIMD.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <vector>

typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef float f16v __attribute__((ext_vector_type(16)));
typedef float f2 __attribute__((ext_vector_type(2)));

enum { M_IDLE, M_FMA, M_PKFMA, M_ADD, M_PKADD, M_MFMA, M_FMA_LIT, M_CVTPK, M_PERM, M_MAX3,
       M_DSW16, M_FMAC_S, M_PKMUL, M_MUL, M_CNDMASK, M_CVTUB, M_CMPV, M_SUBABS, M_PKADDH, M_MFMA16, M_FMA_ABS, M_MIX8, M_MIX16, M_MIX32, M_MIX16S, M_DPP_HM, M_DPP_QP, M_ADDLIT, M_FMAAK, M_DPP_MUL, M_PKFMA_BC, M_CVTUB0, M_NMODES };
static const char *kName[] = {"idle", "v_fma_f32 (vgpr)", "v_pk_fma_f32", "v_add_f32",
                              "v_pk_add_f32", "mfma_32x32x16_f16", "v_fmamk_f32 literal",
                              "v_cvt_pkrtz_f16_f32", "v_perm_b32", "v_max3_f32", "ds_write_b16",
                              "v_fmac_f32 sgpr", "v_pk_mul_f32", "v_mul_f32", "v_cndmask_b32",
"v_cvt_f32_ubyte1", "v_cmp_ge vgpr->sgpr", "v_sub_f32 |a|", "v_pk_add_f16", "mfma_16x16x32_f16", "v_fma_f32 |a|", "mix 1mfma32:8fma", "mix 1mfma32:16fma", "mix 1mfma32:32fma", "mix 1mfma16:16fma", "v_fmac_dpp half_mirror", "v_fmac_dpp quad_perm", "v_add_f32 literal", "v_fmaak_f32", "v_mul_f32_dpp qp", "v_pk_fma op_sel bcast", "v_cvt_f32_ubyte0"};
constexpr int ITERS = 64;     // outer iterations
constexpr int UNR = 16;       // instructions per chain per iteration (x8 chains)

template <int MODE>
__device__ __forceinline__ void stream(float *o, float s, unsigned *lds)
{
    if (MODE == M_IDLE) return;
    if (MODE == M_MFMA16) {
        h8 a, b;
        for (int i = 0; i < 8; i++) {
            a[i] = (_Float16)(threadIdx.x * 0.01f + i);
            b[i] = (_Float16)(s + i);
        }
        typedef float f4v __attribute__((ext_vector_type(4)));
        f4v c0 = {}, c1 = {}, c2 = {}, c3 = {};
        for (int it = 0; it < ITERS; it++) {
#pragma unroll
            for (int r = 0; r < UNR * 2; r++) {
                c0 = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c0, 0, 0, 0);
                c1 = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c1, 0, 0, 0);
                c2 = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c2, 0, 0, 0);
                c3 = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c3, 0, 0, 0);
            }
        }
        float t = 0;
        for (int i = 0; i < 4; i++) t += c0[i] + c1[i] + c2[i] + c3[i];
        o[threadIdx.x] = t;
        return;
    }
    if (MODE == M_MIX8 || MODE == M_MIX16 || MODE == M_MIX32 || MODE == M_MIX16S) {
        constexpr int K = MODE == M_MIX8 ? 8 : (MODE == M_MIX32 ? 32 : 16);
        h8 ha, hb;
        for (int i = 0; i < 8; i++) {
            ha[i] = (_Float16)(threadIdx.x * 0.01f + i);
            hb[i] = (_Float16)(s + i);
        }
        typedef float f4v __attribute__((ext_vector_type(4)));
        f16v c0 = {}, c1 = {};
        f4v d0 = {}, d1 = {};
        float a[8];
        for (int i = 0; i < 8; i++) a[i] = (float)threadIdx.x + i;
        for (int it = 0; it < ITERS; it++) {
#pragma unroll
            for (int r = 0; r < 16; r++) {
                if (MODE == M_MIX16S) {
                    if (r & 1) d0 = __builtin_amdgcn_mfma_f32_16x16x32_f16(ha, hb, d0, 0, 0, 0);
                    else d1 = __builtin_amdgcn_mfma_f32_16x16x32_f16(ha, hb, d1, 0, 0, 0);
                } else {
                    if (r & 1) c0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(ha, hb, c0, 0, 0, 0);
                    else c1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(ha, hb, c1, 0, 0, 0);
                }
#pragma unroll
                for (int j = 0; j < K; j++) {
                    const int i = j & 7;
                    asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(a[i]) : "v"(a[(i + 1) & 7]), "v"(a[(i + 2) & 7]));
                }
            }
        }
        float t = 0;
        for (int i = 0; i < 16; i++) t += c0[i] + c1[i];
        for (int i = 0; i < 4; i++) t += d0[i] + d1[i];
        for (int i = 0; i < 8; i++) t += a[i];
        o[threadIdx.x] = t;
        return;
    }
    if (MODE == M_MFMA) {
        h8 a, b;
        for (int i = 0; i < 8; i++) {
            a[i] = (_Float16)(threadIdx.x * 0.01f + i);
            b[i] = (_Float16)(s + i);
        }
        f16v c0 = {}, c1 = {}, c2 = {}, c3 = {};
        for (int it = 0; it < ITERS; it++) {
#pragma unroll
            for (int r = 0; r < UNR * 2; r++) {   // 128 MFMAs per iteration, 4 accumulators
                c0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c0, 0, 0, 0);
                c1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c1, 0, 0, 0);
                c2 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c2, 0, 0, 0);
                c3 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c3, 0, 0, 0);
            }
        }
        float t = 0;
        for (int i = 0; i < 16; i++) t += c0[i] + c1[i] + c2[i] + c3[i];
        o[threadIdx.x] = t;
        return;
    }
    float a[8];
    f2 p[8];
    unsigned u[8];
    for (int i = 0; i < 8; i++) {
        a[i] = (float)threadIdx.x + i;
        p[i] = f2{a[i], a[i] + 1.0f};
        u[i] = threadIdx.x * 0x01010101u + i;
    }
    const f2 sp = f2{s, s * 0.5f};
    for (int it = 0; it < ITERS; it++) {
#pragma unroll
        for (int r = 0; r < UNR; r++)
#pragma unroll
            for (int i = 0; i < 8; i++) {
                if (MODE == M_FMA)
                    asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(a[i]) : "v"(a[(i + 1) & 7]), "v"(a[(i + 2) & 7]));
                else if (MODE == M_FMA_LIT)
                    asm volatile("v_fmamk_f32 %0, %0, 0x3f7b14be, %1" : "+v"(a[i]) : "v"(a[(i + 2) & 7]));
                else if (MODE == M_FMAC_S)
                    asm volatile("v_fmac_f32_e32 %0, %1, %2" : "+v"(a[i]) : "s"(s), "v"(a[(i + 1) & 7]));
                else if (MODE == M_PKFMA)
                    asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(p[i]) : "v"(p[(i + 1) & 7]), "v"(p[(i + 2) & 7]));
                else if (MODE == M_ADD)
                    asm volatile("v_add_f32_e32 %0, %1, %0" : "+v"(a[i]) : "v"(a[(i + 1) & 7]));
                else if (MODE == M_MUL)
                    asm volatile("v_mul_f32_e32 %0, %1, %0" : "+v"(a[i]) : "v"(a[(i + 1) & 7]));
                else if (MODE == M_PKADD)
                    asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(p[i]) : "v"(p[(i + 1) & 7]));
                else if (MODE == M_PKMUL)
                    asm volatile("v_pk_mul_f32 %0, %0, %1" : "+v"(p[i]) : "v"(p[(i + 1) & 7]));
                else if (MODE == M_CVTPK)
                    asm volatile("v_cvt_pkrtz_f16_f32 %0, %1, %2" : "=v"(u[i]) : "v"(a[i]), "v"(a[(i + 1) & 7]));
                else if (MODE == M_PERM)
                    asm volatile("v_perm_b32 %0, %0, %1, %2" : "+v"(u[i]) : "v"(u[(i + 1) & 7]), "v"(u[(i + 3) & 7]));
                else if (MODE == M_MAX3)
                    asm volatile("v_max3_f32 %0, %0, %1, %2" : "+v"(a[i]) : "v"(a[(i + 1) & 7]), "v"(a[(i + 2) & 7]));
                else if (MODE == M_CNDMASK)
                    asm volatile("v_cndmask_b32_e32 %0, %0, %1, vcc" : "+v"(u[i]) : "v"(u[(i + 1) & 7]));
                else if (MODE == M_CVTUB)
                    asm volatile("v_cvt_f32_ubyte1_e32 %0, %1" : "=v"(a[i]) : "v"(u[(i + 1) & 7]));
                else if (MODE == M_CMPV) {
                    unsigned long long m;
                    asm volatile("v_cmp_ge_f32_e64 %0, |%1|, %2" : "=s"(m) : "v"(a[i]), "v"(a[(i + 1) & 7]));
                } else if (MODE == M_SUBABS)
                    asm volatile("v_sub_f32_e64 %0, |%0|, %1" : "+v"(a[i]) : "v"(a[(i + 1) & 7]));
                else if (MODE == M_FMA_ABS)
                    asm volatile("v_fma_f32 %0, |%0|, %1, %2" : "+v"(a[i]) : "v"(a[(i + 1) & 7]), "v"(a[(i + 2) & 7]));
                else if (MODE == M_PKADDH)
                    asm volatile("v_pk_add_f16 %0, %0, %1" : "+v"(u[i]) : "v"(u[(i + 1) & 7]));
                else if (MODE == M_DPP_HM)
                    asm volatile("v_fmac_f32_dpp %0, %1, %2 row_half_mirror row_mask:0xf bank_mask:0xf" : "+v"(a[i]) : "v"(a[(i + 3) & 7]), "v"(a[(i + 5) & 7]));
                else if (MODE == M_DPP_QP)
                    asm volatile("v_fmac_f32_dpp %0, %1, %2 quad_perm:[1,1,1,1] row_mask:0xf bank_mask:0xf" : "+v"(a[i]) : "v"(a[(i + 3) & 7]), "v"(a[(i + 5) & 7]));
                else if (MODE == M_DPP_MUL)
                    asm volatile("v_mul_f32_dpp %0, %1, %2 quad_perm:[2,2,2,2] row_mask:0xf bank_mask:0xf" : "=v"(a[i]) : "v"(a[(i + 3) & 7]), "v"(a[(i + 5) & 7]));
                else if (MODE == M_ADDLIT)
                    asm volatile("v_add_f32_e32 %0, 0x4b400000, %0" : "+v"(a[i]));
                else if (MODE == M_FMAAK)
                    asm volatile("v_fmaak_f32 %0, %0, %1, 0x4b400000" : "+v"(a[i]) : "v"(a[(i + 1) & 7]));
                else if (MODE == M_PKFMA_BC)
                    asm volatile("v_pk_fma_f32 %0, %0, %1, %2 op_sel_hi:[1,0,1]" : "+v"(p[i]) : "v"(p[(i + 1) & 7]), "v"(p[(i + 2) & 7]));
                else if (MODE == M_CVTUB0)
                    asm volatile("v_cvt_f32_ubyte0_e32 %0, %1" : "=v"(a[i]) : "v"(u[(i + 1) & 7]));
                else if (MODE == M_DSW16)
                    asm volatile("ds_write_b16 %0, %1 offset:%2" ::"v"(threadIdx.x * 130u), "v"(u[i]), "i"(i * 2) : "memory");
            }
    }
    float t = 0;
    for (int i = 0; i < 8; i++) t += a[i] + p[i].x + p[i].y + (float)u[i];
    o[threadIdx.x] = t;
}

template <int MA, int MB>
__global__ void k(float *o, unsigned long long *cyc, int wa, float s)
{
    __shared__ unsigned lds[256 * 96];
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    __syncthreads();
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    if (w < wa)
        stream<MA>(o + blockIdx.x * blockDim.x, s, lds);
    else
        stream<MB>(o + blockIdx.x * blockDim.x, s, lds);
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * 16 + w] = t1 - t0;
}

template <int MA, int MB>
void run(int wps, int wa_per_simd, float *o, unsigned long long *cyc, int cus)
{
    const int threads = 256 * wps, wa = 4 * wa_per_simd;
    hipLaunchKernelGGL((k<MA, MB>), dim3(cus), dim3(threads), 0, 0, o, cyc, wa, 1.0001f);
    hipDeviceSynchronize();
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipEventRecord(e0);
    hipLaunchKernelGGL((k<MA, MB>), dim3(cus), dim3(threads), 0, 0, o, cyc, wa, 1.0001f);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    std::vector<unsigned long long> h((size_t)cus * 16);
    hipMemcpy(h.data(), cyc, h.size() * 8, hipMemcpyDeviceToHost);
    std::vector<double> ca, cb;
    for (int b = 0; b < cus; b++)
        for (int w = 0; w < 4 * wps; w++) (w < wa ? ca : cb).push_back((double)h[b * 16 + w]);
    auto med = [](std::vector<double> &v) {
        if (v.empty()) return 0.0;
        std::nth_element(v.begin(), v.begin() + v.size() / 2, v.end());
        return v[v.size() / 2];
    };
    const double ma = med(ca), mb = med(cb);
    const double nA = MA >= M_MIX8 ? ITERS * 16 * (1 + (MA == M_MIX8 ? 8 : MA == M_MIX32 ? 32 : 16)) : (MA == M_MFMA || MA == M_MFMA16) ? ITERS * UNR * 2 * 4 : ITERS * UNR * 8;
    const double nB = MB >= M_MIX8 ? ITERS * 16 * (1 + (MB == M_MIX8 ? 8 : MB == M_MIX32 ? 32 : 16)) : (MB == M_MFMA || MB == M_MFMA16) ? ITERS * UNR * 2 * 4 : ITERS * UNR * 8;
    // cycles per instruction per SIMD if the role's waves of a SIMD share it for the whole span
    printf("%-22s x%d | %-22s x%d : A %8.0f cyc (%5.2f cyc/instr/SIMD)  B %8.0f cyc (%5.2f)  kernel %.3f ms\n",
           kName[MA], wa_per_simd, kName[MB], wps - wa_per_simd, ma,
           ma / (nA * wa_per_simd), mb, MB == M_IDLE ? 0.0 : mb / (nB * (wps - wa_per_simd)), ms);
}

int main()
{
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    float *o;
    unsigned long long *cyc;
    hipMalloc(&o, (size_t)cus * 1024 * sizeof(float));
    hipMalloc(&cyc, (size_t)cus * 16 * 8);
    for (int wps : {2, 3, 4}) {
        run<M_DPP_HM, M_IDLE>(wps, wps, o, cyc, cus);
        run<M_DPP_QP, M_IDLE>(wps, wps, o, cyc, cus);
        run<M_DPP_MUL, M_IDLE>(wps, wps, o, cyc, cus);
        run<M_ADDLIT, M_IDLE>(wps, wps, o, cyc, cus);
        run<M_FMAAK, M_IDLE>(wps, wps, o, cyc, cus);
        run<M_PKFMA_BC, M_IDLE>(wps, wps, o, cyc, cus);
        run<M_CVTUB0, M_IDLE>(wps, wps, o, cyc, cus);
        run<M_FMA, M_IDLE>(wps, wps, o, cyc, cus);
    }
    return 0;
}
