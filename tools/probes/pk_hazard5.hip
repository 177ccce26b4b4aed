/*
 * pk_hazard5.hip -- round-5 probe: WHICH packed-fp32 form goes wrong in lanes 48..63 after the same
 * wave's MFMAs (pk_hazard4.hip: the packed DCT does, in 1.7e-4 of its runs; never without MFMAs in
 * the wave).  Each wave, per iteration: eight v_mfma_f32_16x16x32_f16 products into AGPR/VGPR
 * accumulators, per-lane pseudo-random inputs made by integer hashing (as pk_hazard4), then ONE
 * inline-asm packed instruction of the form under test on a register pair whose halves the compiler
 * has just written, compared with the scalar result.  Forms (MODE):
 *   0 v_pk_add_f32 d, a, b                       1 v_pk_add_f32 with op_sel:[0,1] op_sel_hi:[1,0]
 *   2 v_pk_fma_f32 d, a, s[k:k+1], b             3 v_pk_mul_f32 d, a, b
 *   4 v_pk_add_f32 with s_nop 7 x 4 before it     5 v_pk_fma_f32 d, a, b, c (all VGPR)
 *   6 v_pk_mov_b32 d, a, b op_sel:[1,0] (swap)    7 two v_add_f32 (scalar control)
 *  (set 1) 1 without MFMA; 10 swap src0; 11 / 12 src0 hi / lo broadcast; 13 src1 lo broadcast;
 *   14 swap src1 after 32 wait states; 15 v_pk_fma src2 lo broadcast; 16 the column pass's
 *   v_pk_fma (src0 hi broadcast, SGPR pair, src2 lo broadcast); 17 swap src1 whose pair was written
 *   an iteration earlier; 1 again
 *  (set 2) fp64 VALU (the exact pass's arithmetic): 20 v_add_f64, 21 v_fma_f64, 22 v_mul_f64,
 *   23 v_add_f64 of a DPP row_half_mirror'd value; 1 again
 *  (set 3, round 6: the cross-lane ops the MFMA kernels still issue after their products, each
 *   checked against the partner lane's value fetched by ds_bpermute, an LDS-path reference)
 *   30 v_permlane16_swap of an fp32 value (no MFMA, then with); 31 v_permlane32_swap fp32;
 *   32 / 33 v_permlane16 / 32_swap of an fp64's halves + v_add_f64 (mx_xsum64); 34 DPP row_mirror
 *   fp32 + v_add_f32; 35 DPP quad_perm [1,0,3,2] fp32 + v_add_f32; 36 DPP row_mirror of an fp64's
 *   halves + v_add_f64; 1 again (the known-failing packed form, as the positive control)
 * Usage: ./pk_hazard5 [blocks] [iters] [set 0 | 1 | 2 | 3]
 * Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -fno-slp-vectorize -o tools/probes/pk_hazard5 tools/probes/pk_hazard5.hip
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

__device__ __forceinline__ uint32_t hash(uint32_t x)
{
    x ^= x >> 16;
    x *= 0x7feb352du;
    x ^= x >> 15;
    x *= 0x846ca68bu;
    return x ^ (x >> 16);
}

template <int MODE, bool MFMA = true>
__global__ __launch_bounds__(256) void k_form(unsigned *bad, int iters, float kx, float ky)
{
    const unsigned gid = blockIdx.x * 256u + threadIdx.x, lane = threadIdx.x & 63u;
    h8 a0, a1, b0, b1;
    for (int i = 0; i < 8; i++) {
        a0[i] = (_Float16)(float)((hash(gid * 8 + i) & 255u) * (1.0f / 64.0f) - 2.0f);
        a1[i] = (_Float16)(float)((hash(gid * 8 + i + 99) & 255u) * (1.0f / 64.0f) - 2.0f);
        b0[i] = (_Float16)(float)((hash(lane * 8 + i + 7) & 255u) * (1.0f / 64.0f) - 2.0f);
        b1[i] = (_Float16)(float)((hash(lane * 8 + i + 77) & 255u) * (1.0f / 64.0f) - 2.0f);
    }
    unsigned nbad = 0;
    uint32_t keep = 0, seed = gid * 0x9E3779B9u;
    const f2 K = {kx, ky};                       /* wave-uniform: an SGPR pair */
    f2 Bold = {1.5f, -2.5f};
    for (int it = 0; it < iters; it++) {
        f4 cr[8] = {};
        if (MFMA) {
#pragma unroll
            for (int k = 0; k < 8; k++) {
                cr[k] = __builtin_amdgcn_mfma_f32_16x16x32_f16((k & 1) ? a1 : a0, (k & 2) ? b1 : b0, f4{}, 0, 0, 0);
                a0[k] = (_Float16)((float)a0[k] + 0.0625f);
            }
        }
        __builtin_amdgcn_sched_barrier(0);
        float in[6];
#pragma unroll
        for (int k = 0; k < 6; k++) {
            seed = hash(seed + (uint32_t)k);
            in[k] = (float)(int)(seed & 0xffffu) * (1.0f / 4096.0f) - 8.0f;
        }
        f2 A = {in[0], in[1]}, B = {in[2], in[3]}, C = {in[4], in[5]}, D;
        if (MODE == 17 && it == 0) Bold = B;
        float wx, wy;
        if (MODE == 0) {
            asm volatile("v_pk_add_f32 %0, %1, %2" : "=v"(D) : "v"(A), "v"(B));
            wx = A.x + B.x, wy = A.y + B.y;
        } else if (MODE == 1) {
            asm volatile("v_pk_add_f32 %0, %1, %2 op_sel:[0,1] op_sel_hi:[1,0]" : "=v"(D) : "v"(A), "v"(B));
            wx = A.x + B.y, wy = A.y + B.x;
        } else if (MODE == 2) {
            asm volatile("v_pk_fma_f32 %0, %1, %2, %3" : "=v"(D) : "v"(A), "s"(K), "v"(B));
            wx = __builtin_fmaf(A.x, K.x, B.x), wy = __builtin_fmaf(A.y, K.y, B.y);
        } else if (MODE == 3) {
            asm volatile("v_pk_mul_f32 %0, %1, %2" : "=v"(D) : "v"(A), "v"(B));
            wx = A.x * B.x, wy = A.y * B.y;
        } else if (MODE == 4) {
            asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7\n\tv_pk_add_f32 %0, %1, %2" : "=v"(D) : "v"(A), "v"(B));
            wx = A.x + B.x, wy = A.y + B.y;
        } else if (MODE == 5) {
            asm volatile("v_pk_fma_f32 %0, %1, %2, %3" : "=v"(D) : "v"(A), "v"(B), "v"(C));
            wx = __builtin_fmaf(A.x, B.x, C.x), wy = __builtin_fmaf(A.y, B.y, C.y);
        } else if (MODE == 6) {
            asm volatile("v_pk_mov_b32 %0, %1, %2 op_sel:[1,0]" : "=v"(D) : "v"(A), "v"(B));
            wx = A.y, wy = B.x;
        } else if (MODE == 7) {
            float dx, dy;
            asm volatile("v_add_f32 %0, %2, %3\n\tv_add_f32 %1, %4, %5" : "=&v"(dx), "=&v"(dy)
                         : "v"(A.x), "v"(B.x), "v"(A.y), "v"(B.y));
            D = f2{dx, dy};
            wx = A.x + B.x, wy = A.y + B.y;
        } else if (MODE == 10) {                 /* swap src0 */
            asm volatile("v_pk_add_f32 %0, %1, %2 op_sel:[1,0] op_sel_hi:[0,1]" : "=v"(D) : "v"(A), "v"(B));
            wx = A.y + B.x, wy = A.x + B.y;
        } else if (MODE == 11) {                 /* src0 hi broadcast */
            asm volatile("v_pk_add_f32 %0, %1, %2 op_sel:[1,0] op_sel_hi:[1,1]" : "=v"(D) : "v"(A), "v"(B));
            wx = A.y + B.x, wy = A.y + B.y;
        } else if (MODE == 12) {                 /* src0 lo broadcast */
            asm volatile("v_pk_add_f32 %0, %1, %2 op_sel_hi:[0,1]" : "=v"(D) : "v"(A), "v"(B));
            wx = A.x + B.x, wy = A.x + B.y;
        } else if (MODE == 13) {                 /* src1 lo broadcast */
            asm volatile("v_pk_add_f32 %0, %1, %2 op_sel_hi:[1,0]" : "=v"(D) : "v"(A), "v"(B));
            wx = A.x + B.x, wy = A.y + B.x;
        } else if (MODE == 14) {                 /* swap src1, 32 wait states before */
            asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7\n\tv_pk_add_f32 %0, %1, %2 op_sel:[0,1] op_sel_hi:[1,0]"
                         : "=v"(D) : "v"(A), "v"(B));
            wx = A.x + B.y, wy = A.y + B.x;
        } else if (MODE == 15) {                 /* fma, src2 lo broadcast */
            asm volatile("v_pk_fma_f32 %0, %1, %2, %3 op_sel_hi:[1,1,0]" : "=v"(D) : "v"(A), "v"(B), "v"(C));
            wx = __builtin_fmaf(A.x, B.x, C.x), wy = __builtin_fmaf(A.y, B.y, C.x);
        } else if (MODE == 16) {                 /* the column pass's form: src0 hi broadcast, SGPR, src2 lo broadcast */
            asm volatile("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[1,0,0] op_sel_hi:[1,1,0]" : "=v"(D) : "v"(A), "s"(K), "v"(C));
            wx = __builtin_fmaf(A.y, K.x, C.x), wy = __builtin_fmaf(A.y, K.y, C.x);
        } else if (MODE == 20 || MODE == 21 || MODE == 22) { /* fp64: v_add_f64 / v_fma_f64 / v_mul_f64 */
            const double da = (double)A.x * 3.0 + (double)A.y, db = (double)B.x - (double)B.y * 0.5,
                         dc = (double)C.x;
            double dd;
            if (MODE == 20) asm volatile("v_add_f64 %0, %1, %2" : "=v"(dd) : "v"(da), "v"(db));
            else if (MODE == 21) asm volatile("v_fma_f64 %0, %1, %2, %3" : "=v"(dd) : "v"(da), "v"(db), "v"(dc));
            else asm volatile("v_mul_f64 %0, %1, %2" : "=v"(dd) : "v"(da), "v"(db));
            const double wd = MODE == 20 ? da + db : (MODE == 21 ? __builtin_fma(da, db, dc) : da * db);
            const uint64_t gb = __builtin_bit_cast(uint64_t, dd), wb = __builtin_bit_cast(uint64_t, wd);
            D = f2{__uint_as_float((uint32_t)gb), __uint_as_float((uint32_t)(gb >> 32))};
            wx = __uint_as_float((uint32_t)wb), wy = __uint_as_float((uint32_t)(wb >> 32));
        } else if (MODE == 23) {                 /* the exact pass's DPP step: v_add_f64 of a row_half_mirror'd value */
            const double da = (double)A.x * 3.0 + (double)A.y;
            const uint64_t b = __builtin_bit_cast(uint64_t, da);
            const uint32_t lo = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)b, 0x141, 0xf, 0xf, false);
            const uint32_t hi = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)(b >> 32), 0x141, 0xf, 0xf, false);
            const double dm = __builtin_bit_cast(double, (uint64_t)lo | ((uint64_t)hi << 32));
            double dd;
            asm volatile("v_add_f64 %0, %1, %2" : "=v"(dd) : "v"(da), "v"(dm));
            /* the reference: the mirrored lane's value via LDS-free recomputation is not possible here,
             * so compare with the same add done after a fence-like dependency chain */
            asm volatile("s_nop 7\n\ts_nop 7" ::: "memory");
            const double wd = da + dm;
            const uint64_t gb = __builtin_bit_cast(uint64_t, dd), wb = __builtin_bit_cast(uint64_t, wd);
            D = f2{__uint_as_float((uint32_t)gb), __uint_as_float((uint32_t)(gb >> 32))};
            wx = __uint_as_float((uint32_t)wb), wy = __uint_as_float((uint32_t)(wb >> 32));
        } else if (MODE >= 30 && MODE <= 36) {   /* cross-lane ops; reference: ds_bpermute of the partner */
            const float x = A.x;
            const double dx = (double)A.x * 3.0 + (double)A.y;
            const uint64_t bx = __builtin_bit_cast(uint64_t, dx);
            const unsigned r = lane >> 4;
            uint32_t g0 = 0, g1 = 0, w0 = 0, w1 = 0;
            if (MODE == 30 || MODE == 31) {
                const auto pr = MODE == 30 ? __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false)
                                           : __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
                g0 = pr[0], g1 = pr[1];
                const unsigned e = MODE == 30 ? ((r & 1u) ? lane - 16u : lane) : (lane & 31u);
                const unsigned o = MODE == 30 ? ((r & 1u) ? lane : lane + 16u) : (lane | 32u);
                w0 = (uint32_t)__shfl((int)__float_as_uint(x), (int)e, 64);
                w1 = (uint32_t)__shfl((int)__float_as_uint(x), (int)o, 64);
            } else if (MODE == 32 || MODE == 33) {
                const uint32_t lo = (uint32_t)bx, hi = (uint32_t)(bx >> 32);
                const auto l2 = MODE == 32 ? __builtin_amdgcn_permlane16_swap(lo, lo, false, false)
                                           : __builtin_amdgcn_permlane32_swap(lo, lo, false, false);
                const auto h2 = MODE == 32 ? __builtin_amdgcn_permlane16_swap(hi, hi, false, false)
                                           : __builtin_amdgcn_permlane32_swap(hi, hi, false, false);
                const double sum = __builtin_bit_cast(double, (uint64_t)l2[0] | ((uint64_t)h2[0] << 32)) +
                                   __builtin_bit_cast(double, (uint64_t)l2[1] | ((uint64_t)h2[1] << 32));
                const unsigned q = MODE == 32 ? (lane ^ 16u) : (lane ^ 32u);
                const uint64_t pb = (uint64_t)(uint32_t)__shfl((int)lo, (int)q, 64) |
                                    ((uint64_t)(uint32_t)__shfl((int)hi, (int)q, 64) << 32);
                const double pd = __builtin_bit_cast(double, pb);
                const bool first = MODE == 32 ? !(r & 1u) : lane < 32u;      /* this lane's value is the even / low one */
                const double ws = first ? dx + pd : pd + dx;
                const uint64_t gs = __builtin_bit_cast(uint64_t, sum), wsb = __builtin_bit_cast(uint64_t, ws);
                g0 = (uint32_t)gs, g1 = (uint32_t)(gs >> 32), w0 = (uint32_t)wsb, w1 = (uint32_t)(wsb >> 32);
            } else if (MODE == 34 || MODE == 35) {
                const uint32_t m = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)__float_as_uint(x), MODE == 34 ? 0x140 : 0xB1, 0xf, 0xf, false);
                const float sum = x + __uint_as_float(m);
                const unsigned q = MODE == 34 ? ((lane & ~15u) | (15u - (lane & 15u))) : (lane ^ 1u);
                const float pv = __uint_as_float((uint32_t)__shfl((int)__float_as_uint(x), (int)q, 64));
                g0 = __float_as_uint(sum), w0 = __float_as_uint(x + pv);
                g1 = m, w1 = __float_as_uint(pv);
            } else {                             /* 36: fp64 row_mirror + v_add_f64 */
                const uint32_t lo = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)bx, 0x140, 0xf, 0xf, false);
                const uint32_t hi = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)(bx >> 32), 0x140, 0xf, 0xf, false);
                const double sum = dx + __builtin_bit_cast(double, (uint64_t)lo | ((uint64_t)hi << 32));
                const unsigned q = (lane & ~15u) | (15u - (lane & 15u));
                const uint64_t pb = (uint64_t)(uint32_t)__shfl((int)(uint32_t)bx, (int)q, 64) |
                                    ((uint64_t)(uint32_t)__shfl((int)(uint32_t)(bx >> 32), (int)q, 64) << 32);
                const double ws = dx + __builtin_bit_cast(double, pb);
                const uint64_t gs = __builtin_bit_cast(uint64_t, sum), wsb = __builtin_bit_cast(uint64_t, ws);
                g0 = (uint32_t)gs, g1 = (uint32_t)(gs >> 32), w0 = (uint32_t)wsb, w1 = (uint32_t)(wsb >> 32);
            }
            D = f2{__uint_as_float(g0), __uint_as_float(g1)};
            wx = __uint_as_float(w0), wy = __uint_as_float(w1);
        } else {                                 /* 17: swap src1, both halves of B old (written one iteration early) */
            asm volatile("v_pk_add_f32 %0, %1, %2 op_sel:[0,1] op_sel_hi:[1,0]" : "=v"(D) : "v"(A), "v"(Bold));
            wx = A.x + Bold.y, wy = A.y + Bold.x;
        }
        asm volatile("s_nop 1" ::: "memory");
        const bool ok = __float_as_uint(D.x) == __float_as_uint(wx) && __float_as_uint(D.y) == __float_as_uint(wy);
        nbad += ok ? 0u : 1u;
        for (int k = 0; k < 8; k++) keep += __float_as_uint(cr[k].w);
        if (MODE == 17) Bold = f2{Bold.y * 0.5f + in[0], Bold.x * 0.25f - in[1]};
    }
    if (nbad) atomicAdd(&bad[lane >> 4], nbad);
    if (keep == 0x12345678u) bad[9] = 1u;
}

template <int MODE, bool MFMA = true>
static void run(unsigned *d_bad, int blocks, int iters)
{
    CK(hipMemset(d_bad, 0, 16 * sizeof(unsigned)));
    hipLaunchKernelGGL((k_form<MODE, MFMA>), dim3(blocks), dim3(256), 0, 0, d_bad, iters, 1.25f, -0.75f);
    CK(hipGetLastError());
    CK(hipDeviceSynchronize());
    unsigned h[16];
    CK(hipMemcpy(h, d_bad, sizeof h, hipMemcpyDeviceToHost));
    printf("form %d%s: wrong results per lane group [0-15, 16-31, 32-47, 48-63]: %u %u %u %u of %.0f\n", MODE, MFMA ? "" : " (no MFMA)", h[0],
           h[1], h[2], h[3], (double)blocks * 256.0 * iters);
    fflush(stdout);
}

int main(int argc, char **argv)
{
    const int blocks = argc > 1 ? atoi(argv[1]) : 8192, iters = argc > 2 ? atoi(argv[2]) : 400;
    unsigned *d_bad;
    CK(hipMalloc(&d_bad, 16 * sizeof(unsigned)));
    const int which = argc > 3 ? atoi(argv[3]) : 0;
    if (which == 0) {
        run<0>(d_bad, blocks, iters);
        run<1>(d_bad, blocks, iters);
        run<2>(d_bad, blocks, iters);
        run<3>(d_bad, blocks, iters);
        run<4>(d_bad, blocks, iters);
        run<5>(d_bad, blocks, iters);
        run<6>(d_bad, blocks, iters);
        run<7>(d_bad, blocks, iters);
    } else if (which == 3) {
        run<30, false>(d_bad, blocks, iters);
        run<30>(d_bad, blocks, iters);
        run<31, false>(d_bad, blocks, iters);
        run<31>(d_bad, blocks, iters);
        run<32, false>(d_bad, blocks, iters);
        run<32>(d_bad, blocks, iters);
        run<33>(d_bad, blocks, iters);
        run<34, false>(d_bad, blocks, iters);
        run<34>(d_bad, blocks, iters);
        run<35>(d_bad, blocks, iters);
        run<36>(d_bad, blocks, iters);
        run<1>(d_bad, blocks, iters);
    } else if (which == 2) {
        run<20>(d_bad, blocks, iters);
        run<21>(d_bad, blocks, iters);
        run<22>(d_bad, blocks, iters);
        run<23>(d_bad, blocks, iters);
        run<1>(d_bad, blocks, iters);
    } else {
        run<1, false>(d_bad, blocks, iters);
        run<10>(d_bad, blocks, iters);
        run<11>(d_bad, blocks, iters);
        run<12>(d_bad, blocks, iters);
        run<13>(d_bad, blocks, iters);
        run<14>(d_bad, blocks, iters);
        run<15>(d_bad, blocks, iters);
        run<16>(d_bad, blocks, iters);
        run<17>(d_bad, blocks, iters);
        run<1>(d_bad, blocks, iters);
    }
    return 0;
}
