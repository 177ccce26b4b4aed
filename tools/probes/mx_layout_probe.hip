// Probe: (1) LDS layout of global_load_lds with 12-byte pieces, (2) the lane map of
// v_mfma_f32_16x16x32_f16 (A[row l&15][k 8(l>>4)+e], B[k][col l&15], C col l&15 rows 4(l>>4)+i).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef float f4 __attribute__((ext_vector_type(4)));

__global__ void k_dma(const uint8_t *src, uint8_t *dst)
{
    __shared__ __attribute__((aligned(16))) uint8_t lds[2048];
    for (int i = threadIdx.x; i < 2048; i += 64) lds[i] = 0xEE;
    __syncthreads();
    const unsigned l = threadIdx.x;
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *)(src + 12 * l),
                                     (__attribute__((address_space(3))) void *)lds, 12, 0, 0);
    __builtin_amdgcn_s_waitcnt(0xF70);
    __syncthreads();
    for (int i = threadIdx.x; i < 2048; i += 64) dst[i] = lds[i];
}

__global__ void k_mma(const _Float16 *A, const _Float16 *B, float *D)
{
    const unsigned l = threadIdx.x;
    h8 a, b;
    for (int e = 0; e < 8; e++) {
        a[e] = A[(l & 15) * 32 + 8 * (l >> 4) + e];
        b[e] = B[(8 * (l >> 4) + e) * 16 + (l & 15)];
    }
    f4 c = {};
    c = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
    for (int i = 0; i < 4; i++) D[(4 * (l >> 4) + i) * 16 + (l & 15)] = c[i];
}

int main()
{
    uint8_t h[2048], *ds, *dd;
    for (int i = 0; i < 2048; i++) h[i] = (uint8_t)(i * 7 + 3);
    hipMalloc(&ds, 2048); hipMalloc(&dd, 2048);
    hipMemcpy(ds, h, 2048, hipMemcpyHostToDevice);
    k_dma<<<1, 64>>>(ds, dd);
    uint8_t o[2048];
    hipMemcpy(o, dd, 2048, hipMemcpyDeviceToHost);
    int ok12 = 1, ok16 = 1;
    for (int l = 0; l < 64; l++)
        for (int b = 0; b < 12; b++) {
            if (o[12 * l + b] != h[12 * l + b]) ok12 = 0;
            if (o[16 * l + b] != h[12 * l + b]) ok16 = 0;
        }
    printf("dma12: stride12 %s stride16 %s; first bytes:", ok12 ? "YES" : "no", ok16 ? "YES" : "no");
    for (int i = 0; i < 32; i++) printf(" %02x", o[i]);
    printf("\n");
    _Float16 A[16 * 32], B[32 * 16];
    float D[256], R[256];
    for (int m = 0; m < 16; m++) for (int k = 0; k < 32; k++) A[m * 32 + k] = (_Float16)(float)((m * 3 + k * 5) % 17 - 8);
    for (int k = 0; k < 32; k++) for (int n = 0; n < 16; n++) B[k * 16 + n] = (_Float16)(float)((k * 7 + n * 11) % 13 - 6);
    for (int m = 0; m < 16; m++) for (int n = 0; n < 16; n++) {
        float s = 0; for (int k = 0; k < 32; k++) s += (float)A[m * 32 + k] * (float)B[k * 16 + n];
        R[m * 16 + n] = s;
    }
    _Float16 *dA, *dB; float *dD;
    hipMalloc(&dA, sizeof A); hipMalloc(&dB, sizeof B); hipMalloc(&dD, sizeof D);
    hipMemcpy(dA, A, sizeof A, hipMemcpyHostToDevice); hipMemcpy(dB, B, sizeof B, hipMemcpyHostToDevice);
    k_mma<<<1, 64>>>(dA, dB, dD);
    hipMemcpy(D, dD, sizeof D, hipMemcpyDeviceToHost);
    int bad = 0;
    for (int i = 0; i < 256; i++) bad += D[i] != R[i];
    printf("mfma16x16x32_f16 map: %d/256 mismatches\n", bad);
    return 0;
}
