/*
 * jpgx_entropy.hip -- entropy-stage statistics on the device.
 *
 * What the reference's host runs on the hot path's output before it writes any bits:
 *   dpcm            src/dpcm.c:6-21        d_i = v_i - d_{i-1} over each channel's DCs, in place
 *   huffman_encode  src/huffman.c:23-44    frequency pass: per block calculate_freq_block_DC
 *                   (class of the dpcm'd DC, :182-185) and calculate_freq_block_AC (run/size
 *                   symbols, ZRL, EOB, :187-222, with the reference's `run | size`), into
 *                   lum_DC, lum_AC, chrom_DC (Cb and Cr), chrom_AC; freq[256] = 1 (:55).
 * (construct_huffman_table, which never terminates, is not part of this.)
 *
 * The recurrence is sequential; it is an alternating prefix sum:
 *     d_l = (-1)^l (P_l - c),  P_l = sum_{k<=l} (-1)^k v_k,  c = the DC carried in
 * so three launches per image: (A) per 256-block chunk, AC symbols into the histogram and the
 * chunk's sum of (-1)^k v_k; (B) one workgroup scans the chunk sums per channel; (C) per chunk,
 * the in-chunk scan, d_l, the DC classes.  Integer work, bound by reading the coefficients
 * once (A) plus their DC words (C).
 */
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "jpgx_internal.h"

namespace {

constexpr int kChunk = 256;     /* blocks per workgroup (one thread per block) */

__device__ __forceinline__ int dc_class(int v)   /* huffman.c:226-235 get_class */
{
    const unsigned a = (unsigned)(v < 0 ? -v : v);
    return a ? 32 - __builtin_clz(a) : 0;
}

struct Chunks {
    const int16_t *coef;        /* Y [nb_y][64] | Cb [nb_c][64] | Cr [nb_c][64]          */
    int32_t *dc;                /* [nb_y + 2 nb_c]                                       */
    uint32_t *hist;             /* [4][257]                                              */
    long long *part;            /* [nchunks] chunk sums of (-1)^k v_k (k local to channel) */
    unsigned nb[3];             /* blocks per channel                                    */
    unsigned first[3];          /* first chunk of each channel                           */
    unsigned off[3];            /* first block of each channel in coef / dc              */
    int carry[3];               /* DC carried in per channel (0 at the image start)      */
};

__device__ __forceinline__ void chunk_of(const Chunks &c, unsigned chunk, int &ch, unsigned &k0)
{
    ch = chunk >= c.first[2] ? 2 : (chunk >= c.first[1] ? 1 : 0);
    k0 = (chunk - c.first[ch]) * kChunk;
}

__global__ __launch_bounds__(kChunk) void k_stats_ac(const Chunks c)
{
    __shared__ uint32_t h[256];
    __shared__ long long wsum[kChunk / 64];
    int ch;
    unsigned k0;
    chunk_of(c, blockIdx.x, ch, k0);
    h[threadIdx.x] = 0;
    __syncthreads();
    const unsigned k = k0 + threadIdx.x;
    long long w = 0;
    if (k < c.nb[ch]) {
        const int16_t *z = c.coef + ((size_t)c.off[ch] + k) * 64;
        int zz[64];
        for (int i = 0; i < 64; i += 8) {            /* 16-byte loads */
            const uint4 q = *(const uint4 *)(z + i);
            const uint32_t u[4] = {q.x, q.y, q.z, q.w};
            for (int j = 0; j < 4; j++) {
                zz[i + 2 * j] = (int16_t)(u[j] & 0xffffu);
                zz[i + 2 * j + 1] = (int16_t)(u[j] >> 16);
            }
        }
        w = (k & 1) ? -(long long)zz[0] : (long long)zz[0];
        int last = 0;                                 /* huffman.c:193-199 */
        for (int i = 63; i > 0; i--)
            if (zz[i] != 0) {
                last = i;
                break;
            }
        int zeros = 0;
        for (int i = 1; i < 64; i++) {                /* :202-221 */
            if (i == last + 1) {
                atomicAdd(&h[0x00], 1u);              /* EOB */
                break;
            }
            if (zz[i] == 0) {
                if (++zeros == 16) {
                    atomicAdd(&h[0xF0], 1u);          /* ZRL */
                    zeros = 0;
                }
            } else {
                atomicAdd(&h[zeros | dc_class(zz[i])], 1u);
                zeros = 0;
            }
        }
    }
    /* chunk sum of (-1)^k v_k */
    for (int o = 32; o > 0; o >>= 1) w += __shfl_xor(w, o, 64);
    if ((threadIdx.x & 63) == 0) wsum[threadIdx.x >> 6] = w;
    __syncthreads();
    if (threadIdx.x == 0) {
        long long s = 0;
        for (int i = 0; i < kChunk / 64; i++) s += wsum[i];
        c.part[blockIdx.x] = s;
    }
    const uint32_t n = h[threadIdx.x];
    if (n) atomicAdd(&c.hist[(ch == 0 ? 1 : 3) * 257 + threadIdx.x], n);
}

/* exclusive scan of the chunk sums, per channel; one workgroup */
__global__ __launch_bounds__(kChunk) void k_stats_scan(const Chunks c, unsigned nchunks)
{
    __shared__ long long sh[kChunk];
    if (threadIdx.x < 4) c.hist[threadIdx.x * 257 + 256] = 1u;   /* reserved code point */
    for (int ch = 0; ch < 3; ch++) {
        const unsigned a = c.first[ch], b = ch < 2 ? c.first[ch + 1] : nchunks;
        long long run = 0;
        for (unsigned base = a; base < b; base += kChunk) {
            const unsigned i = base + threadIdx.x;
            const long long v = i < b ? c.part[i] : 0;
            sh[threadIdx.x] = v;
            __syncthreads();
            for (int o = 1; o < kChunk; o <<= 1) {    /* Hillis-Steele, inclusive */
                const long long t = threadIdx.x >= (unsigned)o ? sh[threadIdx.x - o] : 0;
                __syncthreads();
                sh[threadIdx.x] += t;
                __syncthreads();
            }
            if (i < b) c.part[i] = run + sh[threadIdx.x] - v;     /* exclusive */
            run += sh[kChunk - 1];
            __syncthreads();
        }
    }
}

__global__ __launch_bounds__(kChunk) void k_stats_dc(const Chunks c)
{
    __shared__ uint32_t h[33];                        /* classes 0..32 of an int */
    __shared__ long long wtot[kChunk / 64];
    int ch;
    unsigned k0;
    chunk_of(c, blockIdx.x, ch, k0);
    if (threadIdx.x < 33) h[threadIdx.x] = 0;
    const unsigned k = k0 + threadIdx.x;
    const bool live = k < c.nb[ch];
    const long long v = live ? (long long)c.coef[((size_t)c.off[ch] + k) * 64] : 0;
    long long p = (k & 1) ? -v : v;                   /* inclusive scan over the chunk */
    const unsigned lane = threadIdx.x & 63;
    for (int o = 1; o < 64; o <<= 1) {
        const long long t = __shfl_up(p, o, 64);
        if (lane >= (unsigned)o) p += t;
    }
    if (lane == 63) wtot[threadIdx.x >> 6] = p;
    __syncthreads();
    for (unsigned wv = 0; wv < (threadIdx.x >> 6); wv++) p += wtot[wv];
    if (live) {
        const long long P = c.part[blockIdx.x] + p;
        const long long d = (k & 1) ? -(P - c.carry[ch]) : (P - c.carry[ch]);
        const int di = (int)d;                        /* the reference's int */
        c.dc[c.off[ch] + k] = di;
        atomicAdd(&h[dc_class(di)], 1u);
    }
    __syncthreads();
    if (threadIdx.x < 33 && h[threadIdx.x])
        atomicAdd(&c.hist[(ch == 0 ? 0 : 2) * 257 + threadIdx.x], h[threadIdx.x]);
}

int hip_rc2(hipError_t e) { return e == hipSuccess ? JPGX_OK : JPGX_EHIP; }

size_t nchunks_of(size_t nb_y, size_t nb_c)
{
    return (nb_y + kChunk - 1) / kChunk + 2 * ((nb_c + kChunk - 1) / kChunk);
}

}  // namespace

extern "C" {

size_t jpgx_entropy_workspace_size(size_t nb_y, size_t nb_c)
{
    return nchunks_of(nb_y, nb_c) * sizeof(long long);
}

int jpgx_entropy_stats_gpu(const int16_t *d_coef, size_t nb_y, size_t nb_c, const int32_t *carry,
                           int32_t *d_dc, uint32_t *d_hist, void *d_workspace,
                           size_t workspace_bytes, void *stream)
{
    if (!d_coef || !d_dc || !d_hist || ((uintptr_t)d_coef & 15) || nb_y == 0 ||
        nb_y + 2 * nb_c >= (1ull << 31))
        return JPGX_EARG;
    const size_t nch = nchunks_of(nb_y, nb_c);
    if (!d_workspace || workspace_bytes < nch * sizeof(long long) || ((uintptr_t)d_workspace & 7))
        return JPGX_EWORKSPACE;
    Chunks c;
    c.coef = d_coef;
    c.dc = d_dc;
    c.hist = d_hist;
    c.part = (long long *)d_workspace;
    c.nb[0] = (unsigned)nb_y;
    c.nb[1] = c.nb[2] = (unsigned)nb_c;
    c.first[0] = 0;
    c.first[1] = (unsigned)((nb_y + kChunk - 1) / kChunk);
    c.first[2] = c.first[1] + (unsigned)((nb_c + kChunk - 1) / kChunk);
    c.off[0] = 0;
    c.off[1] = (unsigned)nb_y;
    c.off[2] = (unsigned)(nb_y + nb_c);
    for (int k = 0; k < 3; k++) c.carry[k] = carry ? carry[k] : 0;
    hipStream_t s = (hipStream_t)stream;
    int rc = hip_rc2(hipMemsetAsync(d_hist, 0, 4 * 257 * sizeof(uint32_t), s));
    if (rc) return rc;
    hipLaunchKernelGGL(k_stats_ac, dim3((unsigned)nch), dim3(kChunk), 0, s, c);
    hipLaunchKernelGGL(k_stats_scan, dim3(1), dim3(kChunk), 0, s, c, (unsigned)nch);
    hipLaunchKernelGGL(k_stats_dc, dim3((unsigned)nch), dim3(kChunk), 0, s, c);
    return hip_rc2(hipGetLastError());
}

}  /* extern "C" */
