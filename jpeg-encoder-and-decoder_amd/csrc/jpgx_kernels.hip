/*
 * jpgx_kernels.hip -- gfx950 kernels of the block-transform hot path + the device C-ABI.
 *
 * k_xform (all-VALU; one lane = one 8x8 block, all 3 channels)
 *   HBM -> VGPR: each lane loads its block's 8 pixel rows (8 x 24 B; a wave covers 64
 *   horizontally adjacent blocks = 1.5 KiB contiguous per pixel row).
 *   Per channel, entirely in the lane's registers (no cross-lane traffic):
 *     byte -> f32, colour + level shift (3 FMAs/px)        src/preprocess.c:160-162,186-188
 *     row DCT then column DCT, even/odd 8-point DCT-II      src/dct.c:36-59
 *     quantise: one FMA with the per-coefficient fp32 scale (1/Q and DCT normalisation
 *       folded) that also rounds to an integer (+1.5*2^23)  src/quantise.c:52-72 (transposed)
 *     each int16 to the wave's LDS stage at its zig-zag position  src/zig_zag.c:48-58
 *   LDS -> HBM: the wave's 64 blocks x 128 B of a channel leave as 8 KiB of contiguous
 *   16-B-per-lane nontemporal stores.
 *   Exactness: a block-channel with a coefficient inside the rigorous guard band of a .5
 *   boundary (jpgx_plan.cpp) is queued in the wave's LDS and, after the wave's last tile,
 *   recomputed eight blocks at a time in the reference's exact fp64 operation order: double
 *   colour conversion in its operand order, -128, the 64-term sum x-outer / y-inner with
 *   (X*c_u[x])*c_v[y] and the glibc cosine doubles, ((0.25*a_u)*a_v)*s, true double division
 *   by the transposed table entry, round() half away from zero.
 * k_chroma<1|2>: true 4:2:2 / 4:2:0 chroma of the test-only cross-check library; k_xform does Y.
 * k_mx / k_mx422 / k_mx420 (csrc/jpgx_mx.hip): the product kernels (4:4:4, true 4:2:2 / 4:2:0)
 *   with the colour conversion and row DCT on the matrix cores.
 *
 * Compiled with FP contraction off; the fast path uses explicit fmaf.  Variants of k_xform
 * measured slower are kept out of this file: tools/probes/k_xform_variants.patch (git history: 63924df).
 */
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <mutex>
#include <thread>
#include <vector>

#include "jpgx_internal.h"
#include "jx_consts.h"
#include "xform_math.h"

#pragma clang fp contract(off)

namespace {

constexpr float kMagic = 12582912.0f; /* 1.5 * 2^23: x + kMagic rounds x to an integer   */
/* per-wave, per-channel queue of blocks with a coefficient inside the guard band */
constexpr int kItems = 128;
static_assert(kItems >= 64, "a tile adds at most 64 items per channel");

/* zig_zag.c:6-15: scan position of natural (row v, column u) */
__host__ __device__ constexpr int zz_of(int v, int u)
{
    constexpr int t[64] = {0,  1,  5,  6,  14, 15, 27, 28, 2,  4,  7,  13, 16, 26, 29, 42,
                           3,  8,  12, 17, 25, 30, 41, 43, 9,  11, 18, 24, 31, 40, 44, 53,
                           10, 19, 23, 32, 39, 45, 52, 54, 20, 22, 33, 38, 46, 51, 55, 60,
                           21, 34, 37, 47, 50, 56, 59, 61, 35, 36, 48, 49, 57, 58, 62, 63};
    return t[v * 8 + u];
}

/* scan position of natural (row v, column u) for a runtime index (jx_consts.h) */
__constant__ int kScan[8][8] = JX_SCAN_ORDER_INIT;
__device__ __forceinline__ int zz_of_rt(int v, int u) { return kScan[v][u]; }

/* cos(((2x+1)*u*M_PI)/16) exactly as glibc returns it for the reference (jx_consts.h) */
__constant__ double kCos[8][8] = JX_COS_INIT;

/* Per-quality tables (index 0 unused), constant address space so that wave-uniform reads
 * become scalar loads; filled once per device by tables_for_current_device(). */
__constant__ jx_qtab g_qtab[JX_MAXQ + 1];
__constant__ jx_limtab g_lim[2][JX_MAXQ + 1];
/* true chroma subsampling (k_chroma): [sub-1][force][q], chroma bounds of averaged samples */
__constant__ jx_limtab g_limsub[2][2][JX_MAXQ + 1];

/* dct.c:13 ALPHA(0) = 1/sqrt(2) as the reference's double */
constexpr double kAlpha0 = JX_ALPHA0;

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef float f2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

/* coefficient stores with the nontemporal bit (streamed, never re-read): 0.186 -> 0.158 ms
 * early on, DESIGN.md 4.1 */
__device__ __forceinline__ void jx_store(u32x4 *p, u32x4 v) { __builtin_nontemporal_store(v, p); }

/* Per-wave LDS: each int16 goes to the stage as it is produced (no register packing: fewer
 * live VGPRs, what lets 3 waves share a SIMD) */
struct WaveLds {
    uint32_t stage[64 * 33];      /* one channel: block k at dwords 33k.. (odd stride: the
                                     16-bit writes of 64 lanes hit 64 different banks)      */
    uint32_t item[3][kItems];     /* per channel: queued launch-global block indices       */
};

/* 16-B unit e (block e/8, zig-zag chunk e%8) of the staged channel */
__device__ __forceinline__ u32x4 stage_unit(const WaveLds &W, unsigned e)
{
    const unsigned o = (e >> 3) * 33 + (e & 7) * 4;
    return u32x4{W.stage[o], W.stage[o + 1], W.stage[o + 2], W.stage[o + 3]};
}

__device__ __forceinline__ uint32_t byte_of(const uint32_t (&row)[6], int k)
{
    return (row[k >> 2] >> (8 * (k & 3))) & 0xffu;
}

/*
 * The 8 pixel rows block `bi` of frame `f` reads, with the reference's addressing:
 * blockToCoords (src/preprocess.c:199-211) gives x0 = -8 for the last block of a block-row,
 * which with offset = (y+y0)*W + x0 + x (:159) means pixel row 8r+y-1, columns W-8..W-1;
 * for frame block-row 0, y = 0 those are the bytes in front of the planes (g.under).
 */
__device__ __forceinline__ void load_block(const jx_geom &g, unsigned f, unsigned bi,
                                           uint32_t (&raw)[8][6])
{
    const unsigned r = bi / (unsigned)g.bpr, c = bi - r * (unsigned)g.bpr;
    const bool last = c == (unsigned)g.bpr - 1;
    const bool under = last && (g.row0 + (int)r == 0);
    const long long row = 8ll * r - (last ? 1 : 0);
    const uint8_t *base = g.rgb + (long long)f * g.in_fstride + row * g.in_pitch + 24ll * c;
#pragma unroll
    for (int y = 0; y < 8; y++) {
        const uint8_t *p = base + (long long)(y == 0 && under ? 1 : y) * g.in_pitch;
        p = (const uint8_t *)__builtin_assume_aligned(p, 8);
        u32x4 a;
        u32x2 b;
        __builtin_memcpy(&a, p, 16);
        __builtin_memcpy(&b, p + 16, 8);
        raw[y][0] = a.x; raw[y][1] = a.y; raw[y][2] = a.z; raw[y][3] = a.w;
        raw[y][4] = b.x; raw[y][5] = b.y;
    }
    if (under) {
#pragma unroll
        for (int k = 0; k < 6; k++) raw[0][k] = g.under[k];
    }
}

/* ---- exact path -------------------------------------------------------------------------- */

/* Exact reference value of one channel pixel, level shift included (preprocess.c:160-162,
 * 186-188); r,g,b promoted int -> double as in the reference. */
__device__ __forceinline__ double exact_pixel(int ch, int r, int g, int b)
{
    if (ch == 0) {
        const double yv = 0.299 * r + 0.587 * g + 0.114 * b;
        return yv - 128;
    }
    if (ch == 1) {
        const double cb = 128 - (0.168736 * r - 0.331264 * g + 0.5 * b);
        return cb - 128;
    }
    const double cr = 128 + (0.5 * r - 0.418688 * g - 0.081312 * b);
    return cr - 128;
}

/* One coefficient in the reference's exact operation order.  raw = the block's 8 pixel rows
 * (24 interleaved bytes each) in registers. */
__device__ __forceinline__ int16_t *coef_ptr(const jx_geom &g, unsigned b, int ch, int zz)
{
    const unsigned nb = (unsigned)g.nb, f = b / nb, bi = b - f * nb;
    return g.out + (long long)f * g.out_fstride + ((long long)ch * nb + bi) * 64 + zz;
}

/* number of set bits of m below this lane */
__device__ __forceinline__ int lane_rank(uint64_t m)
{
    return (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                          __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

/* ---- fast path --------------------------------------------------------------------------- */

/* jx_pixel<FOps, CH> for a (uniform) runtime channel: the same fmaf sequence, constants by
 * select; fma(b, k, -0) is the plain product b*k bit for bit (sign of zero included). */
__device__ __forceinline__ float pixel_k(const int CH, float r, float g, float b)
{
    const float k0 = CH == 0 ? JX_K(0.299).f : (CH == 1 ? JX_K(-0.168736).f : JX_K(0.5).f);
    const float k1 = CH == 0 ? JX_K(0.587).f : (CH == 1 ? JX_K(0.331264).f : JX_K(-0.418688).f);
    const float k2 = CH == 0 ? JX_K(0.114).f : (CH == 1 ? JX_K(-0.5).f : JX_K(-0.081312).f);
    const float k3 = CH == 0 ? JX_K(-128.0).f : -0.0f;
    return __builtin_fmaf(r, k0, __builtin_fmaf(g, k1, __builtin_fmaf(b, k2, k3)));
}

__device__ __forceinline__ void row_pixels(const int CH, const uint32_t (&row)[6], float (&px)[8])
{
#pragma unroll
    for (int x = 0; x < 8; x++) {
        const float r = (float)byte_of(row, 3 * x);
        const float gg = (float)byte_of(row, 3 * x + 1);
        const float bb = (float)byte_of(row, 3 * x + 2);
        px[x] = pixel_k(CH, r, gg, bb);
    }
}

/* Row pass of channel CH: bytes -> pixel values -> 1-D DCT of each of the 8 pixel rows. */
__device__ __forceinline__ void xform_rows(const int CH, uint32_t (&raw)[8][6], float (&T)[8][8])
{
    /* Opaque to the optimiser: forces each channel to re-convert its bytes instead of
     * keeping 192 converted floats alive across the three channel passes (CSE). */
#pragma unroll
    for (int y = 0; y < 8; y++)
#pragma unroll
        for (int k = 0; k < 6; k++) asm volatile("" : "+v"(raw[y][k]));
#pragma unroll
    for (int y = 0; y < 8; y++) {
        float px[8];
        row_pixels(CH, raw[y], px);
        jx_fdct8<FOps>(px, T[y]);
    }
}

/* Quantise one coefficient in fp32: tm = rint(F*w) + 1.5*2^23 (its low 16 bits are the int16)
 * and d = F*w - rint(F*w), exact (the guard band tests |d|). */
__device__ __forceinline__ void quant_coef(float F, float w, float &tm, float &d)
{
    tm = __builtin_fmaf(F, w, kMagic);
    const float rr = tm - kMagic;                /* exact */
    d = __builtin_fmaf(F, w, -rr);
}

/* per-wave queue state (wave-uniform) */
struct Queue {
    int n[3];               /* items in the LDS queue                                     */
    unsigned done[3];       /* items already moved to the wave's global region            */
};

/* The staged channel CH of tile t leaves as coalesced stores; lanes in `seen` (a coefficient
 * of this channel inside the guard band) queue their block-channel for the exact pass. */
__device__ __forceinline__ void store_and_queue(const int CH, const jx_xform_args &a, WaveLds &W, Queue &Q,
                                                bool active, unsigned b, unsigned t,
                                                unsigned lane, uint64_t seen)
{
    const jx_geom &g = a.g;
    /* coalesced store: the wave's 64 blocks x 128 B of this channel, 1 KiB per instruction */
    const unsigned nb = (unsigned)g.nb, total = nb * (unsigned)g.nframes;
    const unsigned b0 = t * 64u;
    const unsigned f0 = b0 / nb, bl = std::min(b0 + 63u, total - 1u), fl = bl / nb;
    if (f0 == fl && b0 + 63u < total) {
        u32x4 *dst = (u32x4 *)(g.out + (long long)f0 * g.out_fstride +
                               ((long long)CH * nb + (b0 - f0 * nb)) * 64);
        /* unit e = 64j + lane is at dword o0 + 264j: one base, recomputed here (opaque) so
         * that eight loop-invariant addresses are not hoisted out of the tile loop and spilled */
        unsigned o0 = (lane >> 3) * 33 + (lane & 7) * 4;
        asm volatile("" : "+v"(o0));
        /* all eight LDS reads first, one wait, then the eight stores (interleaved, every
         * store waited for its own read) */
        u32x4 unit[8];
#pragma unroll
        for (int j = 0; j < 8; j++) {
            const unsigned o = o0 + 264u * (unsigned)j;
            unit[j] = u32x4{W.stage[o], W.stage[o + 1], W.stage[o + 2], W.stage[o + 3]};
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int j = 0; j < 8; j++) jx_store(dst + (unsigned)j * 64u + lane, unit[j]);
    } else {                                   /* tile crosses a frame end or the last tile */
        /* units past the end hold block total-1's coefficients (inactive lanes computed the
         * clamped block): they are written there again, identical bytes */
#pragma unroll
        for (int j = 0; j < 8; j++) {
            const unsigned e = (unsigned)j * 64u + lane, bb = std::min(b0 + (e >> 3), total - 1u);
            jx_store((u32x4 *)coef_ptr(g, bb, CH, (int)(e & 7) * 8), stage_unit(W, e));
        }
    }
    /* some lane has a coefficient inside the guard band (about 40% of the channel-tiles of
     * random data at q90; wave-uniform branch): queue its block-channel */
    if (seen != 0) {
        const uint64_t M = seen & __ballot(active);
        /* (selects, not Q.n[CH]: a runtime index would put Q in scratch memory) */
        const int n = CH == 0 ? Q.n[0] : (CH == 1 ? Q.n[1] : Q.n[2]);
        if ((M >> lane) & 1u) W.item[CH][n + lane_rank(M)] = b;
        const int nn = n + __popcll(M);
        Q.n[0] = CH == 0 ? nn : Q.n[0];
        Q.n[1] = CH == 1 ? nn : Q.n[1];
        Q.n[2] = CH == 2 ? nn : Q.n[2];
    }
}

/* Column pass, quantisation, zig-zag, LDS staging + coalesced store of channel CH; block-
 * channels with a coefficient inside the guard band are queued for the exact path. */
__device__ __forceinline__ void xform_cols(const int CH, float (&T)[8][8], const jx_xform_args &a, WaveLds &W,
                                           Queue &Q, bool active, unsigned b, unsigned t,
                                           unsigned lane)
{
    const jx_qtab &tab = g_qtab[a.quality];
    const int fe = a.force_exact ? 1 : 0;
    const jx_limtab &band = a.sub ? g_limsub[a.sub - 1][fe][a.quality] : g_lim[fe][a.quality];
    /* wave mask of lanes with a coefficient of this channel inside the guard band */
    uint64_t seen = 0;
#pragma unroll
    for (int u = 0; u < 8; u++) {
        /* column u's 16 table values: wave-uniform, scalar loads */
        float wc[8], lc[8];
#pragma unroll
        for (int v = 0; v < 8; v++) {
            wc[v] = tab.w[CH][u][v];
            lc[v] = band.lim[CH][u][v];
        }
        float col[8], F[8];
#pragma unroll
        for (int y = 0; y < 8; y++) col[y] = T[y][u];
        jx_fdct8<FOps>(col, F);
#pragma unroll
        for (int v = 0; v < 8; v++) {
            float tm, d;
            quant_coef(F[v], wc[v], tm, d);
            ((uint16_t *)W.stage)[lane * 66 + zz_of(v, u)] = (uint16_t)__float_as_uint(tm);
            /* compare straight into a lane mask, OR-ed at once (left to the compiler, the 64
             * masks of a channel are kept alive until the end and spilled) */
            uint64_t m;
            asm("v_cmp_ge_f32_e64 %[m], |%[d]|, %[l]\n\t"
                "s_or_b64 %[seen], %[seen], %[m]"
                : [m] "=&s"(m), [seen] "+s"(seen)
                : [d] "v"(d), [l] "s"(lc[v])
                : "scc");
        }
        /* scheduling fence between the column DCTs of a channel (measured faster) */
        __builtin_amdgcn_sched_barrier(0);
    }
    store_and_queue(CH, a, W, Q, active, b, t, lane, seen);
}

/* exact_coef's last step: F(u,v) = 1/4 a(u) a(v) s (dct.c:54), round(F / Q) (quantise.c:58) */
__device__ __forceinline__ int16_t exact_finish(double s, int u, int v, int q)
{
    const double F = 0.25 * (u == 0 ? kAlpha0 : 1.0) * (v == 0 ? kAlpha0 : 1.0) * s;
    return (int16_t)(int)round(F / (double)q);
}

/* pixel row y of block bi of frame f, with load_block's addressing (x0 = -8 quirk) */
__device__ __forceinline__ void load_row(const jx_geom &g, unsigned f, unsigned bi, unsigned y,
                                         uint32_t (&row)[6])
{
    const unsigned r = bi / (unsigned)g.bpr, c = bi - r * (unsigned)g.bpr;
    const bool last = c == (unsigned)g.bpr - 1;
    if (last && y == 0 && g.row0 + (int)r == 0) {
#pragma unroll
        for (int k = 0; k < 6; k++) row[k] = g.under[k];
        return;
    }
    const long long pr = 8ll * r - (last ? 1 : 0) + y;
    const uint8_t *p = g.rgb + (long long)f * g.in_fstride + pr * g.in_pitch + 24ll * c;
    p = (const uint8_t *)__builtin_assume_aligned(p, 8);
    u32x4 a;
    u32x2 b;
    __builtin_memcpy(&a, p, 16);
    __builtin_memcpy(&b, p + 16, 8);
    row[0] = a.x; row[1] = a.y; row[2] = a.z; row[3] = a.w;
    row[4] = b.x; row[5] = b.y;
}

__device__ __forceinline__ void wave_sync_lds()
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

/* LDS of one k_fix wave, 8 blocks at a time */
struct FixLds8 {
    uint32_t px[8][8][6];                      /* [block][row] pixel rows                    */
    union {
        float T[64 * 9];                       /* (A) row-DCT outputs, (block*8 + row)*9 + u */
        double prod[8][8][8];                  /* (B) [task slot][x][y] terms of exact sums  */
    };
    uint32_t blk[8];                           /* launch-global block indices                */
    uint8_t bch[8];                            /* and their channels                         */
    uint16_t task[8 * 64];                     /* block << 6 | natural coefficient index     */
};

/* jx_pixel for a per-lane channel (all three formed, one kept: same fp32 operations) */
__device__ __forceinline__ float pixel_rt(int ch, float r, float g, float b)
{
    const float y = jx_pixel<FOps, 0>(r, g, b), cb = jx_pixel<FOps, 1>(r, g, b),
                cr = jx_pixel<FOps, 2>(r, g, b);
    return ch == 0 ? y : (ch == 1 ? cb : cr);
}

/*
 * Exact pass over up to 8 blocks, eight lanes each (lane = block << 3 | j):
 * (A) lane j loads pixel row j, parks it in LDS and runs the fp32 row transform; then lane j
 *     runs column j (the same FOps code as k_xform, so the same coefficients come out inside
 *     the guard band) and tests its 8 coefficients;
 * (B) eight flagged coefficients at a time, eight lanes each: lane x forms the 8 terms
 *     (X(x,y) c_u[x]) c_v[y] of its column in fp64, then one lane sums the 64 terms in the
 *     reference's x-outer / y-inner order (dct.c:46-50) -- the same additions in the same
 *     order as exact_sum, spread so that the products run in parallel.
 */
__device__ __forceinline__ void fix_chunk8(FixLds8 &L, const jx_xform_args &a, unsigned b, int ch,
                                           bool has, unsigned lane)
{
    const jx_geom &g = a.g;
    const unsigned nb = (unsigned)g.nb;
    const unsigned i = lane >> 3, j = lane & 7u;
    const jx_qtab &tab = g_qtab[a.quality];
    const jx_limtab &band = g_lim[a.force_exact ? 1 : 0][a.quality];
    if (has) {                                             /* (A) rows */
        const unsigned f = b / nb;
        uint32_t row[6];
        load_row(g, f, b - f * nb, j, row);
#pragma unroll
        for (int k = 0; k < 6; k++) L.px[i][j][k] = row[k];
        if (j == 0) {
            L.blk[i] = b;
            L.bch[i] = (uint8_t)ch;
        }
        float px[8], T[8];
#pragma unroll
        for (int x = 0; x < 8; x++) {
            const float r = (float)byte_of(row, 3 * x);
            const float gg = (float)byte_of(row, 3 * x + 1);
            const float bb = (float)byte_of(row, 3 * x + 2);
            px[x] = pixel_rt(ch, r, gg, bb);
        }
        jx_fdct8<FOps>(px, T);
#pragma unroll
        for (int u = 0; u < 8; u++) L.T[(i * 8 + j) * 9 + u] = T[u];
    }
    wave_sync_lds();
    unsigned flags = 0;                                    /* bit v: coefficient (u = j, v) */
    if (has) {                                             /* (A) column u = j */
        float col[8], F[8];
#pragma unroll
        for (int y = 0; y < 8; y++) col[y] = L.T[(i * 8 + y) * 9 + j];
        jx_fdct8<FOps>(col, F);
#pragma unroll
        for (int v = 0; v < 8; v++) {
            float tm, d;
            quant_coef(F[v], tab.w[ch][j][v], tm, d);
            if (__builtin_fabsf(d) >= band.lim[ch][j][v]) flags |= 1u << v;
        }
    }
    /* exclusive prefix of the per-lane task counts -> task list */
    const unsigned n = (unsigned)__popc(flags);
    unsigned incl = n;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const unsigned o = __shfl_up(incl, d, 64);
        if ((int)lane >= d) incl += o;
    }
    const unsigned total = __builtin_amdgcn_readlane(incl, 63);
    unsigned pos = incl - n;
    while (flags) {
        const unsigned v = (unsigned)__builtin_ctz(flags);
        flags &= flags - 1;
        L.task[pos++] = (uint16_t)(i << 6 | v << 3 | j);
    }
    wave_sync_lds();
    const unsigned x = j;
    /* the blocks' tile stores came from other lanes: they must
     * have landed before the exact values are written over them */
    if (total) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    for (unsigned t0 = 0; t0 < total; t0 += 8) {           /* (B) */
        const unsigned t = t0 + i;
        const bool live = t < total;
        const unsigned tk = live ? L.task[t] : 0u, src = tk >> 6, k = tk & 63u;
        const int u = (int)(k & 7u), v = (int)(k >> 3);
        const int tch = live ? (int)L.bch[src] : 0;
        if (live) {
            const double cu = kCos[u][x];
            const int k0 = (int)(3 * x) >> 2, sh = (int)(3 * x) & 3;
#pragma unroll
            for (int y = 0; y < 8; y++) {
                /* the 3 bytes of pixel x: dwords k0 and k0+1 (k0 + 1 <= 5) */
                const uint64_t w = (uint64_t)L.px[src][y][k0] |
                                   ((uint64_t)L.px[src][y][k0 + 1 < 6 ? k0 + 1 : 5] << 32);
                const uint32_t p3 = (uint32_t)(w >> (8 * sh));
                const int r = (int)(p3 & 0xffu), gg = (int)((p3 >> 8) & 0xffu),
                          bb = (int)((p3 >> 16) & 0xffu);
                L.prod[i][x][y] = exact_pixel(tch, r, gg, bb) * cu * kCos[v][y];
            }
        }
        wave_sync_lds();
        if (live && x == 0) {
            double s = 0.0;
#pragma unroll
            for (int xx = 0; xx < 8; xx++)
#pragma unroll
                for (int y = 0; y < 8; y++) s += L.prod[i][xx][y];
            *coef_ptr(g, L.blk[src], tch, zz_of_rt(v, u)) =
                exact_finish(s, u, v, tab.q[tch == 0 ? 0 : 1][u * 8 + v]);
        }
        wave_sync_lds();                                   /* prod reused */
    }
}

static_assert(sizeof(FixLds8) <= sizeof(WaveLds::stage), "FixLds8 lives in the staging area");


/* Exact pass of up to 8 queued blocks, taken from the tails of the three channel queues in
 * turn, inside k_xform (the staging area is free between tiles; fix_chunk8 waits for the
 * wave's tile stores before it writes). */
template <class WL>
__device__ __forceinline__ void fix_queued(WL &W, int (&n)[3], const jx_xform_args &a,
                                        unsigned lane)
{
    const int k0 = std::min(n[0], 8), k1 = std::min(n[1], 8 - k0),
              k2 = std::min(n[2], 8 - k0 - k1);
    const int i = (int)(lane >> 3);
    int ch = 2, at = n[2] - k2 + (i - k0 - k1);
    if (i < k0) {
        ch = 0;
        at = n[0] - k0 + i;
    } else if (i < k0 + k1) {
        ch = 1;
        at = n[1] - k1 + (i - k0);
    }
    const bool has = i < k0 + k1 + k2;
    const unsigned b = has ? W.item[ch][at] : 0u;
    n[0] -= k0;
    n[1] -= k1;
    n[2] -= k2;
    fix_chunk8(*reinterpret_cast<FixLds8 *>(W.stage), a, b, ch, has, lane);
}

/*
 * Persistent: each wave walks tiles t, t + waves, ...; per tile: load the tile's pixel rows
 * (the wait also drains the previous tile's stores), the three channels, and an exact pass
 * only when a queue could overflow (rare); the rest of the exact pass runs after the wave's
 * last tile.
 */
__global__ __launch_bounds__(JX_WG, 3) void k_xform(const jx_xform_args a)
{
    __shared__ WaveLds s_wave[JX_WG / 64];
    const jx_geom &g = a.g;
    const unsigned nb = (unsigned)g.nb;
    const unsigned total = nb * (unsigned)g.nframes;
    const unsigned ntiles = (total + 63u) / 64u;
    const unsigned lane = threadIdx.x & 63u;
    const unsigned nwaves = gridDim.x * (JX_WG / 64);
    /* wave-uniform (readfirstlane: the compiler cannot see that threadIdx.x >> 6 is), so the
     * tile loop and its branches are scalar */
    unsigned t = __builtin_amdgcn_readfirstlane(blockIdx.x * (JX_WG / 64) + (threadIdx.x >> 6));
    if (t >= ntiles) return;
    WaveLds &W = s_wave[threadIdx.x >> 6];
    Queue Q{{0, 0, 0}, {0u, 0u, 0u}};
    uint32_t raw[8][6];
    for (; t < ntiles; t += nwaves) {
        const unsigned b0 = t * 64u + lane;
        const bool active = b0 < total;
        const unsigned b = active ? b0 : total - 1;
        {
            const unsigned f = b / nb;
            load_block(g, f, b - f * nb, raw);
        }
        float T[8][8];
        xform_rows(0, raw, T);
        xform_cols(0, T, a, W, Q, active, b, t, lane);
        __builtin_amdgcn_sched_barrier(0);
        if (!a.luma_only) {                      /* (true subsampling: chroma in k_chroma) */
            xform_rows(1, raw, T);
            xform_cols(1, T, a, W, Q, active, b, t, lane);
            __builtin_amdgcn_sched_barrier(0);
            xform_rows(2, raw, T);
            xform_cols(2, T, a, W, Q, active, b, t, lane);
            __builtin_amdgcn_sched_barrier(0);
        }
        /* only when a queue could overflow (rare): the rest waits for the kernel's end */
        while (Q.n[0] > kItems - 64 || Q.n[1] > kItems - 64 || Q.n[2] > kItems - 64)
            fix_queued(W, Q.n, a, lane);
    }
    while (Q.n[0] + Q.n[1] + Q.n[2] > 0) fix_queued(W, Q.n, a, lane);
}

/* ---- k_chroma: true 4:2:2 / 4:2:0 chroma (extension) ---------------------------------------
 * The reference's subsample_422/420 (src/downsample.c:24-32) only print; oracle/cpu_ref.h
 * defines the semantics this kernel implements: level-shifted Cb/Cr (preprocess.c:161-162,
 * 186-188) averaged over the horizontal pixel pair (4:2:2) or the 2x2 quad (4:2:0) -- the
 * Notes' "level shift before chroma subsample" -- tiled in raster order on the (W/2) x H or
 * (W/2) x (H/2) plane, then the same DCT, transposed chroma quantisation, zig-zag, guard band
 * (bounds of the averaged samples, g_limsub) and exact fallback.  One lane per chroma block,
 * one channel at a time, pixel rows read as they are transformed (no 96-register tile).
 * g.bpr = chroma blocks per row, g.nb = chroma blocks per frame stripe, g.out offset so that
 * channel ch lands at out + (nb_y + (ch-1) nbc) * 64 of each frame. */

/* exact sample (level shift, then the average), the oracle's double operations */
__device__ __forceinline__ double exact_chroma(const jx_geom &g, int sub, int ch, unsigned f,
                                               unsigned X, unsigned Y)
{
    const uint8_t *p = g.rgb + (long long)f * g.in_fstride +
                       (long long)(sub == 2 ? 2 * Y : Y) * g.in_pitch + 6ll * X;
    const double e0 = exact_pixel(ch, p[0], p[1], p[2]), e1 = exact_pixel(ch, p[3], p[4], p[5]);
    if (sub == 1) return (e0 + e1) * 0.5;
    const uint8_t *q = p + g.in_pitch;
    const double e2 = exact_pixel(ch, q[0], q[1], q[2]), e3 = exact_pixel(ch, q[3], q[4], q[5]);
    return ((e0 + e1) + (e2 + e3)) * 0.25;
}

/* Exact recomputation of every queued block of channel ch (the whole block: the exact value
 * is the definition), one coefficient per lane; written over the fast values once the
 * tile's stores have landed. */
__device__ void fix_chroma(WaveLds &W, Queue &Q, int ch, const jx_xform_args &a, unsigned lane)
{
    const jx_geom &g = a.g;
    const int n = ch == 1 ? Q.n[1] : Q.n[2];
    if (n == 0) return;
    double *smp = reinterpret_cast<double *>(W.stage);
    const unsigned nb = (unsigned)g.nb, bpr = (unsigned)g.bpr;
    const int u = (int)(lane & 7u), v = (int)(lane >> 3);
    const int qd = g_qtab[a.quality].q[1][u * 8 + v];
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    for (int i = 0; i < n; i++) {
        const unsigned b = W.item[ch][i];
        const unsigned f = b / nb, bi = b - f * nb, by = bi / bpr, bx = bi - by * bpr;
        smp[lane] = exact_chroma(g, a.sub, ch, f, 8 * bx + (lane & 7u), 8 * by + (lane >> 3));
        wave_sync_lds();
        double s = 0.0;
#pragma unroll
        for (int x = 0; x < 8; x++)              /* dct.c:46-50: x outer, y inner */
#pragma unroll
            for (int y = 0; y < 8; y++) s += smp[y * 8 + x] * kCos[u][x] * kCos[v][y];
        *coef_ptr(g, b, ch, zz_of_rt(v, u)) = exact_finish(s, u, v, qd);
        wave_sync_lds();
    }
    if (ch == 1) Q.n[1] = 0; else Q.n[2] = 0;
}

template <int SUB>
__device__ __forceinline__ void chroma_rows(const int CH, const jx_geom &g, unsigned f, unsigned bx,
                                            unsigned by, float (&T)[8][8])
{
#pragma unroll
    for (int y = 0; y < 8; y++) {
        const unsigned Y = 8 * by + y;
        const uint8_t *p = g.rgb + (long long)f * g.in_fstride +
                           (long long)(SUB == 2 ? 2 * Y : Y) * g.in_pitch + 48ll * bx;
        p = (const uint8_t *)__builtin_assume_aligned(p, 8);
        uint32_t r0[12], r1[12];
#pragma unroll
        for (int k = 0; k < 6; k++) {
            u32x2 w;
            __builtin_memcpy(&w, p + 8 * k, 8);
            r0[2 * k] = w.x; r0[2 * k + 1] = w.y;
            if (SUB == 2) {
                __builtin_memcpy(&w, p + g.in_pitch + 8 * k, 8);
                r1[2 * k] = w.x; r1[2 * k + 1] = w.y;
            }
        }
        const auto bt = [](const uint32_t (&r)[12], int i) {
            return (float)((r[i >> 2] >> (8 * (i & 3))) & 0xffu);
        };
        float smp[8];
#pragma unroll
        for (int x = 0; x < 8; x++) {
            /* the colour transform is linear: convert the byte sums of the pair / quad (exact
             * in fp32) once and scale (the guard band, jpgx_plan.cpp coef_bounds, is derived
             * for this sequence; the exact pass keeps the definition's average of samples) */
            const int i0 = 6 * x, i1 = 6 * x + 3;        /* bytes of pixels 2x, 2x+1 */
            float R = bt(r0, i0) + bt(r0, i1), G = bt(r0, i0 + 1) + bt(r0, i1 + 1),
                  B = bt(r0, i0 + 2) + bt(r0, i1 + 2);
            if (SUB == 2) {
                R = R + (bt(r1, i0) + bt(r1, i1));
                G = G + (bt(r1, i0 + 1) + bt(r1, i1 + 1));
                B = B + (bt(r1, i0 + 2) + bt(r1, i1 + 2));
            }
            smp[x] = pixel_k(CH, R, G, B) * (SUB == 1 ? 0.5f : 0.25f);
        }
        jx_fdct8<FOps>(smp, T[y]);
    }
}

template <int SUB>
__global__ __launch_bounds__(JX_WG, 3) void k_chroma(const jx_xform_args a)
{
    __shared__ WaveLds s_wave[JX_WG / 64];
    const jx_geom &g = a.g;
    const unsigned nb = (unsigned)g.nb, bpr = (unsigned)g.bpr;
    const unsigned total = nb * (unsigned)g.nframes;
    const unsigned ntiles = (total + 63u) / 64u;
    const unsigned lane = threadIdx.x & 63u;
    const unsigned nwaves = gridDim.x * (JX_WG / 64);
    /* wave-uniform (readfirstlane: the compiler cannot see that threadIdx.x >> 6 is), so the
     * tile loop and its branches are scalar */
    unsigned t = __builtin_amdgcn_readfirstlane(blockIdx.x * (JX_WG / 64) + (threadIdx.x >> 6));
    if (t >= ntiles) return;
    WaveLds &W = s_wave[threadIdx.x >> 6];
    Queue Q{{0, 0, 0}, {0u, 0u, 0u}};
    for (; t < ntiles; t += nwaves) {
        const unsigned b0 = t * 64u + lane;
        const bool active = b0 < total;
        const unsigned b = active ? b0 : total - 1;
        const unsigned f = b / nb, bi = b - f * nb, by = bi / bpr, bx = bi - by * bpr;
#pragma unroll
        for (int ch = 1; ch <= 2; ch++) {
            float T[8][8];
            chroma_rows<SUB>(ch, g, f, bx, by, T);
            xform_cols(ch, T, a, W, Q, active, b, t, lane);
            __builtin_amdgcn_sched_barrier(0);
            fix_chroma(W, Q, ch, a, lane);
        }
    }
}

__device__ __forceinline__ uint8_t splitmix_byte(uint64_t seed, uint64_t k)
{
    uint64_t z = seed + (k + 1) * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z ^= z >> 31;
    return (uint8_t)(z >> 56);
}

__global__ void k_gen_splitmix(uint8_t *dst, size_t n, uint64_t seed)
{
    const size_t stride = (size_t)gridDim.x * blockDim.x * 16;
    for (size_t k0 = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) * 16; k0 < n; k0 += stride) {
        if (k0 + 16 <= n && (((uintptr_t)(dst + k0)) & 15) == 0) {
            uint32_t w[4];
#pragma unroll
            for (int j = 0; j < 4; j++) {
                w[j] = 0;
#pragma unroll
                for (int i = 0; i < 4; i++)
                    w[j] |= (uint32_t)splitmix_byte(seed, k0 + 4 * j + i) << (8 * i);
            }
            *(u32x4 *)(dst + k0) = u32x4{w[0], w[1], w[2], w[3]};
        } else {
            for (size_t k = k0; k < k0 + 16 && k < n; k++) dst[k] = splitmix_byte(seed, k);
        }
    }
}

__global__ void k_gen_tie(uint8_t *dst, int W, int H)
{
    const size_t npx = (size_t)W * H;
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < npx; i += stride) {
        const size_t y = i / W, x = i - y * W;
        const size_t bi = (y / 8) * (W / 8) + x / 8;
        const uint8_t v = (uint8_t)(97 + 2 * (bi % 40));
        dst[3 * i] = v;
        dst[3 * i + 1] = v;
        dst[3 * i + 2] = v;
    }
}

int hip_rc(hipError_t e) { return e == hipSuccess ? JPGX_OK : JPGX_EHIP; }

constexpr int kMaxDev = 64;
std::once_flag g_tab_once[kMaxDev];
int g_tab_rc[kMaxDev];

int tables_for_current_device()
{
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDev) return JPGX_ENODEV;
    std::call_once(g_tab_once[dev], [dev]() {
        std::vector<jx_qtab> host(JX_MAXQ + 1);
        std::vector<jx_limtab> band(2 * (JX_MAXQ + 1));
        memset(host.data(), 0, host.size() * sizeof(jx_qtab));
        memset(band.data(), 0, band.size() * sizeof(jx_limtab));
        for (int q = 1; q <= JX_MAXQ; q++) {
            float w[3][64], lim[3][64];
            jx_plan_tables(q, w, lim, host[q].q);
            for (int ch = 0; ch < 3; ch++)
                for (int u = 0; u < 8; u++)
                    for (int v = 0; v < 8; v++) {
                        host[q].w[ch][u][v] = w[ch][v * 8 + u];
                        band[q].lim[ch][u][v] = lim[ch][v * 8 + u];
                        band[JX_MAXQ + 1 + q].lim[ch][u][v] = -1.0f;   /* FORCE_EXACT */
                    }
        }
        /* true subsampling: chroma bounds of the averaged samples, [sub-1][force][q] */
        std::vector<jx_limtab> bsub(2 * 2 * (JX_MAXQ + 1));
        memset(bsub.data(), 0, bsub.size() * sizeof(jx_limtab));
        for (int sm = 1; sm <= 2; sm++)
            for (int q = 1; q <= JX_MAXQ; q++) {
                float w[3][64], lim[3][64];
                int16_t qq[2][64];
                jx_plan_tables_mode(q, sm, w, lim, qq);
                jx_limtab &bn = bsub[((sm - 1) * 2 + 0) * (JX_MAXQ + 1) + q];
                jx_limtab &bf = bsub[((sm - 1) * 2 + 1) * (JX_MAXQ + 1) + q];
                for (int ch = 0; ch < 3; ch++)
                    for (int u = 0; u < 8; u++)
                        for (int v = 0; v < 8; v++) {
                            /* k_chroma reads the chroma slots; slot 0 (luma is never
                             * averaged) holds the joint Cb / Cr band */
                            const int k = v * 8 + u;
                            bn.lim[ch][u][v] = ch ? lim[ch][k] : std::min(lim[1][k], lim[2][k]);
                            bf.lim[ch][u][v] = -1.0f;
                        }
            }
        g_tab_rc[dev] = hip_rc(hipMemcpyToSymbol(HIP_SYMBOL(g_qtab), host.data(),
                                                 host.size() * sizeof(jx_qtab)));
        if (!g_tab_rc[dev])
            g_tab_rc[dev] = hip_rc(hipMemcpyToSymbol(HIP_SYMBOL(g_limsub), bsub.data(),
                                                     bsub.size() * sizeof(jx_limtab)));
        if (!g_tab_rc[dev])
            g_tab_rc[dev] = hip_rc(hipMemcpyToSymbol(HIP_SYMBOL(g_lim), band.data(),
                                                     band.size() * sizeof(jx_limtab)));
    });
    return g_tab_rc[dev];
}

/* resident waves of k_xform on the current device (persistent grid size) */
int g_resident_waves[kMaxDev];
std::once_flag g_res_once[kMaxDev];

int resident_waves()
{
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDev) return 0;
    std::call_once(g_res_once[dev], [dev]() {
        int cus = 0, per_cu = 0;
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
            cus = 256;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_xform, JX_WG, 0) != hipSuccess ||
            per_cu < 1)
            per_cu = 2;
        g_resident_waves[dev] = cus * per_cu * (JX_WG / 64);
    });
    return g_resident_waves[dev];
}

/* Dispatch.  The product library (libjpgx.so) runs one kernel per mode: k_mx for 4:4:4,
 * k_mx422 / k_mx420 for true 4:2:2 / 4:2:0.  The test-only cross-check library
 * (libjpgx_alt.so, built from the same sources with -DJPGX_ALT_DISPATCH) runs the second
 * implementations instead: k_xform for 4:4:4 and k_xform (Y) + k_chroma<1|2> for true 4:2:x. */
#ifndef JPGX_ALT_DISPATCH
#define JPGX_ALT_DISPATCH 0
#endif
constexpr bool kAltDispatch = JPGX_ALT_DISPATCH != 0;
constexpr size_t kMaxPitch = (size_t)1 << 27;     /* 16 rows x pitch + 256 < 2^32 */

}  // namespace

static int blocks_gpu(const jpgx_frames *fr, const jpgx_params *p, const uint8_t *d_rgb, int16_t *d_out,
                      void *d_workspace, size_t workspace_bytes, void *stream, void *event_after, void *ev_start,
                      void *ev_stop);

extern "C" {

int jpgx_blocks_gpu(const jpgx_frames *fr, const jpgx_params *p, const uint8_t *d_rgb,
                    int16_t *d_out, void *d_workspace, size_t workspace_bytes, void *stream)
{
    return jpgx_blocks_gpu_ev(fr, p, d_rgb, d_out, d_workspace, workspace_bytes, stream, nullptr);
}

int jpgx_blocks_gpu_ev(const jpgx_frames *fr, const jpgx_params *p, const uint8_t *d_rgb,
                       int16_t *d_out, void *d_workspace, size_t workspace_bytes, void *stream,
                       void *event_after)
{
    return blocks_gpu(fr, p, d_rgb, d_out, d_workspace, workspace_bytes, stream, event_after, nullptr, nullptr);
}

int jpgx_blocks_gpu_timed(const jpgx_frames *fr, const jpgx_params *p, const uint8_t *d_rgb,
                          int16_t *d_out, void *d_workspace, size_t workspace_bytes, void *stream,
                          void *ev_start, void *ev_stop)
{
    if (!ev_start || !ev_stop) return JPGX_EARG;
    return blocks_gpu(fr, p, d_rgb, d_out, d_workspace, workspace_bytes, stream, nullptr, ev_start, ev_stop);
}

}  /* extern "C" */

static int blocks_gpu(const jpgx_frames *fr, const jpgx_params *p, const uint8_t *d_rgb, int16_t *d_out,
                      void *d_workspace, size_t workspace_bytes, void *stream, void *event_after, void *ev_start,
                      void *ev_stop)
{
    if (!fr || !p) return JPGX_EARG;
    int rc = jpgx_validate(fr->width, fr->height, p);
    if (rc) return rc;
    if (fr->row_begin < 0 || fr->row_end > fr->height / 8 || fr->row_begin > fr->row_end ||
        fr->nframes < 1)
        return JPGX_EARG;
    const bool sub = (p->flags & JPGX_FLAG_SUBSAMPLE) != 0;
    if (sub && p->sample_ratio == 0) return JPGX_ESAMPLE;
    if (sub && p->sample_ratio == 2 && ((fr->row_begin | fr->row_end) & 1)) return JPGX_EARG;
    if (fr->row_begin == fr->row_end) return JPGX_OK;
    if (!d_rgb || !d_out) return JPGX_EARG;
    if (fr->in_pitch < (size_t)fr->width * 3 || fr->in_pitch % 8 || fr->in_frame_stride % 8 ||
        ((uintptr_t)d_rgb & 7) || ((uintptr_t)d_out & 15) || fr->out_frame_stride % 8)
        return JPGX_EARG;
    /* the MFMA kernels address a step's pixel rows (up to 16 of them) with 32-bit lane offsets */
    if (fr->in_pitch > kMaxPitch) return JPGX_EARG;
    const int bpr = fr->width / 8;
    const size_t nb = (size_t)(fr->row_end - fr->row_begin) * bpr;
    const size_t total = nb * fr->nframes;
    if (total + 64 >= (1ull << 32)) return JPGX_EARG;
    const size_t nbc = sub ? jpgx_chroma_blocks(fr->width, fr->row_begin, fr->row_end,
                                                p->sample_ratio, p->flags)
                           : nb;
    if (fr->nframes > 1 && fr->out_frame_stride < (nb + 2 * nbc) * 64) return JPGX_EARG;
    if (fr->nframes > 1 && fr->in_frame_stride < fr->in_pitch * (size_t)(fr->row_end - fr->row_begin) * 8)
        return JPGX_EARG;
    if (workspace_bytes < jpgx_workspace_size(fr) || ((uintptr_t)d_workspace & 15))
        return JPGX_EWORKSPACE;

    jx_xform_args xa;
    memset(&xa, 0, sizeof xa);
    jx_geom &g = xa.g;
    g.rgb = d_rgb;
    g.out = d_out;
    g.in_pitch = (long long)fr->in_pitch;
    g.in_fstride = (long long)fr->in_frame_stride;
    g.out_fstride = (long long)fr->out_frame_stride;
    g.bpr = bpr;
    g.nb = (int)nb;
    g.nframes = fr->nframes;
    g.row0 = fr->row_begin;
    g.dnb = jx_udiv_make((uint32_t)nb);
    g.dbpr = jx_udiv_make((uint32_t)bpr);
    g.mpr = (uint32_t)bpr / 2u;
    g.nmcu = (uint32_t)(nb / (size_t)bpr / 2u) * g.mpr;
    g.dmpr = jx_udiv_make(g.mpr ? g.mpr : 1u);
    g.dnmcu = jx_udiv_make(g.nmcu ? g.nmcu : 1u);
    jx_under_dwords(p->underflow, g.under);
    rc = tables_for_current_device();
    if (rc) return rc;
    xa.quality = p->quality;
    xa.force_exact = (p->flags & JPGX_FLAG_FORCE_EXACT) ? 1 : 0;
    hipStream_t s = (hipStream_t)stream;
    xa.luma_only = sub ? 1 : 0;
    if (!sub && !kAltDispatch) {
        /* k_mx: colour + row DCT on the matrix cores, exact pass inside (csrc/jpgx_mx.hip) */
        rc = jx_launch_mx(&xa, stream, ev_start, ev_stop);
        if (rc) return rc;
        if (event_after) rc = hip_rc(hipEventRecord((hipEvent_t)event_after, s));
        return rc;
    }
    /* k_xform: persistent, one wave per resident slot (at most one per tile) */
    const size_t ntiles = (total + 63) / 64;
    const size_t waves = std::min<size_t>(ntiles, (size_t)std::max(resident_waves(), 4));
    const unsigned grid = (unsigned)((waves + JX_WG / 64 - 1) / (JX_WG / 64));
    if (sub && p->sample_ratio == 2 && !kAltDispatch) {
        /* true 4:2:0 in one pass on the matrix cores (k_mx420, csrc/jpgx_mx.hip) */
        rc = jx_launch_mx420(&xa, stream, ev_start, ev_stop);
        if (!rc && event_after) rc = hip_rc(hipEventRecord((hipEvent_t)event_after, s));
        return rc;
    }
    if (sub && p->sample_ratio == 1 && !kAltDispatch) {
        /* true 4:2:2 in one pass on the matrix cores (k_mx422, csrc/jpgx_mx.hip) */
        rc = jx_launch_mx422(&xa, stream, ev_start, ev_stop);
        if (!rc && event_after) rc = hip_rc(hipEventRecord((hipEvent_t)event_after, s));
        return rc;
    }
    if (ev_start) {                                   /* the test library: events around its kernels */
        rc = hip_rc(hipEventRecord((hipEvent_t)ev_start, s));
        if (rc) return rc;
    }
    hipLaunchKernelGGL(k_xform, dim3(grid), dim3(JX_WG), 0, s, xa);
    rc = hip_rc(hipGetLastError());
    if (rc) return rc;
    if (sub) {
        /* true 4:2:2 / 4:2:0 chroma: Cb at out + nb*64, Cr at out + (nb + nbc)*64 per frame */
        jx_xform_args xc = xa;
        xc.luma_only = 0;
        xc.sub = p->sample_ratio;
        xc.g.bpr = fr->width / 16;
        xc.g.nb = (int)nbc;
        xc.g.out = d_out + (long long)nb * 64 - (long long)nbc * 64;
        const size_t ctiles = (nbc * fr->nframes + 63) / 64;
        const size_t cw = std::min<size_t>(ctiles, (size_t)std::max(resident_waves(), 4));
        const unsigned cgrid = (unsigned)((cw + JX_WG / 64 - 1) / (JX_WG / 64));
        if (p->sample_ratio == 1)
            hipLaunchKernelGGL(k_chroma<1>, dim3(cgrid), dim3(JX_WG), 0, s, xc);
        else
            hipLaunchKernelGGL(k_chroma<2>, dim3(cgrid), dim3(JX_WG), 0, s, xc);
        rc = hip_rc(hipGetLastError());
        if (rc) return rc;
    }
    if (ev_stop) rc = hip_rc(hipEventRecord((hipEvent_t)ev_stop, s));
    if (!rc && event_after) rc = hip_rc(hipEventRecord((hipEvent_t)event_after, s));
    return rc;
}

extern "C" {

int jpgx_gen_splitmix_gpu(uint8_t *d_dst, size_t nbytes, uint64_t seed, void *stream)
{
    if (!d_dst) return JPGX_EARG;
    if (!nbytes) return JPGX_OK;
    const size_t threads = (nbytes + 15) / 16;
    const unsigned grid = (unsigned)std::min<size_t>((threads + 255) / 256, 65536);
    hipLaunchKernelGGL(k_gen_splitmix, dim3(grid), dim3(256), 0, (hipStream_t)stream, d_dst,
                       nbytes, seed);
    return hip_rc(hipGetLastError());
}

int jpgx_gen_tie_gpu(uint8_t *d_dst, int width, int height, void *stream)
{
    if (!d_dst || width <= 0 || height <= 0 || width % 8 || height % 8) return JPGX_EARG;
    const size_t npx = (size_t)width * height;
    const unsigned grid = (unsigned)std::min<size_t>((npx + 255) / 256, 65536);
    hipLaunchKernelGGL(k_gen_tie, dim3(grid), dim3(256), 0, (hipStream_t)stream, d_dst, width,
                       height);
    return hip_rc(hipGetLastError());
}

int jpgx_device_count(void)
{
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

}  /* extern "C" */
