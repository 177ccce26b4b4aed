/*
 * jpgx_kernels.hip -- gfx950 kernels of the block-transform hot path + the device C-ABI.
 *
 * k_xform (one kernel does the whole hot path; one lane = one 8x8 block, all 3 channels)
 *   HBM -> VGPR: each lane loads its block's 8 pixel rows (8 x 24 B; a wave covers 64
 *   horizontally adjacent blocks = 1.5 KiB contiguous per pixel row), one tile ahead.
 *   Per channel, entirely in the lane's registers (no cross-lane traffic):
 *     byte -> f32, colour + level shift (3 FMAs/px)        src/preprocess.c:160-162,186-188
 *     row DCT then column DCT, even/odd 8-point DCT-II      src/dct.c:36-59
 *     quantise: one FMA with the per-coefficient fp32 scale (1/Q and DCT normalisation
 *       folded) that also rounds to an integer (+1.5*2^23)  src/quantise.c:52-72 (transposed)
 *     zig-zag as a compile-time register permutation, int16 pairs packed with v_perm
 *                                                           src/zig_zag.c:48-58
 *   LDS -> HBM: the wave's 64 blocks x 128 B of a channel are staged in LDS and written as
 *   8 KiB of contiguous 16-B-per-lane stores (coalesced).
 *   Exactness: a coefficient whose fp32 quotient lies within the rigorous guard band of a
 *   .5 boundary (jpgx_plan.cpp) is queued in the wave's LDS (block pixels + item) and later
 *   recomputed, many lanes at once, in the reference's exact fp64 operation order:
 *   double colour conversion in its operand order, -128, the 64-term sum x-outer / y-inner
 *   with (X*c_u[x])*c_v[y] and the glibc cosine doubles, ((0.25*a_u)*a_v)*s, true double
 *   division by the transposed table entry, round() half away from zero.
 *
 * Compiled with FP contraction off; the fast path uses explicit fmaf.
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

#ifndef JX_PREFETCH
#define JX_PREFETCH 0   /* input prefetch mode, see k_xform */
#endif
#ifndef JX_TPF          /* 1: quantiser tables of the next column loaded one column ahead
                           (0 measured 1-2% faster, tools/variant_bench.py, 6 interleaved rounds) */
#define JX_TPF 0
#endif
#ifndef JX_CHLOOP       /* 1: the three channels run one rolled copy of the channel body */
#define JX_CHLOOP 0
#endif
#ifndef JX_RELOAD       /* 1: pixels re-read (L2) per channel, issued during the previous
                           column pass: they are not kept in registers across channels */
#define JX_RELOAD 0
#endif
#ifndef JX_RELOAD_COL   /* column of the column pass at which the next loads are issued  */
#define JX_RELOAD_COL 4
#endif
#ifndef JX_ROW_SB       /* scheduling fence between the row DCTs of a channel
                           (0 measured 1-2% faster together with JX_TPF 0)             */
#define JX_ROW_SB 0
#endif
#ifndef JX_COL_SB       /* scheduling fence between the column DCTs of a channel       */
#define JX_COL_SB 1
#endif
#if JX_ROW_SB
#define JX_SB_ROW() __builtin_amdgcn_sched_barrier(0)
#else
#define JX_SB_ROW() ((void)0)
#endif
#if JX_COL_SB
#define JX_SB_COL() __builtin_amdgcn_sched_barrier(0)
#else
#define JX_SB_COL() ((void)0)
#endif
#ifndef JX_WPE          /* minimum waves per SIMD the register allocation must allow:
                           3 (<= 168 VGPRs; a few spills outside the tile loop) measured
                           faster than 2 (no spills)                                     */
#define JX_WPE 3
#endif
#ifndef JX_FLAG_MODE     /* guard-band test: 0 v_cmp into SGPR masks + s_or; 1 VALU max of
                            |d|-lim; 2 VALU compare-or; 3 VALU max of |d| per column against
                            the column's tightest limit (more flags, fewer instructions)     */
#define JX_FLAG_MODE 0
#endif
#ifndef JX_DBG_NO_EXACT  /* debug/measurement only: drop the exact path (NOT bit-exact)    */
#define JX_DBG_NO_EXACT 0
#endif

constexpr float kMagic = 12582912.0f; /* 1.5 * 2^23: x + kMagic rounds x to an integer   */
#ifndef JX_QUEUE_ITEMS
#define JX_QUEUE_ITEMS 128
#endif
#ifndef JX_FIX_STAGGER  /* 1: one mid-run exact pass per wave at a wave-dependent tile; 2: one
                           before the wave's last tile (plus the end-of-kernel pass)          */
#define JX_FIX_STAGGER 0
#endif
#ifndef JX_FUSED_FIX    /* k_xform runs the exact pass itself, 8 queued blocks at a time: 1 after its
                           last tile, 2 also at each tile start, under the pixel loads;
                           0: a second kernel (k_fix) does it */
#define JX_FUSED_FIX 1
#endif
/* per-wave, per-channel queue of blocks with a coefficient inside the guard band */
constexpr int kItems = JX_QUEUE_ITEMS;
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

/* column u of zig-zag index z */
__host__ __device__ constexpr int zz_col(int z)
{
    for (int v = 0; v < 8; v++)
        for (int u = 0; u < 8; u++)
            if (zz_of(v, u) == z) return u;
    return -1;
}
/* the column pass after which zig-zag entries z0 and z1 are both available */
[[maybe_unused]] __host__ __device__ constexpr int zz_col_done(int z0, int z1)
{
    return zz_col(z0) > zz_col(z1) ? zz_col(z0) : zz_col(z1);
}
/* the column pass after which the 16-byte output chunk j (zig-zag 8j..8j+7) is complete */
[[maybe_unused]] __host__ __device__ constexpr int zz_chunk_done(int j)
{
    int m = 0;
    for (int z = 8 * j; z < 8 * j + 8; z++) m = zz_col(z) > m ? zz_col(z) : m;
    return m;
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

#ifndef JX_NT_STORE     /* coefficient stores with the nontemporal bit (streamed, never re-read) */
#define JX_NT_STORE 1
#endif
#ifndef JX_NT_LOAD      /* pixel loads with the nontemporal bit                                 */
#define JX_NT_LOAD 0
#endif

__device__ __forceinline__ void jx_store(u32x4 *p, u32x4 v)
{
#ifdef JX_DBG_NO_STORE      /* timing experiments only: keep the work, drop the bytes */
    if ((v.x ^ v.y ^ v.z ^ v.w) == 0x9e3779b9u) *p = v;
    return;
#endif
#if JX_NT_STORE
    __builtin_nontemporal_store(v, p);
#else
    *p = v;
#endif
}

#ifndef JX_STAGE16      /* 1: each int16 goes to LDS as produced (no register packing:
                           fewer live VGPRs, what lets 3 waves share a SIMD)             */
#define JX_STAGE16 1
#endif

/* Per-wave LDS */
struct WaveLds {
#if JX_STAGE16
    uint32_t stage[64 * 33];      /* one channel: block k at dwords 33k.. (odd stride: the
                                     16-bit writes of 64 lanes hit 64 different banks)      */
#else
    u32x4 stage[64 * 9];          /* one channel: block k's 8 chunks at units 9k..9k+7     */
#endif
    uint32_t item[3][kItems];     /* per channel: queued launch-global block indices       */
};

/* 16-B unit e (block e/8, zig-zag chunk e%8) of the staged channel */
__device__ __forceinline__ u32x4 stage_unit(const WaveLds &W, unsigned e)
{
#if JX_STAGE16
    const unsigned o = (e >> 3) * 33 + (e & 7) * 4;
    return u32x4{W.stage[o], W.stage[o + 1], W.stage[o + 2], W.stage[o + 3]};
#else
    return W.stage[(e >> 3) * 9 + (e & 7)];
#endif
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
#if defined(JX_DBG_NO_LOAD)  /* timing experiments only: synthetic bytes, no HBM reads */
        {
            const uint32_t s = (uint32_t)(uintptr_t)p * 2654435761u;
            a = u32x4{s, s ^ 0x5bd1e995u, s + 0x6a09e667u, s * 3u};
            b = u32x2{s ^ 0xbb67ae85u, s + 0x3c6ef372u};
        }
#elif JX_NT_LOAD
        a = __builtin_nontemporal_load((const u32x4 *)p);
        b = __builtin_nontemporal_load((const u32x2 *)(p + 16));
#else
        __builtin_memcpy(&a, p, 16);
        __builtin_memcpy(&b, p + 16, 8);
#endif
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
template <int CH>
__device__ __forceinline__ double exact_sum(const uint32_t (&raw)[8][6], int u, int v)
{
    double cu[8], cv[8];
#pragma unroll
    for (int k = 0; k < 8; k++) {
        cu[k] = kCos[u][k];
        cv[k] = kCos[v][k];
    }
    double s = 0.0;
#pragma unroll
    for (int x = 0; x < 8; x++)              /* dct.c:46 x outer */
#pragma unroll
        for (int y = 0; y < 8; y++) {        /* dct.c:47 y inner */
            const int r = (int)byte_of(raw[y], 3 * x);
            const int g = (int)byte_of(raw[y], 3 * x + 1);
            const int b = (int)byte_of(raw[y], 3 * x + 2);
            s += exact_pixel(CH, r, g, b) * cu[x] * cv[y];   /* (X*c_u[x])*c_v[y], :48-50 */
        }
    return s;
}

template <int CH>
__device__ __forceinline__ int16_t exact_coef(const uint32_t (&raw)[8][6], int u, int v, int q)
{
    const double s = exact_sum<CH>(raw, u, v);
    const double F = 0.25 * (u == 0 ? kAlpha0 : 1.0) * (v == 0 ? kAlpha0 : 1.0) * s;
    return (int16_t)(int)round(F / (double)q);      /* quantise.c:58 */
}

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

#ifndef JX_MIX           /* 1: colour conversion by v_fma_mix_f32 straight from the bytes */
#define JX_MIX 0
#endif

/* The eight pixel values of channel CH (level shift included) of one pixel row (24 bytes).
 * JX_MIX: each pair of bytes becomes two f16 subnormals b*2^-24 (one v_perm_b32), which
 * v_fma_mix_f32 multiplies exactly by the f32 constant k*2^24: fma(b*2^-24, k*2^24, c) rounds
 * b*k + c once, the very value of jx_pixel's fmaf(b, k, c) (the plain product b*k as
 * fma(., ., -0), also exact with its sign) -- no byte->f32 conversions at all.  Needs f16
 * denormals (the default kernel mode); the parity tests check every output bit. */
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
#if JX_MIX
    uint32_t h[12];                          /* h[k] = bytes 2k, 2k+1 as f16 subnormals */
#pragma unroll
    for (int k = 0; k < 12; k++)
        h[k] = __builtin_amdgcn_perm(row[k >> 1], row[k >> 1], (k & 1) ? 0x0c070c06u : 0x0c050c04u);
    const auto in = [&](int i) {              /* byte i of the row, times 2^-24 */
        const uint32_t w = h[i >> 1];
        const uint16_t b16 = (i & 1) ? (uint16_t)(w >> 16) : (uint16_t)w;
        return (float)__builtin_bit_cast(_Float16, b16);
    };
    constexpr float S = 16777216.0f;
    float nz = -0.0f;                      /* opaque: fma(x, y, -0) must not become a mul */
    asm volatile("" : "+v"(nz));
#define JX_KS(v) (JX_K(v).f * S)
#pragma unroll
    for (int x = 0; x < 8; x++) {
        const float r = in(3 * x), gg = in(3 * x + 1), bb = in(3 * x + 2);
        if (CH == 0)
            px[x] = __builtin_fmaf(r, JX_KS(0.299), __builtin_fmaf(gg, JX_KS(0.587),
                    __builtin_fmaf(bb, JX_KS(0.114), JX_K(-128.0).f)));
        else if (CH == 1)
            px[x] = __builtin_fmaf(r, JX_KS(-0.168736), __builtin_fmaf(gg, JX_KS(0.331264),
                    __builtin_fmaf(bb, JX_KS(-0.5), nz)));
        else
            px[x] = __builtin_fmaf(r, JX_KS(0.5), __builtin_fmaf(gg, JX_KS(-0.418688),
                    __builtin_fmaf(bb, JX_KS(-0.081312), nz)));
    }
#undef JX_KS
#else
#pragma unroll
    for (int x = 0; x < 8; x++) {
        const float r = (float)byte_of(row, 3 * x);
        const float gg = (float)byte_of(row, 3 * x + 1);
        const float bb = (float)byte_of(row, 3 * x + 2);
        px[x] = pixel_k(CH, r, gg, bb);
    }
#endif
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
        JX_SB_ROW();
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
         * clamped block): they are written there again, identical bytes, so every path issues
         * the same 8 stores (which the vmcnt accounting of JX_PREFETCH 2 relies on) */
#pragma unroll
        for (int j = 0; j < 8; j++) {
            const unsigned e = (unsigned)j * 64u + lane, bb = std::min(b0 + (e >> 3), total - 1u);
            jx_store((u32x4 *)coef_ptr(g, bb, CH, (int)(e & 7) * 8), stage_unit(W, e));
        }
    }
    /* some lane has a coefficient inside the guard band (about 40% of the channel-tiles of
     * random data at q90; wave-uniform branch): queue its block-channel */
    if (!JX_DBG_NO_EXACT && seen != 0) {
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
template <class Pre>
__device__ __forceinline__ void xform_cols(const int CH, float (&T)[8][8], const jx_xform_args &a, WaveLds &W,
                                           Queue &Q, bool active, unsigned b, unsigned t,
                                           unsigned lane, Pre &&pre)
{
#if !JX_STAGE16
    uint32_t bits[64];     /* tm bit patterns by zig-zag index; low 16 bits = the int16    */
    uint32_t packed[32];   /* zig-zag pairs (2k, 2k+1) as one dword, formed when complete */
#endif
    const jx_qtab &tab = g_qtab[a.quality];
    const int fe = a.force_exact ? 1 : 0;
    const jx_limtab &band = a.sub ? g_limsub[a.sub - 1][fe][a.quality] : g_lim[fe][a.quality];
    /* wave mask of lanes with a coefficient of this channel inside the guard band */
    uint64_t seen = 0;
#if JX_FLAG_MODE == 1 || JX_FLAG_MODE == 3 || JX_FLAG_MODE == 4
    float flagacc = -1.0f, epair = 0.0f, colmax = 0.0f;
    (void)epair;
    (void)colmax;
#elif JX_FLAG_MODE == 2
    uint32_t flagany = 0;
#endif
#ifdef JX_DBG_NO_STAGE
    uint32_t dbg_acc = 0;
#endif
    /* JX_TPF: column u+1's scale and band values are read at the top of column u (scalar loads
     * in flight under its DCT) instead of right before their use, where every column paid the
     * scalar-load latency plus, through the shared lgkm counter, its pending LDS writes */
    float wc[8], lc[8];
#pragma unroll
    for (int v = 0; v < 8; v++) {
        wc[v] = tab.w[CH][0][v];
        lc[v] = JX_FLAG_MODE == 4 ? band.lsqn[CH][0][v] : band.lim[CH][0][v];
    }
#pragma unroll
    for (int u = 0; u < 8; u++) {
        if (u == JX_RELOAD_COL) pre();      /* e.g. issue the next pixel loads (JX_RELOAD) */
        float wn[8], ln[8];
#pragma unroll
        for (int v = 0; v < 8; v++) {
            wn[v] = JX_TPF && u < 7 ? tab.w[CH][u + 1][v] : 0.0f;
            ln[v] = JX_TPF && u < 7 ? (JX_FLAG_MODE == 4 ? band.lsqn[CH][u + 1][v]
                                                         : band.lim[CH][u + 1][v])
                                    : 0.0f;
            if (!JX_TPF) {
                wc[v] = tab.w[CH][u][v];
                lc[v] = JX_FLAG_MODE == 4 ? band.lsqn[CH][u][v] : band.lim[CH][u][v];
            }
        }
        float col[8], F[8];
#pragma unroll
        for (int y = 0; y < 8; y++) col[y] = T[y][u];
        jx_fdct8<FOps>(col, F);
#if JX_FLAG_MODE == 4
        /* quantiser and band test two coefficients (v, v+1) per v_pk_*_f32: tm, rint and d are
         * lane for lane quant_coef's values; the test d*d - lsq >= 0 (lsq <= lim^2) flags every
         * coefficient |d| >= lim flags, into one running max per lane (no compare, no SALU) */
#pragma unroll
        for (int v = 0; v < 8; v += 2) {
            const f2 Fp = f2{F[v], F[v + 1]}, wp = f2{wc[v], wc[v + 1]};
            const f2 M2 = f2{kMagic, kMagic};
            const f2 tm = __builtin_elementwise_fma(Fp, wp, M2);
            ((uint16_t *)W.stage)[lane * 66 + zz_of(v, u)] = (uint16_t)__float_as_uint(tm.x);
            ((uint16_t *)W.stage)[lane * 66 + zz_of(v + 1, u)] = (uint16_t)__float_as_uint(tm.y);
            if (!JX_DBG_NO_EXACT) {
                const f2 rr = tm - M2;
                const f2 d = __builtin_elementwise_fma(Fp, wp, -rr);
                const f2 e = __builtin_elementwise_fma(d, d, -f2{lc[v], lc[v + 1]});
                flagacc = __builtin_fmaxf(flagacc, __builtin_fmaxf(e.x, e.y));
            }
        }
        if (false)
#endif
#pragma unroll
        for (int v = 0; v < 8; v++) {
            float tm, d;
            quant_coef(F[v], wc[v], tm, d);
#if JX_STAGE16
#ifdef JX_DBG_NO_STAGE              /* timing experiments only: no LDS staging writes */
            dbg_acc ^= __float_as_uint(tm);
#else
            ((uint16_t *)W.stage)[lane * 66 + zz_of(v, u)] = (uint16_t)__float_as_uint(tm);
#endif
#else
            bits[zz_of(v, u)] = __float_as_uint(tm);
#endif
            if (!JX_DBG_NO_EXACT) {
#if JX_FLAG_MODE == 0
                /* compare straight into a lane mask, OR-ed at once (left to the compiler,
                 * the 64 masks of a channel are kept alive until the end and spilled) */
                uint64_t m;
                asm("v_cmp_ge_f32_e64 %[m], |%[d]|, %[l]\n\t"
                    "s_or_b64 %[seen], %[seen], %[m]"
                    : [m] "=&s"(m), [seen] "+s"(seen)
                    : [d] "v"(d), [l] "s"(lc[v])
                    : "scc");
#elif JX_FLAG_MODE == 1
                /* all in VALU: e = |d| - lim, running max (>= 0 means flagged); pinned asm
                 * like mode 0 (left to the compiler, the table loads are hoisted and spill) */
                if (v & 1) {
                    float e;
                    asm("v_sub_f32_e64 %[e], |%[d]|, %[l]\n\t"
                        "v_max3_f32 %[acc], %[acc], %[p], %[e]"
                        : [e] "=&v"(e), [acc] "+v"(flagacc)
                        : [d] "v"(d), [l] "s"(lc[v]), [p] "v"(epair));
                } else {
                    asm("v_sub_f32_e64 %[e], |%[d]|, %[l]"
                        : [e] "=v"(epair)
                        : [d] "v"(d), [l] "s"(lc[v]));
                }
#elif JX_FLAG_MODE == 2
                asm("v_cmp_ge_f32_e64 vcc, |%[d]|, %[l]\n\t"
                    "v_cndmask_b32_e64 %[f], %[f], -1, vcc"
                    : [f] "+v"(flagany)
                    : [d] "v"(d), [l] "s"(lc[v])
                    : "vcc");
#elif JX_FLAG_MODE == 3
                /* one limit per column (the column's tightest): running max of |d| */
                if (v == 0)
                    asm("v_max_f32_e64 %[c], |%[d]|, |%[d]|" : [c] "=v"(colmax) : [d] "v"(d));
                else
                    asm("v_max_f32_e64 %[c], %[c], |%[d]|" : [c] "+v"(colmax) : [d] "v"(d));
                if (v == 7)
                    asm("v_sub_f32_e64 %[c], %[c], %[l]\n\t"
                        "v_max_f32_e32 %[acc], %[acc], %[c]"
                        : [c] "+v"(colmax), [acc] "+v"(flagacc)
                        : [l] "s"(band.limcol[CH][u]));
#endif
            }
        }
#if !JX_STAGE16
        /* pack zig-zag pairs completed by this column; stage the 16-B chunks it completes
         * (compile-time decisions: the loops are fully unrolled) */
#pragma unroll
        for (int k = 0; k < 32; k++)
            if (zz_col_done(2 * k, 2 * k + 1) == u)
                packed[k] = __builtin_amdgcn_perm(bits[2 * k + 1], bits[2 * k], 0x05040100u);
#pragma unroll
        for (int j = 0; j < 8; j++)
            if (zz_chunk_done(j) == u)
                W.stage[lane * 9 + j] =
                    u32x4{packed[4 * j], packed[4 * j + 1], packed[4 * j + 2], packed[4 * j + 3]};
#endif
        if (JX_TPF) {
#pragma unroll
            for (int v = 0; v < 8; v++) {
                wc[v] = wn[v];
                lc[v] = ln[v];
            }
        }
        JX_SB_COL();
    }

#ifdef JX_DBG_NO_STAGE
    W.stage[lane] = dbg_acc;
#endif
#if JX_FLAG_MODE == 1 || JX_FLAG_MODE == 3 || JX_FLAG_MODE == 4
    seen = __ballot(flagacc >= 0.0f);
#elif JX_FLAG_MODE == 2
    seen = __ballot(flagany != 0u);
#endif
    store_and_queue(CH, a, W, Q, active, b, t, lane, seen);
}

/* ---- fast path, packed ------------------------------------------------------------------
 * The same fp32 operations as xform_rows / xform_cols, two per v_pk_*_f32 instruction
 * (xform_math.h, checked bit for bit against the scalar code by jx_selftest_pk):
 *   rows:    pixel pairs (x, x+1); jx_fdct8_pk splits each row DCT over the pair's two lanes
 *            and leaves the row's coefficients in the pairs (0,4) (2,6) (1,3) (5,7);
 *   columns: each such pair of columns runs jx_fdct8 in lock-step, one column per lane;
 *   quantiser and guard band per coefficient pair, the band test as d*d - lsq >= 0 (lsq <=
 *   lim^2) folded into one running max per lane: no per-coefficient compare or scalar op.
 */
#ifndef JX_PACKED
#define JX_PACKED 0
#endif
#ifndef JX_PK_ROWS
#define JX_PK_ROWS 2
#endif
#ifndef JX_Q_SB          /* scheduling fences between the quantiser stages (packed path) */
#define JX_Q_SB 1
#endif
#if JX_Q_SB
#define JX_SB_Q() __builtin_amdgcn_sched_barrier(0)
#else
#define JX_SB_Q() ((void)0)
#endif

struct DevPair {
    typedef f2 V;
    static __host__ __device__ __forceinline__ V mk(float a, float b) { return V{a, b}; }
    static __host__ __device__ __forceinline__ float lo(V a) { return a.x; }
    static __host__ __device__ __forceinline__ float hi(V a) { return a.y; }
    static __host__ __device__ __forceinline__ V add(V a, V b) { return a + b; }
    static __host__ __device__ __forceinline__ V sub(V a, V b) { return a - b; }
    static __host__ __device__ __forceinline__ V mul(V a, V b) { return a * b; }
    static __host__ __device__ __forceinline__ V fma(V a, V b, V c)
    {
        return __builtin_elementwise_fma(a, b, c);
    }
};
typedef PairOps<DevPair> DevPO;

/* Row pass of channel CH, packed: T[y][j] = row y's coefficient pair j (jx_pk_k order). */
template <int CH>
__device__ __forceinline__ void xform_rows_pk(uint32_t (&raw)[8][6], f2 (&T)[8][4])
{
#pragma unroll
    for (int y = 0; y < 8; y++)
#pragma unroll
        for (int k = 0; k < 6; k++) asm volatile("" : "+v"(raw[y][k]));
#pragma unroll
    for (int y = 0; y < 8; y++) {
        if (y % JX_PK_ROWS == 0) JX_SB_ROW();   /* JX_PK_ROWS rows interleave (hides the
                                                   dependent-issue gaps of one row's chain) */
        f2 px[4];
#if JX_MIX
        {
            float p1[8];
            row_pixels(CH, raw[y], p1);
#pragma unroll
            for (int k = 0; k < 4; k++) px[k] = f2{p1[2 * k], p1[2 * k + 1]};
        }
#else
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const int x0 = 6 * k, x1 = 6 * k + 3;      /* byte offsets of pixels 2k, 2k+1 */
            const f2 r = f2{(float)byte_of(raw[y], x0), (float)byte_of(raw[y], x1)};
            const f2 gg = f2{(float)byte_of(raw[y], x0 + 1), (float)byte_of(raw[y], x1 + 1)};
            const f2 bb = f2{(float)byte_of(raw[y], x0 + 2), (float)byte_of(raw[y], x1 + 2)};
            px[k] = jx_pixel<DevPO, CH>(r, gg, bb);
        }
#endif
        jx_fdct8_pk<DevPair>(px, T[y]);
    }
}

/* Column pass, quantisation, guard band, zig-zag staging of channel CH, packed.  Each column
 * pair's eight coefficient pairs go through the quantiser stage by stage (eight independent
 * packed operations per stage: no dependent back-to-back pairs, which would cost wait states),
 * and the band test reduces through a max3 tree. */
template <int CH>
__device__ __forceinline__ void xform_cols_pk(f2 (&T)[8][4], const jx_xform_args &a, WaveLds &W,
                                              Queue &Q, bool active, unsigned b, unsigned t,
                                              unsigned lane)
{
    /* table addresses re-derived per channel from opaque scalars (hoisted, they were kept
     * in spilled registers and reloaded from scratch behind vmcnt waits) */
    int qv = a.quality * 2 + (a.force_exact ? 1 : 0);
    asm volatile("" : "+v"(qv));
    const int qf = __builtin_amdgcn_readfirstlane(qv), qq = qf >> 1, fe = qf & 1;
    const jx_qtab &tab = g_qtab[qq];
    const jx_limtab &band = g_lim[fe][qq];
    const f2 M2 = f2{kMagic, kMagic};
    float acc = -1.0f;                   /* max over the channel of d*d - lsq (>= 0: flagged) */
    uint16_t *st = (uint16_t *)W.stage + lane * 66;
#pragma unroll
    for (int j = 0; j < 4; j++) {
        f2 col[8], F[8], tm[8], rr[8], d[8];
#pragma unroll
        for (int y = 0; y < 8; y++) col[y] = T[y][j];
        jx_fdct8<DevPO>(col, F);
        JX_SB_Q();
#pragma unroll
        for (int v = 0; v < 8; v++)
            tm[v] = DevPair::fma(F[v], f2{tab.wp[CH][j][v][0], tab.wp[CH][j][v][1]}, M2);
        JX_SB_Q();
#pragma unroll
        for (int v = 0; v < 8; v++) {
            st[zz_of(v, jx_pk_k(j, 0))] = (uint16_t)__float_as_uint(tm[v].x);
            st[zz_of(v, jx_pk_k(j, 1))] = (uint16_t)__float_as_uint(tm[v].y);
        }
        if (!JX_DBG_NO_EXACT) {
#pragma unroll
            for (int v = 0; v < 8; v++) rr[v] = tm[v] - M2;
            JX_SB_Q();
#pragma unroll
            for (int v = 0; v < 8; v++)
                d[v] = DevPair::fma(F[v], f2{tab.wp[CH][j][v][0], tab.wp[CH][j][v][1]}, -rr[v]);
            JX_SB_Q();
#pragma unroll
            for (int v = 0; v < 8; v++)
                d[v] = DevPair::fma(d[v], d[v], -f2{band.lsq[CH][j][v][0], band.lsq[CH][j][v][1]});
            JX_SB_Q();
            /* 16 values + acc through 8 max3: el(i) = element i of d[0].x, d[0].y, d[1].x, ... */
            const auto el = [&](int i) { return (i & 1) ? d[i >> 1].y : d[i >> 1].x; };
            const auto mx3 = [](float x, float y, float z) {
                return __builtin_fmaxf(__builtin_fmaxf(x, y), z);
            };
            const float m0 = mx3(acc, el(0), el(1)), m1 = mx3(el(2), el(3), el(4));
            const float m2 = mx3(el(5), el(6), el(7)), m3 = mx3(el(8), el(9), el(10));
            const float m4 = mx3(el(11), el(12), el(13)), m5 = __builtin_fmaxf(el(14), el(15));
            acc = __builtin_fmaxf(mx3(m0, m1, m2), mx3(m3, m4, m5));
        }
        JX_SB_COL();
    }
    const uint64_t seen = JX_DBG_NO_EXACT ? 0ull : __ballot(acc >= 0.0f);
    store_and_queue(CH, a, W, Q, active, b, t, lane, seen);
}

/* ---- exact path -------------------------------------------------------------------------- */

/*
 * Guard-band test of one block-channel (raw = its pixel rows, reloaded): the fp32 transform
 * is recomputed by the same code, so exactly the coefficients the fast pass found inside the
 * guard band are found again.  Bit v*8+u of the result = coefficient (u, v) is flagged.
 */
template <int CH>
__device__ __forceinline__ uint64_t flagged_coefs(uint32_t (&raw)[8][6], int quality, int force)
{
    const jx_qtab &tab = g_qtab[quality];
    const jx_limtab &band = g_lim[force][quality];
    float T[8][8];
    xform_rows(CH, raw, T);
    uint64_t flagged = 0;
#pragma unroll
    for (int u = 0; u < 8; u++) {
        float col[8], F[8];
#pragma unroll
        for (int y = 0; y < 8; y++) col[y] = T[y][u];
        jx_fdct8<FOps>(col, F);
#pragma unroll
        for (int v = 0; v < 8; v++) {
            float tm, d;
            quant_coef(F[v], tab.w[CH][u][v], tm, d);
            if (__builtin_fabsf(d) >= band.lim[CH][u][v]) flagged |= 1ull << (v * 8 + u);
        }
    }
    return flagged;
}

#if !JX_FUSED_FIX
/* Move the wave's queued blocks of channel ch to its region of the launch's lists and empty
 * the queue.  Wave-uniform; `wave` = the k_xform wave index, `done` = items already moved. */
__device__ __forceinline__ void flush_queue(WaveLds &W, Queue &Q, int ch, const jx_fixlist &fx,
                                            unsigned wave, unsigned lane)
{
    const int n = Q.n[ch];
    uint32_t *dst = fx.items + ((size_t)ch * fx.nwaves + wave) * fx.capw + Q.done[ch];
    for (int i = (int)lane; i < n; i += 64) dst[i] = W.item[ch][i];
    Q.done[ch] += n;
    Q.n[ch] = 0;
}
#endif

#ifndef JX_FIX_PAR      /* 1: eight lanes per block and per exact coefficient (see fix_chunk8) */
#define JX_FIX_PAR 1
#endif
#ifndef JX_FIX_GROUP
#define JX_FIX_GROUP (JX_FIX_PAR ? 2 : 8)
#endif
constexpr unsigned kFixGroup = JX_FIX_GROUP;
constexpr int kFixTasks = 64 * 64;             /* FORCE_EXACT: every coefficient of 64 blocks */

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
#ifdef JX_DBG_FIX_NO_DETECT             /* timing experiments only (NOT exact) */
            (void)band;
            if (v == 0 && ((__float_as_uint(d) >> 7) & 7u) == j) flags |= 1u;
#else
            if (__builtin_fabsf(d) >= band.lim[ch][j][v]) flags |= 1u << v;
#endif
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
    /* in k_xform (JX_FUSED_FIX) the blocks' tile stores came from other lanes: they must
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
#ifdef JX_DBG_FIX_NO_EXACT             /* timing experiments only (NOT exact) */
            *coef_ptr(g, L.blk[src], tch, zz_of_rt(v, u)) = (int16_t)s;
#else
            *coef_ptr(g, L.blk[src], tch, zz_of_rt(v, u)) =
                exact_finish(s, u, v, tab.q[tch == 0 ? 0 : 1][u * 8 + v]);
#endif
        }
        wave_sync_lds();                                   /* prod reused */
    }
}

static_assert(sizeof(FixLds8) <= sizeof(WaveLds::stage), "FixLds8 lives in the staging area");
#if JX_FUSED_FIX

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
#endif

/* block index of this lane in tile t (clamped into range for the tail tile) */
[[maybe_unused]] __device__ __forceinline__ unsigned tile_block(unsigned t, unsigned lane,
                                                                unsigned total)
{
    const unsigned b = t * 64u + lane;
    return b < total ? b : total - 1;
}

/*
 * Persistent: each wave walks tiles t, t + waves, ...  Input prefetch (JX_PREFETCH):
 *   0  load the tile's rows at its start (the wait also drains the previous tile's stores)
 *   1  load tile t+1 into a second register set at the start of tile t (+48 VGPRs)
 *   2  load tile t+1 into the same registers once the last row pass has consumed them (the
 *      exact path reloads its pixels)
 */
__global__ __launch_bounds__(JX_WG, JX_WPE) void k_xform(const jx_xform_args a)
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
    const unsigned wave = t;
    if (t >= ntiles) {                             /* whole wave: nothing to queue */
        if (!JX_DBG_NO_EXACT && lane < 3) a.fix.count[lane * a.fix.nwaves + wave] = 0;
        return;
    }
    WaveLds &W = s_wave[threadIdx.x >> 6];
    Queue Q{{0, 0, 0}, {0u, 0u, 0u}};
    unsigned iter = 0;                             /* tiles done by this wave (uniform) */
    const unsigned tpw = (ntiles + nwaves - 1) / nwaves;
    const unsigned stagger_at = tpw > 2 ? wave % (tpw - 1) : 0u;
    (void)stagger_at;
    (void)iter;
    uint32_t raw[8][6];
#if JX_PREFETCH || JX_RELOAD
    {
        const unsigned b = tile_block(t, lane, total), f = b / nb;
        load_block(g, f, b - f * nb, raw);
    }
#if JX_PREFETCH == 2
    __builtin_amdgcn_s_waitcnt(0xF70);              /* vmcnt(0): same state as the back edge */
#pragma unroll
    for (int y = 0; y < 8; y++)
#pragma unroll
        for (int k = 0; k < 6; k++) asm volatile("" : "+v"(raw[y][k]));
#endif
#endif
    for (; t < ntiles; t += nwaves) {
        const unsigned b0 = t * 64u + lane;
        const bool active = b0 < total;
        const unsigned b = active ? b0 : total - 1;
        const unsigned tn = t + nwaves;
#if JX_PREFETCH == 1
        uint32_t nxt[8][6];
        if (tn < ntiles) {
            const unsigned bn = tile_block(tn, lane, total), fn = bn / nb;
            load_block(g, fn, bn - fn * nb, nxt);
        }
#elif JX_PREFETCH == 0 && !JX_RELOAD
        {
            const unsigned f = b / nb;
            load_block(g, f, b - f * nb, raw);
        }
#endif
#if JX_FUSED_FIX == 2
        /* exact pass of earlier tiles' blocks while this tile's pixels are in flight */
        if (!JX_DBG_NO_EXACT && Q.n[0] + Q.n[1] + Q.n[2] > 0) fix_queued(W, Q.n, a, lane);
#endif
        float T[8][8];
#if JX_RELOAD
        const unsigned f = b / nb, bi = b - f * nb;
        const auto reload = [&]() { load_block(g, f, bi, raw); };
        const auto next = [&]() {
            if (tn < ntiles) {
                const unsigned bn = tile_block(tn, lane, total), fn = bn / nb;
                load_block(g, fn, bn - fn * nb, raw);
            }
        };
        xform_rows(0, raw, T);
        xform_cols(0, T, a, W, Q, active, b, t, lane, reload);
        __builtin_amdgcn_sched_barrier(0);
        xform_rows(1, raw, T);
        xform_cols(1, T, a, W, Q, active, b, t, lane, reload);
        __builtin_amdgcn_sched_barrier(0);
        xform_rows(2, raw, T);
        xform_cols(2, T, a, W, Q, active, b, t, lane, next);
        __builtin_amdgcn_sched_barrier(0);
#elif JX_PACKED
        f2 TP[8][4];
        (void)T;
        xform_rows_pk<0>(raw, TP);
        xform_cols_pk<0>(TP, a, W, Q, active, b, t, lane);
        __builtin_amdgcn_sched_barrier(0);
        xform_rows_pk<1>(raw, TP);
        xform_cols_pk<1>(TP, a, W, Q, active, b, t, lane);
        __builtin_amdgcn_sched_barrier(0);
        xform_rows_pk<2>(raw, TP);
#if JX_PREFETCH == 2
        if (tn < ntiles) {                          /* raw is dead: refill it for tile tn */
            const unsigned bn = tile_block(tn, lane, total), fn = bn / nb;
            load_block(g, fn, bn - fn * nb, raw);
        }
#endif
        xform_cols_pk<2>(TP, a, W, Q, active, b, t, lane);
        __builtin_amdgcn_sched_barrier(0);
#elif defined(JX_DBG_NO_COMPUTE)
        /* timing experiments only: the same loads, LDS staging and stores, no transform */
        (void)T;
#pragma unroll
        for (int ch = 0; ch < 3; ch++) {
#pragma unroll
            for (int z = 0; z < 64; z += 2)
                W.stage[lane * 33 + z / 2] = raw[(z >> 3) & 7][(z + ch) % 6] + (uint32_t)z;
            store_and_queue(ch, a, W, Q, active, b, t, lane, 0ull);
            __builtin_amdgcn_sched_barrier(0);
        }
#elif JX_CHLOOP
        /* one copy of the channel body (a third of the code), channel as a uniform value */
        const auto none = []() {};
#pragma nounroll
        for (int ch = 0; ch < 3; ch++) {
            int chv = ch;
            asm volatile("" : "+s"(chv));           /* keep the loop rolled */
            xform_rows(chv, raw, T);
            xform_cols(chv, T, a, W, Q, active, b, t, lane, none);
            __builtin_amdgcn_sched_barrier(0);
        }
#else
        const auto none = []() {};
        xform_rows(0, raw, T);
        xform_cols(0, T, a, W, Q, active, b, t, lane, none);
        __builtin_amdgcn_sched_barrier(0);
        if (!a.luma_only) {                      /* (true subsampling: chroma in k_chroma) */
        xform_rows(1, raw, T);
        xform_cols(1, T, a, W, Q, active, b, t, lane, none);
        __builtin_amdgcn_sched_barrier(0);
        xform_rows(2, raw, T);
#if JX_PREFETCH == 2
        if (tn < ntiles) {                          /* raw is dead: refill it for tile tn */
            const unsigned bn = tile_block(tn, lane, total), fn = bn / nb;
            load_block(g, fn, bn - fn * nb, raw);
        }
        __builtin_amdgcn_sched_barrier(0);          /* issue them here, ahead of the column pass */
#endif
        xform_cols(2, T, a, W, Q, active, b, t, lane, none);
        __builtin_amdgcn_sched_barrier(0);
        }
#if JX_PREFETCH == 2
        /* the next tile's pixels, but not this channel's 8 coefficient stores issued after
         * them: vmcnt counts loads and stores in order, and without this explicit count the
         * wait at the loop head is vmcnt(0), which also drains those stores every tile */
        __builtin_amdgcn_s_waitcnt(0xF78);          /* vmcnt(8), expcnt/lgkmcnt: no wait */
        /* re-define raw here: at the loop head it then comes from this (already waited) point
         * on both paths, not from loads the wait analysis would drain the stores for */
#pragma unroll
        for (int y = 0; y < 8; y++)
#pragma unroll
            for (int k = 0; k < 6; k++) asm volatile("" : "+v"(raw[y][k]));
#endif
#endif
#if JX_FUSED_FIX
        if (!JX_DBG_NO_EXACT) {
            /* only when a queue could overflow (rare): the rest waits for the kernel's end */
            while (Q.n[0] > kItems - 64 || Q.n[1] > kItems - 64 || Q.n[2] > kItems - 64)
                fix_queued(W, Q.n, a, lane);
#if JX_FIX_STAGGER == 1
            /* one mid-run drain per wave, at a wave-dependent tile: the waves' exact passes
             * overlap the others' streaming instead of all landing at the end */
            if (iter == stagger_at)
                while (Q.n[0] + Q.n[1] + Q.n[2] > 0) fix_queued(W, Q.n, a, lane);
#elif JX_FIX_STAGGER == 2
            if (t + 2 * nwaves >= ntiles)        /* before the wave's last tile */
                while (Q.n[0] + Q.n[1] + Q.n[2] > 0) fix_queued(W, Q.n, a, lane);
#endif
        }
        iter++;
#else
        /* keep room for the next tile's 64 possible items per channel */
        if (!JX_DBG_NO_EXACT) {
#pragma unroll
            for (int ch = 0; ch < 3; ch++)
                if (Q.n[ch] > kItems - 64) flush_queue(W, Q, ch, a.fix, wave, lane);
        }
#endif
#if JX_PREFETCH == 1
        if (tn < ntiles) {
#pragma unroll
            for (int y = 0; y < 8; y++)
#pragma unroll
                for (int k = 0; k < 6; k++) raw[y][k] = nxt[y][k];
        }
#else
        (void)tn;
#endif
    }
#if JX_FUSED_FIX
    if (!JX_DBG_NO_EXACT) {
#ifdef JX_DBG_NO_FIXPASS  /* timing experiments only: band test and queueing, no exact pass */
        Q.n[0] = Q.n[1] = Q.n[2] = 0;
#endif
        while (Q.n[0] + Q.n[1] + Q.n[2] > 0) fix_queued(W, Q.n, a, lane);
    }
    (void)wave;
#else
    if (!JX_DBG_NO_EXACT) {
#pragma unroll
        for (int ch = 0; ch < 3; ch++) flush_queue(W, Q, ch, a.fix, wave, lane);
        /* (no runtime index into Q: that would put it in scratch memory) */
        const unsigned mine = lane == 0 ? Q.done[0] : (lane == 1 ? Q.done[1] : Q.done[2]);
        if (lane < 3) a.fix.count[lane * a.fix.nwaves + wave] = mine;
    }
#endif
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
        JX_SB_ROW();
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
            const int i0 = 6 * x, i1 = 6 * x + 3;        /* bytes of pixels 2x, 2x+1 */
            const float p0 = pixel_k(CH, bt(r0, i0), bt(r0, i0 + 1), bt(r0, i0 + 2));
            const float p1 = pixel_k(CH, bt(r0, i1), bt(r0, i1 + 1), bt(r0, i1 + 2));
            if (SUB == 1) {
                smp[x] = (p0 + p1) * 0.5f;
            } else {
                const float q0 = pixel_k(CH, bt(r1, i0), bt(r1, i0 + 1), bt(r1, i0 + 2));
                const float q1 = pixel_k(CH, bt(r1, i1), bt(r1, i1 + 1), bt(r1, i1 + 2));
                smp[x] = ((p0 + p1) + (q0 + q1)) * 0.25f;
            }
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
    const auto none = []() {};
    for (; t < ntiles; t += nwaves) {
        const unsigned b0 = t * 64u + lane;
        const bool active = b0 < total;
        const unsigned b = active ? b0 : total - 1;
        const unsigned f = b / nb, bi = b - f * nb, by = bi / bpr, bx = bi - by * bpr;
#pragma unroll
        for (int ch = 1; ch <= 2; ch++) {
            float T[8][8];
            chroma_rows<SUB>(ch, g, f, bx, by, T);
            xform_cols(ch, T, a, W, Q, active, b, t, lane, none);
            __builtin_amdgcn_sched_barrier(0);
            if (!JX_DBG_NO_EXACT) fix_chroma(W, Q, ch, a, lane);
        }
    }
}

/* ---- k_xform2: two lanes per block ----------------------------------------------------------
 * Lane l < 32 holds pixel rows 0-3 of block l of the tile, lane l + 32 rows 4-7: half the
 * registers of one lane per block (raw 24, row outputs 32), so five waves share a SIMD instead
 * of three.  Row pass: each lane transforms its four rows.  Transpose: v_permlane32_swap
 * exchanges, per (row r, column k < 4), the lower lanes' column 4+k against the upper lanes'
 * column k, after which lane l has columns 0-3 and lane l + 32 columns 4-7 of the block, all
 * eight rows.  Column pass: four columns per lane, the same jx_fdct8 in the same input order,
 * so every fp32 value equals the one-lane kernel's (and the guard band holds unchanged).  The
 * quantiser's scale and band now differ between the two half-waves: they come from a small
 * per-workgroup LDS copy of the quality's tables, [ch][half][k][v] = (w, lim). */
#ifndef JX_K2
#define JX_K2 0
#endif
#ifndef JX_K2_WPE
#define JX_K2_WPE 4
#endif
constexpr int kItems2 = 64;                 /* per channel; a tile adds at most 32 */

struct WaveLds2 {
    union {
        uint32_t stage[32 * 33];            /* one channel: block k at dwords 33k..      */
        FixLds8 fix;                        /* exact pass, between tiles                 */
    };
    uint32_t item[3][kItems2];
};

/* pixel rows 4h..4h+3 of block bi of frame f (load_block's addressing, x0 = -8 quirk) */
__device__ __forceinline__ void load_half(const jx_geom &g, unsigned f, unsigned bi, unsigned h,
                                          uint32_t (&raw)[4][6])
{
    const unsigned r = bi / (unsigned)g.bpr, c = bi - r * (unsigned)g.bpr;
    const bool last = c == (unsigned)g.bpr - 1;
    const bool under = last && (g.row0 + (int)r == 0) && h == 0;
    const long long row = 8ll * r - (last ? 1 : 0) + 4 * (long long)h;
    const uint8_t *base = g.rgb + (long long)f * g.in_fstride + row * g.in_pitch + 24ll * c;
#pragma unroll
    for (int y = 0; y < 4; y++) {
        const uint8_t *p = base + (long long)(y == 0 && under ? 1 : y) * g.in_pitch;
        p = (const uint8_t *)__builtin_assume_aligned(p, 8);
        u32x4 a4;
        u32x2 b2;
        __builtin_memcpy(&a4, p, 16);
        __builtin_memcpy(&b2, p + 16, 8);
        raw[y][0] = a4.x; raw[y][1] = a4.y; raw[y][2] = a4.z; raw[y][3] = a4.w;
        raw[y][4] = b2.x; raw[y][5] = b2.y;
    }
    if (under) {                    /* one lane in rare tiles: a real branch, not six selects
                                       whose operands would have to stay live in registers */
        asm volatile("" ::: "memory");
#pragma unroll
        for (int k = 0; k < 6; k++) raw[0][k] = g.under[k];
    }
}

/* one channel of the tile: rows, transpose, columns, quantiser, staging, store, queue */
__shared__ __attribute__((aligned(16))) float s_tab2[3][2][4][8];  /* [ch][half][k][v] = w(4half+k, v) */

__device__ __forceinline__ void xform2_channel(const int CH, uint32_t (&raw)[4][6],
                                               const jx_xform_args &a, WaveLds2 &W, int (&qn)[3],
                                               bool active, unsigned b, unsigned t, unsigned lane)
{
    const jx_geom &g = a.g;
    const unsigned h = lane >> 5, bl = lane & 31u;
#pragma unroll
    for (int y = 0; y < 4; y++)
#pragma unroll
        for (int k = 0; k < 6; k++) asm volatile("" : "+v"(raw[y][k]));
    float T[4][8];
#pragma unroll
    for (int y = 0; y < 4; y++) {
        JX_SB_ROW();
        float px[8];
        row_pixels(CH, raw[y], px);
        jx_fdct8<FOps>(px, T[y]);
    }
    /* transpose: C[k][y] = column (4h + k), row y */
    float C[4][8];
#pragma unroll
    for (int r = 0; r < 4; r++)
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(T[r][k]),
                                                             __float_as_uint(T[r][4 + k]), false, false);
            C[k][r] = __uint_as_float(sw[0]);
            C[k][4 + r] = __uint_as_float(sw[1]);
        }
    uint64_t seen = 0;
    /* per-lane staging base and half index, opaque here: the 32 per-coefficient addresses
     * (base + zig-zag offset, which differs between the halves) are formed in the loop, one
     * multiply-add each, instead of being hoisted into 32 spilled registers */
    unsigned hv = h, sbase = bl * 66;
    asm volatile("" : "+v"(hv), "+v"(sbase));
    uint16_t *st = (uint16_t *)W.stage + sbase;
    /* this half's scales: one LDS base per channel (opaque, so the per-coefficient addresses
     * become instruction offsets, not hoisted registers); the band is shared by the two
     * halves (limh: the tighter of columns k and 4+k), a scalar operand */
    unsigned tqo = (unsigned)(CH * 2 + h) * 32u;
    asm volatile("" : "+v"(tqo));
    const float4 *tq = (const float4 *)(&s_tab2[0][0][0][0] + tqo);   /* 16-B aligned rows */
    int qv = a.quality * 2 + (a.force_exact ? 1 : 0);
    asm volatile("" : "+v"(qv));
    const int qf = __builtin_amdgcn_readfirstlane(qv);
    const jx_limtab &band = g_lim[qf & 1][qf >> 1];
    float wc[8], lc[8];
    {
        const float4 w0 = tq[0], w1 = tq[1];
        wc[0] = w0.x; wc[1] = w0.y; wc[2] = w0.z; wc[3] = w0.w;
        wc[4] = w1.x; wc[5] = w1.y; wc[6] = w1.z; wc[7] = w1.w;
    }
#pragma unroll
    for (int v = 0; v < 8; v++) lc[v] = band.limh[CH][0][v];
#pragma unroll
    for (int k = 0; k < 4; k++) {
        JX_SB_COL();
        float wn[8], ln[8];
        {
            const float4 w0 = k < 3 ? tq[2 * k + 2] : float4{}, w1 = k < 3 ? tq[2 * k + 3] : float4{};
            wn[0] = w0.x; wn[1] = w0.y; wn[2] = w0.z; wn[3] = w0.w;
            wn[4] = w1.x; wn[5] = w1.y; wn[6] = w1.z; wn[7] = w1.w;
        }
#pragma unroll
        for (int v = 0; v < 8; v++) ln[v] = k < 3 ? band.limh[CH][k + 1][v] : 0.0f;
        float F[8];
        jx_fdct8<FOps>(C[k], F);
#pragma unroll
        for (int v = 0; v < 8; v++) {
            float tm, d;
            quant_coef(F[v], wc[v], tm, d);
            /* zig-zag position of (u = 4h + k, v) as arithmetic on compile-time constants (a
             * select of two constants became a per-lane table load) */
            const int z0 = zz_of(v, k), dz = zz_of(v, 4 + k) - zz_of(v, k);
            st[z0 + (int)hv * dz] = (uint16_t)__float_as_uint(tm);
            if (!JX_DBG_NO_EXACT) {
                uint64_t m;
                asm("v_cmp_ge_f32_e64 %[m], |%[d]|, %[l]\n\t"
                    "s_or_b64 %[seen], %[seen], %[m]"
                    : [m] "=&s"(m), [seen] "+s"(seen)
                    : [d] "v"(d), [l] "s"(lc[v])
                    : "scc");
            }
        }
#pragma unroll
        for (int v = 0; v < 8; v++) {
            wc[v] = wn[v];
            lc[v] = ln[v];
        }
    }
    /* 32 blocks x 128 B: four 1-KiB coalesced stores */
    const unsigned nb = (unsigned)g.nb, total = nb * (unsigned)g.nframes;
    const unsigned b0 = t * 32u;
    const unsigned f0 = b0 / nb, blast = std::min(b0 + 31u, total - 1u), fl = blast / nb;
    if (f0 == fl && b0 + 31u < total) {
        u32x4 *dst = (u32x4 *)(g.out + (long long)f0 * g.out_fstride +
                               ((long long)CH * nb + (b0 - f0 * nb)) * 64);
        unsigned o0 = (lane >> 3) * 33 + (lane & 7) * 4;
        asm volatile("" : "+v"(o0));
        u32x4 unit[4];
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const unsigned o = o0 + 264u * (unsigned)j;
            unit[j] = u32x4{W.stage[o], W.stage[o + 1], W.stage[o + 2], W.stage[o + 3]};
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int j = 0; j < 4; j++) jx_store(dst + (unsigned)j * 64u + lane, unit[j]);
    } else {
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const unsigned e = (unsigned)j * 64u + lane, bb = b0 + (e >> 3);
            if (bb < total) {
                const unsigned o = (e >> 3) * 33 + (e & 7) * 4;
                jx_store((u32x4 *)coef_ptr(g, bb, CH, (int)(e & 7) * 8),
                         u32x4{W.stage[o], W.stage[o + 1], W.stage[o + 2], W.stage[o + 3]});
            }
        }
    }
    /* a block is flagged when either of its lanes is: fold the upper half onto the lower */
    if (!JX_DBG_NO_EXACT && seen != 0) {
        const uint64_t act = __ballot(active);
        const uint32_t M = (uint32_t)((seen | (seen >> 32)) & act);
        const int n = CH == 0 ? qn[0] : (CH == 1 ? qn[1] : qn[2]);
        if (h == 0 && ((M >> bl) & 1u))
            W.item[CH][n + __builtin_amdgcn_mbcnt_lo(M, 0u)] = b;
        const int nn = n + __popc(M);
        qn[0] = CH == 0 ? nn : qn[0];
        qn[1] = CH == 1 ? nn : qn[1];
        qn[2] = CH == 2 ? nn : qn[2];
    }
}

__global__ __launch_bounds__(JX_WG, JX_K2_WPE) void k_xform2(const jx_xform_args a)
{
    __shared__ WaveLds2 s_wave[JX_WG / 64];
    const jx_geom &g = a.g;
    {
        const jx_qtab &tab = g_qtab[a.quality];
        for (unsigned i = threadIdx.x; i < 3 * 2 * 4 * 8; i += blockDim.x) {
            const unsigned ch = i / 64, hh = (i / 32) & 1, k = (i / 8) & 3, v = i & 7;
            s_tab2[ch][hh][k][v] = tab.w[ch][4 * hh + k][v];
        }
        __syncthreads();
    }
    const unsigned nb = (unsigned)g.nb;
    const unsigned total = nb * (unsigned)g.nframes;
    const unsigned ntiles = (total + 31u) / 32u;
    const unsigned lane = threadIdx.x & 63u, h = lane >> 5, bl = lane & 31u;
    const unsigned nwaves = gridDim.x * (JX_WG / 64);
    /* wave-uniform (readfirstlane: the compiler cannot see that threadIdx.x >> 6 is), so the
     * tile loop and its branches are scalar */
    unsigned t = __builtin_amdgcn_readfirstlane(blockIdx.x * (JX_WG / 64) + (threadIdx.x >> 6));
    if (t >= ntiles) return;
    WaveLds2 &W = s_wave[threadIdx.x >> 6];
    int qn[3] = {0, 0, 0};
    for (; t < ntiles; t += nwaves) {
        const unsigned b0 = t * 32u + bl;
        const bool active = b0 < total;
        const unsigned b = active ? b0 : total - 1;
        uint32_t raw[4][6];
        {
            const unsigned f = b / nb;
            load_half(g, f, b - f * nb, h, raw);
        }
        xform2_channel(0, raw, a, W, qn, active, b, t, lane);
        __builtin_amdgcn_sched_barrier(0);
        xform2_channel(1, raw, a, W, qn, active, b, t, lane);
        __builtin_amdgcn_sched_barrier(0);
        xform2_channel(2, raw, a, W, qn, active, b, t, lane);
        __builtin_amdgcn_sched_barrier(0);
        if (!JX_DBG_NO_EXACT) {
            while (qn[0] > kItems2 - 32 || qn[1] > kItems2 - 32 || qn[2] > kItems2 - 32)
                fix_queued(W, qn, a, lane);
        }
    }
    if (!JX_DBG_NO_EXACT) {
        while (qn[0] + qn[1] + qn[2] > 0) fix_queued(W, qn, a, lane);
    }
}

/*
 * The exact pass over the blocks k_xform queued.  Wave (ch, group) takes the lists of channel
 * ch of k_xform waves [kFixGroup*group, +kFixGroup) (waves never mix channels), 64 blocks at
 * a time: (A) one lane per block reloads its pixels, re-finds its flagged coefficients and
 * parks the pixels in LDS; (B) one lane per flagged coefficient recomputes it exactly.
 */
struct FixLds {
    u32x4 px[64][12];                          /* pixel rows of the chunk's blocks           */
    uint32_t blk[64];                          /* their launch-global block indices          */
    uint16_t task[kFixTasks];                  /* lane << 6 | natural coefficient index      */
};

template <int CH>
__device__ __forceinline__ void fix_chunk(FixLds &L, const jx_xform_args &a, unsigned b,
                                          bool has, unsigned lane)
{
    const jx_geom &g = a.g;
    const unsigned nb = (unsigned)g.nb;
    const int force = a.force_exact ? 1 : 0;
    uint64_t flagged = 0;
    if (has) {                                             /* (A) */
        const unsigned f = b / nb;
        uint32_t raw[8][6];
        load_block(g, f, b - f * nb, raw);
#pragma unroll
        for (int k = 0; k < 12; k++) {
            const int d = 4 * k;
            L.px[lane][k] = u32x4{raw[d / 6][d % 6], raw[(d + 1) / 6][(d + 1) % 6],
                                  raw[(d + 2) / 6][(d + 2) % 6], raw[(d + 3) / 6][(d + 3) % 6]};
        }
        L.blk[lane] = b;
#ifdef JX_DBG_FIX_NO_DETECT             /* timing experiments only (NOT exact) */
        flagged = 1ull << (raw[0][0] & 63u);
#else
        flagged = flagged_coefs<CH>(raw, a.quality, force);
#endif
    }
    /* exclusive prefix of the per-lane task counts */
    const unsigned n = (unsigned)__popcll(flagged);
    unsigned incl = n;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const unsigned o = __shfl_up(incl, d, 64);
        if ((int)lane >= d) incl += o;
    }
    const unsigned total = __builtin_amdgcn_readlane(incl, 63);
    unsigned pos = incl - n;
    while (flagged) {
        const unsigned k = (unsigned)__builtin_ctzll(flagged);
        flagged &= flagged - 1;
        L.task[pos++] = (uint16_t)(lane << 6 | k);
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const jx_qtab &tab = g_qtab[a.quality];
    for (unsigned t = lane; t < total; t += 64) {         /* (B) */
        const unsigned tk = L.task[t], src = tk >> 6, k = tk & 63u;
        const int u = (int)(k & 7u), v = (int)(k >> 3);
        uint32_t raw[8][6];
#pragma unroll
        for (int j = 0; j < 12; j++) {
            const u32x4 q4 = L.px[src][j];
            const int d = 4 * j;
            raw[d / 6][d % 6] = q4.x;
            raw[(d + 1) / 6][(d + 1) % 6] = q4.y;
            raw[(d + 2) / 6][(d + 2) % 6] = q4.z;
            raw[(d + 3) / 6][(d + 3) % 6] = q4.w;
        }
#ifdef JX_DBG_FIX_NO_EXACT             /* timing experiments only (NOT exact) */
        *coef_ptr(g, L.blk[src], CH, zz_of_rt(v, u)) = (int16_t)raw[0][0];
#else
        *coef_ptr(g, L.blk[src], CH, zz_of_rt(v, u)) =
            exact_coef<CH>(raw, u, v, tab.q[CH == 0 ? 0 : 1][u * 8 + v]);
#endif
    }
    __builtin_amdgcn_wave_barrier();                       /* LDS reused by the next chunk */
}

#if !JX_FUSED_FIX
#if JX_FIX_PAR
__global__ __launch_bounds__(256) void k_fix(const jx_xform_args a)
{
    __shared__ FixLds8 s_fix[4];
    const jx_fixlist &fx = a.fix;
    const unsigned lane = threadIdx.x & 63u;
    const unsigned groups = (fx.nwaves + kFixGroup - 1) / kFixGroup;
    const unsigned job = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (job >= 3 * groups) return;
    FixLds8 &L = s_fix[threadIdx.x >> 6];
    const int ch = (int)(job / groups);
    const unsigned w0 = (job - ch * groups) * kFixGroup;
    unsigned cnt = 0;
    if (lane < kFixGroup && w0 + lane < fx.nwaves) cnt = fx.count[ch * fx.nwaves + w0 + lane];
    unsigned incl[kFixGroup];
    unsigned run = 0;
#pragma unroll
    for (unsigned s = 0; s < kFixGroup; s++) {
        run += __builtin_amdgcn_readlane(cnt, s);
        incl[s] = run;
    }
    for (unsigned c0 = 0; c0 < run; c0 += 8) {
        const unsigned idx = c0 + (lane >> 3);
        const bool has = idx < run;
        unsigned b = 0;
        if (has) {
            unsigned s = 0, excl = 0;
#pragma unroll
            for (unsigned k = 0; k < kFixGroup; k++)
                if (incl[k] <= idx) {
                    s = k + 1;
                    excl = incl[k];
                }
            b = fx.items[((size_t)ch * fx.nwaves + w0 + s) * fx.capw + (idx - excl)];
        }
        fix_chunk8(L, a, b, ch, has, lane);
    }
}
#else
__global__ __launch_bounds__(256) void k_fix(const jx_xform_args a)
{
    __shared__ FixLds s_fix[4];
    const jx_fixlist &fx = a.fix;
    const unsigned lane = threadIdx.x & 63u;
    const unsigned groups = (fx.nwaves + kFixGroup - 1) / kFixGroup;
    const unsigned job = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (job >= 3 * groups) return;
    FixLds &L = s_fix[threadIdx.x >> 6];
    const int ch = (int)(job / groups);
    const unsigned w0 = (job - ch * groups) * kFixGroup;
    /* counts of the group's waves -> inclusive prefix sums, broadcast to scalars */
    unsigned cnt = 0;
    if (lane < kFixGroup && w0 + lane < fx.nwaves) cnt = fx.count[ch * fx.nwaves + w0 + lane];
    unsigned incl[kFixGroup];
    unsigned run = 0;
#pragma unroll
    for (unsigned s = 0; s < kFixGroup; s++) {
        run += __builtin_amdgcn_readlane(cnt, s);
        incl[s] = run;
    }
    for (unsigned c0 = 0; c0 < run; c0 += 64) {
        const unsigned i = c0 + lane;
        const bool has = i < run;
        unsigned b = 0;
        if (has) {
            unsigned s = 0, excl = 0;
#pragma unroll
            for (unsigned k = 0; k < kFixGroup; k++)
                if (incl[k] <= i) {
                    s = k + 1;
                    excl = incl[k];
                }
            b = fx.items[((size_t)ch * fx.nwaves + w0 + s) * fx.capw + (i - excl)];
        }
        if (ch == 0) fix_chunk<0>(L, a, b, has, lane);
        else if (ch == 1) fix_chunk<1>(L, a, b, has, lane);
        else fix_chunk<2>(L, a, b, has, lane);
    }
}
#endif
#endif  /* !JX_FUSED_FIX */

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

/* a float <= lim^2 (exactly representable squares of floats fit in a double); -1 for lim < 0 */
float lim_square_down(float lim)
{
    if (!(lim > 0.0f)) return -1.0f;
    const double l2 = (double)lim * (double)lim;
    float s = (float)l2;
    if ((double)s > l2) s = nextafterf(s, 0.0f);
    return s;
}

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
            for (int ch = 0; ch < 3; ch++)
                for (int u = 0; u < 8; u++) {
                    float m = band[q].lim[ch][u][0];
                    for (int v = 1; v < 8; v++) m = std::min(m, band[q].lim[ch][u][v]);
                    band[q].limcol[ch][u] = m;
                    band[JX_MAXQ + 1 + q].limcol[ch][u] = -1.0f;
                }
            for (int ch = 0; ch < 3; ch++)
                for (int u = 0; u < 8; u++)
                    for (int v = 0; v < 8; v++) {
                        band[q].lsqn[ch][u][v] = lim_square_down(band[q].lim[ch][u][v]);
                        band[JX_MAXQ + 1 + q].lsqn[ch][u][v] = -1.0f;
                    }
            for (int ch = 0; ch < 3; ch++)
                for (int k = 0; k < 4; k++)
                    for (int v = 0; v < 8; v++) {
                        band[q].limh[ch][k][v] =
                            std::min(band[q].lim[ch][k][v], band[q].lim[ch][4 + k][v]);
                        band[JX_MAXQ + 1 + q].limh[ch][k][v] = -1.0f;
                    }
            /* packed path: pair order, squared limits rounded down (d*d >= lsq is implied by
             * |d| >= lim, so every coefficient the band flags is still flagged) */
            for (int ch = 0; ch < 3; ch++)
                for (int j = 0; j < 4; j++)
                    for (int v = 0; v < 8; v++)
                        for (int l = 0; l < 2; l++) {
                            const int u = jx_pk_k(j, l);
                            host[q].wp[ch][j][v][l] = w[ch][v * 8 + u];
                            const double lm = (double)band[q].lim[ch][u][v];
                            float s = -1.0f;
                            if (lm > 0) {
                                s = (float)(lm * lm);
                                if ((double)s > lm * lm) s = nextafterf(s, 0.0f);
                            }
                            band[q].lsq[ch][j][v][l] = s;
                            band[JX_MAXQ + 1 + q].lsq[ch][j][v][l] = -1.0f;
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
                            bn.lim[ch][u][v] = lim[ch][v * 8 + u];
                            bf.lim[ch][u][v] = -1.0f;
                            bn.lsqn[ch][u][v] = lim_square_down(lim[ch][v * 8 + u]);
                            bf.lsqn[ch][u][v] = -1.0f;
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
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, JX_K2 ? k_xform2 : k_xform, JX_WG,
                                                          0) != hipSuccess ||
            per_cu < 1)
            per_cu = 2;
#ifdef JX_DBG_GRID_WGS_PER_CU   /* timing experiments: fewer resident workgroups per CU */
        per_cu = std::min(per_cu, JX_DBG_GRID_WGS_PER_CU);
#endif
        g_resident_waves[dev] = cus * per_cu * (JX_WG / 64);
    });
    return g_resident_waves[dev];
}

/* the 4:4:4 transform kernel: k_xform (all-VALU), or k_mx (matrix-core row pass,
 * csrc/jpgx_mx.hip) with JPGX_KERNEL=mx -- bit-exact, measured slower so far */
bool mx_selected()
{
    const char *e = getenv("JPGX_KERNEL");
    return e && strcmp(e, "mx") == 0;
}

}  // namespace

extern "C" {

size_t jpgx_chroma_blocks(int width, int row_begin, int row_end, int sample_ratio, unsigned flags)
{
    if (width <= 0 || row_end < row_begin) return 0;
    const size_t rows = (size_t)(row_end - row_begin);
    if (!(flags & JPGX_FLAG_SUBSAMPLE) || sample_ratio == 0) return rows * (size_t)(width / 8);
    return (sample_ratio == 2 ? rows / 2 : rows) * (size_t)(width / 16);
}

size_t jpgx_workspace_size(const jpgx_frames *fr)
{
    if (!fr || fr->row_end <= fr->row_begin || fr->nframes < 1 || fr->width < 8) return 0;
    const size_t total = (size_t)(fr->row_end - fr->row_begin) * (fr->width / 8) * fr->nframes;
    const size_t ntiles = (total + 63) / 64;
    /* per k_xform wave (at most tiles + 3 of them) and channel: a count, and room for 64
     * items per tile the wave walks (waves x ceil(tiles / waves) < 2 x tiles + 3) */
    const size_t counts = (3 * (ntiles + 3) * sizeof(unsigned) + 255) & ~(size_t)255;
    const size_t xform = JX_WS_HEADER + counts + 3 * (2 * ntiles + 3) * 64 * sizeof(uint32_t);
    return xform;
}

int jpgx_blocks_gpu(const jpgx_frames *fr, const jpgx_params *p, const uint8_t *d_rgb,
                    int16_t *d_out, void *d_workspace, size_t workspace_bytes, void *stream)
{
    return jpgx_blocks_gpu_ev(fr, p, d_rgb, d_out, d_workspace, workspace_bytes, stream, nullptr);
}

int jpgx_blocks_gpu_ev(const jpgx_frames *fr, const jpgx_params *p, const uint8_t *d_rgb,
                       int16_t *d_out, void *d_workspace, size_t workspace_bytes, void *stream,
                       void *event_after)
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
    if (workspace_bytes < jpgx_workspace_size(fr) || !d_workspace ||
        ((uintptr_t)d_workspace & 15))
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
    jx_under_dwords(p->underflow, g.under);
    rc = tables_for_current_device();
    if (rc) return rc;
    xa.quality = p->quality;
    xa.force_exact = (p->flags & JPGX_FLAG_FORCE_EXACT) ? 1 : 0;
    hipStream_t s = (hipStream_t)stream;
    xa.luma_only = sub ? 1 : 0;
    if (!sub && mx_selected()) {
        /* k_mx: colour + row DCT on the matrix cores, exact pass inside (csrc/jpgx_mx.hip) */
        rc = jx_launch_mx(&xa, stream);
        if (rc) return rc;
        if (event_after) rc = hip_rc(hipEventRecord((hipEvent_t)event_after, s));
        return rc;
    }
    if (JX_K2 && !sub) {
        /* two lanes per block: 32-block tiles, persistent grid, exact pass inside */
        const size_t nt2 = (total + 31) / 32;
        const size_t w2 = std::min<size_t>(nt2, (size_t)std::max(resident_waves(), 4));
        const unsigned grid2 = (unsigned)((w2 + JX_WG / 64 - 1) / (JX_WG / 64));
        hipLaunchKernelGGL(k_xform2, dim3(grid2), dim3(JX_WG), 0, s, xa);
        rc = hip_rc(hipGetLastError());
        if (rc) return rc;
        if (event_after) rc = hip_rc(hipEventRecord((hipEvent_t)event_after, s));
        return rc;
    }
    const size_t ntiles = (total + 63) / 64;
#ifndef JX_PERSISTENT     /* 0: one wave per tile (the dispatcher refills SIMDs as waves end) */
#define JX_PERSISTENT 1
#endif
    size_t waves = JX_PERSISTENT ? std::min<size_t>(ntiles, (size_t)std::max(resident_waves(), 4))
                                 : ntiles;
#ifndef JX_GRID_BALANCE   /* 1: fewest waves that still finish in the same number of rounds */
#define JX_GRID_BALANCE 0
#endif
    if (JX_GRID_BALANCE) {
        const size_t rounds = (ntiles + waves - 1) / waves;
        waves = (ntiles + rounds - 1) / rounds;
    }
    const unsigned grid = (unsigned)((waves + JX_WG / 64 - 1) / (JX_WG / 64));
    const size_t nwaves = (size_t)grid * (JX_WG / 64);      /* >= waves, <= ntiles + 3   */
    const size_t tpw = (ntiles + nwaves - 1) / nwaves;
    xa.fix.nwaves = (unsigned)nwaves;
    xa.fix.capw = (unsigned)(tpw * 64);
    xa.fix.count = (unsigned *)((uint8_t *)d_workspace + JX_WS_HEADER);
    xa.fix.items = (uint32_t *)((uint8_t *)d_workspace + JX_WS_HEADER +
                                ((3 * nwaves * sizeof(unsigned) + 255) & ~(size_t)255));
    /* the layout must fit the size promised by jpgx_workspace_size */
    if (JX_WS_HEADER + ((3 * nwaves * sizeof(unsigned) + 255) & ~(size_t)255) +
            3 * nwaves * tpw * 64 * sizeof(uint32_t) > workspace_bytes)
        return JPGX_EWORKSPACE;
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
    if (event_after) rc = hip_rc(hipEventRecord((hipEvent_t)event_after, s));
    if (rc) return rc;
    /* exact pass: one wave per channel and group of kFixGroup k_xform waves */
    const size_t jobs = 3 * ((nwaves + kFixGroup - 1) / kFixGroup);
    const unsigned fgrid = (unsigned)((jobs + 3) / 4);
#if !defined(JX_DBG_HOST_NO_FIX) && !JX_FUSED_FIX   /* (HOST_NO_FIX: timing only, NOT exact) */
    if (!JX_DBG_NO_EXACT) hipLaunchKernelGGL(k_fix, dim3(fgrid), dim3(256), 0, s, xa);
#else
    (void)fgrid;
#endif
    return hip_rc(hipGetLastError());
}

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

/* One GPU, one stripe: H2D of the stripe (+ the pixel row above it), run, D2H of the
 * stripe's three channel ranges into the whole-image host output: [3][nb][64], or with
 * JPGX_FLAG_SUBSAMPLE Y [nb][64] + Cb, Cr [nbc][64]. */
static int run_stripe(const uint8_t *rgb, int width, int height, size_t pitch,
                      const jpgx_params *p, int16_t *out, int device, int r0, int r1)
{
    if (r0 == r1) return JPGX_OK;
    if (hipSetDevice(device) != hipSuccess) return JPGX_ENODEV;
    const int bpr = width / 8;
    const size_t row_bytes = (size_t)width * 3;
    const size_t dpitch = (row_bytes + 7) & ~(size_t)7;
    const int halo = r0 > 0 ? 1 : 0;
    const size_t rows = (size_t)(r1 - r0) * 8 + halo;
    const size_t nb_s = (size_t)(r1 - r0) * bpr, nb = (size_t)(height / 8) * bpr;
    const size_t nbc_s = jpgx_chroma_blocks(width, r0, r1, p->sample_ratio, p->flags);
    const size_t nbc = jpgx_chroma_blocks(width, 0, height / 8, p->sample_ratio, p->flags);
    const size_t c0 = jpgx_chroma_blocks(width, 0, r0, p->sample_ratio, p->flags);
    jpgx_frames fr;
    memset(&fr, 0, sizeof fr);
    fr.width = width;
    fr.height = height;
    fr.row_begin = r0;
    fr.row_end = r1;
    fr.nframes = 1;
    fr.in_pitch = dpitch;
    fr.in_frame_stride = dpitch * rows;
    fr.out_frame_stride = (nb_s + 2 * nbc_s) * 64;
    uint8_t *d_in = nullptr;
    int16_t *d_out = nullptr;
    void *d_ws = nullptr;
    const size_t ws = jpgx_workspace_size(&fr);
    hipStream_t s = nullptr;
    int rc = JPGX_OK;
    if (hipMalloc(&d_in, rows * dpitch) != hipSuccess ||
        hipMalloc(&d_out, (nb_s + 2 * nbc_s) * 64 * sizeof(int16_t)) != hipSuccess ||
        hipMalloc(&d_ws, ws) != hipSuccess || hipStreamCreate(&s) != hipSuccess) {
        rc = JPGX_EHIP;
    }
    if (!rc) {
        const uint8_t *src = rgb + ((size_t)r0 * 8 - halo) * pitch;
        rc = hip_rc(hipMemcpy2DAsync(d_in, dpitch, src, pitch, row_bytes, rows,
                                     hipMemcpyHostToDevice, s));
    }
    if (!rc) rc = jpgx_blocks_gpu(&fr, p, d_in + halo * dpitch, d_out, d_ws, ws, s);
    for (int ch = 0; ch < 3 && !rc; ch++) {
        const size_t dst = ch == 0 ? (size_t)r0 * bpr : nb + (size_t)(ch - 1) * nbc + c0;
        const size_t srcb = ch == 0 ? 0 : nb_s + (size_t)(ch - 1) * nbc_s;
        const size_t cnt = ch == 0 ? nb_s : nbc_s;
        rc = hip_rc(hipMemcpyAsync(out + dst * 64, d_out + srcb * 64, cnt * 64 * sizeof(int16_t),
                                   hipMemcpyDeviceToHost, s));
    }
    if (!rc) rc = hip_rc(hipStreamSynchronize(s));
    if (s) (void)hipStreamDestroy(s);
    (void)hipFree(d_in);
    (void)hipFree(d_out);
    (void)hipFree(d_ws);
    return rc;
}

int jpgx_blocks(const uint8_t *rgb, int width, int height, size_t pitch, const jpgx_params *p,
                int16_t *out, int device)
{
    if (!rgb || !out || !p) return JPGX_EARG;
    int rc = jpgx_validate(width, height, p);
    if (rc) return rc;
    if (pitch < (size_t)width * 3) return JPGX_EARG;
    if (device < 0 || device >= jpgx_device_count()) return JPGX_ENODEV;
    return run_stripe(rgb, width, height, pitch, p, out, device, 0, height / 8);
}

int jpgx_blocks_multi(const uint8_t *rgb, int width, int height, size_t pitch,
                      const jpgx_params *p, int16_t *out, int ngpus)
{
    if (!rgb || !out || !p || ngpus < 1) return JPGX_EARG;
    int rc = jpgx_validate(width, height, p);
    if (rc) return rc;
    if (pitch < (size_t)width * 3) return JPGX_EARG;
    if (ngpus > jpgx_device_count()) return JPGX_ENODEV;
    std::vector<int> rcs(ngpus, JPGX_OK);
    std::vector<std::thread> th;
    /* true 4:2:0 stripes split MCU rows (pairs of block rows) */
    const int unit = (p->flags & JPGX_FLAG_SUBSAMPLE) && p->sample_ratio == 2 ? 2 : 1;
    for (int k = 0; k < ngpus; k++) {
        th.emplace_back([&, k]() {
            int r0, r1;
            jpgx_stripe(height / 8 / unit, ngpus, k, &r0, &r1);
            r0 *= unit;
            r1 *= unit;
            rcs[k] = run_stripe(rgb, width, height, pitch, p, out, k, r0, r1);
        });
    }
    for (auto &t : th) t.join();
    for (int k = 0; k < ngpus; k++)
        if (rcs[k]) return rcs[k];
    return JPGX_OK;
}

}  /* extern "C" */
