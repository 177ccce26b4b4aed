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
#ifndef JX_ROW_SB       /* scheduling fence between the row DCTs of a channel          */
#define JX_ROW_SB 1
#endif
#ifndef JX_COL_SB       /* scheduling fence between the column DCTs of a channel       */
#define JX_COL_SB 1
#endif
#ifndef JX_EXACT_INLINE /* inline the rare exact-path helpers (vs real calls)           */
#define JX_EXACT_INLINE 1
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
#ifndef JX_WPE          /* minimum waves per SIMD the register allocation must allow    */
#define JX_WPE 2
#endif
#ifndef JX_DBG_FLAGMODE  /* guard-band bookkeeping: 0 SALU masks in asm, 3 VALU count+select */
#define JX_DBG_FLAGMODE 0
#endif
#ifndef JX_DBG_UNIFORM_LIM
#define JX_DBG_UNIFORM_LIM 0
#endif
#ifndef JX_DBG_NO_ADMIT
#define JX_DBG_NO_ADMIT 0
#endif
#ifndef JX_FLAG_ASM_VOLATILE    /* 1: the flag bookkeeping asm also fences scheduling     */
#define JX_FLAG_ASM_VOLATILE 0  /*    (measured 6% slower; kept as a knob)                */
#endif
#if JX_FLAG_ASM_VOLATILE
#define JX_FLAG_ASM_Q volatile
#else
#define JX_FLAG_ASM_Q
#endif
#ifndef JX_DBG_NO_EXACT  /* debug/measurement only: drop the exact path (NOT bit-exact)    */
#define JX_DBG_NO_EXACT 0
#endif
#if JX_EXACT_INLINE
#define JX_RARE __device__
#else
#define JX_RARE __device__ __noinline__
#endif

constexpr float kMagic = 12582912.0f; /* 1.5 * 2^23: x + kMagic rounds x to an integer   */
#ifndef JX_SLOTS_PER_WAVE
#define JX_SLOTS_PER_WAVE 32
#endif
constexpr int kSlots = JX_SLOTS_PER_WAVE; /* per-wave deferred-exact queue: pixel slots    */
constexpr int kItems = 128;               /*                             and coefficients  */
static_assert(kSlots <= 32, "item encoding keeps 5 bits for the slot");

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
__host__ __device__ constexpr int zz_col_done(int z0, int z1)
{
    return zz_col(z0) > zz_col(z1) ? zz_col(z0) : zz_col(z1);
}
/* the column pass after which the 16-byte output chunk j (zig-zag 8j..8j+7) is complete */
__host__ __device__ constexpr int zz_chunk_done(int j)
{
    int m = 0;
    for (int z = 8 * j; z < 8 * j + 8; z++) m = zz_col(z) > m ? zz_col(z) : m;
    return m;
}

/* inverse scan: zig-zag index -> (v << 3) | u */
__constant__ uint8_t kUnZZ[64] = {
    0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,
    12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13, 6,  7,  14, 21, 28,
    35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51,
    58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63};

/* cos(((2x+1)*u*M_PI)/16) exactly as glibc returns it for the reference (jx_consts.h) */
__constant__ double kCos[8][8] = JX_COS_INIT;

/* Per-quality tables (index 0 unused), constant address space so that wave-uniform reads
 * become scalar loads; filled once per device by tables_for_current_device(). */
__constant__ jx_qtab g_qtab[JX_MAXQ + 1];
__constant__ jx_limtab g_lim[2][JX_MAXQ + 1];

/* dct.c:13 ALPHA(0) = 1/sqrt(2) as the reference's double */
constexpr double kAlpha0 = JX_ALPHA0;

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

#ifndef JX_NT_STORE     /* coefficient stores with the nontemporal bit (streamed, never re-read) */
#define JX_NT_STORE 1
#endif
#ifndef JX_NT_LOAD      /* pixel loads with the nontemporal bit                                 */
#define JX_NT_LOAD 0
#endif

__device__ __forceinline__ void jx_store(u32x4 *p, u32x4 v)
{
#if JX_NT_STORE
    __builtin_nontemporal_store(v, p);
#else
    *p = v;
#endif
}

/* Per-wave LDS.  `stage` and `px` are adjacent: after a flush the pair is reused as 64 x
 * 192 B to stage every lane's block for a whole-block exact recompute (overflow path). */
struct WaveLds {
    u32x4 stage[64 * 9];          /* one channel: block k's 8 chunks at units 9k..9k+7     */
    u32x4 px[kSlots][12];         /* pixel rows (8 x 24 B) of blocks with queued items     */
    uint32_t slot_blk[kSlots];    /* launch-global block index of each slot                */
    uint32_t item[kItems];        /* slot | ch << 5 | zigzag << 7                          */
};
static_assert(sizeof(u32x4) * (64 * 9 + kSlots * 12) >= 64 * 192, "overflow staging");

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
#if JX_NT_LOAD
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

__device__ __forceinline__ void raw_to_lds(const uint32_t (&raw)[8][6], u32x4 *dst)
{
#pragma unroll
    for (int k = 0; k < 12; k++) {
        const int d = 4 * k;
        dst[k] = u32x4{raw[d / 6][d % 6], raw[(d + 1) / 6][(d + 1) % 6],
                       raw[(d + 2) / 6][(d + 2) % 6], raw[(d + 3) / 6][(d + 3) % 6]};
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

/* One coefficient in the reference's exact operation order.  px = the block's 8 pixel rows
 * (24 interleaved bytes each, 48 dwords), already in registers. */
template <int CH>
__device__ __forceinline__ double exact_sum(const uint32_t (&px)[48], int u, int v)
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
            const int o = y * 24 + 3 * x;
            const int r = (int)((px[o >> 2] >> (8 * (o & 3))) & 0xffu);
            const int g = (int)((px[(o + 1) >> 2] >> (8 * ((o + 1) & 3))) & 0xffu);
            const int b = (int)((px[(o + 2) >> 2] >> (8 * ((o + 2) & 3))) & 0xffu);
            s += exact_pixel(CH, r, g, b) * cu[x] * cv[y];   /* (X*c_u[x])*c_v[y], :48-50 */
        }
    return s;
}

__device__ int16_t exact_coef(const uint32_t (&px)[48], int ch, int u, int v, int q)
{
    const double s = ch == 0 ? exact_sum<0>(px, u, v)
                             : (ch == 1 ? exact_sum<1>(px, u, v) : exact_sum<2>(px, u, v));
    const double F = 0.25 * (u == 0 ? kAlpha0 : 1.0) * (v == 0 ? kAlpha0 : 1.0) * s;
    return (int16_t)(int)round(F / (double)q);      /* quantise.c:58 */
}

__device__ __forceinline__ int16_t *coef_ptr(const jx_geom &g, unsigned b, int ch, int zz)
{
    const unsigned nb = (unsigned)g.nb, f = b / nb, bi = b - f * nb;
    return g.out + (long long)f * g.out_fstride + ((long long)ch * nb + bi) * 64 + zz;
}

/* Process every queued coefficient of the wave, lanes in parallel.  Wave-uniform call. */
JX_RARE void flush_queue(WaveLds &W, int nitem, const jx_geom &g, int quality,
                                         unsigned lane)
{
    /* the fast-path values these overwrite were stored earlier by this wave */
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    for (int i = (int)lane; i < nitem; i += 64) {
        const uint32_t it = W.item[i];
        const int slot = (int)(it & 31u), ch = (int)((it >> 5) & 3u), zz = (int)(it >> 7);
        const int uv = kUnZZ[zz], u = uv & 7, v = uv >> 3;
        const int q = g_qtab[quality].q[ch == 0 ? 0 : 1][u * 8 + v];
        uint32_t px[48];
#pragma unroll
        for (int k = 0; k < 12; k++) {
            const u32x4 d4 = W.px[slot][k];
            px[4 * k] = d4.x; px[4 * k + 1] = d4.y; px[4 * k + 2] = d4.z; px[4 * k + 3] = d4.w;
        }
        *coef_ptr(g, W.slot_blk[slot], ch, zz) = exact_coef(px, ch, u, v, q);
    }
}

/* wave-uniform deferred-exact queue state */
struct Queue {
    int nslot, nitem;
};

/* number of set bits of m below this lane */
__device__ __forceinline__ int lane_rank(uint64_t m)
{
    return (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                          __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

__device__ __forceinline__ void drain(WaveLds &W, Queue &Q, int &myslot, const jx_geom &g,
                                      int quality, unsigned lane)
{
    if (Q.nitem) flush_queue(W, Q.nitem, g, quality, lane);
    Q.nitem = Q.nslot = 0;
    myslot = -1;
}

/* Per lane: block-channels whose exact work did not fit the queue during the tile. */
struct Pending {
    unsigned bits;          /* bit ch: channel ch of this lane's block is pending          */
    int idx0, idx1, idx2;   /* per channel: the single flagged zig-zag index, or -1 = all 64 */
};

/*
 * Admit `single` lanes (one flagged coefficient, zig-zag `idx`) of channel CH into the
 * queue without draining it (the channel passes run at full register pressure): lanes that
 * do not fit, and block-channels with several flags (`multi`, all 64 coefficients), are
 * left pending for settle_pending() at the end of the tile.  Wave-uniform call.
 */
template <int CH>
__device__ __forceinline__ void admit_flags(WaveLds &W, Queue &Q, int &myslot,
                                            const uint32_t (&raw)[8][6], unsigned b, bool single,
                                            bool multi, int idx, unsigned lane, Pending &P)
{
    const uint64_t S = __ballot(single);
    const uint64_t needs = S & __ballot(myslot < 0);
    const bool admit = single && lane_rank(S) < kItems - Q.nitem &&
                       (myslot >= 0 || lane_rank(needs) < kSlots - Q.nslot);
    const uint64_t A = __ballot(admit);
    const uint64_t fresh = A & needs;
    if (admit && myslot < 0) {
        myslot = Q.nslot + lane_rank(fresh);
        raw_to_lds(raw, W.px[myslot]);
        W.slot_blk[myslot] = b;
    }
    if (admit)
        W.item[Q.nitem + lane_rank(A)] = (uint32_t)myslot | (uint32_t)CH << 5 | (uint32_t)idx << 7;
    Q.nslot += __popcll(fresh);
    Q.nitem += __popcll(A);
    if ((single && !admit) || multi) {
        P.bits |= 1u << CH;
        const int id = multi ? -1 : idx;
        if (CH == 0) P.idx0 = id;
        if (CH == 1) P.idx1 = id;
        if (CH == 2) P.idx2 = id;
    }
}

/*
 * End of tile: queue every pending block-channel, draining the queue (lane-parallel exact
 * pass) as often as needed.  Pixel rows come from `raw`, still this tile's.  Wave-uniform.
 */
__device__ void settle_pending(WaveLds &W, Queue &Q, int &myslot, const uint32_t (&raw)[8][6],
                               unsigned b, Pending &P, const jx_geom &g, int quality,
                               unsigned lane)
{
#pragma unroll 1
    for (int ch = 0; ch < 3; ch++) {
        const bool pend = (P.bits >> ch) & 1u;
        const int id = ch == 0 ? P.idx0 : (ch == 1 ? P.idx1 : P.idx2);
        uint64_t S = __ballot(pend && id >= 0);
        while (S) {                               /* singles, as many as fit per drain */
            const uint64_t needs = S & __ballot(myslot < 0);
            const bool admit = ((S >> lane) & 1u) && lane_rank(S) < kItems - Q.nitem &&
                               (myslot >= 0 || lane_rank(needs) < kSlots - Q.nslot);
            const uint64_t A = __ballot(admit);
            if (!A) {
                drain(W, Q, myslot, g, quality, lane);
                continue;
            }
            const uint64_t fresh = A & needs;
            if (admit && myslot < 0) {
                myslot = Q.nslot + lane_rank(fresh);
                raw_to_lds(raw, W.px[myslot]);
                W.slot_blk[myslot] = b;
            }
            if (admit)
                W.item[Q.nitem + lane_rank(A)] =
                    (uint32_t)myslot | (uint32_t)ch << 5 | (uint32_t)id << 7;
            Q.nslot += __popcll(fresh);
            Q.nitem += __popcll(A);
            S &= ~A;
        }
        uint64_t M = __ballot(pend && id < 0);
        while (M) {                               /* whole block-channels: 64 items each */
            const unsigned L = (unsigned)__builtin_ctzll(M);
            M &= M - 1;
            drain(W, Q, myslot, g, quality, lane);
            if (lane == L) {
                raw_to_lds(raw, W.px[0]);
                W.slot_blk[0] = b;
            }
            W.item[lane] = 0u | (uint32_t)ch << 5 | lane << 7;   /* zig-zag index = lane */
            Q.nslot = 1;
            Q.nitem = 64;
            drain(W, Q, myslot, g, quality, lane);
        }
    }
    P.bits = 0;
}

/* ---- fast path --------------------------------------------------------------------------- */

/* Row pass of channel CH: bytes -> pixel values -> 1-D DCT of each of the 8 pixel rows. */
template <int CH>
__device__ __forceinline__ void xform_rows(uint32_t (&raw)[8][6], float (&T)[8][8])
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
#pragma unroll
        for (int x = 0; x < 8; x++) {
            const float r = (float)byte_of(raw[y], 3 * x);
            const float gg = (float)byte_of(raw[y], 3 * x + 1);
            const float bb = (float)byte_of(raw[y], 3 * x + 2);
            px[x] = jx_pixel<FOps, CH>(r, gg, bb);
        }
        jx_fdct8<FOps>(px, T[y]);
    }
}

/* Column pass, quantisation, zig-zag, LDS staging + coalesced store of channel CH. */
template <int CH>
__device__ __forceinline__ void xform_cols(float (&T)[8][8], const uint32_t (&raw)[8][6],
                                           const jx_xform_args &a, WaveLds &W, Queue &Q,
                                           int &myslot, Pending &P, bool active, unsigned b,
                                           unsigned t, unsigned lane)
{
    const jx_geom &g = a.g;
    uint32_t bits[64];     /* tm bit patterns by zig-zag index; low 16 bits = the int16    */
    uint32_t packed[32];   /* zig-zag pairs (2k, 2k+1) as one dword, formed when complete */
    const jx_qtab &tab = g_qtab[a.quality];
    const jx_limtab &band = g_lim[a.force_exact ? 1 : 0][a.quality];
    const bool force = a.force_exact != 0;
    /* guard-band bookkeeping, branch-free: per lane the zig-zag index of its (last) flagged
     * coefficient; wave masks of lanes with >= 1 and with >= 2 flags in this channel */
    int idx = 0;
    uint64_t seen = 0, dup = 0;
#if JX_DBG_FLAGMODE == 3
    int nfl = 0;
#endif
#pragma unroll
    for (int u = 0; u < 8; u++) {
        float col[8], F[8];
#pragma unroll
        for (int y = 0; y < 8; y++) col[y] = T[y][u];
        jx_fdct8<FOps>(col, F);
#pragma unroll
        for (int v = 0; v < 8; v++) {
            const float w = tab.w[CH][u][v];
            const float tm = __builtin_fmaf(F[v], w, kMagic);   /* rint(F*w) + magic  */
            const float rr = tm - kMagic;                         /* exact             */
            const float d = __builtin_fmaf(F[v], w, -rr);         /* F*w - rint(F*w)   */
            bits[zz_of(v, u)] = __float_as_uint(tm);              /* low 16 bits = int16 */
            if (!JX_DBG_NO_EXACT) {
#if JX_DBG_UNIFORM_LIM   /* timing experiment only: one limit per channel (NOT the product) */
                const bool fl = __builtin_fabsf(d) >= band.lim[CH][0][0];
#else
                const bool fl = __builtin_fabsf(d) >= band.lim[CH][u][v];
#endif
#if JX_DBG_FLAGMODE == 3
                /* per-lane count and index, all VALU (compare + 2 selects) */
                nfl += fl ? 1 : 0;
                idx = fl ? zz_of(v, u) : idx;
#else
                const uint64_t m = __ballot(fl);
                /* SALU mask bookkeeping kept next to its compare: left to the compiler, the
                 * 64 masks of a channel are kept alive until the end and spilled */
                uint64_t tmp;
                asm JX_FLAG_ASM_Q("s_and_b64 %[t], %[m], %[seen]\n\t"
                             "s_or_b64 %[dup], %[dup], %[t]\n\t"
                             "s_or_b64 %[seen], %[seen], %[m]\n\t"
                             "v_cndmask_b32_e64 %[idx], %[idx], %[z], %[m]"
                             : [dup] "+s"(dup), [seen] "+s"(seen), [t] "=&s"(tmp),
                               [idx] "+v"(idx)
                             : [m] "s"(m), [z] "n"(zz_of(v, u))
                             : "scc");
#endif
            }
        }
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
        JX_SB_COL();
    }

    /* coalesced store: the wave's 64 blocks x 128 B of this channel, 1 KiB per instruction */
    const unsigned nb = (unsigned)g.nb, total = nb * (unsigned)g.nframes;
    const unsigned b0 = t * 64u;
    const unsigned f0 = b0 / nb, bl = std::min(b0 + 63u, total - 1u), fl = bl / nb;
    if (f0 == fl && b0 + 63u < total) {
        u32x4 *dst = (u32x4 *)(g.out + (long long)f0 * g.out_fstride +
                               ((long long)CH * nb + (b0 - f0 * nb)) * 64);
#pragma unroll
        for (int j = 0; j < 8; j++) {
            const unsigned e = (unsigned)j * 64u + lane;
            jx_store(dst + e, W.stage[(e >> 3) * 9 + (e & 7)]);
        }
    } else {                                   /* tile crosses a frame end or the last tile */
#pragma unroll
        for (int j = 0; j < 8; j++) {
            const unsigned e = (unsigned)j * 64u + lane, bb = b0 + (e >> 3);
            if (bb < total)
                jx_store((u32x4 *)coef_ptr(g, bb, CH, (int)(e & 7) * 8),
                         W.stage[(e >> 3) * 9 + (e & 7)]);
        }
    }
    /* some lane has a coefficient inside the guard band (about half the channel-tiles of
     * random data at q90; wave-uniform branch): queue the exact recomputation */
#if JX_DBG_FLAGMODE == 3
    seen = __ballot(nfl > 0);
    dup = __ballot(nfl > 1);
#endif
#if JX_DBG_NO_ADMIT      /* timing experiment only: bookkeeping without acting on it */
    if (seen != 0 && lane == 0) W.item[0] = (uint32_t)idx ^ (uint32_t)dup;
#else
    if (!JX_DBG_NO_EXACT && seen != 0) {
        const bool mine = active && ((seen >> lane) & 1u);
        const bool multi = mine && (force || ((dup >> lane) & 1u));
        admit_flags<CH>(W, Q, myslot, raw, b, mine && !multi, multi, idx, lane, P);
    }
#endif
}

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
 *   2  (timing builds without the exact path only) load tile t+1 into the same registers
 *      once the last row pass has consumed them -- the exact path still needs them.
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
    unsigned t = blockIdx.x * (JX_WG / 64) + (threadIdx.x >> 6);
    if (t >= ntiles) return;                       /* whole wave */
    WaveLds &W = s_wave[threadIdx.x >> 6];
    Queue Q{0, 0};
    uint32_t raw[8][6];
#if JX_PREFETCH
    {
        const unsigned b = tile_block(t, lane, total), f = b / nb;
        load_block(g, f, b - f * nb, raw);
    }
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
#elif JX_PREFETCH == 0
        {
            const unsigned f = b / nb;
            load_block(g, f, b - f * nb, raw);
        }
#endif
        int myslot = -1;
        Pending P{0u, 0, 0, 0};
        float T[8][8];
        xform_rows<0>(raw, T);
        xform_cols<0>(T, raw, a, W, Q, myslot, P, active, b, t, lane);
        __builtin_amdgcn_sched_barrier(0);
        xform_rows<1>(raw, T);
        xform_cols<1>(T, raw, a, W, Q, myslot, P, active, b, t, lane);
        __builtin_amdgcn_sched_barrier(0);
        xform_rows<2>(raw, T);
#if JX_PREFETCH == 2
        static_assert(JX_DBG_NO_EXACT, "late prefetch overwrites pixels the exact path needs");
        if (tn < ntiles) {                          /* raw is dead: refill it for tile tn */
            const unsigned bn = tile_block(tn, lane, total), fn = bn / nb;
            load_block(g, fn, bn - fn * nb, raw);
        }
#endif
        xform_cols<2>(T, raw, a, W, Q, myslot, P, active, b, t, lane);
        __builtin_amdgcn_sched_barrier(0);
        if (!JX_DBG_NO_EXACT) {
            /* exact work that did not fit during the tile, then drain a nearly full queue */
            if (__ballot(P.bits != 0)) settle_pending(W, Q, myslot, raw, b, P, g, a.quality, lane);
            if (Q.nslot > kSlots - 4 || Q.nitem > kItems - 16)
                drain(W, Q, myslot, g, a.quality, lane);
        }
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
    if (Q.nitem) flush_queue(W, Q.nitem, g, a.quality, lane);
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
        g_tab_rc[dev] = hip_rc(hipMemcpyToSymbol(HIP_SYMBOL(g_qtab), host.data(),
                                                 host.size() * sizeof(jx_qtab)));
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

}  // namespace

extern "C" {

size_t jpgx_workspace_size(const jpgx_frames *fr)
{
    (void)fr;
    return 0;   /* the exact-fixup queue lives in LDS; no device workspace is needed */
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
    (void)d_workspace;
    if (!fr || !p) return JPGX_EARG;
    int rc = jpgx_validate(fr->width, fr->height, p);
    if (rc) return rc;
    if (fr->row_begin < 0 || fr->row_end > fr->height / 8 || fr->row_begin > fr->row_end ||
        fr->nframes < 1)
        return JPGX_EARG;
    if (fr->row_begin == fr->row_end) return JPGX_OK;
    if (!d_rgb || !d_out) return JPGX_EARG;
    if (fr->in_pitch < (size_t)fr->width * 3 || fr->in_pitch % 8 || fr->in_frame_stride % 8 ||
        ((uintptr_t)d_rgb & 7) || ((uintptr_t)d_out & 15) || fr->out_frame_stride % 8)
        return JPGX_EARG;
    const int bpr = fr->width / 8;
    const size_t nb = (size_t)(fr->row_end - fr->row_begin) * bpr;
    const size_t total = nb * fr->nframes;
    if (total + 64 >= (1ull << 32)) return JPGX_EARG;
    if (fr->nframes > 1 && fr->out_frame_stride < 3 * nb * 64) return JPGX_EARG;
    if (fr->nframes > 1 && fr->in_frame_stride < fr->in_pitch * (size_t)(fr->row_end - fr->row_begin) * 8)
        return JPGX_EARG;
    if (workspace_bytes < jpgx_workspace_size(fr)) return JPGX_EWORKSPACE;

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
    const size_t ntiles = (total + 63) / 64;
    const size_t waves = std::min<size_t>(ntiles, (size_t)std::max(resident_waves(), 4));
    const unsigned grid = (unsigned)((waves + JX_WG / 64 - 1) / (JX_WG / 64));
    hipLaunchKernelGGL(k_xform, dim3(grid), dim3(JX_WG), 0, s, xa);
    rc = hip_rc(hipGetLastError());
    if (rc) return rc;
    if (event_after) rc = hip_rc(hipEventRecord((hipEvent_t)event_after, s));
    return rc;
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
 * stripe's three channel ranges into the whole-image [3][nb][64] host output. */
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
    jpgx_frames fr;
    memset(&fr, 0, sizeof fr);
    fr.width = width;
    fr.height = height;
    fr.row_begin = r0;
    fr.row_end = r1;
    fr.nframes = 1;
    fr.in_pitch = dpitch;
    fr.in_frame_stride = dpitch * rows;
    fr.out_frame_stride = 3 * nb_s * 64;
    uint8_t *d_in = nullptr;
    int16_t *d_out = nullptr;
    hipStream_t s = nullptr;
    int rc = JPGX_OK;
    if (hipMalloc(&d_in, rows * dpitch) != hipSuccess ||
        hipMalloc(&d_out, 3 * nb_s * 64 * sizeof(int16_t)) != hipSuccess ||
        hipStreamCreate(&s) != hipSuccess) {
        rc = JPGX_EHIP;
    }
    if (!rc) {
        const uint8_t *src = rgb + ((size_t)r0 * 8 - halo) * pitch;
        rc = hip_rc(hipMemcpy2DAsync(d_in, dpitch, src, pitch, row_bytes, rows,
                                     hipMemcpyHostToDevice, s));
    }
    if (!rc) rc = jpgx_blocks_gpu(&fr, p, d_in + halo * dpitch, d_out, nullptr, 0, s);
    for (int ch = 0; ch < 3 && !rc; ch++)
        rc = hip_rc(hipMemcpyAsync(out + ((size_t)ch * nb + (size_t)r0 * bpr) * 64,
                                   d_out + (size_t)ch * nb_s * 64, nb_s * 64 * sizeof(int16_t),
                                   hipMemcpyDeviceToHost, s));
    if (!rc) rc = hip_rc(hipStreamSynchronize(s));
    if (s) (void)hipStreamDestroy(s);
    (void)hipFree(d_in);
    (void)hipFree(d_out);
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
    for (int k = 0; k < ngpus; k++) {
        th.emplace_back([&, k]() {
            int r0, r1;
            jpgx_stripe(height / 8, ngpus, k, &r0, &r1);
            rcs[k] = run_stripe(rgb, width, height, pitch, p, out, k, r0, r1);
        });
    }
    for (auto &t : th) t.join();
    for (int k = 0; k < ngpus; k++)
        if (rcs[k]) return rcs[k];
    return JPGX_OK;
}

}  /* extern "C" */
