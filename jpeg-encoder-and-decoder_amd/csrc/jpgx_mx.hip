/*
 * jpgx_mx.hip -- k_mx, the gfx950 block-transform kernel with the colour conversion and the
 * row DCT on the matrix cores (v_mfma_f32_32x32x16_f16), the column DCT, quantiser, guard
 * band and zig-zag in VALU.
 *
 * Reference path: preprocess.c:160-162,186-188 (colour + level shift) -> dct.c:36-59 ->
 * quantise.c:52-72 (transposed divisor, round()) -> zig_zag.c:48-58; output = the three
 * JpgData.zig_zag_* arrays, [frame][Y|Cb|Cr][nb][64] int16.
 *
 * Mapping.  A wave takes a "pair-group" of 8 consecutive blocks of one frame, as two MFMA
 * groups of 4 blocks.  MFMA row m (0..31) of a group is pixel row y of block blk with
 * m = 8i + 4hh + j -> blk = 2hh + (i >> 1), y = 4(i & 1) + j, so that in the 32x32 result
 * (column n on the lane, rows (r & 3) + 8(r >> 2) + 4(lane >> 5) in register r) lane half h
 * holds all eight pixel rows of blocks 2h and 2h+1 for its column n = 8c + u:
 *     A[m][k]  = b_k - 128 of the pixel row (k = 3x + p; exact in f16), k = 24 the bias 1.0
 *     B[k][n]  = a[c][p] cos((2x+1)u pi/16), B[24][n] = the level-shift bias (jpgx_plan.cpp)
 *     R[m][n]  = (A Bh) + 2^-12 fl(A Bl + A Bm) (acc_h exact: jpgx_plan.cpp explains why;
 *                                                the lo parts are stored scaled by 2^12)
 * i.e. the colour-converted, level-shifted row transform of all three channels in 6 MFMAs
 * per 4 blocks.  Each lane then runs the column DCT (jx_fdct8, the FOps code the guard band
 * is derived from) of its column for two blocks, quantises with the per-lane (c,u) scales,
 * tests the guard band (v_cmp into an SGPR mask), and writes each int16 to the wave's LDS
 * stage at its zig-zag position.  The 8 blocks x 3 channels x 128 B leave as three 1-KiB
 * nontemporal stores (64 lanes x 16 B, contiguous per channel).
 *
 * Exactness (as k_xform): coefficients inside the rigorous guard band
 * (jx_plan_tables_mx) are recorded per block-channel as 64-bit masks, turned into tasks in
 * an LDS queue after the pair-group's stores, and recomputed in the reference's fp64
 * operation order (8 lanes per coefficient: lane x forms (X(x,y) c_u[x]) c_v[y] for y = 0..7,
 * the 64-term sum runs x-outer / y-inner through the 8 lanes in turn) when the queue fills
 * and at the end of the wave's work.
 */
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <mutex>
#include <vector>

#include "jpgx_internal.h"
#include "jx_consts.h"
#include "xform_math.h"

#pragma clang fp contract(off)

namespace {

typedef _Float16 mx_h8 __attribute__((ext_vector_type(8)));
typedef _Float16 mx_h2 __attribute__((ext_vector_type(2)));
typedef float mx_f16 __attribute__((ext_vector_type(16)));
typedef uint32_t mx_u4 __attribute__((ext_vector_type(4)));
typedef uint32_t mx_u2 __attribute__((ext_vector_type(2)));
typedef float mx_f2 __attribute__((ext_vector_type(2)));

constexpr float kMagic = 12582912.0f;   /* 1.5 * 2^23 */
constexpr int kMxCap = 256;             /* exact tasks queued per wave                     */
#ifndef JX_MX_DBG_NORARE         /* measurement only: no exact pass (NOT bit-exact) */
#define JX_MX_DBG_NORARE 0
#endif
#ifndef JX_MX_RARE               /* inlining of the rare paths (exact pass, flag masks)  */
#define JX_MX_RARE __forceinline__
#endif
#ifndef JX_MX_DBG_NODRAIN        /* measurement only: band test, no exact pass (NOT bit-exact) */
#define JX_MX_DBG_NODRAIN 0
#endif
#ifndef JX_MX_DRAIN              /* the exact pass: out of line (its registers would
                                    otherwise count against the tile loop's)            */
#define JX_MX_DRAIN __forceinline__
#endif
#ifndef JX_MX_WPE
#define JX_MX_WPE 3                     /* waves per SIMD the register allocation targets  */
#endif

__device__ jx_mxtab g_mxtab[JX_MAXQ + 1];
__device__ mx_u4 g_mxB[6][64];          /* B operands: (part, kstep) x lane, 8 f16 each     */
__device__ uint32_t g_mxzo[64][8];      /* LDS stage offset of (lane, v): column n = 8c + u,
                                           lane half h (blocks 2h, 2h + 1)                 */
__constant__ double kMxCos[8][8] = JX_COS_INIT;
__constant__ int kMxScan[8][8] = JX_SCAN_ORDER_INIT;
constexpr double kMxAlpha0 = JX_ALPHA0;

struct MxLds {
    uint8_t stage[4096];                /* [c][8 blocks][64] int16; c = 3: unused columns  */
    uint32_t tblk[kMxCap];              /* queued tasks: launch-global block               */
    uint16_t tcode[kMxCap];             /*               ch << 6 | v << 3 | u              */
};

/* four pixel bytes -> two f16 (b - 128): bytes as 0x64bb = 1024 + b, minus 1152 (exact) */
__device__ __forceinline__ mx_h2 mx_bytes2(uint32_t d, uint32_t sel)
{
    const uint32_t v = __builtin_amdgcn_perm(0x64646464u, d, sel);
    return __builtin_bit_cast(mx_h2, v) - (mx_h2){(_Float16)1152.0f, (_Float16)1152.0f};
}

__device__ __forceinline__ mx_h8 mx_cvt8(mx_u2 b)
{
    const mx_h2 p0 = mx_bytes2(b.x, 0x04010400u), p1 = mx_bytes2(b.x, 0x04030402u);
    const mx_h2 p2 = mx_bytes2(b.y, 0x04010400u), p3 = mx_bytes2(b.y, 0x04030402u);
    return (mx_h8){p0[0], p0[1], p1[0], p1[1], p2[0], p2[1], p3[0], p3[1]};
}

__device__ __forceinline__ void mx_wave_sync()
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ int mx_rank(uint64_t m)
{
    return (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                          __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

/* The launch geometry as plain values (kernel-argument fields copied out: references into
 * the argument struct, or indexed reads of its arrays, make the compiler copy it to scratch) */
struct MxG {
    const uint8_t *rgb;
    int16_t *out;
    long long pitch, fstride, ofstride;
    unsigned bpr, nb;
    int row0, quality;
    uint32_t u0, u1, u2, u3, u4, u5;   /* the underflow pixel row (jx_geom.under) */
};

__device__ __forceinline__ MxG mx_geom(const jx_xform_args &a)
{
    MxG G;
    G.rgb = a.g.rgb;
    G.out = a.g.out;
    G.pitch = a.g.in_pitch;
    G.fstride = a.g.in_fstride;
    G.ofstride = a.g.out_fstride;
    G.bpr = (unsigned)a.g.bpr;
    G.nb = (unsigned)a.g.nb;
    G.row0 = a.g.row0;
    G.quality = a.quality;
    G.u0 = a.g.under[0];
    G.u1 = a.g.under[1];
    G.u2 = a.g.under[2];
    G.u3 = a.g.under[3];
    G.u4 = a.g.under[4];
    G.u5 = a.g.under[5];
    return G;
}

/*
 * Pixel row pointer of block (frame f, row r, column c), pixel row y, with the reference's
 * addressing: blockToCoords (preprocess.c:199-211) gives x0 = -8 for the last block of a
 * block-row, i.e. pixel row 8r+y-1, columns W-8..W-1; at frame block-row 0, y = 0 those are
 * the bytes in front of the planes (g.under; *under = true, the pointer is then unused).
 */
__device__ __forceinline__ const uint8_t *mx_row(MxG g, unsigned f, unsigned r,
                                                 unsigned c, unsigned y, bool *under)
{
    const bool last = c == g.bpr - 1u;
    *under = last && y == 0 && g.row0 + (int)r == 0;
    const long long pr = 8ll * r + y - (last ? 1 : 0);
    return g.rgb + (long long)f * g.fstride + (*under ? 0 : pr * g.pitch) + 24ll * c;
}

/*
 * Exact pass over the wave's queued tasks (after its stores: s_waitcnt vmcnt(0)), 8 at a
 * time, 8 lanes each: lane x of task i forms the products (X(x,y) c_u[x]) c_v[y], y = 0..7
 * (dct.c:48-50, exact_pixel in double), and the sum runs x-outer / y-inner (dct.c:46-47)
 * through lanes x = 0..7 in turn; then F = ((1/4 a(u)) a(v)) s (dct.c:54) and round(F / Q)
 * with the transposed divisor (quantise.c:58).
 */
__device__ JX_MX_DRAIN void mx_drain(MxLds &L, int nq, MxG g, unsigned lane)
{
    const jx_mxtab &T = g_mxtab[g.quality];
    const unsigned i = lane >> 3, x = lane & 7u;
    uint32_t(*px)[8][6] = reinterpret_cast<uint32_t(*)[8][6]>(L.stage);  /* [task][row][dword] */
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    mx_wave_sync();
    for (int t0 = 0; t0 < nq; t0 += 8) {
        const int t = t0 + (int)i;
        const bool live = t < nq;
        const unsigned blk = L.tblk[live ? t : t0];
        const unsigned code = L.tcode[live ? t : t0];
        const int ch = (int)(code >> 6), v = (int)((code >> 3) & 7u), u = (int)(code & 7u);
        const unsigned nb = g.nb, f = blk / nb, bi = blk - f * nb;
        const unsigned r = bi / g.bpr, c = bi - r * g.bpr;
        {   /* lane x of task i stages pixel row x of the task's block */
            bool under;
            const uint8_t *p = mx_row(g, f, r, c, x, &under);
            const mx_u2 *pw = (const mx_u2 *)__builtin_assume_aligned(p, 8);
            const mx_u2 d0 = pw[0], d1 = pw[1], d2 = pw[2];
            px[i][x][0] = under ? g.u0 : d0.x;
            px[i][x][1] = under ? g.u1 : d0.y;
            px[i][x][2] = under ? g.u2 : d1.x;
            px[i][x][3] = under ? g.u3 : d1.y;
            px[i][x][4] = under ? g.u4 : d2.x;
            px[i][x][5] = under ? g.u5 : d2.y;
        }
        mx_wave_sync();
        /* lane x: the 8 products of pixel column x */
        const int k0 = (int)(3 * x) >> 2, sh = (int)(3 * x) & 3, k1 = k0 + 1 < 6 ? k0 + 1 : 5;
        const double cu = kMxCos[u][x];
        /* mx_exact_pixel with the channel's constants selected once: t = (k0 r + k1 g) + k2 b
         * (the signs of the reference's subtractions folded into k1, k2: a - b*k == a + b*(-k)
         * exactly), then (A + S t) - 128 with (A, S) = (0, 1) Y, (128, -1) Cb, (128, 1) Cr */
        const double k0c = ch == 0 ? 0.299 : (ch == 1 ? 0.168736 : 0.5);
        const double k1c = ch == 0 ? 0.587 : (ch == 1 ? -0.331264 : -0.418688);
        const double k2c = ch == 0 ? 0.114 : (ch == 1 ? 0.5 : -0.081312);
        const double Ac = ch == 0 ? 0.0 : 128.0, Sc = ch == 1 ? -1.0 : 1.0;
        double prod[8];
#pragma unroll
        for (int y = 0; y < 8; y++) {
            const uint64_t w = (uint64_t)px[i][y][k0] | ((uint64_t)px[i][y][k1] << 32);
            const uint32_t p3 = (uint32_t)(w >> (8 * sh));
            const double rr = (double)(p3 & 0xffu), gg = (double)((p3 >> 8) & 0xffu),
                         bb = (double)((p3 >> 16) & 0xffu);
            const double t = (k0c * rr + k1c * gg) + k2c * bb;
            const double X = (Ac + Sc * t) - 128.0;
            prod[y] = X * cu * kMxCos[v][y];
        }
        double s = 0.0;
#pragma unroll
        for (int xx = 0; xx < 8; xx++) {
            if ((int)x == xx) {
#pragma unroll
                for (int y = 0; y < 8; y++) s += prod[y];
            }
            s = __shfl(s, (int)((lane & ~7u) | (unsigned)xx), 64);
        }
        if (live && x == 0) {
            const double F = 0.25 * (u == 0 ? kMxAlpha0 : 1.0) * (v == 0 ? kMxAlpha0 : 1.0) * s;
            const int q = T.q[ch == 0 ? 0 : 1][u * 8 + v];
            g.out[(long long)f * g.ofstride + ((long long)ch * nb + bi) * 64 + kMxScan[v][u]] =
                (int16_t)(int)round(F / (double)q);
        }
        mx_wave_sync();                                    /* px reused by the next chunk */
    }
}

/* The pair-group's flagged coefficients as per-lane task bits: lane t < 24 <-> block
 * bl = t / 3 of the pair-group, channel c = t % 3, bit 8v + u for coefficient (u, v).
 * L.seenv[q][v] holds the lanes (h, n = 8c + u) of group q that flagged row v in either of
 * their two blocks 2h, 2h + 1: both blocks get the task. */
__device__ __forceinline__ uint64_t mx_task_bits(const uint64_t *seenv, unsigned lane,
                                                 unsigned seenq, unsigned nvalid)
{
    uint64_t M = 0;
    const unsigned bl = lane / 3u, c = lane - 3u * bl, q = bl >> 2, hh = (bl >> 1) & 1u;
    if (lane < 24 && bl < nvalid && ((seenq >> q) & 1u)) {
#pragma unroll
        for (int v = 0; v < 8; v++)
            M |= ((seenv[8 * q + v] >> (32u * hh + 8u * c)) & 0xffull) << (8 * v);
    }
    return M;
}

/* Move task bits M (blocks blk0 + lane / 3) into the LDS queue while it has room; the bits
 * that did not fit stay in M.  Returns the new queue length. */
__device__ __forceinline__ int mx_enqueue(MxLds &L, int nq, uint64_t &M, unsigned blk0,
                                          unsigned lane)
{
    const unsigned bl = lane / 3u, c = lane - 3u * bl;
    for (;;) {
        const uint64_t act = __ballot(M != 0);
        if (!act || nq == kMxCap) break;
        const int room = kMxCap - nq, rk = mx_rank(act);
        if (M != 0 && rk < room) {
            const int k = __builtin_ctzll(M);
            M &= M - 1;
            L.tblk[nq + rk] = blk0 + bl;
            L.tcode[nq + rk] = (uint16_t)(c << 6 | k);
        }
        nq += std::min((int)__popcll(act), room);
    }
    return nq;
}

/* Rows of one 4-block group through the matrix cores.  Register r of the 32x32 result holds
 * block 2h + (r & 1), pixel row r >> 1 of column n = lane & 31 (the A-row mapping in k_mx),
 * so R[y] = (block 2h, block 2h + 1) at pixel row y is an aligned register pair. */
__device__ __forceinline__ void mx_rows(mx_h8 A0, mx_h8 A1, const mx_h8 (&B)[6], mx_f2 (&R)[8])
{
    mx_f16 ah = {}, al = {};
    ah = __builtin_amdgcn_mfma_f32_32x32x16_f16(A0, B[0], ah, 0, 0, 0);
    ah = __builtin_amdgcn_mfma_f32_32x32x16_f16(A1, B[1], ah, 0, 0, 0);
    al = __builtin_amdgcn_mfma_f32_32x32x16_f16(A0, B[2], al, 0, 0, 0);
    al = __builtin_amdgcn_mfma_f32_32x32x16_f16(A1, B[3], al, 0, 0, 0);
    al = __builtin_amdgcn_mfma_f32_32x32x16_f16(A0, B[4], al, 0, 0, 0);
    al = __builtin_amdgcn_mfma_f32_32x32x16_f16(A1, B[5], al, 0, 0, 0);
#pragma unroll
    for (int y = 0; y < 8; y++)
        R[y] = __builtin_elementwise_fma(mx_f2{al[2 * y], al[2 * y + 1]},
                                         mx_f2{0x1p-12f, 0x1p-12f},
                                         mx_f2{ah[2 * y], ah[2 * y + 1]});
}

/* v_pk_*_f32 pairs: two blocks' columns in lock-step, lane by lane the FOps sequence */
struct MxPair {
    typedef mx_f2 V;
    static __device__ __forceinline__ V mk(float a, float b) { return V{a, b}; }
    static __device__ __forceinline__ float lo(V a) { return a.x; }
    static __device__ __forceinline__ float hi(V a) { return a.y; }
    static __device__ __forceinline__ V add(V a, V b) { return a + b; }
    static __device__ __forceinline__ V sub(V a, V b) { return a - b; }
    static __device__ __forceinline__ V mul(V a, V b) { return a * b; }
    static __device__ __forceinline__ V fma(V a, V b, V c) { return __builtin_elementwise_fma(a, b, c); }
};

__global__ __launch_bounds__(256, JX_MX_WPE) void k_mx(const jx_xform_args a)
{
    __shared__ MxLds s_lds[4];
    const MxG g = mx_geom(a);
    const unsigned lane = threadIdx.x & 63u;
    MxLds &L = s_lds[threadIdx.x >> 6];
    const unsigned nb = g.nb, bpr = g.bpr;
    const unsigned pgf = (nb + 7u) / 8u, npg = pgf * (unsigned)a.g.nframes;
    const bool force = a.force_exact != 0;
    /* each wave walks a contiguous range of pair-groups (incremental addressing, no division
     * per pair-group) */
    const unsigned nw = gridDim.x * 4u;
    const unsigned wv = __builtin_amdgcn_readfirstlane(blockIdx.x * 4u + (threadIdx.x >> 6));
    const unsigned pg_end = (unsigned)(((unsigned long long)npg * (wv + 1)) / nw);
    unsigned pg = (unsigned)(((unsigned long long)npg * wv) / nw);
    if (pg >= pg_end) return;
    /* position of pair-group pg: frame f, pair-group pgi in it, first block b0 = (r0, c0) */
    unsigned f = pg / pgf, pgi = pg - f * pgf;
    unsigned r0 = (8u * pgi) / bpr, c0 = 8u * pgi - r0 * bpr;

    /* A-operand row of this lane (both groups): register r = (m & 3) + 4 (m >> 3) of lane
     * half (m >> 2) & 1 of the result is block 2((m >> 2) & 1) + (r & 1), pixel row r >> 1 */
    const unsigned h = lane >> 5, m = lane & 31u;
    const unsigned rA = (m & 3u) + 4u * (m >> 3);
    const unsigned blkA = 2u * ((m >> 2) & 1u) + (rA & 1u), yA = rA >> 1;
    const long long laneoff = (long long)yA * g.pitch + 24 * blkA;   /* within the group */
    const unsigned n = lane & 31u;
    const unsigned last_b = nb - 1u, last_r = last_b / bpr, last_c = last_b - last_r * bpr;
    const uint32_t ua0 = h ? g.u2 : g.u0, ua1 = h ? g.u3 : g.u1;

    /* The lane's 8-byte loads (bytes 8h.., and 16..23) of both groups of the pair-group at
     * (F, R0, C0, B0).  Pair-groups inside one block-row, clear of its last block, take one
     * add per load; the others (row wrap, the x0 = -8 quirk, underflow, frame tail) the
     * general per-lane path. */
    mx_u2 LdA[2][2], LdB[2][2];
#define MX_LOAD(Ld, F, R0, C0, B0)                                                          \
    do {                                                                                    \
        if ((C0) + 8u < bpr) {                                                              \
            const uint8_t *base = g.rgb + (long long)(F) * g.fstride +                      \
                                  (long long)(8u * (R0)) * g.pitch + 24ll * (C0) + laneoff; \
            _Pragma("unroll") for (int q = 0; q < 2; q++) {                                 \
                const mx_u2 *pw = (const mx_u2 *)__builtin_assume_aligned(base + 96 * q, 8); \
                (Ld)[q][0] = pw[h];                                                         \
                (Ld)[q][1] = pw[2];                                                         \
            }                                                                               \
        } else {                                                                            \
            _Pragma("unroll") for (int q = 0; q < 2; q++) {                                 \
                const unsigned off = 4u * (unsigned)q + blkA;                               \
                unsigned c = (C0) + off, r = (R0);                                          \
                while (c >= bpr) {                                                          \
                    c -= bpr;                                                               \
                    r++;                                                                    \
                }                                                                           \
                const bool tail = (B0) + off > last_b;                                      \
                r = tail ? last_r : r;                                                      \
                c = tail ? last_c : c;                                                      \
                bool un;                                                                    \
                const uint8_t *p8 = mx_row(g, (F), r, c, yA, &un);                          \
                const mx_u2 *pw = (const mx_u2 *)__builtin_assume_aligned(p8, 8);           \
                const mx_u2 l0 = pw[h], l1 = pw[2];                                         \
                (Ld)[q][0] = un ? mx_u2{ua0, ua1} : l0;                                     \
                (Ld)[q][1] = un ? mx_u2{g.u4, g.u5} : l1;                                   \
            }                                                                               \
        }                                                                                   \
    } while (0)

    /* flagged pair-groups: record k of this wave at slot pg_begin + k of the workspace
     * (rec_pg = pair-group | seenq << 30, rec_sv = its 16 lane masks), exact pass after the
     * tile loop, where none of its values are live */
    const unsigned pg_begin = pg;
    unsigned nrec = 0;
    const jx_mxtab &T = g_mxtab[g.quality];
    float w[8], lim[8];
    uint32_t zo[8];
#pragma unroll
    for (int v = 0; v < 8; v++) {
        w[v] = T.w[n][v];
        lim[v] = force && n < 24 ? -1.0f : T.lim[n][v];
        zo[v] = g_mxzo[lane][v];
    }
    mx_h8 B[6];
#pragma unroll
    for (int i = 0; i < 6; i++) B[i] = __builtin_bit_cast(mx_h8, g_mxB[i][lane]);
    /* position of the pair-group after (F, P, R, C): scalar */
#define MX_NEXT(F, P, R, C, FN, PN, RN, CN)                                                 \
    do {                                                                                    \
        FN = F;                                                                             \
        PN = (P) + 1u;                                                                      \
        RN = R;                                                                             \
        CN = (C) + 8u;                                                                      \
        if (PN == pgf) {                                                                    \
            FN = (F) + 1u;                                                                  \
            PN = 0;                                                                         \
            RN = 0;                                                                         \
            CN = 0;                                                                         \
        } else {                                                                            \
            while (CN >= bpr) {                                                             \
                CN -= bpr;                                                                  \
                RN++;                                                                       \
            }                                                                               \
        }                                                                                   \
    } while (0)
    /* One pair-group from the pixels in LC; the pixels of pair-group pg + 2 are loaded into
     * LC as soon as its A operands are formed (two pair-groups in flight per wave). */
#define MX_STEP(LC)                                                                         \
    do {                                                                                    \
        unsigned f2_, p2_, r2_, c2_;                                                        \
        MX_NEXT(f1, p1, r1, c1, f2_, p2_, r2_, c2_);                                        \
        const mx_h8 bias = (mx_h8){(_Float16)1.0f, 0, 0, 0, 0, 0, 0, 0};                    \
        mx_h8 A[2][2];                                                                      \
        _Pragma("unroll") for (int q = 0; q < 2; q++) {                                     \
            A[q][0] = mx_cvt8(LC[q][0]);                                                    \
            A[q][1] = h ? bias : mx_cvt8(LC[q][1]);                                         \
        }                                                                                   \
        if (pg + 2u < pg_end) MX_LOAD(LC, f2_, r2_, c2_, 8u * p2_);                          \
        const unsigned b0 = 8u * pgi;                                                       \
        const unsigned slot = pg_begin + nrec;                                              \
        unsigned seenq = 0;                                                                 \
        _Pragma("unroll") for (int q = 0; q < 2; q++) {                                     \
            mx_f2 R[8], F[8];                                                               \
            mx_rows(A[q][0], A[q][1], B, R);                                                \
            jx_fdct8<PairOps<MxPair>>(R, F);                                                \
            uint64_t sv[8];                                                                 \
            _Pragma("unroll") for (int v = 0; v < 8; v++) {                                 \
                const mx_f2 wv2 = mx_f2{w[v], w[v]}, M2 = mx_f2{kMagic, kMagic};            \
                const mx_f2 tm = __builtin_elementwise_fma(F[v], wv2, M2);                  \
                const mx_f2 rr = tm - M2;                                                   \
                const mx_f2 d = __builtin_elementwise_fma(F[v], wv2, -rr);                  \
                /* blocks 2h and 2h + 1 of group q: stage offsets (4q + 2h + b) * 128 */    \
                *(uint16_t *)(L.stage + zo[v] + 512u * q) = (uint16_t)__float_as_uint(tm.x); \
                *(uint16_t *)(L.stage + zo[v] + 512u * q + 128u) =                          \
                    (uint16_t)__float_as_uint(tm.y);                                        \
                const float e = __builtin_fmaxf(__builtin_fabsf(d.x), __builtin_fabsf(d.y)); \
                sv[v] = __builtin_amdgcn_ballot_w64(e >= lim[v]);                           \
            }                                                                               \
            const uint64_t seen =                                                           \
                ((sv[0] | sv[1]) | (sv[2] | sv[3])) | ((sv[4] | sv[5]) | (sv[6] | sv[7]));  \
            if (!JX_MX_DBG_NORARE && seen) {   /* rare: record which lanes, per row v */    \
                seenq |= 1u << q;                                                           \
                if (lane == 0) {                                                            \
                    uint64_t *rs = a.rec_sv + (size_t)slot * 16 + 8 * q;                    \
                    _Pragma("unroll") for (int v = 0; v < 8; v++) rs[v] = sv[v];            \
                }                                                                           \
            }                                                                               \
        }                                                                                   \
        if (seenq) {                                                                        \
            if (lane == 0) a.rec_pg[slot] = pg | seenq << 30;                               \
            nrec++;                                                                         \
        }                                                                                   \
        mx_wave_sync();                                                                     \
        /* stores: channel c's 8 blocks x 128 B are contiguous, 16 B per lane */            \
        int16_t *ob = g.out + (long long)f * g.ofstride + (long long)b0 * 64 + lane * 8;    \
        const bool st = b0 + (lane >> 3) < nb;                                              \
        _Pragma("unroll") for (int c = 0; c < 3; c++) {                                     \
            const mx_u4 val = *(const mx_u4 *)(L.stage + c * 1024 + lane * 16);             \
            if (st) __builtin_nontemporal_store(val, (mx_u4 *)(ob + (long long)c * nb * 64)); \
        }                                                                                   \
        mx_wave_sync();                                                                     \
        f = f1; pgi = p1; r0 = r1; c0 = c1;                                                 \
        f1 = f2_; p1 = p2_; r1 = r2_; c1 = c2_;                                             \
        pg++;                                                                               \
    } while (0)

    unsigned f1, p1, r1, c1;                 /* position of pair-group pg + 1 */
    MX_NEXT(f, pgi, r0, c0, f1, p1, r1, c1);
    MX_LOAD(LdA, f, r0, c0, 8u * pgi);
    if (pg + 1u < pg_end) MX_LOAD(LdB, f1, r1, c1, 8u * p1);
    while (pg < pg_end) {
        MX_STEP(LdA);
        if (pg >= pg_end) break;
        MX_STEP(LdB);
    }
#undef MX_STEP
#undef MX_NEXT
    if (JX_MX_DBG_NODRAIN || !nrec) return;
    /* exact pass over the recorded pair-groups' flagged coefficients */
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    int nq = 0;
    for (unsigned k = 0; k < nrec; k++) {
        const unsigned rec = a.rec_pg[pg_begin + k];
        const unsigned p = rec & 0x3fffffffu, sq = rec >> 30;
        const unsigned fr = p / pgf, bb0 = 8u * (p - fr * pgf);
        uint64_t M = mx_task_bits(a.rec_sv + (size_t)(pg_begin + k) * 16, lane, sq,
                                  std::min(8u, nb - bb0));
        for (;;) {
            nq = mx_enqueue(L, nq, M, fr * nb + bb0, lane);
            if (__ballot(M != 0) == 0) break;
            mx_drain(L, nq, g, lane);
            nq = 0;
        }
    }
    if (nq) mx_drain(L, nq, g, lane);
#undef MX_LOAD
}

int mx_rc(hipError_t e) { return e == hipSuccess ? JPGX_OK : JPGX_EHIP; }

constexpr int kMaxDev = 64;
std::once_flag g_mx_once[kMaxDev];
int g_mx_rc[kMaxDev];
int g_mx_waves[kMaxDev];

int mx_tables_for_current_device(int *waves)
{
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDev) return JPGX_ENODEV;
    std::call_once(g_mx_once[dev], [dev]() {
        std::vector<jx_mxtab> tab(JX_MAXQ + 1);
        memset(tab.data(), 0, tab.size() * sizeof(jx_mxtab));
        int rc = JPGX_OK;
        for (int q = 1; q <= JX_MAXQ && !rc; q++) {
            rc = jx_plan_tables_mx(q, tab[q].w, tab[q].lim, tab[q].q);
            for (int n = 24; n < 32; n++)
                for (int v = 0; v < 8; v++) {
                    tab[q].w[n][v] = 0.0f;
                    tab[q].lim[n][v] = 3.0e38f;
                }
        }
        uint16_t ops[6][64][8];
        if (!rc) rc = jx_mx_operands(ops);
        static const int scan[8][8] = JX_SCAN_ORDER_INIT;
        uint32_t zo[64][8];
        for (int l = 0; l < 64; l++)
            for (int v = 0; v < 8; v++) {   /* columns 24..31 (padding) write to stage[3] */
                const int n = l & 31;
                zo[l][v] = (uint32_t)((n >> 3) * 1024 + 256 * (l >> 5) +
                                      2 * (n < 24 ? scan[v][n & 7] : v * 8 + (n & 7)));
            }
        if (!rc) rc = mx_rc(hipMemcpyToSymbol(HIP_SYMBOL(g_mxzo), zo, sizeof zo));
        if (!rc) rc = mx_rc(hipMemcpyToSymbol(HIP_SYMBOL(g_mxtab), tab.data(),
                                              tab.size() * sizeof(jx_mxtab)));
        if (!rc) rc = mx_rc(hipMemcpyToSymbol(HIP_SYMBOL(g_mxB), ops, sizeof ops));
        int cus = 0, per_cu = 0;
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
            cus = 256;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_mx, 256, 0) != hipSuccess ||
            per_cu < 1)
            per_cu = 2;
        g_mx_waves[dev] = cus * per_cu * 4;
        g_mx_rc[dev] = rc;
    });
    if (waves) *waves = g_mx_waves[dev];
    return g_mx_rc[dev];
}

}  // namespace

/* workspace bytes k_mx needs: a record slot per pair-group */
extern "C" size_t jx_mx_workspace(size_t nb, int nframes)
{
    const size_t npg = (nb + 7) / 8 * (size_t)nframes;
    return npg * (16 * sizeof(uint64_t) + sizeof(unsigned)) + 256;
}

/* k_mx over every frame of the stripe (4:4:4 / reference-parity output). */
extern "C" int jx_launch_mx(const jx_xform_args *xa_in, void *ws, size_t ws_bytes, void *stream)
{
    int waves = 0;
    const int rc = mx_tables_for_current_device(&waves);
    if (rc) return rc;
    jx_xform_args xa = *xa_in;
    const size_t nb = (size_t)xa.g.nb, npg = (nb + 7) / 8 * (size_t)xa.g.nframes;
    if (npg >= (1u << 30) || ws_bytes < jx_mx_workspace(nb, xa.g.nframes) || ((uintptr_t)ws & 15))
        return JPGX_EWORKSPACE;
    xa.rec_sv = (uint64_t *)ws;
    xa.rec_pg = (unsigned *)((uint8_t *)ws + npg * 16 * sizeof(uint64_t));
    const size_t w = std::min<size_t>(npg, (size_t)std::max(waves, 4));
    const unsigned grid = (unsigned)((w + 3) / 4);
    hipLaunchKernelGGL(k_mx, dim3(grid), dim3(256), 0, (hipStream_t)stream, xa);
    return mx_rc(hipGetLastError());
}
