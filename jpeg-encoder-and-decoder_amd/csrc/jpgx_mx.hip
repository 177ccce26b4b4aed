/*
 * jpgx_mx.hip -- k_mx, the gfx950 block-transform kernel with the colour conversion and the
 * row DCT on the matrix cores (v_mfma_f32_16x16x32_f16), the column DCT, quantiser, guard
 * band and zig-zag in packed fp32 VALU (v_pk_*_f32), and the exact-order fp64 pass for
 * guard-band coefficients inline, from the pixels already in LDS.
 *
 * Reference path: preprocess.c:160-162,186-188 (colour + level shift) -> dct.c:36-59 ->
 * quantise.c:52-72 (transposed divisor, round()) -> zig_zag.c:48-58; output = the three
 * JpgData.zig_zag_* arrays, [frame][Y|Cb|Cr][nb][64] int16.
 *
 * Work unit: a "step" of 8 consecutive blocks (launch-global block index, frames
 * concatenated).  The launched kernel (round 4) is k_mxs: short-lived waves, JX_MXS_C = 3
 * steps per wave, one workgroup of JX_MXS_WPG = 4 waves sharing an LDS image of the B operands
 * and tables; a wave issues the DMA of all its steps up front and exits after its third store.
 * k_mx (JX_MX_SHORT=0) is the round-3 persistent form: chunks of kChunk steps grid-stride
 * (mx_span_init), DMA two steps ahead in a 3-slot ring.
 *   Input   the step's 8 pixel rows x 8 blocks x 24 B land in a 1.5-KiB LDS slot ([y][24 jb + k])
 *           by LDS-DMA (16-byte pieces).
 *   Rows    set s (blocks 4s..4s+3), half h (pixel rows 4h..4h+3): a 16 x 32 f16 A operand,
 *           row m = 4 jb + y, k = byte k of the pixel row (zero-extended: the f16 b 2^-24,
 *           exact, one v_perm per two bytes; k = 24 the bias 1.0).  One product with B = colour x cosine gives, in C row m, column j, the
 *           row transform of channel j/8 (Y, Cb), frequency u = j%8.  Cr: the two sets
 *           concatenated along K (B zero outside its set's columns), so column j of the Cr tile
 *           is set j/8's Cr at u = j%8.  B = Bh + Bl (JX_MX_PARTS = 2 f16 parts; 3 adds a
 *           second lo part for a 1.28x narrower band at 50% more MFMAs, measured slower); acc_h =
 *           A Bh is EXACT in any summation order (jpgx_plan.cpp); R = acc_h + acc_l (JX_MX_LOEXP
 *           = 0: Bl encoded at Bh's scale, so the combine is one packed add).
 *   Columns every lane then holds three whole columns (8 rows, registers 0..3 of the two
 *           halves): (set 0, c = j/8, u), (set 1, same), (Cr, set j/8, u).  Each runs jx_fdct8_pk
 *           (lane by lane the FOps code the band is derived for), the quantiser tm = F w +
 *           1.5 2^23 (low 16 bits = the rounded int16) per v_pk_fma pair, the int16 to the LDS
 *           stage at its zig-zag position, and the band test d^2 - lsq >= 0 (d = F w - rint,
 *           exact) folded into a running max.
 *   Exact   (rare) a column whose max says "some coefficient in the band" records its flagged
 *           v's; k_mxs recomputes them in the step, from the pixels still in its LDS slot, into
 *           the stage before the store (mx_exact_inline); k_mx defers them to a per-wave side
 *           buffer (mx_defer / mx_flush).  Eight tasks at a time, eight lanes each: lane x forms
 *           (X(x,y) c_u[x]) c_v[y] in fp64, the sum runs x-outer / y-inner (dct.c:46-50) lane
 *           to lane over DPP, F = ((1/4 a(u)) a(v)) s, round(F / Q).
 *   Output  channel c's 8 blocks x 128 B leave as one 1-KiB nontemporal store.
 */
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <memory>
#include <mutex>
#include <type_traits>
#include <vector>

#include "jpgx_internal.h"
#include "jx_consts.h"
#include "xform_math.h"

#pragma clang fp contract(off)

namespace {

typedef _Float16 mx_h8 __attribute__((ext_vector_type(8)));
typedef _Float16 mx_h2 __attribute__((ext_vector_type(2)));
typedef float mx_f4 __attribute__((ext_vector_type(4)));
typedef float mx_f2 __attribute__((ext_vector_type(2)));
typedef uint32_t mx_u4 __attribute__((ext_vector_type(4)));
typedef uint32_t mx_u2 __attribute__((ext_vector_type(2)));

constexpr float kMagic = 12582912.0f;   /* 1.5 * 2^23: x + kMagic rounds x to an integer     */
constexpr int kParts = JX_MX_PARTS;     /* f16 parts of B: hi (exact products) + lo [+ lo2]  */
constexpr unsigned kSlot = 1536;        /* one step's pixels: [y][8 blocks x 24 B]           */
#ifndef JX_MX_DIST
#define JX_MX_DIST 2                    /* DMA issued this many steps ahead                  */
#endif
constexpr unsigned kDist = JX_MX_DIST;
constexpr unsigned kSteps = 3;          /* steps per chunk = LDS input slots (step k in slot k) */
/* s_waitcnt immediate for vmcnt(5 kDist - 2): the VMEM operations younger than a step's DMA
 * (kDist steps' 3 stores each, kDist - 1 steps' 2 DMA pieces each) */
constexpr unsigned kVmWait = 5 * kDist - 2;
constexpr int kWaitImm = (int)((kVmWait & 15u) | ((kVmWait >> 4) << 14) | 0xF70u);
static_assert(kVmWait < 64, "vmcnt is 6 bits");
#ifndef JX_MX_DYNLDS
#define JX_MX_DYNLDS 0                  /* timing experiments only: extra LDS per workgroup (lower occupancy) */
#endif
#ifndef JX_MX_WPE
#define JX_MX_WPE 4                     /* waves per SIMD the register allocation targets    */
#endif

/* LDS stage: 128 B per block in zig-zag order, 16 B of padding between blocks (kBS).  k_mx's
 * block (c, jb) sits at slot mx_pos(c, jb): Y 0..7, Cr 0..3 at 8..11, Cb at 12..19, Cr 4..7 at
 * 20..23 -- so that a lane's three columns, (c = j / 8, gq), (c = j / 8, 4 + gq) and (Cr,
 * 4 (j / 8) + gq), lie at one lane address plus 0, 4 and 8 slots (one set of address registers
 * with immediate offsets). */
constexpr unsigned kBS = 144;
__host__ __device__ constexpr unsigned mx_pos(unsigned c, unsigned jb)
{
    return c == 0 ? jb : (c == 1 ? 12u + jb : (jb < 4 ? 8u + jb : 16u + jb));
}
constexpr unsigned kStageBytes = 24 * kBS;
/* k_mxs's lean stage (JX_MXS_LEAN): Y 0..7, Cb 8..15; the Cr column is computed after the Y and
 * Cb stores and takes the set-0 slots of its lane (Cr 0..3 at 0..3, Cr 4..7 at 8..11) */
__host__ __device__ constexpr unsigned mx_pos_lean(unsigned c, unsigned jb)
{
    return c == 0 ? jb : (c == 1 ? 8u + jb : (jb < 4 ? jb : 4u + jb));
}

constexpr int kSide = 8;                /* deferred exact tasks per flush (8-lane groups)    */
constexpr int kSidePix = 6;             /* k_mx: deferred blocks' pixel slots per wave       */
struct alignas(16) MxLds {          /* 16-byte aligned: every wave's DMA slots and stage */
    uint8_t ring[kSteps][kSlot];
    uint8_t stage[kStageBytes];
    uint8_t pix[kSidePix][192];         /* deferred blocks' pixel rows, [y][24]              */
    uint32_t sblk[kSidePix];            /* and their launch-global block indices             */
    uint16_t dtask[kSide];              /* deferred columns: slot << 13 | c << 11 | u << 8 | v-mask */
    uint16_t task[8];                   /* inline batch: source lane << 8 | column << 3 | v  */
    uint32_t dummy[64];                 /* landing area of padding DMA operations            */
};
static_assert(kSlot % 16 == 0 && kStageBytes % 16 == 0 && sizeof(MxLds) % 16 == 0, "16-byte aligned LDS regions");
/* per-lane scales / band limits, shared by the workgroup: table t, half h (pairs 2h, 2h + 1 in
 * jx_pk_k order), profile j = lane & 15 -- a column's read of one (t, h) by the wave touches 16
 * consecutive 16-byte entries, every bank once.  k_mx: t = Wy|b, Ly|b (plan column j), Wr, Lr
 * (16 + j % 8); k_mx422: Wy, Ly (j % 8), Wc, Lc (8 + j). */
struct MxTab {
    mx_f4 wl[4][2][16];
};
static_assert(sizeof(MxLds) * 4 + sizeof(MxTab) <= 40 * 1024, "4 workgroups of 4 waves per CU");

__device__ mx_u4 g_mxB[3 * JX_MX_PARTS][64];     /* B operands: (part, which) x lane        */
__device__ jx_mxtab g_mxtab[2][JX_MAXQ + 1];     /* [force][quality]                        */
__constant__ double kMxCos[8][8] = JX_COS_INIT;
__constant__ int kMxScan[8][8] = JX_SCAN_ORDER_INIT;
/* ((0.25 a(u)) a(v)) of dct.c:54, 0.25 a(u) exact in a double */
__constant__ double kMxQuarterAlpha[8] = {0.25 * JX_ALPHA0, 0.25, 0.25, 0.25, 0.25, 0.25, 0.25, 0.25};
__constant__ double kMxAlpha[8] = {JX_ALPHA0, 1.0, 1.0, 1.0, 1.0, 1.0, 1.0, 1.0};
/* per channel the reference's colour constants as the exact pass uses them: t = (k0 r + k1 g)
 * + k2 b (the signs of its subtractions folded into k1, k2: a - b*k == a + b*(-k) exactly),
 * then (A + S t) - 128 with (A, S) = (0, 1) Y, (128, -1) Cb, (128, 1) Cr */
#define JX_MX_COLOUR_INIT                                                                          \
    {{0.299, 0.587, 0.114, 0.0, 1.0}, {0.168736, -0.331264, 0.5, 128.0, -1.0}, {0.5, -0.418688, -0.081312, 128.0, 1.0}}
__constant__ double kMxColour[3][5] = JX_MX_COLOUR_INIT;

/* Keep the compiler from moving this wave's LDS accesses across this point (a wave's LDS
 * instructions execute in program order; no fence: that would drain the memory counters). */
__device__ __forceinline__ void mx_wave_sync()
{
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");
}

__device__ __forceinline__ int mx_rank(uint64_t m)
{
    return (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                          __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

/* the lane id, opaque, for rare paths (lane-derived values are then not kept live) */
__device__ __forceinline__ unsigned mx_lane()
{
    unsigned l;
    asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
    return l;
}

/* Two pixel bytes -> two f16: one perm zero-extends each selected byte of d to 16 bits, the
 * f16 subnormal b 2^-24 (exact; jpgx_plan.cpp stores B's byte rows x 2^15, so the products are
 * b B 2^-9).  Selector byte 0x0c gives 0x00; for the bias lanes 0x05 picks 0x3C from K, i.e.
 * the f16 1.0 (0x3C00).  Data: 0x0c010c00 (bytes 0, 1) / 0x0c030c02 (2, 3); bias 1.0, 0.0:
 * 0x0c0c050c; zeros 0x0c0c0c0c. */
__device__ __forceinline__ uint32_t mx_cvt2(uint32_t d, uint32_t sel)
{
    return __builtin_amdgcn_perm(0x00003C00u, d, sel);
}
constexpr uint32_t kSelLo = 0x0c010c00u, kSelHi = 0x0c030c02u, kSelOne = 0x0c0c050cu, kSelZero = 0x0c0c0c0cu;
/* the MFMA results are R 2^-9 (jpgx_plan.cpp kMxBiasExp): the quantiser's w carries 2^9 */
constexpr float kRScale = 512.0f;

__device__ __forceinline__ mx_h8 mx_aop(mx_u2 d, uint32_t s0, uint32_t s1, uint32_t s2)
{
    const mx_u4 a = {mx_cvt2(d.x, s0), mx_cvt2(d.x, s1), mx_cvt2(d.y, s2), mx_cvt2(d.y, s1)};
    return __builtin_bit_cast(mx_h8, a);
}

__device__ __forceinline__ mx_f4 mx_mma(mx_h8 a, mx_u4 b, mx_f4 c)
{
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, __builtin_bit_cast(mx_h8, b), c, 0, 0, 0);
}

/* v_pk_*_f32 pairs for jx_fdct8_pk (lane by lane the scalar FOps operations) */
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

/* The launch geometry as plain values */
struct MxG {
    const uint8_t *rgb;
    int16_t *out;
    long long pitch, fstride, ofstride;
    unsigned bpr, nb, total;
    int row0, quality, force;
    bool lin_store;                     /* plane offsets fit the stores' 32-bit lane offsets */
    uint32_t u[6];                      /* the underflow pixel row (jx_geom.under) */
    jx_udiv dnb, dbpr;                  /* division by nb, by bpr (jx_geom) */
};

__device__ __forceinline__ unsigned mx_udiv(unsigned n, const jx_udiv &d)
{
    const unsigned t = __umulhi(d.m, n);
    return (t + ((n - t) >> d.s1)) >> d.s2;
}

/* A step's position: frame f, block bi in the frame, block-row r, column c, and running
 * pointers to its pixel (8c, 8r) and to its first block's channel-0 output. */
struct MxCur {
    unsigned f, bi, r, c;
    const uint8_t *src;
    int16_t *dst;
};

/* P's pixel and output pointers from its position */
__device__ __forceinline__ void mx_ptrs(MxCur &P, const MxG &g)
{
    P.src = g.rgb + (long long)P.f * g.fstride + 8ll * P.r * g.pitch + 24ll * P.c;
    P.dst = g.out + (long long)P.f * g.ofstride + 64ll * P.bi;
}

__device__ __forceinline__ void mx_seek(MxCur &P, const MxG &g, unsigned b0)
{
    P.f = mx_udiv(b0, g.dnb);
    P.bi = b0 - P.f * g.nb;
    P.r = mx_udiv(P.bi, g.dbpr);
    P.c = P.bi - P.r * g.bpr;
    mx_ptrs(P, g);
}

/* the step's 8 blocks lie in one block-row of one frame, none is the row's last block, all in
 * range: lane-linear source addresses */
__device__ __forceinline__ bool mx_simple_load(const MxCur &p, const MxG &g, unsigned b0)
{
    return p.c + 8u < g.bpr && b0 + 8u <= g.total;
}

/*
 * Which steps a wave computes: the launch's blocks cut into chunks of kChunk steps (32 blocks);
 * wave wv takes chunks wv, wv + nw, wv + 2 nw, ... (grid-stride), so the waves in flight stream
 * through one window of about nw chunks at a time -- neighbouring waves on neighbouring bytes.
 * All the bookkeeping is per chunk: its position (one division at the wave's start, then a
 * constant jump of 32 nw blocks), its base pointers, and whether all its steps are "simple"
 * (one block-row of one frame, not the row's last block, in range): then every step of it is
 * two LDS-DMA instructions and three stores off SGPR bases with loop-invariant lane offsets.
 * The rare other chunks (a row's last 32 blocks, frame / stripe / launch ends) take the general
 * per-step path.
 */
static_assert(kSteps == 3 && kDist == 2, "the ring holds one chunk: step k of a chunk in slot k");
constexpr unsigned kCB = 8 * kSteps;    /* blocks per chunk */
struct MxChunk {
    unsigned b0;                        /* first block (launch-global); >= total: none        */
    unsigned f, bi, r, c;               /* frame, block in frame, block-row, column of b0      */
    const uint8_t *src;                 /* pixel (8c, 8r) of frame f                           */
    int16_t *dst;                       /* frame f's channel-0 output of block bi              */
    int16_t *cdst;                      /* k_mx422: frame f's Cb output of chroma block bi / 2 */
    bool simple;
};
struct MxJump {
    unsigned jb, jr, jc, rows;          /* 32 nw blocks = jr block-rows + jc blocks; rows/frame */
};

/* CB = blocks per chunk (k_mx 32, k_mx422 24) */
template <unsigned CB>
__device__ __forceinline__ void mx_chunk_ptrs(MxChunk &C, const MxG &g)
{
    C.src = g.rgb + (long long)C.f * g.fstride + 8ll * C.r * g.pitch + 24ll * C.c;
    C.dst = g.out + (long long)C.f * g.ofstride + 64ll * C.bi;
    C.cdst = g.out + (long long)C.f * g.ofstride + 64ll * (g.nb + C.bi / 2u);
    C.simple = C.b0 + CB <= g.total && C.c + CB < g.bpr && g.lin_store;
}

template <unsigned CB>
__device__ __forceinline__ void mx_chunk_at(MxChunk &C, const MxG &g, unsigned b0)
{
    C.b0 = b0;
    C.f = b0 / g.nb;
    C.bi = b0 - C.f * g.nb;
    C.r = C.bi / g.bpr;
    C.c = C.bi - C.r * g.bpr;
    mx_chunk_ptrs<CB>(C, g);
}

/* the wave's next chunk, CB nw blocks on: no division */
template <unsigned CB>
__device__ __forceinline__ void mx_chunk_next(MxChunk &C, const MxG &g, const MxJump &J)
{
    C.b0 += J.jb;
    if (C.b0 >= g.total) return;
    C.bi += J.jb;
    C.c += J.jc;
    C.r += J.jr;
    if (C.c >= g.bpr) {
        C.c -= g.bpr;
        C.r++;
    }
    while (C.bi >= g.nb) {
        C.bi -= g.nb;
        C.r -= J.rows;
        C.f++;
    }
    mx_chunk_ptrs<CB>(C, g);
}

typedef __attribute__((address_space(3))) uint8_t lds_u8;
/* LDS pointer as the DMA builtin wants it */
typedef __attribute__((address_space(3))) void *mx_lp;
typedef const __attribute__((address_space(1))) void *mx_gp;

/*
 * The pixels of the step starting at block b0 (position P) into `slot` ([y][24 jb + k]).
 * Simple steps: two LDS-DMA instructions of 16-byte pieces (piece p = lane, and 64 + lane for
 * lanes < 32: row p / 12, bytes 16 (p % 12); the LDS destination of an LDS-DMA is base + 16 lane
 * for 12- and 16-byte pieces alike, so the slot is filled contiguously).  Other steps (a row's
 * last block, row or frame crossings, the launch's last step): lane l loads pixel row y = l & 7
 * of block jb = l >> 3 with the reference's addressing -- blockToCoords (preprocess.c:199-211)
 * gives x0 = -8 for the last block of a block-row, i.e. pixel row 8r + y - 1, columns W-8..W-1,
 * and at frame block-row 0, y = 0 those are the bytes in front of the planes (g.u) -- and
 * writes it to the slot itself; it waits for every outstanding VMEM operation (rare), so the
 * caller's vmcnt accounting, which counts two DMA operations per step, stays conservative.
 */
__device__ __forceinline__ void mx_issue(const MxG &g, const MxCur &P, unsigned b0, bool simple,
                                         uint32_t off0, uint32_t off1, uint8_t *slot)
{
    if (simple) {
        const uint8_t *base = P.src;
        __builtin_amdgcn_global_load_lds((mx_gp)(base + off0), (mx_lp)slot, 16, 0, 0);
        if (mx_lane() < 32)
            __builtin_amdgcn_global_load_lds((mx_gp)(base + off1), (mx_lp)(slot + 1024u), 16, 0, 0);
        return;
    }
    const unsigned lane = mx_lane(), y = lane & 7u, jb = lane >> 3;
    unsigned b = b0 + jb;
    b = b < g.total ? b : g.total - 1u;
    const unsigned f = b / g.nb, bi = b - f * g.nb;
    const unsigned r = bi / g.bpr, c = bi - r * g.bpr;
    const bool last = c == g.bpr - 1u;
    const bool under = last && y == 0 && g.row0 + (int)r == 0;
    const long long prow = under ? 8ll * r : 8ll * r + y - (last ? 1 : 0);
    typedef const __attribute__((address_space(1))) mx_u2 gu2;
    const gu2 *src = (const gu2 *)(g.rgb + (long long)f * g.fstride + prow * g.pitch + 24ll * c);
    mx_u2 v0 = src[0], v1 = src[1], v2 = src[2];
    if (under) {
        v0 = mx_u2{g.u[0], g.u[1]};
        v1 = mx_u2{g.u[2], g.u[3]};
        v2 = mx_u2{g.u[4], g.u[5]};
    }
    uint8_t *d = slot + 192u * y + 24u * jb;
    *(mx_u2 *)d = v0;
    *(mx_u2 *)(d + 8) = v1;
    *(mx_u2 *)(d + 16) = v2;
    __builtin_amdgcn_s_waitcnt(0xF70);                 /* vmcnt(0) (see above) */
}

/* s of lane x - 1 (DPP row shift by one; lane 0 of a 16-lane row gets 0) */
__device__ __forceinline__ double mx_shr1(double s)
{
    const uint64_t b = __builtin_bit_cast(uint64_t, s);
    const uint32_t lo = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)b, 0x111, 0xf, 0xf, false);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)(b >> 32), 0x111, 0xf, 0xf, false);
    return __builtin_bit_cast(double, (uint64_t)lo | ((uint64_t)hi << 32));
}

/* n padding VMEM operations (4-byte LDS-DMA of the input's first bytes into L.dummy): they keep
 * the number of VMEM operations per step constant, so that one vmcnt(8) always waits for exactly
 * the step's own DMA */
template <class Lds>
__device__ __forceinline__ void mx_pad(const MxG &g, Lds &L, int n)
{
    for (int i = 0; i < n; i++)
        __builtin_amdgcn_global_load_lds((mx_gp)g.rgb, (mx_lp)L.dummy, 4, 0, 0);
}

/*
 * One exact coefficient per 8-lane group (lane = 8 i + x), in the reference's operation order:
 * lane x forms X(x,y) in double colour arithmetic (preprocess.c:160-162,186-188) and the
 * products (X c_u[x]) c_v[y] (dct.c:48-50); the 64-term sum runs x-outer / y-inner
 * (dct.c:46-47) lane to lane; F = ((1/4 a(u)) a(v)) s (dct.c:54) and round(F / Q) with the
 * transposed divisor (quantise.c:58).  px = the block's pixel row 0, rows rs bytes apart.  The
 * result is valid in lane x == 7.
 */
/* s of lane (x ^ 1), (x ^ 2) or (7 - x) of an 8-lane group (DPP quad_perm / row_half_mirror) */
template <int CTRL>
__device__ __forceinline__ double mx_dpp64(double s)
{
    const uint64_t b = __builtin_bit_cast(uint64_t, s);
    const uint32_t lo = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)b, CTRL, 0xf, 0xf, false);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)(b >> 32), CTRL, 0xf, 0xf, false);
    return __builtin_bit_cast(double, (uint64_t)lo | ((uint64_t)hi << 32));
}

/*
 * The x-outer / y-inner sum of the products (lane x holds the 8 of its x), F and round(F / Q).
 *
 * Fast decision (round 5, JX_MX_FASTEXACT): the reference's 64-term sum runs sequentially
 * (dct.c:46-50), but only round(F / Q) is kept.  Each lane sums its 8 products in order, the 8
 * partial sums meet in a 3-level butterfly (every lane ends with the same total, a + b == b + a):
 * every term passes at most 10 additions.  Terms: |X| <= 171 (the Cb quirk, preprocess.c:161:
 * 128 - (0.168736 r - 0.331264 g + 0.5 b) spans [-170.6, 84.5]; Y, Cr and the 4:2:x averages stay
 * inside), |c| <= 1, so sum |t| <= 64 * 171 (1 + u)^2 <= 10944.01 (u = 2^-53).  Recursive
 * summation (Higham, Thm 4.4): |s_seq - s| <= g63 sum|t|, |s_par - s| <= g10 sum|t| (g_n = n u /
 * (1 - n u)), so |s_seq - s_par| <= 73.01 u 10944.01 < 8.9e-11.  The reference's t = fl(fl(K s) /
 * Q) (K = (1/4 a(u)) a(v) in (0, 0.25], Q >= 1, |t| <= 2736) and the fast t' = fl(s_par R), R =
 * fl(K / Q) from the table (jx_mxtab.r, R), differ by at most 0.25 * 8.9e-11 + 4.01 u 2736 < 2.4e-11.
 * So when t' is more than 2^-33 (1.16e-10) away from every half-integer (|t' - rint(t')| < 1/2 -
 * 2^-33; the difference is exact), no half-integer lies between t' and the reference's t, and
 * round(t) == rint(t').  Otherwise (near-ties: flat blocks, exact DC halves) the whole batch takes
 * the sequential sum -- wave-uniform, rare.
 * Valid in lane x == 7 (fast path: every lane).
 */
/* The inline exact pass ends with every LDS operation retired (JX_MX_EXEND_LGKM).  Round 5
 * (profiles/r05_exact_pass.txt): with the pass's tables in LDS -- no global read, hence no
 * vmcnt / lgkmcnt(0) wait anywhere in it -- a later step's Cr tile came out wrong in rows 12..15
 * in ~2 % of launches; an s_waitcnt vmcnt(0) at the pass's start did not help, lgkmcnt(0) at its
 * end did (0 of 80 launches + 8 golden frames). */
#ifndef JX_MX_EXSTART_VM
#define JX_MX_EXSTART_VM 0              /* diagnostics: vmcnt(0) before the pass */
#endif
#ifndef JX_MX_EXEND_LGKM
#define JX_MX_EXEND_LGKM 1
#endif
#ifndef JX_MX_FASTEXACT
#define JX_MX_FASTEXACT 1
#endif
template <bool FAST = (JX_MX_FASTEXACT != 0)>
__device__ __forceinline__ int mx_exact_sum(const double (&prod)[8], unsigned ch, unsigned u, unsigned v,
                                            unsigned x, const jx_mxtab &T, double R)
{
    if constexpr (FAST) {
        double p = prod[0];
#pragma unroll
        for (int y = 1; y < 8; y++) p += prod[y];
        p += mx_dpp64<0xB1>(p);                  /* quad_perm [1,0,3,2]: lane x ^ 1 */
        p += mx_dpp64<0x4E>(p);                  /* quad_perm [2,3,0,1]: lane x ^ 2 */
        p += mx_dpp64<0x141>(p);                 /* row_half_mirror: lane 7 - x      */
        const double t = p * R, r = __builtin_rint(t);
        if (__ballot(0.5 - __builtin_fabs(t - r) <= 0x1p-33) == 0) return (int)r;   /* t - r: exact */
    }
    double sum = 0.0;
#pragma unroll
    for (int xx = 0; xx < 8; xx++) {
        if ((int)x == xx) {
#pragma unroll
            for (int y = 0; y < 8; y++) sum += prod[y];
        }
        if (xx < 7) sum = mx_shr1(sum);
    }
    const double F = kMxQuarterAlpha[u] * kMxAlpha[v] * sum;
    const int q = T.q[ch == 0 ? 0 : 1][u * 8 + v];
    return (int)round(F / (double)q);
}

/* where the exact pass's constants come from: the __constant__ tables (MxExConst; k_mx, the
 * 4:2:x kernels) or the workgroup's LDS image and literals (MxExLds; k_mxs).  Round 5: a global
 * read in the exact pass waits, through the in-order vmcnt, for every older VMEM operation of the
 * wave -- the later steps' pixel DMA -- so it costs the wave microseconds under full HBM load. */
struct MxExConst {
    const jx_mxtab &T;
    __device__ double cosx(unsigned k, unsigned i) const { return kMxCos[k][i]; }
    __device__ double colour(unsigned ch, unsigned i) const { return kMxColour[ch][i]; }
    __device__ double recip(unsigned c, unsigned i) const { return T.r[c][i]; }
    __device__ unsigned scan(unsigned u, unsigned v) const { return (unsigned)kMxScan[v][u]; }
};
struct alignas(16) MxExTab {
    double cosx_[8][8];                 /* kMxCos                                    */
    int16_t q_[2][64];                  /* jx_mxtab.q of the workgroup's quality     */
};
struct MxExLds {
    const MxExTab &X;
    const uint8_t (&scan_t)[8][8];
    __device__ double cosx(unsigned k, unsigned i) const { return X.cosx_[k][i]; }
    /* kMxColour as literals (i is a compile-time constant at every use) */
    __device__ double colour(unsigned ch, unsigned i) const
    {
        const double y[5] = {0.299, 0.587, 0.114, 0.0, 1.0}, b[5] = {0.168736, -0.331264, 0.5, 128.0, -1.0},
                     r[5] = {0.5, -0.418688, -0.081312, 128.0, 1.0};
        return ch == 0 ? y[i] : (ch == 1 ? b[i] : r[i]);
    }
    /* jx_mxtab.r: fl(fl((1/4 a(u)) a(v)) / Q), the same IEEE operations as the host's */
    __device__ double recip(unsigned c, unsigned i) const
    {
        const double K = ((i >> 3) == 0 ? 0.25 * JX_ALPHA0 : 0.25) * ((i & 7u) == 0 ? JX_ALPHA0 : 1.0);
        return K / (double)X.q_[c][i];
    }
    __device__ unsigned scan(unsigned u, unsigned v) const { return scan_t[u][v]; }
};

template <class XT>
__device__ __forceinline__ int mx_exact_coef(const lds_u8 *px, unsigned rs, unsigned ch, unsigned u,
                                             unsigned v, unsigned x, const jx_mxtab &T, const XT &xt)
{
    const double cu = xt.cosx(u, x);
    const double k0c = xt.colour(ch, 0), k1c = xt.colour(ch, 1), k2c = xt.colour(ch, 2);
    const double Ac = xt.colour(ch, 3), Sc = xt.colour(ch, 4);
    double prod[8];
#pragma unroll
    for (int y = 0; y < 8; y++) {
        const lds_u8 *p = px + rs * (unsigned)y + 3u * x;
        const double rr = (double)p[0], gv = (double)p[1], bv = (double)p[2];
        const double tt = (k0c * rr + k1c * gv) + k2c * bv;
        const double X = (Ac + Sc * tt) - 128.0;
        prod[y] = X * cu * xt.cosx(v, y);
    }
    return mx_exact_sum(prod, ch, u, v, x, T, xt.recip(ch == 0 ? 0 : 1, u * 8 + v));
}

__device__ __forceinline__ lds_u8 *mx_lds(void *p) { return (lds_u8 *)p; }

/* the step's block jb and channel of a lane's column k (k_mx column layout) */
__device__ __forceinline__ unsigned mx_col_block(unsigned k, unsigned sl)
{
    const unsigned gg = sl >> 4, jj = sl & 15u;
    return k == 0 ? gg : (k == 1 ? 4u + gg : (jj < 8 ? gg : 4u + gg));
}

/* Inline exact pass of one step (a step with more tasks than the deferred queue holds, e.g.
 * FLAG_FORCE_EXACT): every flagged coefficient (bit 8 col + v of a lane's `bits`), eight at a
 * time, patching the stage. */
template <bool LEAN = false, class Lds, class XT>
__device__ __forceinline__ void mx_exact_inline(Lds &L, const uint8_t *slot, uint32_t bits,
                                                const jx_mxtab &T, const XT &xt)
{
    const unsigned lane = mx_lane();
#if JX_MX_EXSTART_VM
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
    mx_wave_sync();
    for (;;) {
        const uint64_t act = __ballot(bits != 0);
        if (!act) break;
        const int rk = mx_rank(act);
        if (bits != 0 && rk < 8) {
            const unsigned b = (unsigned)__builtin_ctz(bits);
            bits &= bits - 1u;
            L.task[rk] = (uint16_t)(lane << 8 | b);
        }
        mx_wave_sync();
        const int nt = std::min((int)__popcll(act), 8);
        const unsigned i = lane >> 3, x = lane & 7u;
        const bool live = (int)i < nt;
        const unsigned code = L.task[live ? i : 0u];
        const unsigned sl = code >> 8, k = (code >> 3) & 3u, v = code & 7u;
        const unsigned jj = sl & 15u, u = jj & 7u, ch = k < 2 ? (jj >> 3) : 2u;
        const unsigned jb = mx_col_block(k, sl);
        const int val = mx_exact_coef(mx_lds((void *)slot) + 24u * jb, 192u, ch, u, v, x, T, xt);
        if (live && x == 7)
            *(__attribute__((address_space(3))) int16_t *)(mx_lds(L.stage) +
                                                           kBS * (LEAN ? mx_pos_lean(ch, jb) : mx_pos(ch, jb)) +
                                                           2u * xt.scan(u, v)) = (int16_t)val;
        mx_wave_sync();
    }
#if JX_MX_EXEND_LGKM
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#endif
}

/* Deferred exact pass: up to kSide queued columns (pixels in L.pix), one per 8-lane group, each
 * group walking its column's flagged v's; results straight to global memory once the wave's
 * earlier stores (of those blocks) have landed. */
__device__ __forceinline__ void mx_flush(MxLds &L, int &nq, int &ns, const MxG &g, const jx_mxtab &T)
{
    __builtin_amdgcn_s_waitcnt(0xF70);                 /* vmcnt(0): the tasks' blocks are stored */
    mx_wave_sync();
    const unsigned lane = mx_lane(), i = lane >> 3, x = lane & 7u;
    const bool live = (int)i < nq;
    const unsigned code = L.dtask[live ? i : 0u];
    const unsigned slot = code >> 13, ch = (code >> 11) & 3u, u = (code >> 8) & 7u;
    uint32_t vb = live ? (code & 0xffu) : 0u;
    const unsigned b = L.sblk[slot], f = b / g.nb, bi = b - f * g.nb;
    int16_t *const dst = g.out + (long long)f * g.ofstride + ((long long)ch * g.nb + bi) * 64;
    while (__ballot(vb != 0)) {
        const bool act = vb != 0;
        const unsigned v = act ? (unsigned)__builtin_ctz(vb) : 0u;
        vb &= vb - 1u;
        const int val = mx_exact_coef(mx_lds(L.pix[slot]), 24u, ch, u, v, x, T, MxExConst{T});
        if (act && x == 7) dst[kMxScan[v][u]] = (int16_t)val;
    }
    mx_wave_sync();
    nq = 0;
    ns = 0;
}

/* A step with flagged coefficients (bit 8 col + v of `bits`): queue each flagged column (its
 * v-mask) with its block's pixels, flushing the queue first if it would overflow; a step with more
 * flagged columns or blocks than the queue holds is done inline.  Queue positions come from the
 * three column ballots (mbcnt), no prefix sum. */
__device__ __forceinline__ void mx_defer(MxLds &L, const uint8_t *sp, uint32_t bits, unsigned b0,
                                         int &nq, int &ns, const MxG &g, const jx_mxtab &T)
{
    const unsigned lane = mx_lane();
    /* a launch's last step fills its missing blocks with copies of the last block (mx_issue
     * clamps): their flags are dropped here, the copies are never stored, and the real last
     * block carries the same tasks */
    if (b0 + 8u > g.total) {
        const unsigned nvalid = g.total - b0;
#pragma unroll
        for (int k = 0; k < 3; k++)
            if (mx_col_block((unsigned)k, lane) >= nvalid) bits &= ~(0xffu << (8 * k));
    }
    /* flagged columns (per column kind) and blocks of the step */
    const uint64_t m0 = __ballot((bits & 0xffu) != 0), m1 = __ballot((bits & 0xff00u) != 0),
                   m2 = __ballot((bits & 0xff0000u) != 0);
    uint32_t blk = 0;
#pragma unroll
    for (int gq = 0; gq < 4; gq++) {
        blk |= (((m0 >> (16 * gq)) & 0xffffu) ? 1u : 0u) << gq;
        blk |= (((m1 >> (16 * gq)) & 0xffffu) ? 1u : 0u) << (4 + gq);
        blk |= (((m2 >> (16 * gq)) & 0xffu) ? 1u : 0u) << gq;
        blk |= (((m2 >> (16 * gq + 8)) & 0xffu) ? 1u : 0u) << (4 + gq);
    }
    const int n0 = __popcll(m0), n1 = __popcll(m1), ncol = n0 + n1 + __popcll(m2);
    const int nblk = __popc(blk);
    if (nq + ncol > kSide || ns + nblk > kSidePix) {
        if (nq) mx_flush(L, nq, ns, g, T);
        if (ncol > kSide || nblk > kSidePix) {
            mx_exact_inline(L, sp, bits, T, MxExConst{T});
            return;
        }
    }
    /* copy the flagged blocks' pixel rows to side slots ns.. (lane: row l / 6, dword l % 6) */
    {
        uint32_t bm = blk;
        int t = ns;
        while (bm) {
            const unsigned jb = (unsigned)__builtin_ctz(bm);
            bm &= bm - 1u;
            if (lane < 48) {
                const unsigned y = lane / 6u, k = lane - 6u * y;
                *(__attribute__((address_space(3))) uint32_t *)(mx_lds(L.pix[t]) + 24u * y + 4u * k) =
                    *(const __attribute__((address_space(3))) uint32_t *)(mx_lds((void *)sp) + 192u * y + 24u * jb + 4u * k);
            }
            if (lane == 0) L.sblk[t] = b0 + jb;
            t++;
        }
    }
    /* this lane's flagged columns: kind-0 columns first, then kind 1, then Cr */
    {
        const unsigned jj = lane & 15u, u = jj & 7u;
        const int base[3] = {nq, nq + n0, nq + n0 + n1};
        const uint64_t mk[3] = {m0, m1, m2};
#pragma unroll
        for (int k = 0; k < 3; k++) {
            const uint32_t vb = (bits >> (8 * k)) & 0xffu;
            if (vb) {
                const unsigned jb = mx_col_block((unsigned)k, lane), ch = k < 2 ? (jj >> 3) : 2u;
                const unsigned slot = (unsigned)ns + (unsigned)__popc(blk & ((1u << jb) - 1u));
                L.dtask[base[k] + mx_rank(mk[k])] = (uint16_t)(slot << 13 | ch << 11 | u << 8 | vb);
            }
        }
    }
    mx_wave_sync();
    nq += ncol;
    ns += nblk;
}

/* rare: the flagged v's of one column (the same arithmetic as mx_column_t) */
__device__ __forceinline__ uint32_t mx_flags(const mx_f2 (&F)[4], const mx_f2 (&W)[4], const mx_f2 (&Lq)[4])
{
    const mx_f2 M2 = {kMagic, kMagic};
    uint32_t m = 0;
#pragma unroll
    for (int p = 0; p < 4; p++) {
        const mx_f2 tm = __builtin_elementwise_fma(F[p], W[p], M2);
        const mx_f2 rr = tm - M2;
        const mx_f2 d = __builtin_elementwise_fma(F[p], W[p], -rr);
        const mx_f2 e = __builtin_elementwise_fma(d, d, -Lq[p]);
        m |= (e.x >= 0.0f ? 1u : 0u) << jx_pk_k(p, 0);
        m |= (e.y >= 0.0f ? 1u : 0u) << jx_pk_k(p, 1);
    }
    return m;
}

/* R pairs (y, y+1) of one column from the lo (rows 0..3) and hi (rows 4..7) tiles */
__device__ __forceinline__ void mx_combine(mx_f4 hl, mx_f4 ll, mx_f4 hh, mx_f4 lh, mx_f2 (&R)[4])
{
    if (JX_MX_LOEXP == 0) {                     /* lo parts at the hi scale: fl(acc_h + acc_l) */
        R[0] = mx_f2{ll.x, ll.y} + mx_f2{hl.x, hl.y};
        R[1] = mx_f2{ll.z, ll.w} + mx_f2{hl.z, hl.w};
        R[2] = mx_f2{lh.x, lh.y} + mx_f2{hh.x, hh.y};
        R[3] = mx_f2{lh.z, lh.w} + mx_f2{hh.z, hh.w};
        return;
    }
    const mx_f2 s = {0x1p-12f, 0x1p-12f};
    R[0] = __builtin_elementwise_fma(mx_f2{ll.x, ll.y}, s, mx_f2{hl.x, hl.y});
    R[1] = __builtin_elementwise_fma(mx_f2{ll.z, ll.w}, s, mx_f2{hl.z, hl.w});
    R[2] = __builtin_elementwise_fma(mx_f2{lh.x, lh.y}, s, mx_f2{hh.x, hh.y});
    R[3] = __builtin_elementwise_fma(mx_f2{lh.z, lh.w}, s, mx_f2{hh.z, hh.w});
}

/* a column's scales from the workgroup table; t0 = 0 (k_mx: Y|Cb, k_mx422/420: Y) or 2 (k_mx: Cr,
 * k_mx422/420: chroma); its squared band limits are table t0 + 1 */
struct MxW {
    mx_f4 w01, w23;
};
__device__ __forceinline__ MxW mx_w(const MxTab &tb, unsigned t0, unsigned j)
{
    return MxW{tb.wl[t0][0][j], tb.wl[t0][1][j]};
}
/* the squared band limits of a column (table t0 + 1): rare path only */
__device__ __forceinline__ MxW mx_l(const MxTab &tb, unsigned t0, unsigned j)
{
    return MxW{tb.wl[t0 + 1][0][j], tb.wl[t0 + 1][1][j]};
}
/* k_mxs with one-wave workgroups: the scales (tables 0 and 2) in the wave's LDS, the limits read
 * from the global image on the rare path */
struct MxsScales {
    mx_f4 w[2][2][16];
};
struct MxsTabRef {
    const MxsScales &s;
    const MxTab &g;
};
__device__ __forceinline__ MxW mx_w(const MxsTabRef &tb, unsigned t0, unsigned j)
{
    return MxW{tb.s.w[t0 >> 1][0][j], tb.s.w[t0 >> 1][1][j]};
}
__device__ __forceinline__ MxW mx_l(const MxsTabRef &tb, unsigned t0, unsigned j)
{
    return MxW{tb.g.wl[t0 + 1][0][j], tb.g.wl[t0 + 1][1][j]};
}
/* k_mxs's image table: MxTab with the Cr tables (2, 3) at 8 profiles -- a Cr column's profile is
 * j % 8 (lanes j and j + 8 read the same entry: an LDS broadcast) -- which frees the 512 bytes
 * per workgroup that the exact pass's tables take (MxExTab) */
struct MxsTab {
    mx_f4 yc[2][2][16];                 /* tables 0 (scales), 1 (squared limits): Y | Cb */
    mx_f4 cr[2][2][8];                  /* tables 2, 3: Cr                              */
};
__device__ __forceinline__ MxW mx_w(const MxsTab &tb, unsigned t0, unsigned j)
{
    return t0 == 0 ? MxW{tb.yc[0][0][j], tb.yc[0][1][j]} : MxW{tb.cr[0][0][j & 7u], tb.cr[0][1][j & 7u]};
}
__device__ __forceinline__ MxW mx_l(const MxsTab &tb, unsigned t0, unsigned j)
{
    return t0 == 0 ? MxW{tb.yc[1][0][j], tb.yc[1][1][j]} : MxW{tb.cr[1][0][j & 7u], tb.cr[1][1][j & 7u]};
}
struct MxsTabRefC {
    const MxsScales &s;
    const MxsTab &g;
};
__device__ __forceinline__ MxW mx_w(const MxsTabRefC &tb, unsigned t0, unsigned j)
{
    return MxW{tb.s.w[t0 >> 1][0][j], tb.s.w[t0 >> 1][1][j]};
}
__device__ __forceinline__ MxW mx_l(const MxsTabRefC &tb, unsigned t0, unsigned j)
{
    return mx_l(tb.g, t0, j);
}

/*
 * One limit per lane and column kind for the hot path's band test: a float <= the square root
 * of the smallest of the column's eight squared limits (-1 with FORCE_EXACT: every column takes
 * the rare path).  |d| >= limc is implied by d * d - lsq >= 0 for each of the eight, so testing
 * max |d| >= limc first and the per-coefficient limits only when it fires (mx_flags) flags
 * exactly the same coefficients with two fewer instructions per coefficient pair.
 */
__host__ __device__ __forceinline__ float mx_limc(const MxTab &tb, unsigned t, unsigned j)
{
    const mx_f4 a = tb.wl[t][0][j], b = tb.wl[t][1][j];
    const float mn = fminf(fminf(fminf(a.x, a.y), fminf(a.z, a.w)), fminf(fminf(b.x, b.y), fminf(b.z, b.w)));
    if (!(mn >= 0.0f)) return -1.0f;
    return (float)sqrt((double)mn) * (1.0f - 0x1p-20f);
}

/*
 * MFMA operand rule (tools/mfma_war_check.py, run by the CPU tests on the built ISA): no load may
 * write a VGPR that an issued MFMA may still read.  The register allocator treats an MFMA's
 * operands as dead once the MFMA is issued -- for a chained product whose destination differs
 * from its SrcC, the SrcC registers -- and may hand them to an LDS read a few instructions later,
 * whose data can land before the MFMA has read its last 16-lane group (C rows 12..15) when the
 * matrix pipe is backed up: nondeterministic wrong rows 12..15 (profiles/r03_mfma_war.txt).  So
 * every LDS read of a step (A operands, scale tables) is issued before the step's first MFMA,
 * behind a scheduling barrier; a load that must follow an MFMA (a rare-path limit read) first
 * waits for the newest MFMA's result (mx_fence: a VALU read of it, which the compiler's wait
 * states hold until the MFMA is done -- and with it every older one of this wave).
 */
__device__ __forceinline__ void mx_fence(const mx_f4 &r)
{
    const uint32_t v = __builtin_amdgcn_readfirstlane(__float_as_uint(r.w));
    asm volatile("" ::"s"(v) : "memory");
}

/* the same for a group of products the compiler may issue in any order: one VALU read of every
 * result (v_add3 + v_add), so the fence waits for the group's last product whichever it is */
template <int N>
__device__ __forceinline__ void mx_fence_all(const mx_f4 (&r)[N])
{
    uint32_t v = 0;
#pragma unroll
    for (int i = 0; i < N; i++) v += __float_as_uint(r[i].w);
    asm volatile("" ::"v"(v) : "memory");
}

/* Keep the C inputs of chained products live (so that no VALU instruction or load reuses their
 * registers) until the chain's results have been read (mx_fence).  Round 4: a VALU write into the
 * C input of a chained product 3 wait states after its issue -- what hipcc's hazard recognizer
 * pads for this form on gfx950 -- gave nondeterministic wrong C rows 12..15 (blocks 3 / 7 of a
 * step; profiles/r04_mfma_valu_war.txt).  tools/mfma_war_check.py --valu-srcc checks the rule. */
#ifndef JX_MX_KEEPC
#define JX_MX_KEEPC 1
#endif
/* diagnostics (JX_MX_GAP = N): N + 1 wait states after each group of products, before the VALU
 * work that follows it */
#ifndef JX_MX_GAP
#define JX_MX_GAP -1
#endif
/* diagnostics (JX_MX_DMABAR = 1): an s_barrier after a one-wave workgroup's step wait */
#ifndef JX_MX_DMABAR
#define JX_MX_DMABAR 0
#endif
__device__ __forceinline__ void mx_dmabar()
{
    if (JX_MX_DMABAR) __builtin_amdgcn_s_barrier();
}
__device__ __forceinline__ void mx_gap()
{
#if JX_MX_GAP >= 0
    asm volatile("s_nop %0" ::"n"(JX_MX_GAP));
#endif
}
__device__ __forceinline__ void mx_keep(const mx_f4 (&x)[4])
{
    if (JX_MX_KEEPC) asm volatile("" ::"v"(x[0]), "v"(x[1]), "v"(x[2]), "v"(x[3]));
}
/* the A / B operands of the products too (JX_MX_KEEPA): a product queued behind a chained one
 * reads its operands late, pass by pass */
#ifndef JX_MX_KEEPA
#define JX_MX_KEEPA 1
#endif
template <class T>
__device__ __forceinline__ int mx_keep1(const T &x)
{
    if (JX_MX_KEEPA) asm volatile("" ::"v"(x));
    return 0;
}
template <class... T>
__device__ __forceinline__ void mx_keep_ops(const T &...x)
{
    const int k[] = {mx_keep1(x)...};
    (void)k;
}

/* Column pass of one column (R pairs), quantiser, stage writes at za[v] + OFF, band flags (rare
 * path: the exact per-coefficient test with the limits of table t0 + 1, after mx_fence(*fence)
 * when an MFMA may be in flight) into fl */
template <unsigned OFF, class TB>
__device__ __forceinline__ void mx_column_r(const mx_f2 (&R)[4], const MxW &t, float limc, const TB &tb,
                                             unsigned t0, unsigned j, const uint32_t (&za)[8], uint32_t &fl, int kc,
                                             const mx_f4 *fence = nullptr)
{
    mx_f2 F[4];
    jx_fdct8_pk<MxPair>(R, F);
    const mx_f4 w01 = t.w01, w23 = t.w23;
    const mx_f2 W[4] = {mx_f2{w01.x, w01.y}, mx_f2{w01.z, w01.w}, mx_f2{w23.x, w23.y}, mx_f2{w23.z, w23.w}};
    const mx_f2 M2 = {kMagic, kMagic};
    typedef __attribute__((address_space(3))) uint16_t l16;
    float em = 0.0f;
#pragma unroll
    for (int p = 0; p < 4; p++) {
        const mx_f2 tm = __builtin_elementwise_fma(F[p], W[p], M2);
        *(l16 *)(uintptr_t)(za[jx_pk_k(p, 0)] + OFF) = (uint16_t)__float_as_uint(tm.x);
        *(l16 *)(uintptr_t)(za[jx_pk_k(p, 1)] + OFF) = (uint16_t)__float_as_uint(tm.y);
        const mx_f2 rr = tm - M2;
        const mx_f2 d = __builtin_elementwise_fma(F[p], W[p], -rr);
        em = __builtin_fmaxf(__builtin_fmaxf(em, __builtin_fabsf(d.x)), __builtin_fabsf(d.y));
    }
    if (__builtin_expect(__ballot(em >= limc) != 0, 0)) {
        if (fence) mx_fence(*fence);
        const MxW lw = mx_l(tb, t0, j);
        const mx_f4 l01 = lw.w01, l23 = lw.w23;
        const mx_f2 Lq[4] = {mx_f2{l01.x, l01.y}, mx_f2{l01.z, l01.w}, mx_f2{l23.x, l23.y}, mx_f2{l23.z, l23.w}};
        fl |= mx_flags(F, W, Lq) << (8 * kc);
    }
}

/* the same from the hi / lo accumulator tiles of rows 0..3 and 4..7; LAZY: the column's scales
 * are read here, after the tiles have been read (and after mx_fence(*fence) when a later MFMA may
 * still be in flight) -- no load meets an MFMA operand */
struct MxNoKeep {
    __device__ void operator()() const {}
};
template <unsigned OFF, bool LAZY = false, class TB, class KF = MxNoKeep>
__device__ __forceinline__ void mx_column_t(const mx_f4 (&acc)[4], const MxW &t, float limc, const TB &tb,
                                             unsigned t0, unsigned j, const uint32_t (&za)[8], uint32_t &fl, int kc,
                                             const mx_f4 *fence = nullptr, const KF &keep = KF{})
{
    mx_f2 R[4];
    mx_combine(acc[0], acc[1], acc[2], acc[3], R);
    if (LAZY) {
        __builtin_amdgcn_sched_barrier(0);
        if (fence) mx_fence(*fence);              /* a later MFMA may still be in flight */
        keep();                                   /* every product up to `fence` is done */
        mx_column_r<OFF>(R, mx_w(tb, t0, j), limc, tb, t0, j, za, fl, kc, nullptr);
    } else {
        keep();                                   /* the tiles are read: their chains are done */
        mx_column_r<OFF>(R, t, limc, tb, t0, j, za, fl, kc, fence);
    }
}

__global__ __launch_bounds__(256, JX_MX_WPE) void k_mx(const jx_xform_args a)
{
    __shared__ __attribute__((aligned(16))) MxLds s_lds[4];
    __shared__ __attribute__((aligned(16))) MxTab s_tab;
    MxG g;
    g.rgb = a.g.rgb;
    g.out = a.g.out;
    g.pitch = a.g.in_pitch;
    g.fstride = a.g.in_fstride;
    g.ofstride = a.g.out_fstride;
    g.bpr = (unsigned)a.g.bpr;
    g.nb = (unsigned)a.g.nb;
    g.total = (unsigned)a.g.nb * (unsigned)a.g.nframes;
    g.row0 = a.g.row0;
    g.quality = a.quality;
    g.force = a.force_exact;
    /* the stores' lane offsets (lane * 16 + plane * nb * 128 bytes) fit 32 bits */
    g.lin_store = (unsigned long long)g.nb * 256ull + 1024ull < (1ull << 31);
#pragma unroll
    for (int k = 0; k < 6; k++) g.u[k] = a.g.under[k];
    g.dnb = a.g.dnb;
    g.dbpr = a.g.dbpr;

    const unsigned lane = threadIdx.x & 63u;
    MxLds &L = s_lds[threadIdx.x >> 6];
    const jx_mxtab &T = g_mxtab[g.force ? 1 : 0][g.quality];
    /* the workgroup's scale / limit table: wave 0, lane (t = lane >> 4, profile j = lane & 15);
     * plan columns n = 8c + u: Y|Cb j, Cr 16 + j % 8 */
    if (threadIdx.x < 64) {
        const unsigned t = lane >> 4, jp = lane & 15u;
        const unsigned n = t < 2 ? jp : 16u + (jp & 7u);
        float x[8];
#pragma unroll
        for (int p = 0; p < 4; p++)
#pragma unroll
            for (int h = 0; h < 2; h++) {
                const int v = jx_pk_k(p, h);
                x[2 * p + h] = (t & 1u) ? T.lsq[n][v] : T.w[n][v];
            }
        s_tab.wl[t][0][jp] = mx_f4{x[0], x[1], x[2], x[3]};
        s_tab.wl[t][1][jp] = mx_f4{x[4], x[5], x[6], x[7]};
    }
    __syncthreads();
    /* hot-path band limits of this lane's two column kinds (mx_limc) */
    const float limc0 = mx_limc(s_tab, 1, threadIdx.x & 15u), limc2 = mx_limc(s_tab, 3, threadIdx.x & 15u);
    const unsigned nw = gridDim.x * 4u;
    const unsigned wv = __builtin_amdgcn_readfirstlane(blockIdx.x * 4u + (threadIdx.x >> 6));
    if (kCB * wv >= g.total) return;

    /* A operand of this lane: row m = lane & 15 (block m >> 2 of the set, pixel row m & 3 of the
     * half), k-group q = lane >> 4 (bytes 8q..8q+7; q = 3: the bias) */
    const unsigned m = lane & 15u, q = lane >> 4;
    const uint32_t aoff = 192u * (m & 3u) + 24u * (m >> 2) + 8u * (q < 3 ? q : 0u);
    const uint32_t s0 = q < 3 ? kSelLo : kSelOne;
    const uint32_t s1 = q < 3 ? kSelHi : kSelZero;
    const uint32_t s2 = q < 3 ? kSelLo : kSelZero;
    /* DMA pieces p = lane, 64 + lane: pixel row p / 12, bytes 16 (p % 12) of the step's row */
    const uint32_t off0 = (uint32_t)((lane / 12u) * (unsigned)g.pitch + 16u * (lane % 12u));
    const uint32_t off1 = (uint32_t)(((64u + lane) / 12u) * (unsigned)g.pitch + 16u * ((64u + lane) % 12u));
    /* stores: lane's 16 bytes of channel c's 8 blocks, as byte offsets from the step's block 0;
     * the stage reads at ro (Y), ro + 12 slots (Cb), rr (Cr: slots 8..11, 20..23) */
    const uint32_t so0 = lane * 16u, so1 = so0 + g.nb * 128u, so2 = so1 + g.nb * 128u;
    const uint32_t ro = (lane >> 3) * kBS + (lane & 7u) * 16u;
    const uint32_t rr = ro + ((lane >> 3) < 4 ? 8u : 16u) * kBS;

    /* C layout: lane (gq = lane >> 4, j = lane & 15) holds column j of rows 4 gq..4 gq + 3;
     * its three columns' coefficients go to za[v] + 0, 4 and 8 slots */
    const unsigned gq = lane >> 4, j = lane & 15u, u = j & 7u;
    uint32_t za[8];
    {
        const uint32_t base = (uint32_t)(uintptr_t)mx_lds(L.stage) + kBS * mx_pos(j >> 3, gq);
#pragma unroll
        for (int v = 0; v < 8; v++) za[v] = base + 2u * (unsigned)kMxScan[v][u];
    }
    mx_u4 B[kParts][3];
#pragma unroll
    for (int p = 0; p < kParts; p++)
#pragma unroll
        for (int w = 0; w < 3; w++) B[p][w] = g_mxB[3 * p + w][lane];
    __builtin_amdgcn_s_waitcnt(0xF70);              /* see k_mx422 */

    /* chunks: cc (computed now), nx (the next one; its first steps are issued during cc's last) */
    MxJump J;
    J.jb = kCB * nw;
    J.jr = J.jb / g.bpr;
    J.jc = J.jb - J.jr * g.bpr;
    J.rows = g.nb / g.bpr;
    MxChunk cc;
    mx_chunk_at<kCB>(cc, g, kCB * wv);
    MxChunk nx = cc;

    /* DMA of step k of chunk C into ring slot k (the slot the step computes from) */
    const auto issue = [&](const MxChunk &C, unsigned k) {
        uint8_t *const slot = L.ring[k];
        const unsigned b = C.b0 + 8u * k;
        if (b >= g.total) {
            mx_pad(g, L, 2);
        } else if (C.simple) {
            const uint8_t *base = C.src + 192u * k;
            __builtin_amdgcn_global_load_lds((mx_gp)(base + off0), (mx_lp)slot, 16, 0, 0);
            if (lane < 32) __builtin_amdgcn_global_load_lds((mx_gp)(base + off1), (mx_lp)(slot + 1024u), 16, 0, 0);
        } else {
            MxCur P;
            mx_seek(P, g, b);
            mx_issue(g, P, b, mx_simple_load(P, g, b), off0, off1, slot);
        }
    };
    /* prologue: the first kDist steps, each followed by three padding operations in place of the
     * stores of the (absent) steps before the first */
    for (unsigned d = 0; d < kDist; d++) {
        issue(cc, d);
        mx_pad(g, L, 3);
    }
    int nq = 0, ns = 0;                            /* deferred exact tasks, their blocks */
    unsigned k = 0;                                /* step of cc */
    for (;;) {
        const unsigned b0 = cc.b0 + 8u * k;
        /* VMEM operations younger than this step's DMA, in issue order: the three stores of each
         * of the kDist steps before it and the two DMA pieces of each of the kDist - 1 after it
         * (padding operations stand in for the ones that do not exist; a general step's loads
         * and the exact flush wait for themselves, which only makes this count conservative) */
        __builtin_amdgcn_s_waitcnt(kWaitImm);
        mx_wave_sync();
        const uint8_t *const sp = L.ring[k];
        /* the step kDist ahead: step k + kDist of this chunk, or of the next */
        if (k + kDist < kSteps) {
            issue(cc, k + kDist);
        } else {
            if (k + kDist == kSteps) mx_chunk_next<kCB>(nx, g, J);
            issue(nx, k + kDist - kSteps);
        }
        /* A operands: set 0/1 x half lo/hi */
        const mx_u2 d00 = *(const mx_u2 *)(sp + aoff);
        const mx_u2 d01 = *(const mx_u2 *)(sp + aoff + 768u);
        const mx_u2 d10 = *(const mx_u2 *)(sp + aoff + 96u);
        const mx_u2 d11 = *(const mx_u2 *)(sp + aoff + 864u);
        /* the step's scale reads too, before any MFMA (MFMA operand rule, mx_fence) */
        const MxW w0 = mx_w(s_tab, 0, j);
        const mx_h8 A00 = mx_aop(d00, s0, s1, s2), A01 = mx_aop(d01, s0, s1, s2);
        const mx_h8 A10 = mx_aop(d10, s0, s1, s2), A11 = mx_aop(d11, s0, s1, s2);
        __builtin_amdgcn_sched_barrier(0);
        const mx_f4 z = {};
        uint32_t fl = 0;                               /* bit 8 col + v: flagged (rare) */
        /* MFMAs one column ahead of the VALU work: MFMA(c0), MFMA(c1), VALU(c0), MFMA(c2),
         * VALU(c1), VALU(c2) -- an accumulator is read only after another column's products or
         * VALU work (no exposed MFMA latency, and far more than the MFMA -> VALU wait states the
         * hardware needs), with two columns' accumulators live at a time */
        mx_f4 acc[3][4];                               /* [column][hl, ll, hh, lh] */
        const auto mma_set = [&](mx_f4(&o)[4], const mx_h8 &Alo, const mx_h8 &Ahi) {
            o[0] = mx_mma(Alo, B[0][0], z);
            o[2] = mx_mma(Ahi, B[0][0], z);
#ifdef JX_MX_DBG_NOLO               /* timing experiments only: no lo-part MFMAs (NOT exact) */
            o[1] = z;
            o[3] = z;
#else
            o[1] = mx_mma(Alo, B[1][0], z);
            o[3] = mx_mma(Ahi, B[1][0], z);
#endif
            if (kParts == 3) {
                o[1] = mx_mma(Alo, B[kParts - 1][0], o[1]);
                o[3] = mx_mma(Ahi, B[kParts - 1][0], o[3]);
            }
        };
        mma_set(acc[0], A00, A01);
        __builtin_amdgcn_sched_barrier(0);
        mma_set(acc[1], A10, A11);
        __builtin_amdgcn_sched_barrier(0);
        mx_column_t<0>(acc[0], w0, limc0, s_tab, 0, j, za, fl, 0);
        __builtin_amdgcn_sched_barrier(0);
        acc[2][0] = mx_mma(A00, B[0][1], z);
        acc[2][2] = mx_mma(A01, B[0][1], z);
#ifdef JX_MX_DBG_NOLO
        acc[2][1] = z;
        acc[2][3] = z;
        acc[2][0] = mx_mma(A10, B[0][2], acc[2][0]);
        acc[2][2] = mx_mma(A11, B[0][2], acc[2][2]);
#else
        acc[2][1] = mx_mma(A00, B[1][1], z);
        acc[2][3] = mx_mma(A01, B[1][1], z);
        acc[2][0] = mx_mma(A10, B[0][2], acc[2][0]);
        acc[2][2] = mx_mma(A11, B[0][2], acc[2][2]);
        acc[2][1] = mx_mma(A10, B[1][2], acc[2][1]);
        acc[2][3] = mx_mma(A11, B[1][2], acc[2][3]);
#endif
        if (kParts == 3) {
            acc[2][1] = mx_mma(A00, B[kParts - 1][1], acc[2][1]);
            acc[2][3] = mx_mma(A01, B[kParts - 1][1], acc[2][3]);
            acc[2][1] = mx_mma(A10, B[kParts - 1][2], acc[2][1]);
            acc[2][3] = mx_mma(A11, B[kParts - 1][2], acc[2][3]);
        }
        __builtin_amdgcn_sched_barrier(0);
        mx_column_t<4 * kBS>(acc[1], w0, limc0, s_tab, 0, j, za, fl, 1, &acc[2][3]);
        __builtin_amdgcn_sched_barrier(0);
        /* Y and Cb leave before the Cr column when they carry no flags (+0.3 %, r03_valu_diet_ab) */
        const bool early = cc.simple && __ballot((fl & 0xffffu) != 0) == 0;
        if (early) {
            mx_fence(acc[2][3]);                       /* the Cr products are done (operand rule) */
            mx_wave_sync();
            const uint8_t *const ob = (const uint8_t *)(cc.dst + 512u * k);
            const mx_u4 v0 = *(const mx_u4 *)(L.stage + ro);
            const mx_u4 v1 = *(const mx_u4 *)(L.stage + 12u * kBS + ro);
            __builtin_nontemporal_store(v0, (mx_u4 *)(ob + so0));
            __builtin_nontemporal_store(v1, (mx_u4 *)(ob + so1));
        }
        __builtin_amdgcn_sched_barrier(0);
        mx_column_t<8 * kBS, true>(acc[2], w0, limc2, s_tab, 2, j, za, fl, 2);
        mx_wave_sync();
        if (__builtin_expect(__ballot(fl != 0) != 0, 0)) {
            mx_defer(L, sp, fl, b0, nq, ns, g, T);
            __builtin_amdgcn_s_waitcnt(0xF70);         /* see mx422_defer_step */
        }
        /* stores: channel c's 8 blocks x 128 B; always three store instructions (the vmcnt
         * accounting above counts on it) */
        if (early) {
            const uint8_t *const ob = (const uint8_t *)(cc.dst + 512u * k);
            const mx_u4 v2 = *(const mx_u4 *)(L.stage + rr);
            __builtin_nontemporal_store(v2, (mx_u4 *)(ob + so2));
        } else if (cc.simple) {
            const uint8_t *const ob = (const uint8_t *)(cc.dst + 512u * k);
            const mx_u4 v0 = *(const mx_u4 *)(L.stage + ro);
            const mx_u4 v1 = *(const mx_u4 *)(L.stage + 12u * kBS + ro);
            const mx_u4 v2 = *(const mx_u4 *)(L.stage + rr);
            __builtin_nontemporal_store(v0, (mx_u4 *)(ob + so0));
            __builtin_nontemporal_store(v1, (mx_u4 *)(ob + so1));
            __builtin_nontemporal_store(v2, (mx_u4 *)(ob + so2));
        } else {
            /* lanes past the launch's end (the clamped copies of the last block) store nothing;
             * block b0 is always in range, so each store instruction still issues (the vmcnt
             * accounting counts three per step) */
            const unsigned l = mx_lane();
            const unsigned bl = b0 + (l >> 3), b = bl < g.total ? bl : g.total - 1u;
            const unsigned f = b / g.nb, bi = b - f * g.nb;
#pragma unroll
            for (int c = 0; c < 3; c++) {
                const mx_u4 val = *(const mx_u4 *)(L.stage + kBS * mx_pos((unsigned)c, l >> 3) + (l & 7u) * 16u);
                if (bl < g.total)
                    __builtin_nontemporal_store(
                        val, (mx_u4 *)(g.out + (long long)f * g.ofstride +
                                       ((long long)c * g.nb + bi) * 64 + (l & 7u) * 8));
            }
        }
        mx_wave_sync();
        if (++k == kSteps) {
            k = 0;
            cc = nx;
            if (cc.b0 >= g.total) break;
        } else if (b0 + 8u >= g.total) {
            break;
        }
    }
    if (nq) mx_flush(L, nq, ns, g, T);
}

/* ==== k_mxs: k_mx's transform in short-lived waves (round 4) =================================
 *
 * The same per-step arithmetic as k_mx (MFMA rows, packed-VALU columns, band, zig-zag stage,
 * inline exact pass), but the launch is NOT persistent: wave w of the grid computes the C
 * consecutive steps w C .. w C + C - 1 (8 C blocks) and exits, so the hardware dispatcher hands
 * the chip one compact, advancing window of the batch (the persistent grid-stride layout drifts:
 * instruction arbitration favours older waves, profiles/r03_skeleton_wgrank.txt; the memory
 * skeleton reads 0.72-0.76 non-persistent vs 0.67-0.70 persistent, profiles/r04_*).  What a
 * short wave needs is a cheap start:
 *   - its pixel DMA for all C steps is issued first (no ring reuse: step k lives in slot k);
 *   - the B operands (6 KiB, quality-independent) and this quality's scale / limit table with
 *     the hot-path band limits (2.1 KiB) are one pre-laid-out image (g_mxs_img) that the
 *     workgroup's four waves copy into LDS with LDS-DMA (16-byte pieces), one s_barrier;
 *   - the exact pass runs inline per step on the stage (no cross-step queue, no side buffer).
 * vmcnt bookkeeping: every step issues exactly two DMA operations up front (padding operations
 * for general / absent steps) and three stores, so step k waits with vmcnt(2 (C - 1 - k) + 3 k).
 */
#ifndef JX_MXS_C
#define JX_MXS_C 3                      /* steps per wave */
#endif
constexpr unsigned kMxsC = JX_MXS_C;
static_assert(kMxsC >= 1, "k_mxs: at least one step per wave");
/* up to three steps: every step's DMA up front, step k in slot k; more: a ring of three slots,
 * DMA two steps ahead (k_mx's scheme), step k in slot k % 3 */
constexpr unsigned kMxsR = kMxsC < 3 ? kMxsC : 3;
constexpr bool kMxsRing = kMxsC > 3;

#ifndef JX_MXS_LEAN
#define JX_MXS_LEAN 0                   /* 1: 16-block stage (mx_pos_lean), Y / Cb stored before the Cr column */
#endif
constexpr bool kMxsLean = JX_MXS_LEAN != 0;
struct alignas(16) MxsLds {
    uint8_t ring[kMxsR][kSlot];         /* pixels, [y][24 jb + k]                       */
    uint8_t stage[(kMxsLean ? 16 : 24) * kBS];  /* zig-zag stage (mx_pos / mx_pos_lean)  */
    uint16_t task[8];                   /* inline exact batch                           */
};
static_assert(sizeof(MxsLds) % 16 == 0, "16-byte aligned LDS regions");
/* the workgroup image: B operands, scale / limit table, hot-path limits (mx_limc) per lane
 * profile and column kind */
#ifndef JX_MXS_BLDS
#define JX_MXS_BLDS 0                   /* 1: B operands read from the LDS image every step (fewer VGPRs) */
#endif
/* Round-5 experiment (profiles/r05_exact_pass.txt, code removed): B operands from global memory
 * (g_mxB) to make room for the exact tables gave wrong C rows 12..15 in 10-100 % of launches
 * (not root-caused); the room comes from the compact Cr tables (MxsTab) instead. */
struct alignas(16) MxsImg {
    mx_u4 B[3 * JX_MX_PARTS][64];
    MxsTab tab;
    float limc[2][16];
    uint8_t scan_t[8][8];               /* zig-zag position of (v, u) at [u][v] */
    MxExTab ex;                         /* the exact pass's tables                      */
};
constexpr unsigned kMxsPieces = sizeof(MxsImg) / 16;
static_assert(sizeof(MxsImg) % 16 == 0 && kMxsPieces <= 768, "three 16-byte pieces per thread");
__device__ MxsImg g_mxs_img[2][JX_MAXQ + 1];     /* [force][quality] */
/* waves per workgroup: 4 (the image above shared through one s_barrier) or 1 (each wave its own
 * small image -- the scales, hot-path limits and zig-zag positions -- and its B operands and band
 * limits from the global image: no barrier, and a finished wave frees its slot at once) */
#ifndef JX_MXS_WPG
#define JX_MXS_WPG 4
#endif
constexpr unsigned kMxsWPG = JX_MXS_WPG;
static_assert(kMxsWPG == 1 || kMxsWPG == 4 || kMxsWPG == 8, "k_mxs: 1, 4 or 8 waves per workgroup");
static_assert(kMxsWPG == 1 || sizeof(MxsLds) * kMxsWPG + sizeof(MxsImg) <= 160 * 1024 / (16 / kMxsWPG),
              "16 waves per CU");
struct alignas(16) MxsImg1 {
    MxsScales sc;
    float limc[2][16];
    uint8_t scan_t[8][8];
};
static_assert(sizeof(MxsImg1) % 16 == 0 && sizeof(MxsImg1) / 16 <= 128, "two 16-byte pieces per lane");
static_assert(kMxsWPG != 1 || (sizeof(MxsLds) + sizeof(MxsImg1) + 511) / 512 * 512 * 16 <= 160 * 1024,
              "16 one-wave workgroups per CU");
__device__ MxsImg1 g_mxs_img1[2][JX_MAXQ + 1];
using MxsShared = std::conditional<kMxsWPG == 1, MxsImg1, MxsImg>::type;
/* where the B operands and the column tables come from (four-wave image / one-wave image) */
typedef mx_u4 MxsBOps[3 * JX_MX_PARTS][64];
__device__ __forceinline__ const MxsBOps &mxs_B(const MxsImg &l, const MxsImg &) { return l.B; }
[[maybe_unused]] __device__ __forceinline__ const MxsBOps &mxs_B(const MxsImg1 &, const MxsImg &g) { return g.B; }
/* the exact pass's tables: the LDS image's copy (four-wave image), or the __constant__ tables */
__device__ __forceinline__ MxExLds mxs_xt(const MxsImg &l, const jx_mxtab &) { return MxExLds{l.ex, l.scan_t}; }
[[maybe_unused]] __device__ __forceinline__ MxExConst mxs_xt(const MxsImg1 &, const jx_mxtab &T) { return MxExConst{T}; }
__device__ __forceinline__ const MxsTab &mxs_tb(const MxsImg &l, const MxsImg &) { return l.tab; }
[[maybe_unused]] __device__ __forceinline__ MxsTabRefC mxs_tb(const MxsImg1 &l, const MxsImg &g) { return MxsTabRefC{l.sc, g.tab}; }
#ifdef JX_MXS_STAMP                    /* timing probe builds only: per-wave timestamps */
__device__ unsigned long long g_mxs_ts[1u << 20];
#define JX_MXS_TS(i, v) do { if (lane == 0 && 8u * wv + 8u <= (1u << 20)) g_mxs_ts[8u * wv + (i)] = (v); } while (0)
#else
#define JX_MXS_TS(i, v) do { } while (0)
#endif

template <unsigned N>
__device__ __forceinline__ void mx_wait_vm()
{
    static_assert(N < 64, "vmcnt is 6 bits");
    __builtin_amdgcn_s_waitcnt((int)((N & 15u) | ((N >> 4) << 14) | 0xF70u));
}

/* LDS-DMA of 16 (or 4) bytes per lane to lds_base + 16 (4) lane.  JX_MXS_ASMDMA issues it from
 * inline asm, which the compiler's wait-count pass does not see: then only k_mxs's own counted
 * vmcnt waits order it (with the builtin, the compiler drains vmcnt(0) before the next LDS read
 * of the wave, since it cannot tell which LDS bytes the DMA writes). */
#ifndef JX_MXS_ASMDMA
#define JX_MXS_ASMDMA 0
#endif
template <int SIZE>
__device__ __forceinline__ void mxs_dma(const void *g, void *lds)
{
    static_assert(SIZE == 16 || SIZE == 4, "dwordx4 or dword pieces");
#if JX_MXS_ASMDMA
    const uint32_t l = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)mx_lds(lds));
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"
    if (SIZE == 16)
        asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(g), "s"(l) : "memory", "m0");
    else
        asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dword %0, off" ::"v"(g), "s"(l) : "memory", "m0");
#pragma clang diagnostic pop
#else
    if constexpr (SIZE == 16)
        __builtin_amdgcn_global_load_lds((mx_gp)g, (mx_lp)lds, 16, 0, 0);
    else
        __builtin_amdgcn_global_load_lds((mx_gp)g, (mx_lp)lds, 4, 0, 0);
#endif
}

/* a step cursor (wave-uniform): launch-global first block, whether the step is simple (one
 * block-row of one frame, not the row's last block, in range: two LDS-DMA operations and three
 * stores off its pointers), its column, pixel (8c, 8r) and channel-0 output pointers */
struct MxsCur {
    unsigned b, c;
    bool simple;
    const uint8_t *src;
    int16_t *dst;
    int16_t *cdst;                      /* k_mxs422: its first chroma block's Cb output */
};

__device__ __forceinline__ void mxs_simple(MxsCur &P, const MxG &g)
{
    P.simple = P.c + 8u < g.bpr && P.b + 8u <= g.total && g.lin_store;
}

__device__ __forceinline__ void mxs_at(MxsCur &P, const MxG &g, unsigned b)
{
    P.b = b;
    P.simple = false;
    if (b >= g.total) return;
    MxCur X;
    mx_seek(X, g, b);
    P.c = X.c;
    P.src = X.src;
    P.dst = X.dst;
    P.cdst = g.out + (long long)X.f * g.ofstride + 64ll * (g.nb + X.bi / 2u);
    mxs_simple(P, g);
}

/* the next step: a simple step's successor is in the same block-row (no division) */
__device__ __forceinline__ void mxs_next(MxsCur &P, const MxG &g)
{
    if (!P.simple) {
        mxs_at(P, g, P.b + 8u);
        return;
    }
    P.b += 8u;
    P.c += 8u;
    P.src += 192;
    P.dst += 512;
    P.cdst += 256;
    mxs_simple(P, g);
}

/* two VMEM operations into `slot`: the step's pixels, or padding (a general step's slot is
 * filled through registers at compute time after a vmcnt(0); an absent step's is never read) */
__device__ __forceinline__ void mxs_issue(const MxsCur &P, const MxG &g, uint8_t *slot, uint32_t off0,
                                          uint32_t off1, unsigned lane)
{
    if (P.simple) {
        mxs_dma<16>(P.src + off0, slot);
        if (lane < 32) mxs_dma<16>(P.src + off1, slot + 1024u);
    } else {
        mxs_dma<4>(g.rgb, slot);
        mxs_dma<4>(g.rgb, slot);
    }
}

#ifdef JX_MXS_NUMVGPR
__attribute__((amdgpu_waves_per_eu(JX_MXS_NUMVGPR, JX_MXS_NUMVGPR)))
#endif
__global__ __launch_bounds__(64 * kMxsWPG, JX_MX_WPE) void k_mxs(const jx_xform_args a)
{
    __shared__ __attribute__((aligned(16))) MxsLds s_lds[kMxsWPG];
    __shared__ __attribute__((aligned(16))) MxsShared s_img;
    MxG g;
    g.rgb = a.g.rgb;
    g.out = a.g.out;
    g.pitch = a.g.in_pitch;
    g.fstride = a.g.in_fstride;
    g.ofstride = a.g.out_fstride;
    g.bpr = (unsigned)a.g.bpr;
    g.nb = (unsigned)a.g.nb;
    g.total = (unsigned)a.g.nb * (unsigned)a.g.nframes;
    g.row0 = a.g.row0;
    g.quality = a.quality;
    g.force = a.force_exact;
    g.lin_store = (unsigned long long)g.nb * 256ull + 1024ull < (1ull << 31);
#pragma unroll
    for (int k = 0; k < 6; k++) g.u[k] = a.g.under[k];
    g.dnb = a.g.dnb;
    g.dbpr = a.g.dbpr;

#ifdef JX_MXS_STAMP
    const unsigned long long ts0 = __builtin_amdgcn_s_memrealtime(), cs0 = __builtin_amdgcn_s_memtime();
#endif
    const unsigned lane = threadIdx.x & 63u;
    const unsigned wave = kMxsWPG == 1 ? 0u : __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    MxsLds &L = s_lds[wave];
    const MxsImg &gimg = g_mxs_img[g.force ? 1 : 0][g.quality];
    /* the image into LDS (LDS-DMA: piece p of thread t lands at 16 p) */
    if constexpr (kMxsWPG >= 2) {
        const uint8_t *img = (const uint8_t *)&gimg;
#pragma unroll
        for (unsigned i = 0; i < (kMxsPieces + 64u * kMxsWPG - 1u) / (64u * kMxsWPG); i++) {
            const unsigned piece = 64u * kMxsWPG * i + threadIdx.x;
            if (64u * kMxsWPG * i + 64u * wave < kMxsPieces && piece < kMxsPieces)
                mxs_dma<16>(img + 16u * piece, (uint8_t *)&s_img + 16u * (64u * kMxsWPG * i + 64u * wave));
        }
    } else {
        constexpr unsigned kP1 = sizeof(MxsImg1) / 16;
        const uint8_t *img = (const uint8_t *)&g_mxs_img1[g.force ? 1 : 0][g.quality];
        mxs_dma<16>(img + 16u * lane, &s_img);
        if (lane < kP1 - 64u) mxs_dma<16>(img + 16u * (64u + lane), (uint8_t *)&s_img + 1024u);
    }
    /* this wave's first steps' DMA (kMxsR of them; ring mode: two) */
    const unsigned wv = blockIdx.x * kMxsWPG + wave;
    const uint32_t off0 = (uint32_t)((lane / 12u) * (unsigned)g.pitch + 16u * (lane % 12u));
    const uint32_t off1 = (uint32_t)(((64u + lane) / 12u) * (unsigned)g.pitch + 16u * ((64u + lane) % 12u));
    MxsCur iss;                                  /* issue cursor */
    mxs_at(iss, g, 8u * kMxsC * wv);
    MxsCur cmp = iss;                            /* compute cursor */
    constexpr unsigned kPro = kMxsRing ? 2u : kMxsR;
#pragma unroll
    for (unsigned k = 0; k < kPro; k++) {
        mxs_issue(iss, g, L.ring[k], off0, off1, lane);
        mxs_next(iss, g);
    }

    /* lane constants (k_mx's) */
    const unsigned m = lane & 15u, q = lane >> 4;
    const uint32_t aoff = 192u * (m & 3u) + 24u * (m >> 2) + 8u * (q < 3 ? q : 0u);
    const uint32_t s0 = q < 3 ? kSelLo : kSelOne;
    const uint32_t s1 = q < 3 ? kSelHi : kSelZero;
    const uint32_t s2 = q < 3 ? kSelLo : kSelZero;
    const uint32_t so0 = lane * 16u, so1 = so0 + g.nb * 128u, so2 = so1 + g.nb * 128u;
    const uint32_t ro = (lane >> 3) * kBS + (lane & 7u) * 16u;
    const uint32_t rr = ro + (kMxsLean ? ((lane >> 3) < 4 ? 0u : 4u) : ((lane >> 3) < 4 ? 8u : 16u)) * kBS;
    const uint32_t rcb = (kMxsLean ? 8u : 12u) * kBS + ro;
    const unsigned gq = lane >> 4, j = lane & 15u, u = j & 7u;
    const jx_mxtab &T = g_mxtab[g.force ? 1 : 0][g.quality];
    const auto xt = mxs_xt(s_img, T);

    /* the image has landed (it is older than the prologue's pixel operations), in every wave */
    if constexpr (kMxsWPG == 1) {
        if (cmp.b >= g.total) return;
    }
    mx_wait_vm<2u * kPro>();
    if constexpr (kMxsWPG >= 2) __builtin_amdgcn_s_barrier();
    mx_wave_sync();
    if (cmp.b >= g.total) return;
    /* stage addresses of this lane's column at v = 0..7: the zig-zag positions from the image (no
     * global load: its wait would drain the pixel DMA too) */
    uint32_t za[8];
    {
        const uint32_t base =
            (uint32_t)(uintptr_t)mx_lds(L.stage) + kBS * (kMxsLean ? mx_pos_lean(j >> 3, gq) : mx_pos(j >> 3, gq));
        const mx_u2 sc = *(const mx_u2 *)&s_img.scan_t[u][0];
#pragma unroll
        for (int v = 0; v < 8; v++) za[v] = base + 2u * ((v < 4 ? sc.x : sc.y) >> (8 * (v & 3)) & 0xffu);
    }
#ifndef JX_MXS_UNCHAIN
#define JX_MXS_UNCHAIN 1                /* 1: the Cr tile from independent products (no chained MFMA) */
#endif
constexpr bool kMxsUnchain = JX_MXS_UNCHAIN != 0 && kParts == 2;
#ifndef JX_MXS_NOEXACT
#define JX_MXS_NOEXACT 0                /* timing probes only: skip the inline exact pass (NOT exact) */
#endif
#if !JX_MXS_BLDS
    mx_u4 B[kParts][3];
#pragma unroll
    for (int p = 0; p < kParts; p++)
#pragma unroll
        for (int w = 0; w < 3; w++) B[p][w] = mxs_B(s_img, gimg)[3 * p + w][lane];
#endif
    const float limc0 = s_img.limc[0][j], limc2 = s_img.limc[1][j];
    const auto &tb = mxs_tb(s_img, gimg);
#ifdef JX_MXS_STAMP
    {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
        JX_MXS_TS(0, ts0);
        JX_MXS_TS(1, t1);
        JX_MXS_TS(5, cs0);
        JX_MXS_TS(7, ((unsigned long long)__builtin_amdgcn_s_getreg((31 << 11) | 20) << 32) |
                         (unsigned)__builtin_amdgcn_s_getreg((31 << 11) | 4));
    }
#endif

    /* one step from `sp` (its DMA has landed): transform, inline exact pass, three stores */
    const auto body = [&](const MxsCur &S, uint8_t *sp) __attribute__((always_inline)) {
        if (!S.simple) {
            MxCur P;
            mx_seek(P, g, S.b);
            mx_issue(g, P, S.b, false, off0, off1, sp);      /* register path; waits vmcnt(0) */
        }
        mx_wave_sync();
#ifdef JX_MXS_NOCOMP                    /* timing probe only: the memory pattern without the transform */
        const uint8_t *const ob = (const uint8_t *)S.dst;
        const bool early = false;
        {
            const mx_u2 d = *(const mx_u2 *)(sp + aoff);
            *(__attribute__((address_space(3))) uint32_t *)(uintptr_t)za[0] = d.x ^ d.y;
            mx_wave_sync();
        }
#else
        const mx_u2 d00 = *(const mx_u2 *)(sp + aoff);
        const mx_u2 d01 = *(const mx_u2 *)(sp + aoff + 768u);
        const mx_u2 d10 = *(const mx_u2 *)(sp + aoff + 96u);
        const mx_u2 d11 = *(const mx_u2 *)(sp + aoff + 864u);
        const MxW w0 = mx_w(tb, 0, j);
#if JX_MXS_BLDS
        mx_u4 B[kParts][3];
#pragma unroll
        for (int p = 0; p < kParts; p++)
#pragma unroll
            for (int w = 0; w < 3; w++) B[p][w] = mxs_B(s_img, gimg)[3 * p + w][lane];
#endif
        const mx_h8 A00 = mx_aop(d00, s0, s1, s2), A01 = mx_aop(d01, s0, s1, s2);
        const mx_h8 A10 = mx_aop(d10, s0, s1, s2), A11 = mx_aop(d11, s0, s1, s2);
        __builtin_amdgcn_sched_barrier(0);
        const mx_f4 z = {};
        uint32_t fl = 0;
        mx_f4 acc[3][4];
        const auto mma_set = [&](mx_f4(&o)[4], const mx_h8 &Alo, const mx_h8 &Ahi) __attribute__((always_inline)) {
            o[0] = mx_mma(Alo, B[0][0], z);
            o[2] = mx_mma(Ahi, B[0][0], z);
            o[1] = mx_mma(Alo, B[1][0], z);
            o[3] = mx_mma(Ahi, B[1][0], z);
            if (kParts == 3) {
                o[1] = mx_mma(Alo, B[kParts - 1][0], o[1]);
                o[3] = mx_mma(Ahi, B[kParts - 1][0], o[3]);
            }
        };
        mma_set(acc[0], A00, A01);
        __builtin_amdgcn_sched_barrier(0);
        mma_set(acc[1], A10, A11);
        mx_gap();
        __builtin_amdgcn_sched_barrier(0);
        mx_column_t<0>(acc[0], w0, limc0, tb, 0, j, za, fl, 0);
        __builtin_amdgcn_sched_barrier(0);
        /* the Cr tile: the two sets' K halves.  Round 5 (kMxsUnchain): eight independent products
         * and one VALU add per element, cr[0] + cr[1] -- bit-identical to the chained form, since in
         * every column one of the two halves is an exact zero (B1 is zero in columns 8..15, B2 in
         * 0..7) -- so no product of k_mxs waits in the matrix pipe for another;
         * the products are issued in source order (cr[1][3] last: the fence) */
        mx_f4 cr[2][4];
        const mx_f4 c0 = mx_mma(A00, B[0][1], z);
        __builtin_amdgcn_sched_barrier(0);
        const mx_f4 c2 = mx_mma(A01, B[0][1], z);
        __builtin_amdgcn_sched_barrier(0);
        const mx_f4 c1 = mx_mma(A00, B[1][1], z);
        __builtin_amdgcn_sched_barrier(0);
        const mx_f4 c3 = mx_mma(A01, B[1][1], z);
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (kMxsUnchain) {
            cr[0][0] = c0;
            cr[0][1] = c1;
            cr[0][2] = c2;
            cr[0][3] = c3;
            cr[1][0] = mx_mma(A10, B[0][2], z);
            __builtin_amdgcn_sched_barrier(0);
            cr[1][2] = mx_mma(A11, B[0][2], z);
            __builtin_amdgcn_sched_barrier(0);
            cr[1][1] = mx_mma(A10, B[1][2], z);
            __builtin_amdgcn_sched_barrier(0);
            cr[1][3] = mx_mma(A11, B[1][2], z);
        } else {
            acc[2][0] = mx_mma(A10, B[0][2], c0);
            acc[2][2] = mx_mma(A11, B[0][2], c2);
            acc[2][1] = mx_mma(A10, B[1][2], c1);
            acc[2][3] = mx_mma(A11, B[1][2], c3);
            cr[1][3] = acc[2][3];
        }
        mx_gap();
        const auto keepc = [&]() __attribute__((always_inline)) {
            if constexpr (!kMxsUnchain) {
                const mx_f4 cc[4] = {c0, c1, c2, c3};
                mx_keep(cc);
                mx_keep_ops(A00, A01, A10, A11, B[0][1], B[1][1], B[0][2], B[1][2]);
            }
        };
        /* the Cr tile (unchained: its two halves' sum, every Cr product done after it) */
        const auto cr_tile = [&]() __attribute__((always_inline)) {
            if constexpr (kMxsUnchain) {
#pragma unroll
                for (int i = 0; i < 4; i++) acc[2][i] = cr[0][i] + cr[1][i];
            }
        };
        if (kParts == 3) {
            acc[2][1] = mx_mma(A00, B[kParts - 1][1], acc[2][1]);
            acc[2][3] = mx_mma(A01, B[kParts - 1][1], acc[2][3]);
            acc[2][1] = mx_mma(A10, B[kParts - 1][2], acc[2][1]);
            acc[2][3] = mx_mma(A11, B[kParts - 1][2], acc[2][3]);
        }
        __builtin_amdgcn_sched_barrier(0);
        mx_column_t<4 * kBS>(acc[1], w0, limc0, tb, 0, j, za, fl, 1, &cr[1][3]);
        __builtin_amdgcn_sched_barrier(0);
        const uint8_t *const ob = (const uint8_t *)S.dst;
        /* the launch's last step: flags of its clamped copies are dropped (never stored) */
        const auto clamp = [&](uint32_t &f) __attribute__((always_inline)) {
            if (S.b + 8u > g.total) {
                const unsigned nvalid = g.total - S.b;
#pragma unroll
                for (int kk = 0; kk < 3; kk++)
                    if (mx_col_block((unsigned)kk, lane) >= nvalid) f &= ~(0xffu << (8 * kk));
            }
        };
        const auto store = [&](int c) __attribute__((always_inline)) {    /* the general path's store c */
            const unsigned l = mx_lane();
            const unsigned bl = S.b + (l >> 3), b = bl < g.total ? bl : g.total - 1u;
            const unsigned f = b / g.nb, bi = b - f * g.nb;
            const unsigned pos = kMxsLean ? mx_pos_lean((unsigned)c, l >> 3) : mx_pos((unsigned)c, l >> 3);
            const mx_u4 val = *(const mx_u4 *)(L.stage + kBS * pos + (l & 7u) * 16u);
            if (bl < g.total)
                __builtin_nontemporal_store(
                    val, (mx_u4 *)(g.out + (long long)f * g.ofstride + ((long long)c * g.nb + bi) * 64 + (l & 7u) * 8));
        };
        if constexpr (kMxsLean) {
            /* Y and Cb leave before the Cr column, which then takes their set-0 slots */
            mx_fence(cr[1][3]);                        /* the Cr products are done (operand rule) */
            keepc();
            cr_tile();
            mx_wave_sync();
            if (__builtin_expect(__ballot((fl & 0xffffu) != 0) != 0, 0)) {
                uint32_t f2 = fl & 0xffffu;
                clamp(f2);
                mx_exact_inline<true>(L, sp, f2, T, xt);
            }
            if (S.simple) {
                const mx_u4 v0 = *(const mx_u4 *)(L.stage + ro);
                const mx_u4 v1 = *(const mx_u4 *)(L.stage + rcb);
                __builtin_nontemporal_store(v0, (mx_u4 *)(ob + so0));
                __builtin_nontemporal_store(v1, (mx_u4 *)(ob + so1));
            } else {
                store(0);
                store(1);
            }
            mx_wave_sync();
            mx_column_t<0, true>(acc[2], w0, limc2, tb, 2, j, za, fl, 2);
            mx_wave_sync();
            if (__builtin_expect(__ballot((fl >> 16) != 0) != 0, 0)) {
                uint32_t f2 = fl & 0xff0000u;
                clamp(f2);
                mx_exact_inline<true>(L, sp, f2, T, xt);
            }
            if (S.simple) {
                const mx_u4 v2 = *(const mx_u4 *)(L.stage + rr);
                __builtin_nontemporal_store(v2, (mx_u4 *)(ob + so2));
            } else {
                store(2);
            }
            mx_wave_sync();
            return;
        }
        const bool early = S.simple && __ballot((fl & 0xffffu) != 0) == 0;
        if (early) {
            mx_fence(cr[1][3]);                        /* the Cr products are done (operand rule) */
            keepc();
            mx_wave_sync();
            const mx_u4 v0 = *(const mx_u4 *)(L.stage + ro);
            const mx_u4 v1 = *(const mx_u4 *)(L.stage + rcb);
            __builtin_nontemporal_store(v0, (mx_u4 *)(ob + so0));
            __builtin_nontemporal_store(v1, (mx_u4 *)(ob + so1));
        }
        __builtin_amdgcn_sched_barrier(0);
        cr_tile();
        mx_column_t<8 * kBS, true>(acc[2], w0, limc2, tb, 2, j, za, fl, 2);
        keepc();
        mx_wave_sync();
        if (!JX_MXS_NOEXACT && __builtin_expect(__ballot(fl != 0) != 0, 0)) {
            clamp(fl);
            mx_exact_inline(L, sp, fl, T, xt);
        }
#endif
        /* stores: always three store instructions (the vmcnt accounting counts on it) */
        if (early) {
            const mx_u4 v2 = *(const mx_u4 *)(L.stage + rr);
            __builtin_nontemporal_store(v2, (mx_u4 *)(ob + so2));
        } else if (S.simple) {
            const mx_u4 v0 = *(const mx_u4 *)(L.stage + ro);
            const mx_u4 v1 = *(const mx_u4 *)(L.stage + rcb);
            const mx_u4 v2 = *(const mx_u4 *)(L.stage + rr);
            __builtin_nontemporal_store(v0, (mx_u4 *)(ob + so0));
            __builtin_nontemporal_store(v1, (mx_u4 *)(ob + so1));
            __builtin_nontemporal_store(v2, (mx_u4 *)(ob + so2));
        } else {
#pragma unroll
            for (int c = 0; c < 3; c++) store(c);
        }
        mx_wave_sync();
    };

    if constexpr (!kMxsRing) {
        /* step k waits for its DMA: younger are kMxsR - 1 - k steps' two DMA operations and k
         * steps' three stores */
        const auto step = [&](auto kc) __attribute__((always_inline)) {
            constexpr unsigned k = decltype(kc)::value < kMxsR ? decltype(kc)::value : kMxsR - 1;
            if (cmp.b >= g.total) return;
            mx_wait_vm<2 * (kMxsR - 1 - k) + 3 * k>();
            body(cmp, L.ring[k]);
            mxs_next(cmp, g);
        };
        step(std::integral_constant<unsigned, 0>{});
#ifdef JX_MXS_STAMP
        JX_MXS_TS(2, __builtin_amdgcn_s_memrealtime());
#endif
        if constexpr (kMxsR > 1) step(std::integral_constant<unsigned, 1>{});
        if constexpr (kMxsR > 2) step(std::integral_constant<unsigned, 2>{});
    } else {
        unsigned slot = 0;
        for (unsigned k = 0; k < kMxsC; k++) {
            if (cmp.b >= g.total) break;
            /* younger than this step's DMA: the step after it (two DMA operations) and the steps
             * since its issue (three stores each): 2 at step 0, 2 + 3 at step 1, then 3 + 2 + 3.
             * (No padding in the prologue: its target slot would also receive a later DMA.) */
            if (k == 0)
                mx_wait_vm<2>();
            else if (k == 1)
                mx_wait_vm<5>();
            else
                mx_wait_vm<8>();
            mx_wave_sync();
            uint8_t *const sp = L.ring[0] + kSlot * slot;
            /* the step two ahead into the slot of the step before (consumed) */
            const unsigned s2 = slot == 0 ? 2u : slot - 1u;
            if (k + 2 < kMxsC) {
                mxs_issue(iss, g, L.ring[0] + kSlot * s2, off0, off1, lane);
                mxs_next(iss, g);
            } else {
                /* padding (two operations keep the count): the slot of step k - 1, never read again */
                mxs_dma<4>(g.rgb, L.ring[0] + kSlot * s2);
                mxs_dma<4>(g.rgb, L.ring[0] + kSlot * s2);
            }
            body(cmp, sp);
            mxs_next(cmp, g);
            slot = slot == 2 ? 0u : slot + 1u;
#ifdef JX_MXS_STAMP
            if (k == 0) JX_MXS_TS(2, __builtin_amdgcn_s_memrealtime());
#endif
        }
    }
#ifdef JX_MXS_STAMP
    JX_MXS_TS(3, __builtin_amdgcn_s_memrealtime());
    JX_MXS_TS(4, __builtin_amdgcn_s_memtime());
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    JX_MXS_TS(6, __builtin_amdgcn_s_memrealtime());
#endif
}

/* ==== k_mx422: true 4:2:2 (extension, JPGX_FLAG_SUBSAMPLE, sample_ratio 1) ==================
 *
 * k_mx's chunk loop, LDS-DMA ring and per-step bookkeeping; a step is 8 Y blocks = 4 MCUs
 * (chroma block cb of the step = Y blocks 2 cb, 2 cb + 1: W is a multiple of 16 and steps start
 * at multiples of 8, so an MCU never straddles a step or a block-row).
 *   Y       k_mx's Y row transform with the two sets concatenated along K (B_Y0 zero in columns
 *           8..15, B_Y1 in 0..7): column j of the C tile is set j / 8's Y at u = j % 8.
 *   Chroma  A row m = chroma block m >> 2, pixel row m & 3 of the half, K = the 48 bytes of the
 *           MCU's pixel row over two K = 32 products; B (jpgx_plan.cpp jx_mx422_operands) holds
 *           0.5 a[c][p] cos((2 floor(x/2) + 1) u pi/16), so column j is the row transform of the
 *           pair-averaged level-shifted chroma: Cb (j < 8) or Cr of chroma block gq at u = j % 8.
 *           Same encoding, split and rigorous band as k_mx (jx_plan_tables_mx422: 65 fp32
 *           additions per lo part instead of 33).
 *   Columns each lane holds two, Y block (j / 8) 4 + gq and chroma block (channel j / 8, gq):
 *           16 MFMAs and 2 x 8 column DCTs per step (k_mx: 16 and 3 x 8); 1 KiB Y + 512 B Cb +
 *           512 B Cr leave in two stores (lanes 0..31 Cb, 32..63 Cr).
 *   Occupancy  four waves per SIMD (the kernel is latency-bound: at two waves it runs 1.5x
 *           slower than at three): <= 128 VGPRs and 40 KiB of LDS per workgroup -- a ring of three
 *           slots (chunks of three steps), the per-lane scales and band limits in a 2-KiB
 *           workgroup table read per column, and one set of stage addresses for both columns
 *           (stage layout: Y block jb at 144 jb, chroma (c, cb) at 1152 + 144 (4 c + cb), so the
 *           chroma column's address is the Y column's plus a constant).
 *   Quirk   the x0 = -8 quirk shifts a row-last Y block's rows by one (Y only); a general step
 *           holding such a block loads the block's true rows into L.qtrue for its chroma block.
 *   Exact   deferred / inline as k_mx; a chroma task carries the MCU's 8 x 48 bytes (two side
 *           slots) and follows the oracle's definition (oracle/cpu_ref.c cpuref_chroma_sample,
 *           dct_coef): X = (ls(2X) + ls(2X+1)) * 0.5, ls = the level-shifted chroma in
 *           preprocess.c's operation order.
 */
constexpr unsigned kSteps422 = 3;             /* steps per chunk = ring slots */
constexpr unsigned kCB422 = 8 * kSteps422;    /* blocks per chunk */
static_assert(kDist == 2, "k_mx422: a ring of three slots holds the step and two ahead");
constexpr unsigned kVmWait422 = 4 * kDist - 2;    /* 2 stores x kDist steps + 2 DMA x (kDist - 1) */
constexpr int kWaitImm422 = (int)((kVmWait422 & 15u) | ((kVmWait422 >> 4) << 14) | 0xF70u);
constexpr unsigned kSt422C = 8 * kBS;         /* chroma (c, cb) at kSt422C + kBS (4 c + cb) */
#ifndef JX_MX422_WPE
#define JX_MX422_WPE 4
#endif

struct alignas(16) Mx422Lds {
    uint8_t ring[kSteps422][kSlot];
    uint8_t stage[16 * kBS];
    uint8_t qtrue[4][192];              /* general step: true rows [y][24] of row-last block 2cb+1 */
    uint8_t pix[kSide][192];            /* deferred blocks: Y [y][24] in one slot, an MCU [y][48]
                                           in two                                                */
    uint32_t sblk[kSide];               /* launch-global Y block (an MCU: its left block)        */
    uint16_t dtask[kSide];              /* a flagged column: slot << 13 | ch << 11 | u << 8 | v-mask */
    uint16_t task[8];
    uint32_t dummy[64];
};
static_assert(sizeof(Mx422Lds) * 4 + sizeof(MxTab) <= 40 * 1024, "4 workgroups of 4 waves per CU");

__device__ mx_u4 g_mx422B[JX_MX_PARTS * 4][64];  /* [part * 4 + which][lane] */
__device__ jx_mxtab g_mx422tab[2][JX_MAXQ + 1];  /* n = 8 c + u: c = 0 Y, 1 Cb, 2 Cr */

/* Y block of a lane's columns (lane (gq, j): set j / 8); also the chroma column's stage slot */
__device__ __forceinline__ unsigned mx422_yblock(unsigned sl)
{
    return (sl & 15u) < 8 ? (sl >> 4) : 4u + (sl >> 4);
}

/*
 * One exact coefficient per 8-lane group from pixel pairs: lane x's samples are the averages
 * (X(p) + X(p + d1)) * 0.5 over rows y of p = row0 + rs y, X = the level-shifted channel value
 * in the reference's colour arithmetic.  Chroma (4:2:2): p = pixel 2x, d1 = 3 (the extension's
 * definition, oracle/cpu_ref.c cpuref_chroma_sample); Y: p = pixel x, d1 = 0 ((X + X) * 0.5 == X
 * exactly, so Y tasks share the code).  Valid in lane x == 7.
 */
template <bool FAST = (JX_MX_FASTEXACT != 0)>
__device__ __forceinline__ int mx_exact_pair(const lds_u8 *row0, unsigned rs, unsigned d1, unsigned ch,
                                             unsigned u, unsigned v, unsigned x, const jx_mxtab &T)
{
    const double cu = kMxCos[u][x];
    const double k0c = kMxColour[ch][0], k1c = kMxColour[ch][1], k2c = kMxColour[ch][2];
    const double Ac = kMxColour[ch][3], Sc = kMxColour[ch][4];
    double prod[8];
#pragma unroll
    for (int y = 0; y < 8; y++) {
        const lds_u8 *p = row0 + rs * (unsigned)y, *p1 = p + d1;
        const double t0 = (k0c * (double)p[0] + k1c * (double)p[1]) + k2c * (double)p[2];
        const double t1 = (k0c * (double)p1[0] + k1c * (double)p1[1]) + k2c * (double)p1[2];
        const double X = (((Ac + Sc * t0) - 128.0) + ((Ac + Sc * t1) - 128.0)) * 0.5;
        prod[y] = X * cu * kMxCos[v][y];
    }
    return mx_exact_sum<FAST>(prod, ch, u, v, x, T, T.r[ch == 0 ? 0 : 1][u * 8 + v]);
}

/* lane x's first pixel (row 0) and row stride of chroma block cb in a step's slot; the right
 * Y block's rows come from L.qtrue when it is a row-last block (bit cb of qmask) */
template <class Lds>
__device__ __forceinline__ const lds_u8 *mx422_mcu_row0(Lds &L, const uint8_t *sp, uint32_t qmask,
                                                        unsigned cb, unsigned x, unsigned &rs)
{
    const bool q = ((qmask >> cb) & 1u) && x >= 4;
    rs = q ? 24u : 192u;
    return q ? mx_lds(L.qtrue[cb]) + 6u * (x - 4u) : mx_lds((void *)sp) + 48u * cb + 6u * x;
}

/* Inline exact pass of one step: bit 8 col + v of a lane's bits (col 0 Y, 1 chroma) */
template <class Lds>
__device__ __forceinline__ void mx422_exact_inline(Lds &L, const uint8_t *sp, uint32_t qmask,
                                                   uint32_t bits, const jx_mxtab &T)
{
    const unsigned lane = mx_lane();
    mx_wave_sync();
    for (;;) {
        const uint64_t act = __ballot(bits != 0);
        if (!act) break;
        const int rk = mx_rank(act);
        if (bits != 0 && rk < 8) {
            const unsigned b = (unsigned)__builtin_ctz(bits);
            bits &= bits - 1u;
            L.task[rk] = (uint16_t)(lane << 8 | b);
        }
        mx_wave_sync();
        const int nt = std::min((int)__popcll(act), 8);
        const unsigned i = lane >> 3, x = lane & 7u;
        const bool live = (int)i < nt;
        const unsigned code = L.task[live ? i : 0u];
        const unsigned sl = code >> 8, k = (code >> 3) & 1u, v = code & 7u;
        const unsigned jj = sl & 15u, u = jj & 7u;
        const unsigned slot = mx422_yblock(sl);       /* Y block, or 4 c + cb for chroma */
        unsigned ch, rs, d1;
        const lds_u8 *row0;
        if (k == 0) {
            ch = 0;
            rs = 192u;
            d1 = 0;
            row0 = mx_lds((void *)sp) + 24u * slot + 3u * x;
        } else {
            ch = 1u + (jj >> 3);
            d1 = 3;
            row0 = mx422_mcu_row0(L, sp, qmask, sl >> 4, x, rs);
        }
        const int val = mx_exact_pair<false>(row0, rs, d1, ch, u, v, x, T);   /* k_mxs422 at 128 VGPRs: no room */
        if (live && x == 7)
            *(__attribute__((address_space(3))) int16_t *)(mx_lds(L.stage) + (k ? kSt422C : 0u) + kBS * slot +
                                                           2u * (unsigned)kMxScan[v][u]) = (int16_t)val;
        mx_wave_sync();
    }
}

__device__ __forceinline__ void mx422_flush(Mx422Lds &L, int &nq, int &ns, const MxG &g, const jx_mxtab &T)
{
    __builtin_amdgcn_s_waitcnt(0xF70);                 /* vmcnt(0): the tasks' blocks are stored */
    mx_wave_sync();
    const unsigned lane = mx_lane(), i = lane >> 3, x = lane & 7u;
    const bool live = (int)i < nq;
    const unsigned code = L.dtask[live ? i : 0u];
    const unsigned slot = code >> 13, ch = (code >> 11) & 3u, u = (code >> 8) & 7u;
    uint32_t vb = live ? (code & 0xffu) : 0u;
    const lds_u8 *px = mx_lds(L.pix[slot]);
    const unsigned b = L.sblk[slot], f = b / g.nb, bi = b - f * g.nb;
    const long long blk = ch == 0 ? (long long)bi : (long long)g.nb + (ch - 1u) * (g.nb / 2u) + bi / 2u;
    int16_t *const dst = g.out + (long long)f * g.ofstride + blk * 64;
    while (__ballot(vb != 0)) {
        const bool act = vb != 0;
        const unsigned v = act ? (unsigned)__builtin_ctz(vb) : 0u;
        vb &= vb - 1u;
        const int val = ch == 0 ? mx_exact_pair<false>(px + 3u * x, 24u, 0u, 0u, u, v, x, T)   /* legacy k_mx422 */
                                : mx_exact_pair<false>(px + 6u * x, 48u, 3u, ch, u, v, x, T);
        if (act && x == 7) dst[kMxScan[v][u]] = (int16_t)val;
    }
    mx_wave_sync();
    nq = 0;
    ns = 0;
}

/* A step with flagged coefficients: queue them with their blocks' pixels (Y: one side slot per
 * block; an MCU: two), flushing first if the queue would overflow; inline if the step alone
 * would. */
__device__ __forceinline__ void mx422_defer(Mx422Lds &L, const uint8_t *sp, uint32_t qmask, uint32_t bits,
                                            unsigned b0, int &nq, int &ns, const MxG &g, const jx_mxtab &T)
{
    const unsigned lane = mx_lane();
    if (b0 + 8u > g.total) {                           /* clamped copies past the end (even count) */
        const unsigned nvalid = g.total - b0;
        if (mx422_yblock(lane) >= nvalid) bits &= ~0xffu;
        if (2u * (lane >> 4) >= nvalid) bits &= ~0xff00u;
    }
    const uint64_t m0 = __ballot((bits & 0xffu) != 0), m1 = __ballot((bits & 0xff00u) != 0);
    uint32_t yblk = 0, cblk = 0;
#pragma unroll
    for (int gq = 0; gq < 4; gq++) {
        yblk |= (((m0 >> (16 * gq)) & 0xffu) ? 1u : 0u) << gq;
        yblk |= (((m0 >> (16 * gq + 8)) & 0xffu) ? 1u : 0u) << (4 + gq);
        cblk |= (((m1 >> (16 * gq)) & 0xffffu) ? 1u : 0u) << gq;
    }
    const int n0 = __popcll(m0), ncol = n0 + __popcll(m1);
    const int ny = __popc(yblk), nslot = ny + 2 * __popc(cblk);
    if (nq + ncol > kSide || ns + nslot > kSide) {
        if (nq) mx422_flush(L, nq, ns, g, T);
        if (ncol > kSide || nslot > kSide) {
            mx422_exact_inline(L, sp, qmask, bits, T);
            return;
        }
    }
    /* copy the pixel rows (lane < 48: row l / 6, dword l % 6) */
    {
        const unsigned y = lane / 6u, k = lane - 6u * y;
        uint32_t bm = yblk;
        int t = ns;
        while (bm) {
            const unsigned jb = (unsigned)__builtin_ctz(bm);
            bm &= bm - 1u;
            if (lane < 48)
                *(__attribute__((address_space(3))) uint32_t *)(mx_lds(L.pix[t]) + 24u * y + 4u * k) =
                    *(const __attribute__((address_space(3))) uint32_t *)(mx_lds((void *)sp) + 192u * y + 24u * jb + 4u * k);
            if (lane == 0) L.sblk[t] = b0 + jb;
            t++;
        }
        bm = cblk;
        while (bm) {
            const unsigned cb = (unsigned)__builtin_ctz(bm);
            bm &= bm - 1u;
            if (lane < 48) {
                typedef __attribute__((address_space(3))) uint32_t l32;
                const lds_u8 *left = mx_lds((void *)sp) + 192u * y + 48u * cb;
                const lds_u8 *right = ((qmask >> cb) & 1u) ? mx_lds(L.qtrue[cb]) + 24u * y : left + 24u;
                lds_u8 *d = mx_lds(L.pix[t]) + 48u * y + 4u * k;
                *(l32 *)d = *(const l32 *)(left + 4u * k);
                *(l32 *)(d + 24) = *(const l32 *)(right + 4u * k);
            }
            if (lane == 0) L.sblk[t] = b0 + 2u * cb;
            t += 2;
        }
    }
    {   /* this lane's flagged columns (Y first, then chroma), one queue entry each */
        const unsigned jj = lane & 15u, u = jj & 7u;
        const uint32_t vy = bits & 0xffu, vc = (bits >> 8) & 0xffu;
        if (vy) {
            const unsigned jb = mx422_yblock(lane);
            const unsigned slot = (unsigned)ns + (unsigned)__popc(yblk & ((1u << jb) - 1u));
            L.dtask[nq + mx_rank(m0)] = (uint16_t)(slot << 13 | u << 8 | vy);
        }
        if (vc) {
            const unsigned cb = lane >> 4;
            const unsigned slot = (unsigned)(ns + ny) + 2u * (unsigned)__popc(cblk & ((1u << cb) - 1u));
            L.dtask[nq + n0 + mx_rank(m1)] = (uint16_t)(slot << 13 | (1u + (jj >> 3)) << 11 | u << 8 | vc);
        }
    }
    mx_wave_sync();
    nq += ncol;
    ns += nslot;
}

/* the rare paths end with their loads complete (the exact pass's constant-table loads), so the
 * compiler's wait for them does not land in the hot path of the next step */
__device__ __forceinline__ void mx422_defer_step(Mx422Lds &L, const uint8_t *sp, uint32_t qmask, uint32_t bits,
                                                 unsigned b0, int &nq, int &ns, const MxG &g, const jx_mxtab &T)
{
    mx422_defer(L, sp, qmask, bits, b0, nq, ns, g, T);
    __builtin_amdgcn_s_waitcnt(0xF70);
}

/* a general step's row-last Y blocks (always odd: bpr is even): their true pixel rows 8r..8r+7
 * into L.qtrue[cb]; returns the mask of chroma blocks cb that have one */
template <class Lds>
__device__ __forceinline__ uint32_t mx422_true_rows(Lds &L, const MxG &g, unsigned b0)
{
    const unsigned l = mx_lane(), y = l & 7u, cb = (l >> 3) & 3u;
    const unsigned b = b0 + 2u * cb + 1u;
    bool last = false;
    unsigned f = 0, r = 0, c = 0;
    if (l < 32 && b < g.total) {
        f = b / g.nb;
        const unsigned bi = b - f * g.nb;
        r = bi / g.bpr;
        c = bi - r * g.bpr;
        last = c == g.bpr - 1u;
    }
    const uint64_t bal = __ballot(last && y == 0);
    uint32_t qm = 0;
#pragma unroll
    for (int k = 0; k < 4; k++) qm |= (uint32_t)((bal >> (8 * k)) & 1u) << k;
    if (qm) {
        if (last) {
            typedef const __attribute__((address_space(1))) mx_u2 gu2;
            const gu2 *src = (const gu2 *)(g.rgb + (long long)f * g.fstride + (8ll * r + y) * g.pitch + 24ll * c);
            const mx_u2 v0 = src[0], v1 = src[1], v2 = src[2];
            uint8_t *d = L.qtrue[cb] + 24u * y;
            *(mx_u2 *)d = v0;
            *(mx_u2 *)(d + 8) = v1;
            *(mx_u2 *)(d + 16) = v2;
        }
        __builtin_amdgcn_s_waitcnt(0xF70);             /* vmcnt(0) (rare; conservative) */
        mx_wave_sync();
    }
    return qm;
}

__global__ __launch_bounds__(256, JX_MX422_WPE) void k_mx422(const jx_xform_args a)
{
    __shared__ __attribute__((aligned(16))) Mx422Lds s_lds[4];
    __shared__ __attribute__((aligned(16))) MxTab s_tab;
    MxG g;
    g.rgb = a.g.rgb;
    g.out = a.g.out;
    g.pitch = a.g.in_pitch;
    g.fstride = a.g.in_fstride;
    g.ofstride = a.g.out_fstride;
    g.bpr = (unsigned)a.g.bpr;
    g.nb = (unsigned)a.g.nb;
    g.total = (unsigned)a.g.nb * (unsigned)a.g.nframes;
    g.row0 = a.g.row0;
    g.quality = a.quality;
    g.force = a.force_exact;
    g.lin_store = (unsigned long long)g.nb * 256ull + 1024ull < (1ull << 31);
#pragma unroll
    for (int k = 0; k < 6; k++) g.u[k] = a.g.under[k];
    g.dnb = a.g.dnb;
    g.dbpr = a.g.dbpr;

    const unsigned lane = threadIdx.x & 63u;
    Mx422Lds &L = s_lds[threadIdx.x >> 6];
    const jx_mxtab &T = g_mx422tab[g.force ? 1 : 0][g.quality];
    /* the workgroup's scale / limit table: wave 0, lane (t = lane >> 4, profile j = lane & 15) */
    if (threadIdx.x < 64) {
        const unsigned t = lane >> 4, jp = lane & 15u;
        const unsigned n = t < 2 ? (jp & 7u) : 8u + jp;
        float x[8];
#pragma unroll
        for (int p = 0; p < 4; p++)
#pragma unroll
            for (int h = 0; h < 2; h++) {
                const int v = jx_pk_k(p, h);
                x[2 * p + h] = (t & 1u) ? T.lsq[n][v] : T.w[n][v];
            }
        s_tab.wl[t][0][jp] = mx_f4{x[0], x[1], x[2], x[3]};
        s_tab.wl[t][1][jp] = mx_f4{x[4], x[5], x[6], x[7]};
    }
    __syncthreads();
    /* hot-path band limits of this lane's two column kinds (mx_limc) */
    const float limc0 = mx_limc(s_tab, 1, threadIdx.x & 15u), limc2 = mx_limc(s_tab, 3, threadIdx.x & 15u);
    const unsigned nw = gridDim.x * 4u;
    const unsigned wv = __builtin_amdgcn_readfirstlane(blockIdx.x * 4u + (threadIdx.x >> 6));
    if (kCB422 * wv >= g.total) return;

    /* Y A operands as k_mx's; chroma: row m = (chroma block m >> 2, pixel row m & 3 of the
     * half), k-step 0 bytes 8q.. of the MCU's 48-byte row, k-step 1 bytes 32 + 8q (q < 2), the
     * bias 1.0 (q = 2), zeros (q = 3) */
    const unsigned m = lane & 15u, q = lane >> 4;
    const uint32_t aoff = 192u * (m & 3u) + 24u * (m >> 2) + 8u * (q < 3 ? q : 0u);
    const uint32_t s0 = q < 3 ? kSelLo : kSelOne;
    const uint32_t s1 = q < 3 ? kSelHi : kSelZero;
    const uint32_t s2 = q < 3 ? kSelLo : kSelZero;
    const uint32_t coff0 = 192u * (m & 3u) + 48u * (m >> 2) + 8u * q;
    const uint32_t coff1 = 192u * (m & 3u) + 48u * (m >> 2) + 32u + 8u * (q < 2 ? q : 0u);
    const uint32_t t0 = q < 2 ? kSelLo : (q == 2 ? kSelOne : kSelZero);
    const uint32_t t1 = q < 2 ? kSelHi : kSelZero;
    const uint32_t t2 = q < 2 ? kSelLo : kSelZero;
    const uint32_t off0 = (uint32_t)((lane / 12u) * (unsigned)g.pitch + 16u * (lane % 12u));
    const uint32_t off1 = (uint32_t)(((64u + lane) / 12u) * (unsigned)g.pitch + 16u * ((64u + lane) % 12u));
    /* stores: Y 8 blocks x 128 B (lane 16 B), chroma lanes 0..31 Cb / 32..63 Cr 4 blocks x 128 B;
     * both read the stage at ro (+ kSt422C) */
    const uint32_t soy = lane * 16u, soc = (lane & 31u) * 16u + (lane >> 5) * (g.nb / 2u) * 128u;
    const uint32_t ro = (lane >> 3) * kBS + (lane & 7u) * 16u;

    const unsigned gq = lane >> 4, j = lane & 15u, u = j & 7u;
    /* LDS addresses of the lane's 8 coefficients in the stage (Y column; chroma + kSt422C) */
    uint32_t za[8];
    {
        const uint32_t base = (uint32_t)(uintptr_t)mx_lds(L.stage) + kBS * ((j >> 3) * 4u + gq);
#pragma unroll
        for (int v = 0; v < 8; v++) za[v] = base + 2u * (unsigned)kMxScan[v][u];
    }
    mx_u4 B[kParts][4];
#pragma unroll
    for (int p = 0; p < kParts; p++)
#pragma unroll
        for (int w = 0; w < 4; w++) B[p][w] = g_mx422B[4 * p + w][lane];
    /* the operand and table loads complete here, once: otherwise the compiler's wait for them
     * (it counts one operation for a DMA whose lane < 32 half might be skipped) lands inside
     * the step loop as a vmcnt(0) that drains the prefetch every step */
    __builtin_amdgcn_s_waitcnt(0xF70);

    MxJump J;
    J.jb = kCB422 * nw;
    J.jr = J.jb / g.bpr;
    J.jc = J.jb - J.jr * g.bpr;
    J.rows = g.nb / g.bpr;
    MxChunk cc;
    mx_chunk_at<kCB422>(cc, g, kCB422 * wv);
    MxChunk nx = cc;

    const auto issue = [&](const MxChunk &C, unsigned k) {
        uint8_t *const slot = L.ring[k];
        const unsigned b = C.b0 + 8u * k;
        if (b >= g.total) {
            mx_pad(g, L, 2);
        } else if (C.simple) {
            const uint8_t *base = C.src + 192u * k;
            __builtin_amdgcn_global_load_lds((mx_gp)(base + off0), (mx_lp)slot, 16, 0, 0);
            if (lane < 32) __builtin_amdgcn_global_load_lds((mx_gp)(base + off1), (mx_lp)(slot + 1024u), 16, 0, 0);
        } else {
            MxCur P;
            mx_seek(P, g, b);
            mx_issue(g, P, b, mx_simple_load(P, g, b), off0, off1, slot);
        }
    };
    for (unsigned d = 0; d < kDist; d++) {
        issue(cc, d);
        mx_pad(g, L, 2);
    }
    int nq = 0, ns = 0;
    unsigned k = 0;
    for (;;) {
        const unsigned b0 = cc.b0 + 8u * k;
        /* younger than this step's DMA: the two stores of each of the kDist steps before it and
         * the DMA of the kDist - 1 steps after it */
        __builtin_amdgcn_s_waitcnt(kWaitImm422);
        mx_wave_sync();
        const uint8_t *const sp = L.ring[k];
        if (k + kDist < kSteps422) {
            issue(cc, k + kDist);
        } else {
            if (k + kDist == kSteps422) mx_chunk_next<kCB422>(nx, g, J);
            issue(nx, k + kDist - kSteps422);
        }
        const uint32_t qmask = cc.simple ? 0u : mx422_true_rows(L, g, b0);
        const mx_f4 z = {};
        uint32_t fl = 0;
        mx_f4 acc[2][4];                               /* [Y, chroma][hl, ll, hh, lh] */
        mx_f4 mid[2][4];                               /* the chains' first products (mx_keep) */
        const auto mma2 = [&](mx_f4(&o)[4], mx_f4(&m)[4], const mx_h8 &Al0, const mx_h8 &Ah0, const mx_h8 &Al1,
                              const mx_h8 &Ah1, int w0) {
            m[0] = mx_mma(Al0, B[0][w0], z);
            m[2] = mx_mma(Ah0, B[0][w0], z);
            m[1] = mx_mma(Al0, B[1][w0], z);
            m[3] = mx_mma(Ah0, B[1][w0], z);
            o[0] = mx_mma(Al1, B[0][w0 + 1], m[0]);
            o[2] = mx_mma(Ah1, B[0][w0 + 1], m[2]);
            o[1] = mx_mma(Al1, B[1][w0 + 1], m[1]);
            o[3] = mx_mma(Ah1, B[1][w0 + 1], m[3]);
            if (kParts == 3) {
                o[1] = mx_mma(Al0, B[kParts - 1][w0], o[1]);
                o[3] = mx_mma(Ah0, B[kParts - 1][w0], o[3]);
                o[1] = mx_mma(Al1, B[kParts - 1][w0 + 1], o[1]);
                o[3] = mx_mma(Ah1, B[kParts - 1][w0 + 1], o[3]);
            }
        };
        /* every LDS read of the step's A operands is issued before its first MFMA; each column
         * reads its scales after its tiles (the Y column after a fence on the chroma products)
         * (MFMA operand rule, mx_fence) */
        const mx_u2 y00 = *(const mx_u2 *)(sp + aoff);
        const mx_u2 y01 = *(const mx_u2 *)(sp + aoff + 768u);
        const mx_u2 y10 = *(const mx_u2 *)(sp + aoff + 96u);
        const mx_u2 y11 = *(const mx_u2 *)(sp + aoff + 864u);
        mx_u2 c00, c01, c10, c11;
        {
            if (__builtin_expect(qmask == 0, 1)) {
                c00 = *(const mx_u2 *)(sp + coff0);
                c01 = *(const mx_u2 *)(sp + coff0 + 768u);
                c10 = *(const mx_u2 *)(sp + coff1);
                c11 = *(const mx_u2 *)(sp + coff1 + 768u);
            } else {
                /* chroma blocks with a row-last right block: its bytes (24..47 of the MCU row)
                 * from the true rows */
                const unsigned l = mx_lane(), mm = l & 15u, qq = l >> 4, cb = mm >> 2;
                const bool qb = (qmask >> cb) & 1u;
                const uint8_t *qt = L.qtrue[cb] + 24u * (mm & 3u);
                const uint8_t *p0 = qb && qq == 3 ? qt : sp + coff0;
                const uint8_t *p1 = qb && qq < 2 ? qt + 8u + 8u * qq : sp + coff1;
                const unsigned h0 = qb && qq == 3 ? 96u : 768u, h1 = qb && qq < 2 ? 96u : 768u;
                c00 = *(const mx_u2 *)p0;
                c01 = *(const mx_u2 *)(p0 + h0);
                c10 = *(const mx_u2 *)p1;
                c11 = *(const mx_u2 *)(p1 + h1);
            }
        }
        /* all A operands before the first product (k_mxs422's order, mx_keep) */
        const mx_h8 Ay0 = mx_aop(y00, s0, s1, s2), Ay1 = mx_aop(y01, s0, s1, s2);
        const mx_h8 Ay2 = mx_aop(y10, s0, s1, s2), Ay3 = mx_aop(y11, s0, s1, s2);
        const mx_h8 Ac0 = mx_aop(c00, kSelLo, kSelHi, kSelLo), Ac1 = mx_aop(c01, kSelLo, kSelHi, kSelLo);
        const mx_h8 Ac2 = mx_aop(c10, t0, t1, t2), Ac3 = mx_aop(c11, t0, t1, t2);
        __builtin_amdgcn_sched_barrier(0);
        mma2(acc[0], mid[0], Ay0, Ay1, Ay2, Ay3, 0);
        __builtin_amdgcn_sched_barrier(0);
        mma2(acc[1], mid[1], Ac0, Ac1, Ac2, Ac3, 2);
        __builtin_amdgcn_sched_barrier(0);
        mx_column_t<0, true>(acc[0], MxW{}, limc0, s_tab, 0, j, za, fl, 0, &acc[1][3],
                             [&]() __attribute__((always_inline)) { mx_keep(mid[1]); });
        __builtin_amdgcn_sched_barrier(0);
        mx_column_t<kSt422C, true>(acc[1], MxW{}, limc2, s_tab, 2, j, za, fl, 1);
        mx_wave_sync();
        if (__builtin_expect(__ballot(fl != 0) != 0, 0)) mx422_defer_step(L, sp, qmask, fl, b0, nq, ns, g, T);
        /* always two store instructions per step (the vmcnt accounting counts on it) */
        if (cc.simple) {
            const mx_u4 vy = *(const mx_u4 *)(L.stage + ro);
            const mx_u4 vc = *(const mx_u4 *)(L.stage + kSt422C + ro);
            __builtin_nontemporal_store(vy, (mx_u4 *)((const uint8_t *)(cc.dst + 512u * k) + soy));
            __builtin_nontemporal_store(vc, (mx_u4 *)((const uint8_t *)(cc.cdst + 256u * k) + soc));
        } else {
            const unsigned l = mx_lane();
            const unsigned by = b0 + (l >> 3), bc = b0 + 2u * ((l >> 3) & 3u);
            const unsigned yb = by < g.total ? by : g.total - 1u, cbk = bc < g.total ? bc : g.total - 1u;
            const unsigned fy = yb / g.nb, biy = yb - fy * g.nb;
            const unsigned fc = cbk / g.nb, bic = cbk - fc * g.nb;
            const uint32_t rl = (l >> 3) * kBS + (l & 7u) * 16u;
            const mx_u4 vy = *(const mx_u4 *)(L.stage + rl);
            const mx_u4 vc = *(const mx_u4 *)(L.stage + kSt422C + rl);
            if (by < g.total)
                __builtin_nontemporal_store(
                    vy, (mx_u4 *)(g.out + (long long)fy * g.ofstride + (long long)biy * 64 + (l & 7u) * 8));
            if (bc < g.total)
                __builtin_nontemporal_store(
                    vc, (mx_u4 *)(g.out + (long long)fc * g.ofstride +
                                  ((long long)g.nb + (l >> 5) * (g.nb / 2u) + bic / 2u) * 64 + (l & 7u) * 8));
        }
        mx_wave_sync();
        if (++k == kSteps422) {
            k = 0;
            cc = nx;
            if (cc.b0 >= g.total) break;
        } else if (b0 + 8u >= g.total) {
            break;
        }
    }
    if (nq) mx422_flush(L, nq, ns, g, T);
}

/* ==== k_mxs422: k_mx422's transform in short-lived one-wave workgroups (round 4) =============
 *
 * k_mxs's scheme (three steps per wave, their DMA up front, step k in slot k, a 1.2-KiB per-wave
 * image of scales / hot-path limits / zig-zag positions by LDS-DMA, the B operands and band limits
 * from the global image, the exact pass inline on the stage) around k_mx422's step: 8 Y blocks =
 * 4 MCUs, Y and chroma row transforms on the matrix cores (16 MFMAs), two column DCTs per lane,
 * two stores (Y 1 KiB; lanes 0..31 Cb, 32..63 Cr).  Two stores per step: step k waits with
 * vmcnt(2 (C - 1 - k) + 2 k).  The quirk (a general step holding a row-last Y block) loads that
 * block's true rows into L.qtrue for its MCU's chroma, as k_mx422.
 */
constexpr unsigned kMxs422C = 3;
struct alignas(16) Mxs422Lds {
    uint8_t ring[kMxs422C][kSlot];
    uint8_t stage[16 * kBS];
    uint8_t qtrue[4][192];
    uint16_t task[8];
};
static_assert(sizeof(Mxs422Lds) % 16 == 0 &&
                  (sizeof(Mxs422Lds) + sizeof(MxsImg1) + 511) / 512 * 512 * 16 <= 160 * 1024,
              "16 one-wave workgroups per CU");
/* the global image: B operands [part * 4 + which][lane], k_mx422's scale / limit table */
struct alignas(16) MxsImg422 {
    mx_u4 B[JX_MX_PARTS * 4][64];
    MxTab tab;
};
__device__ MxsImg422 g_mxs422_img[2][JX_MAXQ + 1];
__device__ MxsImg1 g_mxs422_img1[2][JX_MAXQ + 1];
/* waves per workgroup: 1 (B operands from the global image) or 4 (B, scales, limc and the zig-zag
 * table in LDS, shared through one s_barrier; band limits from the global image, rare path) */
#ifndef JX_MXS422_WPG
#define JX_MXS422_WPG 4
#endif
constexpr unsigned kMxs422WPG = JX_MXS422_WPG;
static_assert(kMxs422WPG == 1 || kMxs422WPG == 4 || kMxs422WPG == 8, "1, 4 or 8 waves per workgroup");
struct alignas(16) MxsImg422w {
    mx_u4 B[JX_MX_PARTS * 4][64];
    MxsImg1 s;
};
constexpr unsigned kMxs422Pieces = sizeof(MxsImg422w) / 16;
static_assert(kMxs422WPG == 1 || sizeof(Mxs422Lds) * kMxs422WPG + sizeof(MxsImg422w) <= 160 * 1024 / (16 / kMxs422WPG),
              "4 workgroups of 4 waves per CU");
__device__ MxsImg422w g_mxs422_imgw[2][JX_MAXQ + 1];
typedef std::conditional<kMxs422WPG >= 2, MxsImg422w, MxsImg1>::type Mxs422Shared;
[[maybe_unused]] __device__ __forceinline__ const MxsImg1 &mxs422_s(const MxsImg422w &l) { return l.s; }
[[maybe_unused]] __device__ __forceinline__ const MxsImg1 &mxs422_s(const MxsImg1 &l) { return l; }
[[maybe_unused]] __device__ __forceinline__ const mx_u4 (&mxs422_B(const MxsImg422w &l, const MxsImg422 &))[JX_MX_PARTS * 4][64]
{
    return l.B;
}
[[maybe_unused]] __device__ __forceinline__ const mx_u4 (&mxs422_B(const MxsImg1 &, const MxsImg422 &g))[JX_MX_PARTS * 4][64]
{
    return g.B;
}

__global__ __launch_bounds__(64 * kMxs422WPG, JX_MX422_WPE) void k_mxs422(const jx_xform_args a)
{
    __shared__ __attribute__((aligned(16))) Mxs422Lds s_lds[kMxs422WPG];
    __shared__ __attribute__((aligned(16))) Mxs422Shared s_img;
    MxG g;
    g.rgb = a.g.rgb;
    g.out = a.g.out;
    g.pitch = a.g.in_pitch;
    g.fstride = a.g.in_fstride;
    g.ofstride = a.g.out_fstride;
    g.bpr = (unsigned)a.g.bpr;
    g.nb = (unsigned)a.g.nb;
    g.total = (unsigned)a.g.nb * (unsigned)a.g.nframes;
    g.row0 = a.g.row0;
    g.quality = a.quality;
    g.force = a.force_exact;
    g.lin_store = (unsigned long long)g.nb * 256ull + 1024ull < (1ull << 31);
#pragma unroll
    for (int k = 0; k < 6; k++) g.u[k] = a.g.under[k];
    g.dnb = a.g.dnb;
    g.dbpr = a.g.dbpr;

    const unsigned lane = threadIdx.x & 63u;
    const unsigned wave = kMxs422WPG == 1 ? 0u : __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    Mxs422Lds &L = s_lds[wave];
    const MxsImg422 &gimg = g_mxs422_img[g.force ? 1 : 0][g.quality];
    if constexpr (kMxs422WPG >= 2) {
        const uint8_t *img = (const uint8_t *)&g_mxs422_imgw[g.force ? 1 : 0][g.quality];
#pragma unroll
        for (unsigned i = 0; i < (kMxs422Pieces + 64u * kMxs422WPG - 1u) / (64u * kMxs422WPG); i++) {
            const unsigned piece = 64u * kMxs422WPG * i + threadIdx.x;
            if (64u * kMxs422WPG * i + 64u * wave < kMxs422Pieces && piece < kMxs422Pieces)
                mxs_dma<16>(img + 16u * piece, (uint8_t *)&s_img + 16u * (64u * kMxs422WPG * i + 64u * wave));
        }
    } else {
        constexpr unsigned kP1 = sizeof(MxsImg1) / 16;
        const uint8_t *img = (const uint8_t *)&g_mxs422_img1[g.force ? 1 : 0][g.quality];
        mxs_dma<16>(img + 16u * lane, &s_img);
        if (lane < kP1 - 64u) mxs_dma<16>(img + 16u * (64u + lane), (uint8_t *)&s_img + 1024u);
    }
    const unsigned wv = blockIdx.x * kMxs422WPG + wave;
    const uint32_t off0 = (uint32_t)((lane / 12u) * (unsigned)g.pitch + 16u * (lane % 12u));
    const uint32_t off1 = (uint32_t)(((64u + lane) / 12u) * (unsigned)g.pitch + 16u * ((64u + lane) % 12u));
    MxsCur iss;
    mxs_at(iss, g, 8u * kMxs422C * wv);
    MxsCur cmp = iss;
#pragma unroll
    for (unsigned k = 0; k < kMxs422C; k++) {
        mxs_issue(iss, g, L.ring[k], off0, off1, lane);
        mxs_next(iss, g);
    }

    /* lane constants (k_mx422's) */
    const unsigned m = lane & 15u, q = lane >> 4;
    const uint32_t aoff = 192u * (m & 3u) + 24u * (m >> 2) + 8u * (q < 3 ? q : 0u);
    const uint32_t s0 = q < 3 ? kSelLo : kSelOne;
    const uint32_t s1 = q < 3 ? kSelHi : kSelZero;
    const uint32_t s2 = q < 3 ? kSelLo : kSelZero;
    const uint32_t coff0 = 192u * (m & 3u) + 48u * (m >> 2) + 8u * q;
    const uint32_t coff1 = 192u * (m & 3u) + 48u * (m >> 2) + 32u + 8u * (q < 2 ? q : 0u);
    const uint32_t t0 = q < 2 ? kSelLo : (q == 2 ? kSelOne : kSelZero);
    const uint32_t t1 = q < 2 ? kSelHi : kSelZero;
    const uint32_t t2 = q < 2 ? kSelLo : kSelZero;
    const uint32_t soy = lane * 16u, soc = (lane & 31u) * 16u + (lane >> 5) * (g.nb / 2u) * 128u;
    const uint32_t ro = (lane >> 3) * kBS + (lane & 7u) * 16u;
    const unsigned gq = lane >> 4, j = lane & 15u, u = j & 7u;
    const jx_mxtab &T = g_mx422tab[g.force ? 1 : 0][g.quality];

    if constexpr (kMxs422WPG == 1) {
        if (cmp.b >= g.total) return;
    }
    mx_wait_vm<2u * kMxs422C>();                    /* the image (older than the pixel DMA) */
    if constexpr (kMxs422WPG >= 2) __builtin_amdgcn_s_barrier();
    mx_wave_sync();
    if (cmp.b >= g.total) return;
    const MxsImg1 &si = mxs422_s(s_img);
    uint32_t za[8];
    {
        const uint32_t base = (uint32_t)(uintptr_t)mx_lds(L.stage) + kBS * ((j >> 3) * 4u + gq);
        const mx_u2 sc = *(const mx_u2 *)&si.scan_t[u][0];
#pragma unroll
        for (int v = 0; v < 8; v++) za[v] = base + 2u * ((v < 4 ? sc.x : sc.y) >> (8 * (v & 3)) & 0xffu);
    }
    mx_u4 B[kParts][4];
#pragma unroll
    for (int p = 0; p < kParts; p++)
#pragma unroll
        for (int w = 0; w < 4; w++) B[p][w] = mxs422_B(s_img, gimg)[4 * p + w][lane];
    const float limc0 = si.limc[0][j], limc2 = si.limc[1][j];
    const MxsTabRef tb{si.sc, gimg.tab};

    const auto body = [&](const MxsCur &S, uint8_t *sp) __attribute__((always_inline)) {
        if (!S.simple) {
            MxCur P;
            mx_seek(P, g, S.b);
            mx_issue(g, P, S.b, false, off0, off1, sp);      /* register path; waits vmcnt(0) */
        }
        const uint32_t qmask = S.simple ? 0u : mx422_true_rows(L, g, S.b);
        mx_wave_sync();
        const mx_f4 z = {};
        uint32_t fl = 0;
        mx_f4 acc[2][4];                               /* [Y, chroma][hl, ll, hh, lh] */
        mx_f4 mid[2][4];                               /* the chains' first products (mx_keep) */
        const auto mma2 = [&](mx_f4(&o)[4], mx_f4(&m)[4], const mx_h8 &Al0, const mx_h8 &Ah0, const mx_h8 &Al1,
                              const mx_h8 &Ah1, int w0) __attribute__((always_inline)) {
            m[0] = mx_mma(Al0, B[0][w0], z);
            m[2] = mx_mma(Ah0, B[0][w0], z);
            m[1] = mx_mma(Al0, B[1][w0], z);
            m[3] = mx_mma(Ah0, B[1][w0], z);
            o[0] = mx_mma(Al1, B[0][w0 + 1], m[0]);
            o[2] = mx_mma(Ah1, B[0][w0 + 1], m[2]);
            o[1] = mx_mma(Al1, B[1][w0 + 1], m[1]);
            o[3] = mx_mma(Ah1, B[1][w0 + 1], m[3]);
            if (kParts == 3) {
                o[1] = mx_mma(Al0, B[kParts - 1][w0], o[1]);
                o[3] = mx_mma(Ah0, B[kParts - 1][w0], o[3]);
                o[1] = mx_mma(Al1, B[kParts - 1][w0 + 1], o[1]);
                o[3] = mx_mma(Ah1, B[kParts - 1][w0 + 1], o[3]);
            }
        };
        /* every LDS read of the step's A operands before its first MFMA; each column reads its
         * scales after its tiles (the Y column after a fence on the chroma products) */
        const mx_u2 y00 = *(const mx_u2 *)(sp + aoff);
        const mx_u2 y01 = *(const mx_u2 *)(sp + aoff + 768u);
        const mx_u2 y10 = *(const mx_u2 *)(sp + aoff + 96u);
        const mx_u2 y11 = *(const mx_u2 *)(sp + aoff + 864u);
        mx_u2 c00, c01, c10, c11;
        if (__builtin_expect(qmask == 0, 1)) {
            c00 = *(const mx_u2 *)(sp + coff0);
            c01 = *(const mx_u2 *)(sp + coff0 + 768u);
            c10 = *(const mx_u2 *)(sp + coff1);
            c11 = *(const mx_u2 *)(sp + coff1 + 768u);
        } else {
            const unsigned l = mx_lane(), mm = l & 15u, qq = l >> 4, cb = mm >> 2;
            const bool qb = (qmask >> cb) & 1u;
            const uint8_t *qt = L.qtrue[cb] + 24u * (mm & 3u);
            const uint8_t *p0 = qb && qq == 3 ? qt : sp + coff0;
            const uint8_t *p1 = qb && qq < 2 ? qt + 8u + 8u * qq : sp + coff1;
            const unsigned h0 = qb && qq == 3 ? 96u : 768u, h1 = qb && qq < 2 ? 96u : 768u;
            c00 = *(const mx_u2 *)p0;
            c01 = *(const mx_u2 *)(p0 + h0);
            c10 = *(const mx_u2 *)p1;
            c11 = *(const mx_u2 *)(p1 + h1);
        }
        /* every A operand is built before the first product, so no VALU write falls between a
         * chain's products and the read of its results (the C inputs need no keeping, mx_keep) */
        const mx_h8 Ay0 = mx_aop(y00, s0, s1, s2), Ay1 = mx_aop(y01, s0, s1, s2);
        const mx_h8 Ay2 = mx_aop(y10, s0, s1, s2), Ay3 = mx_aop(y11, s0, s1, s2);
        const mx_h8 Ac0 = mx_aop(c00, kSelLo, kSelHi, kSelLo), Ac1 = mx_aop(c01, kSelLo, kSelHi, kSelLo);
        const mx_h8 Ac2 = mx_aop(c10, t0, t1, t2), Ac3 = mx_aop(c11, t0, t1, t2);
        __builtin_amdgcn_sched_barrier(0);
        mma2(acc[0], mid[0], Ay0, Ay1, Ay2, Ay3, 0);
        __builtin_amdgcn_sched_barrier(0);
        mma2(acc[1], mid[1], Ac0, Ac1, Ac2, Ac3, 2);
        mx_gap();
        __builtin_amdgcn_sched_barrier(0);
        /* the Y column fences on the chroma products: after it, every chain of the step is done */
        const auto keep422 = [&]() __attribute__((always_inline)) {
            mx_keep(mid[1]);
            mx_keep_ops(Ay2, Ay3, Ac2, Ac3, B[0][1], B[1][1], B[0][3], B[1][3]);
        };
        mx_column_t<0, true>(acc[0], MxW{}, limc0, tb, 0, j, za, fl, 0, &acc[1][3], keep422);
        __builtin_amdgcn_sched_barrier(0);
        mx_column_t<kSt422C, true>(acc[1], MxW{}, limc2, tb, 2, j, za, fl, 1);
        mx_wave_sync();
        if (__builtin_expect(__ballot(fl != 0) != 0, 0)) {
            if (S.b + 8u > g.total) {                  /* clamped copies past the end */
                const unsigned nvalid = g.total - S.b;
                if (mx422_yblock(lane) >= nvalid) fl &= ~0xffu;
                if (2u * (lane >> 4) >= nvalid) fl &= ~0xff00u;
            }
            mx422_exact_inline(L, sp, qmask, fl, T);
        }
        /* always two store instructions (the vmcnt accounting counts on it) */
        if (S.simple) {
            const mx_u4 vy = *(const mx_u4 *)(L.stage + ro);
            const mx_u4 vc = *(const mx_u4 *)(L.stage + kSt422C + ro);
            __builtin_nontemporal_store(vy, (mx_u4 *)((const uint8_t *)S.dst + soy));
            __builtin_nontemporal_store(vc, (mx_u4 *)((const uint8_t *)S.cdst + soc));
        } else {
            const unsigned l = mx_lane();
            const unsigned by = S.b + (l >> 3), bc = S.b + 2u * ((l >> 3) & 3u);
            const unsigned yb = by < g.total ? by : g.total - 1u, cbk = bc < g.total ? bc : g.total - 1u;
            const unsigned fy = yb / g.nb, biy = yb - fy * g.nb;
            const unsigned fc = cbk / g.nb, bic = cbk - fc * g.nb;
            const uint32_t rl = (l >> 3) * kBS + (l & 7u) * 16u;
            const mx_u4 vy = *(const mx_u4 *)(L.stage + rl);
            const mx_u4 vc = *(const mx_u4 *)(L.stage + kSt422C + rl);
            if (by < g.total)
                __builtin_nontemporal_store(
                    vy, (mx_u4 *)(g.out + (long long)fy * g.ofstride + (long long)biy * 64 + (l & 7u) * 8));
            if (bc < g.total)
                __builtin_nontemporal_store(
                    vc, (mx_u4 *)(g.out + (long long)fc * g.ofstride +
                                  ((long long)g.nb + (l >> 5) * (g.nb / 2u) + bic / 2u) * 64 + (l & 7u) * 8));
        }
        mx_wave_sync();
    };
    const auto step = [&](auto kc) __attribute__((always_inline)) {
        constexpr unsigned k = decltype(kc)::value;
        if (cmp.b >= g.total) return;
        mx_wait_vm<2 * (kMxs422C - 1 - k) + 2 * k>();
        if (kMxs422WPG == 1) mx_dmabar();
        body(cmp, L.ring[k]);
        mxs_next(cmp, g);
    };
    step(std::integral_constant<unsigned, 0>{});
    step(std::integral_constant<unsigned, 1>{});
    step(std::integral_constant<unsigned, 2>{});
}

/* ==== k_mx420: true 4:2:0 (extension, JPGX_FLAG_SUBSAMPLE, sample_ratio 2) ==================
 *
 * A step is two consecutive MCUs (MCU-linear launch-global index, frames concatenated): their
 * 16 pixel rows x 96 bytes (8 Y blocks: the top block row of the two MCUs is set 0, the bottom
 * one set 1) land in a 1.5-KiB ring slot by the same LDS-DMA as k_mx; chunks of 6 steps (12
 * MCUs) grid-stride, the ring's three slots holding step k in slot k % 3.
 *   Y       k_mx422's Y: the two sets K-concatenated, column j = set j / 8 at u = j % 8.
 *   Chroma  A row m = (MCU cb = m >> 3, chroma row Y' = m & 7), K = the 96 bytes of the MCU's
 *           pixel rows 2Y', 2Y'+1 over three K = 32 products; B (jpgx_plan.cpp
 *           jx_mx420_operands) holds 0.25 a[c][p] cos((2 floor(x/2) + 1) u pi/16): column j of
 *           the one C tile is the row transform of the quad-averaged chroma, Cb (j < 8) or Cr, at
 *           rows 4gq..4gq+3 of the tile.  Two consecutive steps form a pair: after the second,
 *           one v_permlane16_swap per row value gives every lane a whole column of one of the
 *           pair's four MCUs (lane gq: MCU (gq & 1) 2 + (gq >> 1) of the pair), so the chroma
 *           column DCTs run once per pair on all 64 lanes: 1.5 column passes per step.
 *   Output  per step 8 Y blocks in one store (lanes 0..31 the top row, 32..63 the bottom row,
 *           bpr blocks further); per pair 4 Cb + 4 Cr blocks in one store (the first step of a
 *           pair issues a padding operation instead, so every step counts two).
 *   Quirk   a general step whose MCU's right block column is a row's last loads that column's
 *           true pixel rows into L.qtrue for the chroma A operands.
 *   Exact   Y tasks as k_mx422's (pixels copied from the slot); chroma tasks carry the MCU index
 *           and read its pixels from global memory at flush time (the pair's first slot is gone
 *           by then), in the oracle's order: ((ls(p00) + ls(p01)) + (ls(p10) + ls(p11))) * 0.25.
 */
constexpr unsigned kSteps420 = 6;             /* steps per chunk (3 pairs); ring slot = k % 3 */
constexpr unsigned kCM420 = 2 * kSteps420;    /* MCUs per chunk */
constexpr unsigned kVmWait420 = 4 * kDist - 2;
constexpr int kWaitImm420 = (int)((kVmWait420 & 15u) | ((kVmWait420 >> 4) << 14) | 0xF70u);
constexpr unsigned kSt420C = 8 * kBS;         /* chroma (c, lane group gq) at kSt420C + kBS (4 c + gq) */
#ifndef JX_MX420_WPE
#define JX_MX420_WPE 4
#endif

struct alignas(16) Mx420Lds {
    uint8_t ring[3][kSlot];             /* [y 0..15][4 blocks x 24 B] */
    uint8_t stage[16 * kBS];
    uint8_t qtrue[2][384];              /* general step: MCU's right column, true rows [16][24] */
    uint8_t pix[kSide][192];            /* deferred Y blocks' pixel rows [y][24] */
    uint32_t sblk[kSide];               /* their launch-global Y block (frame-concatenated) */
    uint32_t tmcu[kSide];               /* chroma task: launch-global MCU */
    uint16_t dtask[kSide];              /* a flagged column: slot << 13 | ch << 11 | u << 8 | v-mask
                                           (chroma: ch 1 / 2, its MCU in tmcu) */
    uint16_t task[8];
    uint32_t dummy[64];
};
static_assert(sizeof(Mx420Lds) % 16 == 0 && sizeof(Mx420Lds) * 4 + sizeof(MxTab) <= 40 * 1024,
              "4 workgroups of 4 waves per CU, 16-byte aligned regions");

__device__ mx_u4 g_mx420B[JX_MX_PARTS * 5][64];  /* [part * 5 + which][lane] */
__device__ jx_mxtab g_mx420tab[2][JX_MAXQ + 1];

/* MCU geometry of the launch */
struct Mx420G {
    unsigned mpr, nmcu, tm, rows;       /* MCUs per row, per frame, in the launch; MCU rows per frame */
    jx_udiv dmpr, dnmcu;                /* division by mpr, nmcu (jx_geom) */
};

struct Mx420Chunk {
    unsigned m0, f, mi, my, mx;         /* first MCU (launch-global), frame, MCU in frame, row, col */
    const uint8_t *src;                 /* pixel (16 mx, 16 my) of frame f */
    int16_t *ydst, *cdst;               /* Y block (2my, 2mx), chroma block mi (Cb) of frame f */
    bool simple;
};

__device__ __forceinline__ void mx420_ptrs(Mx420Chunk &C, const MxG &g, const Mx420G &h)
{
    C.src = g.rgb + (long long)C.f * g.fstride + 16ll * C.my * g.pitch + 48ll * C.mx;
    C.ydst = g.out + (long long)C.f * g.ofstride + 64ll * (2ull * C.my * g.bpr + 2u * C.mx);
    C.cdst = g.out + (long long)C.f * g.ofstride + 64ll * (g.nb + C.mi);
    C.simple = C.m0 + kCM420 <= h.tm && C.mx + kCM420 < h.mpr && g.lin_store;
}

__device__ __forceinline__ void mx420_at(Mx420Chunk &C, const MxG &g, const Mx420G &h, unsigned m0)
{
    C.m0 = m0;
    C.f = mx_udiv(m0, h.dnmcu);
    C.mi = m0 - C.f * h.nmcu;
    C.my = mx_udiv(C.mi, h.dmpr);
    C.mx = C.mi - C.my * h.mpr;
    mx420_ptrs(C, g, h);
}

__device__ __forceinline__ void mx420_next(Mx420Chunk &C, const MxG &g, const Mx420G &h, const MxJump &J)
{
    C.m0 += J.jb;
    if (C.m0 >= h.tm) return;
    C.mi += J.jb;
    C.mx += J.jc;
    C.my += J.jr;
    if (C.mx >= h.mpr) {
        C.mx -= h.mpr;
        C.my++;
    }
    while (C.mi >= h.nmcu) {
        C.mi -= h.nmcu;
        C.my -= h.rows;
        C.f++;
    }
    mx420_ptrs(C, g, h);
}

/* Position of the launch-global MCU m: frame, MCU in frame, row, column */
__device__ __forceinline__ void mx420_mcu(const Mx420G &h, unsigned m, unsigned &f, unsigned &mi,
                                          unsigned &my, unsigned &mx)
{
    f = mx_udiv(m, h.dnmcu);
    mi = m - f * h.nmcu;
    my = mx_udiv(mi, h.dmpr);
    mx = mi - my * h.mpr;
}

/* A general step's pixels (row / frame crossings, a row's last MCU, the launch's end): lane l
 * loads pixel row y = l & 15 of block column jb = l >> 4 (MCU m0 + jb / 2, its column jb % 2)
 * with the reference's addressing (the x0 = -8 quirk for the row's last block, the underflow
 * bytes at frame block-row 0) into the slot; MCUs past the launch's end are clamped copies. */
__device__ __forceinline__ void mx420_issue_general(const MxG &g, const Mx420G &h, unsigned m0, uint8_t *slot)
{
    const unsigned lane = mx_lane(), y = lane & 15u, jb = lane >> 4;
    unsigned m = m0 + (jb >> 1);
    m = m < h.tm ? m : h.tm - 1u;
    unsigned f, mi, my, mx;
    mx420_mcu(h, m, f, mi, my, mx);
    const unsigned br = 2u * my + (y >> 3), bc = 2u * mx + (jb & 1u), yy = y & 7u;
    const bool last = bc == g.bpr - 1u;
    const bool under = last && yy == 0 && g.row0 + (int)br == 0;
    const long long prow = under ? 8ll * br : 8ll * br + yy - (last ? 1 : 0);
    typedef const __attribute__((address_space(1))) mx_u2 gu2;
    const gu2 *src = (const gu2 *)(g.rgb + (long long)f * g.fstride + prow * g.pitch + 24ll * bc);
    mx_u2 v0 = src[0], v1 = src[1], v2 = src[2];
    if (under) {
        v0 = mx_u2{g.u[0], g.u[1]};
        v1 = mx_u2{g.u[2], g.u[3]};
        v2 = mx_u2{g.u[4], g.u[5]};
    }
    uint8_t *d = slot + 96u * y + 24u * jb;
    *(mx_u2 *)d = v0;
    *(mx_u2 *)(d + 8) = v1;
    *(mx_u2 *)(d + 16) = v2;
    __builtin_amdgcn_s_waitcnt(0xF70);                 /* vmcnt(0) (rare; conservative) */
}

/* a general step's MCUs whose right block column is a row's last: its true pixel rows (16 x 24 B)
 * into L.qtrue[MCU of the step]; returns the mask of those MCUs */
template <class Lds>
__device__ __forceinline__ uint32_t mx420_true_rows(Lds &L, const MxG &g, const Mx420G &h, unsigned m0)
{
    const unsigned l = mx_lane(), y = l & 15u, ms = (l >> 4) & 1u;
    const unsigned m = m0 + ms;
    bool last = false;
    unsigned f = 0, mi = 0, my = 0, mx = 0;
    if (l < 32 && m < h.tm) {
        mx420_mcu(h, m, f, mi, my, mx);
        last = 2u * mx + 1u == g.bpr - 1u;
    }
    const uint64_t bal = __ballot(last && y == 0);
    const uint32_t qm = (uint32_t)(bal & 1u) | (uint32_t)((bal >> 16) & 1u) << 1;
    if (qm) {
        if (last) {
            typedef const __attribute__((address_space(1))) mx_u2 gu2;
            const gu2 *src = (const gu2 *)(g.rgb + (long long)f * g.fstride + (16ll * my + y) * g.pitch +
                                           24ll * (2u * mx + 1u));
            const mx_u2 v0 = src[0], v1 = src[1], v2 = src[2];
            uint8_t *d = L.qtrue[ms] + 24u * y;
            *(mx_u2 *)d = v0;
            *(mx_u2 *)(d + 8) = v1;
            *(mx_u2 *)(d + 16) = v2;
        }
        __builtin_amdgcn_s_waitcnt(0xF70);
        mx_wave_sync();
    }
    return qm;
}

/* One exact chroma coefficient per 8-lane group from the MCU's pixels in global memory: lane x
 * averages the quad ((ls(p00) + ls(p01)) + (ls(p10) + ls(p11))) * 0.25 of chroma row y
 * (oracle/cpu_ref.c cpuref_chroma_sample), then as mx_exact_coef.  row0 = the MCU's pixel (0, 0).
 * Valid in lane x == 7. */
template <bool FAST = (JX_MX_FASTEXACT != 0)>
__device__ __forceinline__ int mx_exact_quad(const uint8_t *row0, long long pitch, unsigned ch, unsigned u,
                                             unsigned v, unsigned x, const jx_mxtab &T)
{
    const double cu = kMxCos[u][x];
    const double k0c = kMxColour[ch][0], k1c = kMxColour[ch][1], k2c = kMxColour[ch][2];
    const double Ac = kMxColour[ch][3], Sc = kMxColour[ch][4];
    double prod[8];
#pragma unroll
    for (int y = 0; y < 8; y++) {
        const uint8_t *p = row0 + (2ll * y) * pitch + 6u * x, *q = p + pitch;
        const double l00 = (Ac + Sc * ((k0c * (double)p[0] + k1c * (double)p[1]) + k2c * (double)p[2])) - 128.0;
        const double l01 = (Ac + Sc * ((k0c * (double)p[3] + k1c * (double)p[4]) + k2c * (double)p[5])) - 128.0;
        const double l10 = (Ac + Sc * ((k0c * (double)q[0] + k1c * (double)q[1]) + k2c * (double)q[2])) - 128.0;
        const double l11 = (Ac + Sc * ((k0c * (double)q[3] + k1c * (double)q[4]) + k2c * (double)q[5])) - 128.0;
        const double X = ((l00 + l01) + (l10 + l11)) * 0.25;
        prod[y] = X * cu * kMxCos[v][y];
    }
    return mx_exact_sum<FAST>(prod, ch, u, v, x, T, T.r[ch == 0 ? 0 : 1][u * 8 + v]);
}

/* the MCU's pixel (0, 0) */
__device__ __forceinline__ const uint8_t *mx420_mcu_src(const MxG &g, const Mx420G &h, unsigned m)
{
    unsigned f, mi, my, mx;
    mx420_mcu(h, m, f, mi, my, mx);
    return g.rgb + (long long)f * g.fstride + 16ll * my * g.pitch + 48ll * mx;
}

/* pair-MCU of a chroma-column lane group (the permlane16 swap's order) */
__device__ __forceinline__ unsigned mx420_pm(unsigned gq) { return (gq & 1u) * 2u + (gq >> 1); }

/* Inline exact pass: Y bits (col 0) of this step and chroma bits (col 1, pair base mp) */
template <class Lds>
__device__ __forceinline__ void mx420_exact_inline(Lds &L, const uint8_t *sp, uint32_t bits, unsigned mp,
                                                   const MxG &g, const Mx420G &h, const jx_mxtab &T)
{
    const unsigned lane = mx_lane();
    mx_wave_sync();
    for (;;) {
        const uint64_t act = __ballot(bits != 0);
        if (!act) break;
        const int rk = mx_rank(act);
        if (bits != 0 && rk < 8) {
            const unsigned b = (unsigned)__builtin_ctz(bits);
            bits &= bits - 1u;
            L.task[rk] = (uint16_t)(lane << 8 | b);
        }
        mx_wave_sync();
        const int nt = std::min((int)__popcll(act), 8);
        const unsigned i = lane >> 3, x = lane & 7u;
        const bool live = (int)i < nt;
        const unsigned code = L.task[live ? i : 0u];
        const unsigned sl = code >> 8, k = (code >> 3) & 1u, v = code & 7u;
        const unsigned jj = sl & 15u, u = jj & 7u, gq = sl >> 4;
        const unsigned slot = 4u * (jj >> 3) + gq;     /* Y: set (j / 8), block gq; chroma: (c, gq) */
        int val;
        if (k == 0) {
            val = mx_exact_pair(mx_lds((void *)sp) + 96u * 8u * (jj >> 3) + 24u * gq + 3u * x, 96u, 0u, 0u, u, v,
                                x, T);
        } else {
            unsigned m = mp + mx420_pm(gq);
            m = m < h.tm ? m : h.tm - 1u;
            val = mx_exact_quad(mx420_mcu_src(g, h, m), g.pitch, 1u + (jj >> 3), u, v, x, T);
        }
        if (live && x == 7)
            *(__attribute__((address_space(3))) int16_t *)(mx_lds(L.stage) + (k ? kSt420C : 0u) + kBS * slot +
                                                           2u * (unsigned)kMxScan[v][u]) = (int16_t)val;
        mx_wave_sync();
    }
}

__device__ __forceinline__ void mx420_flush(Mx420Lds &L, int &nq, int &ns, const MxG &g, const Mx420G &h,
                                            const jx_mxtab &T)
{
    __builtin_amdgcn_s_waitcnt(0xF70);                 /* vmcnt(0): the tasks' blocks are stored */
    mx_wave_sync();
    const unsigned lane = mx_lane(), i = lane >> 3, x = lane & 7u;
    const bool live = (int)i < nq;
    const unsigned code = L.dtask[live ? i : 0u];
    const unsigned slot = code >> 13, ch = (code >> 11) & 3u, u = (code >> 8) & 7u;
    uint32_t vb = live ? (code & 0xffu) : 0u;
    long long dst;
    const uint8_t *src = g.rgb;
    if (ch) {
        const unsigned m = L.tmcu[live ? i : 0u];
        unsigned f, mi, my, mx;
        mx420_mcu(h, m, f, mi, my, mx);
        src = g.rgb + (long long)f * g.fstride + 16ll * my * g.pitch + 48ll * mx;
        dst = (long long)f * g.ofstride + ((long long)g.nb + (ch - 1u) * h.nmcu + mi) * 64;
    } else {
        const unsigned b = L.sblk[slot], f = b / g.nb, bi = b - f * g.nb;
        dst = (long long)f * g.ofstride + (long long)bi * 64;
    }
    while (__ballot(vb != 0)) {
        const bool act = vb != 0;
        const unsigned v = act ? (unsigned)__builtin_ctz(vb) : 0u;
        vb &= vb - 1u;
        const int val = ch ? mx_exact_quad<false>(src, g.pitch, ch, u, v, x, T)   /* legacy k_mx420 */
                           : mx_exact_pair<false>(mx_lds(L.pix[slot]) + 3u * x, 24u, 0u, 0u, u, v, x, T);
        if (act && x == 7) g.out[dst + kMxScan[v][u]] = (int16_t)val;
    }
    mx_wave_sync();
    nq = 0;
    ns = 0;
}

/* Y block (launch-global, frame-concatenated) of step m0's block (set, jb) */
__device__ __forceinline__ unsigned mx420_yblock(const MxG &g, const Mx420G &h, unsigned m0, unsigned set,
                                                 unsigned jb)
{
    unsigned f, mi, my, mx;
    mx420_mcu(h, m0 + (jb >> 1), f, mi, my, mx);
    return f * g.nb + (2u * my + set) * g.bpr + 2u * mx + (jb & 1u);
}

/* Queue a step's flagged coefficients: bits 0..7 Y (this step's blocks), 8..15 chroma (pair base
 * mp, only on a pair's second step) */
__device__ __forceinline__ void mx420_defer(Mx420Lds &L, const uint8_t *sp, uint32_t bits, unsigned m0, unsigned mp,
                                            int &nq, int &ns, const MxG &g, const Mx420G &h, const jx_mxtab &T)
{
    const unsigned lane = mx_lane();
    {   /* clamped MCUs past the launch's end: no tasks (Y block (set, gq) is MCU m0 + gq / 2) */
        const unsigned gq = lane >> 4;
        if (m0 + (gq >> 1) >= h.tm) bits &= ~0xffu;
        if (mp + mx420_pm(gq) >= h.tm) bits &= ~0xff00u;
    }
    const uint64_t m0b = __ballot((bits & 0xffu) != 0);
    uint32_t yblk = 0;
#pragma unroll
    for (int gq = 0; gq < 4; gq++) {
        yblk |= (((m0b >> (16 * gq)) & 0xffu) ? 1u : 0u) << gq;              /* set 0, block gq */
        yblk |= (((m0b >> (16 * gq + 8)) & 0xffu) ? 1u : 0u) << (4 + gq);    /* set 1 */
    }
    const uint64_t m1b = __ballot((bits & 0xff00u) != 0);
    const int n0 = __popcll(m0b), ncol = n0 + __popcll(m1b);
    const int ny = __popc(yblk);
    if (nq + ncol > kSide || ns + ny > kSide) {
        if (nq) mx420_flush(L, nq, ns, g, h, T);
        if (ncol > kSide) {
            mx420_exact_inline(L, sp, bits, mp, g, h, T);
            return;
        }
    }
    {   /* Y blocks' pixel rows to side slots (lane < 48: row l / 6, dword l % 6) */
        const unsigned y = lane / 6u, k = lane - 6u * y;
        uint32_t bm = yblk;
        int t = ns;
        while (bm) {
            const unsigned yb = (unsigned)__builtin_ctz(bm), set = yb >> 2, jb = yb & 3u;
            bm &= bm - 1u;
            if (lane < 48)
                *(__attribute__((address_space(3))) uint32_t *)(mx_lds(L.pix[t]) + 24u * y + 4u * k) =
                    *(const __attribute__((address_space(3))) uint32_t *)(mx_lds((void *)sp) + 96u * (8u * set + y) +
                                                                          24u * jb + 4u * k);
            if (lane == 0) L.sblk[t] = mx420_yblock(g, h, m0, set, jb);
            t++;
        }
    }
    {   /* this lane's flagged columns (Y first, then chroma), one queue entry each */
        const unsigned jj = lane & 15u, u = jj & 7u, gq = lane >> 4;
        const uint32_t vy = bits & 0xffu, vc = (bits >> 8) & 0xffu;
        if (vy) {
            const unsigned yb = 4u * (jj >> 3) + gq;
            const unsigned slot = (unsigned)ns + (unsigned)__popc(yblk & ((1u << yb) - 1u));
            L.dtask[nq + mx_rank(m0b)] = (uint16_t)(slot << 13 | u << 8 | vy);
        }
        if (vc) {
            const unsigned pos = (unsigned)(nq + n0) + (unsigned)mx_rank(m1b);
            L.dtask[pos] = (uint16_t)((1u + (jj >> 3)) << 11 | u << 8 | vc);
            L.tmcu[pos] = mp + mx420_pm(gq);
        }
    }
    mx_wave_sync();
    nq += ncol;
    ns += ny;
}

__global__ __launch_bounds__(256, JX_MX420_WPE) void k_mx420(const jx_xform_args a)
{
    __shared__ __attribute__((aligned(16))) Mx420Lds s_lds[4];
    __shared__ __attribute__((aligned(16))) MxTab s_tab;
    MxG g;
    g.rgb = a.g.rgb;
    g.out = a.g.out;
    g.pitch = a.g.in_pitch;
    g.fstride = a.g.in_fstride;
    g.ofstride = a.g.out_fstride;
    g.bpr = (unsigned)a.g.bpr;
    g.nb = (unsigned)a.g.nb;
    g.total = (unsigned)a.g.nb * (unsigned)a.g.nframes;
    g.row0 = a.g.row0;
    g.quality = a.quality;
    g.force = a.force_exact;
    g.lin_store = (unsigned long long)g.nb * 256ull + 1024ull < (1ull << 31);
#pragma unroll
    for (int k = 0; k < 6; k++) g.u[k] = a.g.under[k];
    g.dnb = a.g.dnb;
    g.dbpr = a.g.dbpr;
    Mx420G h;
    h.mpr = a.g.mpr;
    h.nmcu = a.g.nmcu;
    h.rows = mx_udiv(h.nmcu, a.g.dmpr);
    h.tm = h.nmcu * (unsigned)a.g.nframes;
    h.dmpr = a.g.dmpr;
    h.dnmcu = a.g.dnmcu;

    const unsigned lane = threadIdx.x & 63u;
    Mx420Lds &L = s_lds[threadIdx.x >> 6];
    const jx_mxtab &T = g_mx420tab[g.force ? 1 : 0][g.quality];
    if (threadIdx.x < 64) {
        const unsigned t = lane >> 4, jp = lane & 15u;
        const unsigned n = t < 2 ? (jp & 7u) : 8u + jp;
        float x[8];
#pragma unroll
        for (int p = 0; p < 4; p++)
#pragma unroll
            for (int hh = 0; hh < 2; hh++) {
                const int v = jx_pk_k(p, hh);
                x[2 * p + hh] = (t & 1u) ? T.lsq[n][v] : T.w[n][v];
            }
        s_tab.wl[t][0][jp] = mx_f4{x[0], x[1], x[2], x[3]};
        s_tab.wl[t][1][jp] = mx_f4{x[4], x[5], x[6], x[7]};
    }
    __syncthreads();
    /* hot-path band limits of this lane's two column kinds (mx_limc) */
    const float limc0 = mx_limc(s_tab, 1, threadIdx.x & 15u), limc2 = mx_limc(s_tab, 3, threadIdx.x & 15u);
    const unsigned nw = gridDim.x * 4u;
    const unsigned wv = __builtin_amdgcn_readfirstlane(blockIdx.x * 4u + (threadIdx.x >> 6));
    if (kCM420 * wv >= h.tm) return;

    /* Y A operand: row m = 4 jb + y' (block jb of the set, pixel row y' of the half), k-group q
     * (bytes 8q.. of the block row; q = 3 the bias); set s / half hh at +768 s + 384 hh.
     * Chroma A operand: row m = (MCU cb = m >> 3, chroma row Y' = m & 7); k-step 0: bytes 8q.. of
     * pixel row 2Y' (48 cb + ..), k-step 1: bytes 32 + 8q (q < 2) of row 2Y', bytes 8 (q - 2) of
     * row 2Y' + 1 (q >= 2), k-step 2: bytes 16 + 8q of row 2Y' + 1 */
    const unsigned m = lane & 15u, q = lane >> 4;
    const uint32_t aoff = 96u * (m & 3u) + 24u * (m >> 2) + 8u * (q < 3 ? q : 0u);
    const uint32_t s0 = q < 3 ? kSelLo : kSelOne;
    const uint32_t s1 = q < 3 ? kSelHi : kSelZero;
    const uint32_t s2 = q < 3 ? kSelLo : kSelZero;
    const uint32_t cof0 = 192u * (m & 7u) + 48u * (m >> 3) + 8u * q;
    const uint32_t cof1 = cof0 + (q < 2 ? 32u : 80u);
    const uint32_t off0 = (uint32_t)((lane / 6u) * (unsigned)g.pitch + 16u * (lane % 6u));
    const uint32_t off1 = (uint32_t)(((64u + lane) / 6u) * (unsigned)g.pitch + 16u * ((64u + lane) % 6u));
    /* stores: Y lanes 0..31 the top block row's 4 blocks, 32..63 the bottom row's; chroma lanes
     * 0..31 Cb of the pair's 4 MCUs, 32..63 Cr; stage reads at ro (Y) and rc (chroma: lane group
     * gq of the column pass holds pair-MCU mx420_pm(gq), an involution) */
    const uint32_t soy = (lane & 31u) * 16u + (lane >> 5) * g.bpr * 128u;
    const uint32_t soc = (lane & 31u) * 16u + (lane >> 5) * h.nmcu * 128u;
    const uint32_t ro = (lane >> 3) * kBS + (lane & 7u) * 16u;
    const uint32_t rc = kSt420C + kBS * (4u * (lane >> 5) + mx420_pm((lane >> 3) & 3u)) + (lane & 7u) * 16u;

    const unsigned gq = lane >> 4, j = lane & 15u, u = j & 7u;
    uint32_t za[8];
    {
        const uint32_t base = (uint32_t)(uintptr_t)mx_lds(L.stage) + kBS * (4u * (j >> 3) + gq);
#pragma unroll
        for (int v = 0; v < 8; v++) za[v] = base + 2u * (unsigned)kMxScan[v][u];
    }
    mx_u4 B[kParts][5];
#pragma unroll
    for (int p = 0; p < kParts; p++)
#pragma unroll
        for (int w = 0; w < 5; w++) B[p][w] = g_mx420B[5 * p + w][lane];
    __builtin_amdgcn_s_waitcnt(0xF70);              /* see k_mx422 */

    MxJump J;
    J.jb = kCM420 * nw;
    J.jr = J.jb / h.mpr;
    J.jc = J.jb - J.jr * h.mpr;
    J.rows = h.rows;
    Mx420Chunk cc;
    mx420_at(cc, g, h, kCM420 * wv);
    Mx420Chunk nx = cc;

    const auto issue = [&](const Mx420Chunk &C, unsigned k) {
        uint8_t *const slot = L.ring[k % 3u];
        const unsigned m0 = C.m0 + 2u * k;
        if (m0 >= h.tm) {
            mx_pad(g, L, 2);
        } else if (C.simple) {
            const uint8_t *base = C.src + 96u * k;
            __builtin_amdgcn_global_load_lds((mx_gp)(base + off0), (mx_lp)slot, 16, 0, 0);
            if (lane < 32) __builtin_amdgcn_global_load_lds((mx_gp)(base + off1), (mx_lp)(slot + 1024u), 16, 0, 0);
        } else {
            mx420_issue_general(g, h, m0, slot);
        }
    };
    for (unsigned d = 0; d < kDist; d++) {
        issue(cc, d);
        mx_pad(g, L, 2);
    }
    int nq = 0, ns = 0;
    unsigned k = 0;
    mx_f4 rA = {};                                 /* chroma R of the pair's first step */
    for (;;) {
        const unsigned m0 = cc.m0 + 2u * k;
        __builtin_amdgcn_s_waitcnt(kWaitImm420);
        mx_wave_sync();
        const uint8_t *const sp = L.ring[k % 3u];
        if (k + kDist < kSteps420) {
            issue(cc, k + kDist);
        } else {
            if (k + kDist == kSteps420) mx420_next(nx, g, h, J);
            issue(nx, k + kDist - kSteps420);
        }
        const uint32_t qmask = cc.simple ? 0u : mx420_true_rows(L, g, h, m0);
        const mx_f4 z = {};
        uint32_t fl = 0;
        mx_f4 accY[4], accC[2];
        const mx_u2 y00 = *(const mx_u2 *)(sp + aoff);
        const mx_u2 y01 = *(const mx_u2 *)(sp + aoff + 384u);
        const mx_u2 y10 = *(const mx_u2 *)(sp + aoff + 768u);
        const mx_u2 y11 = *(const mx_u2 *)(sp + aoff + 1152u);
        mx_u2 c0, c1, c2;
        if (__builtin_expect(qmask == 0, 1)) {
            c0 = *(const mx_u2 *)(sp + cof0);
            c1 = *(const mx_u2 *)(sp + cof1);
            c2 = *(const mx_u2 *)(sp + cof0 + 112u);
        } else {
            /* MCUs whose right block column is a row's last: bytes 24..47 of a 48-byte MCU row
             * from the true rows (k-step 0: q = 3; k-step 1: q < 2; k-step 2: q >= 1) */
            const unsigned l = mx_lane(), mm = l & 15u, qq = l >> 4, cb = mm >> 3, yr = 2u * (mm & 7u);
            const bool qb = (qmask >> cb) & 1u;
            const uint8_t *qt = L.qtrue[cb];
            const uint8_t *p0 = qb && qq == 3 ? qt + 24u * yr : sp + cof0;
            const uint8_t *p1 = qb && qq < 2 ? qt + 24u * yr + 8u + 8u * qq : sp + cof1;
            const uint8_t *p2 = qb && qq >= 1 ? qt + 24u * (yr + 1u) + 8u * (qq - 1u) : sp + cof0 + 112u;
            c0 = *(const mx_u2 *)p0;
            c1 = *(const mx_u2 *)p1;
            c2 = *(const mx_u2 *)p2;
        }
        /* A operands before the first MFMA; each column reads its scales after its tiles (the Y
         * column after a fence on the chroma products) (MFMA operand rule, mx_fence) */
        __builtin_amdgcn_sched_barrier(0);
        {
            const mx_h8 Al0 = mx_aop(y00, s0, s1, s2), Ah0 = mx_aop(y01, s0, s1, s2);
            const mx_h8 Al1 = mx_aop(y10, s0, s1, s2), Ah1 = mx_aop(y11, s0, s1, s2);
            accY[0] = mx_mma(Al0, B[0][0], z);
            accY[2] = mx_mma(Ah0, B[0][0], z);
            accY[1] = mx_mma(Al0, B[1][0], z);
            accY[3] = mx_mma(Ah0, B[1][0], z);
            accY[0] = mx_mma(Al1, B[0][1], accY[0]);
            accY[2] = mx_mma(Ah1, B[0][1], accY[2]);
            accY[1] = mx_mma(Al1, B[1][1], accY[1]);
            accY[3] = mx_mma(Ah1, B[1][1], accY[3]);
            if (kParts == 3) {
                accY[1] = mx_mma(Al0, B[kParts - 1][0], accY[1]);
                accY[3] = mx_mma(Ah0, B[kParts - 1][0], accY[3]);
                accY[1] = mx_mma(Al1, B[kParts - 1][1], accY[1]);
                accY[3] = mx_mma(Ah1, B[kParts - 1][1], accY[3]);
            }
        }
        __builtin_amdgcn_sched_barrier(0);
        {
            const mx_h8 C0 = mx_aop(c0, kSelLo, kSelHi, kSelLo), C1 = mx_aop(c1, kSelLo, kSelHi, kSelLo);
            const mx_h8 C2 = mx_aop(c2, kSelLo, kSelHi, kSelLo);
            accC[0] = mx_mma(C0, B[0][2], z);
            accC[1] = mx_mma(C0, B[1][2], z);
            accC[0] = mx_mma(C1, B[0][3], accC[0]);
            accC[1] = mx_mma(C1, B[1][3], accC[1]);
            accC[0] = mx_mma(C2, B[0][4], accC[0]);
            accC[1] = mx_mma(C2, B[1][4], accC[1]);
            if (kParts == 3) {
                accC[1] = mx_mma(C0, B[kParts - 1][2], accC[1]);
                accC[1] = mx_mma(C1, B[kParts - 1][3], accC[1]);
                accC[1] = mx_mma(C2, B[kParts - 1][4], accC[1]);
            }
        }
        __builtin_amdgcn_sched_barrier(0);
        mx_column_t<0, true>(accY, MxW{}, limc0, s_tab, 0, j, za, fl, 0, &accC[1]);
        __builtin_amdgcn_sched_barrier(0);
        const float sl = JX_MX_LOEXP == 0 ? 1.0f : 0x1p-12f;
        const mx_f4 s12 = {sl, sl, sl, sl};
        const mx_f4 rc4 = JX_MX_LOEXP == 0 ? accC[1] + accC[0] : __builtin_elementwise_fma(accC[1], s12, accC[0]);
        __builtin_amdgcn_sched_barrier(0);
        const bool second = (k & 1u) != 0;
        if (second) {
            /* rows Y' 0..3 / 4..7 of the lane's pair-MCU column: lanes in even 16-lane rows take
             * the first step's tile, odd rows the second's */
            mx_f2 R[4];
            float lo4[4], hi4[4];
#pragma unroll
            for (int i = 0; i < 4; i++) {
                const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(rA[i]), __float_as_uint(rc4[i]),
                                                                false, false);
                lo4[i] = __uint_as_float(r[0]);
                hi4[i] = __uint_as_float(r[1]);
            }
            R[0] = mx_f2{lo4[0], lo4[1]};
            R[1] = mx_f2{lo4[2], lo4[3]};
            R[2] = mx_f2{hi4[0], hi4[1]};
            R[3] = mx_f2{hi4[2], hi4[3]};
            mx_column_r<kSt420C>(R, mx_w(s_tab, 2, j), limc2, s_tab, 2, j, za, fl, 1);
        } else {
            rA = rc4;
        }
        mx_wave_sync();
        const unsigned mp = m0 - 2u;                   /* the pair's first MCU (second step) */
        if (__builtin_expect(__ballot(fl != 0) != 0, 0)) {
            mx420_defer(L, sp, fl, m0, second ? mp : 0u, nq, ns, g, h, T);
            __builtin_amdgcn_s_waitcnt(0xF70);         /* see mx422_defer_step */
        }
        /* always two VMEM operations per step: the Y store, and the chroma store or a pad */
        if (cc.simple) {
            const mx_u4 vy = *(const mx_u4 *)(L.stage + ro);
            __builtin_nontemporal_store(vy, (mx_u4 *)((const uint8_t *)(cc.ydst + 256u * k) + soy));
            if (second) {
                const mx_u4 vc = *(const mx_u4 *)(L.stage + rc);
                __builtin_nontemporal_store(vc, (mx_u4 *)((const uint8_t *)(cc.cdst + 256u * (k >> 1)) + soc));
            } else {
                mx_pad(g, L, 1);
            }
        } else {
            const unsigned l = mx_lane();
            {   /* Y: lane's block (set l >> 5, block column (l >> 3) & 3 of the step) */
                const unsigned jb = (l >> 3) & 3u, mm = m0 + (jb >> 1);
                const unsigned mc = mm < h.tm ? mm : h.tm - 1u;
                const unsigned yb = mx420_yblock(g, h, mc - (jb >> 1), l >> 5, jb);
                const unsigned f = yb / g.nb, bi = yb - f * g.nb;
                const mx_u4 vy = *(const mx_u4 *)(L.stage + (l >> 3) * kBS + (l & 7u) * 16u);
                if (mm < h.tm)
                    __builtin_nontemporal_store(
                        vy, (mx_u4 *)(g.out + (long long)f * g.ofstride + (long long)bi * 64 + (l & 7u) * 8));
            }
            if (second) {
                const unsigned pm = (l >> 3) & 3u, mm = mp + pm;
                const unsigned mc = mm < h.tm ? mm : h.tm - 1u;
                unsigned f, mi, my, mx;
                mx420_mcu(h, mc, f, mi, my, mx);
                const mx_u4 vc = *(const mx_u4 *)(L.stage + kSt420C + kBS * (4u * (l >> 5) + mx420_pm(pm)) +
                                                   (l & 7u) * 16u);
                if (mm < h.tm)
                    __builtin_nontemporal_store(
                        vc, (mx_u4 *)(g.out + (long long)f * g.ofstride +
                                      ((long long)g.nb + (l >> 5) * h.nmcu + mi) * 64 + (l & 7u) * 8));
            } else {
                mx_pad(g, L, 1);
            }
        }
        mx_wave_sync();
        if (++k == kSteps420) {
            k = 0;
            cc = nx;
            if (cc.m0 >= h.tm) break;
        } else if (m0 + 2u >= h.tm && second) {
            break;
        }
    }
    if (nq) mx420_flush(L, nq, ns, g, h, T);
}

/* ==== k_mxs420: k_mx420's transform in short-lived one-wave workgroups (round 4) =============
 *
 * One wave = one step pair (two steps of two MCUs each: 16 Y blocks, 4 Cb + 4 Cr blocks), both
 * steps' DMA up front (slots 0 and 1), the 1.2-KiB per-wave image by LDS-DMA, B operands and band
 * limits from the global image, the exact pass inline on the stage (chroma tasks read their
 * MCU's pixels from global memory, as k_mx420's flush).  Step 0 stores its Y (one operation), step
 * 1 its Y and the pair's chroma: step 0 waits vmcnt(2), step 1 vmcnt(1).
 */
struct alignas(16) Mxs420Lds {
    uint8_t ring[2][kSlot];             /* [y 0..15][4 blocks x 24 B] */
    union {
        uint8_t stage[16 * kBS];
        struct {                        /* general step: MCU's right column, true rows [16][24]; read
                                           for the A operands before the chroma column writes here */
            uint8_t y_[kSt420C];
            uint8_t qtrue[2][384];
        };
    };
    mx_f4 rA[64];                       /* step 0's chroma R (not held across step 0's exact pass) */
    uint16_t task[8];
};
static_assert(2 * 384 <= 16 * kBS - kSt420C, "qtrue inside the chroma stage");
/* waves per workgroup: 1 (B operands from the global image, the scales in the wave's LDS) or 4
 * (the whole image in LDS, shared through one s_barrier) */
#ifndef JX_MXS420_WPG
#define JX_MXS420_WPG 4
#endif
constexpr unsigned kMxs420WPG = JX_MXS420_WPG;
static_assert(kMxs420WPG == 1 || kMxs420WPG == 4 || kMxs420WPG == 8, "1, 4 or 8 waves per workgroup");
struct alignas(16) MxsImg420 {
    mx_u4 B[JX_MX_PARTS * 5][64];
    MxTab tab;
    float limc[2][16];
    uint8_t scan_t[8][8];
};
constexpr unsigned kMxs420Pieces = sizeof(MxsImg420) / 16;
static_assert(sizeof(MxsImg420) % 16 == 0 && kMxs420Pieces <= 1024, "four 16-byte pieces per thread");
static_assert(sizeof(Mxs420Lds) % 16 == 0 &&
                  (kMxs420WPG >= 2 ? sizeof(Mxs420Lds) * kMxs420WPG + sizeof(MxsImg420) <= 160 * 1024 / (16 / kMxs420WPG)
                                   : sizeof(Mxs420Lds) + sizeof(MxsImg1) <= 10 * 1024),
              "16 waves per CU");
__device__ MxsImg420 g_mxs420_img[2][JX_MAXQ + 1];
__device__ MxsImg1 g_mxs420_img1[2][JX_MAXQ + 1];
typedef std::conditional<kMxs420WPG >= 2, MxsImg420, MxsImg1>::type Mxs420Shared;
[[maybe_unused]] __device__ __forceinline__ const mx_u4 (&mxs420_B(const MxsImg420 &l, const MxsImg420 &))[JX_MX_PARTS * 5][64]
{
    return l.B;
}
[[maybe_unused]] __device__ __forceinline__ const mx_u4 (&mxs420_B(const MxsImg1 &, const MxsImg420 &g))[JX_MX_PARTS * 5][64]
{
    return g.B;
}
[[maybe_unused]] __device__ __forceinline__ const MxTab &mxs420_tb(const MxsImg420 &l, const MxsImg420 &) { return l.tab; }
[[maybe_unused]] __device__ __forceinline__ MxsTabRef mxs420_tb(const MxsImg1 &l, const MxsImg420 &g)
{
    return MxsTabRef{l.sc, g.tab};
}

__global__ __launch_bounds__(64 * kMxs420WPG, JX_MX420_WPE) void k_mxs420(const jx_xform_args a)
{
    __shared__ __attribute__((aligned(16))) Mxs420Lds s_lds[kMxs420WPG];
    __shared__ __attribute__((aligned(16))) Mxs420Shared s_img;
    MxG g;
    g.rgb = a.g.rgb;
    g.out = a.g.out;
    g.pitch = a.g.in_pitch;
    g.fstride = a.g.in_fstride;
    g.ofstride = a.g.out_fstride;
    g.bpr = (unsigned)a.g.bpr;
    g.nb = (unsigned)a.g.nb;
    g.total = (unsigned)a.g.nb * (unsigned)a.g.nframes;
    g.row0 = a.g.row0;
    g.quality = a.quality;
    g.force = a.force_exact;
    g.lin_store = (unsigned long long)g.nb * 256ull + 1024ull < (1ull << 31);
#pragma unroll
    for (int k = 0; k < 6; k++) g.u[k] = a.g.under[k];
    g.dnb = a.g.dnb;
    g.dbpr = a.g.dbpr;
    Mx420G h;
    h.mpr = a.g.mpr;
    h.nmcu = a.g.nmcu;
    h.rows = mx_udiv(h.nmcu, a.g.dmpr);
    h.tm = h.nmcu * (unsigned)a.g.nframes;
    h.dmpr = a.g.dmpr;
    h.dnmcu = a.g.dnmcu;

    const unsigned lane = threadIdx.x & 63u;
    const unsigned wave = kMxs420WPG == 1 ? 0u : __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    Mxs420Lds &L = s_lds[wave];
    const MxsImg420 &gimg = g_mxs420_img[g.force ? 1 : 0][g.quality];
    if constexpr (kMxs420WPG >= 2) {
        const uint8_t *img = (const uint8_t *)&gimg;
#pragma unroll
        for (unsigned i = 0; i < (kMxs420Pieces + 64u * kMxs420WPG - 1u) / (64u * kMxs420WPG); i++) {
            const unsigned piece = 64u * kMxs420WPG * i + threadIdx.x;
            if (64u * kMxs420WPG * i + 64u * wave < kMxs420Pieces && piece < kMxs420Pieces)
                mxs_dma<16>(img + 16u * piece, (uint8_t *)&s_img + 16u * (64u * kMxs420WPG * i + 64u * wave));
        }
    } else {
        constexpr unsigned kP1 = sizeof(MxsImg1) / 16;
        const uint8_t *img = (const uint8_t *)&g_mxs420_img1[g.force ? 1 : 0][g.quality];
        mxs_dma<16>(img + 16u * lane, &s_img);
        if (lane < kP1 - 64u) mxs_dma<16>(img + 16u * (64u + lane), (uint8_t *)&s_img + 1024u);
    }
    /* the pair: MCUs m0 .. m0 + 3; simple = one MCU row of one frame, no row-last MCU, in range */
    const unsigned m0 = 4u * (blockIdx.x * kMxs420WPG + wave);
    const uint32_t off0 = (uint32_t)((lane / 6u) * (unsigned)g.pitch + 16u * (lane % 6u));
    const uint32_t off1 = (uint32_t)(((64u + lane) / 6u) * (unsigned)g.pitch + 16u * ((64u + lane) % 6u));
    Mx420Chunk cc;
    bool simple = false;
    if (m0 < h.tm) {
        mx420_at(cc, g, h, m0);
        simple = m0 + 4u <= h.tm && cc.mx + 4u < h.mpr && g.lin_store;
    }
#pragma unroll
    for (unsigned k = 0; k < 2; k++) {
        if (simple) {
            mxs_dma<16>(cc.src + 96u * k + off0, L.ring[k]);
            if (lane < 32) mxs_dma<16>(cc.src + 96u * k + off1, L.ring[k] + 1024u);
        } else {
            mxs_dma<4>(g.rgb, L.ring[k]);                   /* padding: filled at compute time */
            mxs_dma<4>(g.rgb, L.ring[k]);
        }
    }

    /* lane constants (k_mx420's) */
    const unsigned m = lane & 15u, q = lane >> 4;
    const uint32_t aoff = 96u * (m & 3u) + 24u * (m >> 2) + 8u * (q < 3 ? q : 0u);
    const uint32_t s0 = q < 3 ? kSelLo : kSelOne;
    const uint32_t s1 = q < 3 ? kSelHi : kSelZero;
    const uint32_t s2 = q < 3 ? kSelLo : kSelZero;
    const uint32_t cof0 = 192u * (m & 7u) + 48u * (m >> 3) + 8u * q;
    const uint32_t cof1 = cof0 + (q < 2 ? 32u : 80u);
    const uint32_t soy = (lane & 31u) * 16u + (lane >> 5) * g.bpr * 128u;
    const uint32_t soc = (lane & 31u) * 16u + (lane >> 5) * h.nmcu * 128u;
    const uint32_t ro = (lane >> 3) * kBS + (lane & 7u) * 16u;
    const uint32_t rc = kSt420C + kBS * (4u * (lane >> 5) + mx420_pm((lane >> 3) & 3u)) + (lane & 7u) * 16u;
    const unsigned gq = lane >> 4, j = lane & 15u, u = j & 7u;
    const jx_mxtab &T = g_mx420tab[g.force ? 1 : 0][g.quality];

    if constexpr (kMxs420WPG == 1) {
        if (m0 >= h.tm) return;
    }
    mx_wait_vm<4>();                                    /* the image (older than the pixel DMA) */
    if constexpr (kMxs420WPG >= 2) __builtin_amdgcn_s_barrier();
    mx_wave_sync();
    if (m0 >= h.tm) return;
    uint32_t za[8];
    {
        const uint32_t base = (uint32_t)(uintptr_t)mx_lds(L.stage) + kBS * (4u * (j >> 3) + gq);
        const mx_u2 sc = *(const mx_u2 *)&s_img.scan_t[u][0];
#pragma unroll
        for (int v = 0; v < 8; v++) za[v] = base + 2u * ((v < 4 ? sc.x : sc.y) >> (8 * (v & 3)) & 0xffu);
    }
    mx_u4 B[kParts][5];
#pragma unroll
    for (int p = 0; p < kParts; p++)
#pragma unroll
        for (int w = 0; w < 5; w++) B[p][w] = mxs420_B(s_img, gimg)[5 * p + w][lane];
    const float limc0 = s_img.limc[0][j], limc2 = s_img.limc[1][j];
    const auto &tb = mxs420_tb(s_img, gimg);

    const auto step = [&](auto kc) __attribute__((always_inline)) {
        constexpr unsigned k = decltype(kc)::value;
        constexpr bool second = k == 1;
        const unsigned ms = m0 + 2u * k;                /* the step's first MCU */
        if (k == 0)
            mx_wait_vm<2>();                            /* younger: step 1's DMA */
        else
            mx_wait_vm<1>();                            /* younger: step 0's Y store */
        if (kMxs420WPG == 1) mx_dmabar();
        uint8_t *const sp = L.ring[k];
        if (!simple) mx420_issue_general(g, h, ms, sp);     /* register path; waits vmcnt(0) */
        const uint32_t qmask = simple ? 0u : mx420_true_rows(L, g, h, ms);
        mx_wave_sync();
        const mx_f4 z = {};
        uint32_t fl = 0;
        mx_f4 accY[4], accC[2], midY[4], midC[4];     /* mid: the chains' earlier products (mx_keep) */
        const mx_u2 y00 = *(const mx_u2 *)(sp + aoff);
        const mx_u2 y01 = *(const mx_u2 *)(sp + aoff + 384u);
        const mx_u2 y10 = *(const mx_u2 *)(sp + aoff + 768u);
        const mx_u2 y11 = *(const mx_u2 *)(sp + aoff + 1152u);
        mx_u2 c0, c1, c2;
        if (__builtin_expect(qmask == 0, 1)) {
            c0 = *(const mx_u2 *)(sp + cof0);
            c1 = *(const mx_u2 *)(sp + cof1);
            c2 = *(const mx_u2 *)(sp + cof0 + 112u);
        } else {
            const unsigned l = mx_lane(), mm = l & 15u, qq = l >> 4, cb = mm >> 3, yr = 2u * (mm & 7u);
            const bool qb = (qmask >> cb) & 1u;
            const uint8_t *qt = L.qtrue[cb];
            const uint8_t *p0 = qb && qq == 3 ? qt + 24u * yr : sp + cof0;
            const uint8_t *p1 = qb && qq < 2 ? qt + 24u * yr + 8u + 8u * qq : sp + cof1;
            const uint8_t *p2 = qb && qq >= 1 ? qt + 24u * (yr + 1u) + 8u * (qq - 1u) : sp + cof0 + 112u;
            c0 = *(const mx_u2 *)p0;
            c1 = *(const mx_u2 *)p1;
            c2 = *(const mx_u2 *)p2;
        }
        __builtin_amdgcn_sched_barrier(0);
        /* every A operand before the first product; all operands stay live until the products are
         * done (mx_keep_ops after the Y column's fence) */
        const mx_h8 Al0 = mx_aop(y00, s0, s1, s2), Ah0 = mx_aop(y01, s0, s1, s2);
        const mx_h8 Al1 = mx_aop(y10, s0, s1, s2), Ah1 = mx_aop(y11, s0, s1, s2);
        __builtin_amdgcn_sched_barrier(0);
        {
            midY[0] = mx_mma(Al0, B[0][0], z);
            midY[2] = mx_mma(Ah0, B[0][0], z);
            midY[1] = mx_mma(Al0, B[1][0], z);
            midY[3] = mx_mma(Ah0, B[1][0], z);
            accY[0] = mx_mma(Al1, B[0][1], midY[0]);
            accY[2] = mx_mma(Ah1, B[0][1], midY[2]);
            accY[1] = mx_mma(Al1, B[1][1], midY[1]);
            accY[3] = mx_mma(Ah1, B[1][1], midY[3]);
            if (kParts == 3) {
                accY[1] = mx_mma(Al0, B[kParts - 1][0], accY[1]);
                accY[3] = mx_mma(Ah0, B[kParts - 1][0], accY[3]);
                accY[1] = mx_mma(Al1, B[kParts - 1][1], accY[1]);
                accY[3] = mx_mma(Ah1, B[kParts - 1][1], accY[3]);
            }
        }
        __builtin_amdgcn_sched_barrier(0);
        /* the Y products are done before anything writes a register again: a chained product may
         * wait in the matrix pipe and read its operands late (profiles/r04_mfma_valu_war.txt) */
        mx_fence_all(accY);
        mx_keep(midY);
        mx_keep_ops(Al1, Ah1);
        __builtin_amdgcn_sched_barrier(0);
        const mx_h8 C0 = mx_aop(c0, kSelLo, kSelHi, kSelLo), C1 = mx_aop(c1, kSelLo, kSelHi, kSelLo);
        const mx_h8 C2 = mx_aop(c2, kSelLo, kSelHi, kSelLo);
        __builtin_amdgcn_sched_barrier(0);
        {
            midC[0] = mx_mma(C0, B[0][2], z);
            midC[1] = mx_mma(C0, B[1][2], z);
            midC[2] = mx_mma(C1, B[0][3], midC[0]);
            midC[3] = mx_mma(C1, B[1][3], midC[1]);
            accC[0] = mx_mma(C2, B[0][4], midC[2]);
            accC[1] = mx_mma(C2, B[1][4], midC[3]);
            mx_gap();
            if (kParts == 3) {
                accC[1] = mx_mma(C0, B[kParts - 1][2], accC[1]);
                accC[1] = mx_mma(C1, B[kParts - 1][3], accC[1]);
                accC[1] = mx_mma(C2, B[kParts - 1][4], accC[1]);
            }
        }
        __builtin_amdgcn_sched_barrier(0);
        /* the same for the chroma products */
        mx_fence_all(accC);
        mx_keep(midC);
        mx_keep_ops(C1, C2);
        __builtin_amdgcn_sched_barrier(0);
        mx_column_t<0, true>(accY, MxW{}, limc0, tb, 0, j, za, fl, 0);
        __builtin_amdgcn_sched_barrier(0);
        const float sl = JX_MX_LOEXP == 0 ? 1.0f : 0x1p-12f;
        const mx_f4 s12 = {sl, sl, sl, sl};
        const mx_f4 rc4 = JX_MX_LOEXP == 0 ? accC[1] + accC[0] : __builtin_elementwise_fma(accC[1], s12, accC[0]);
        __builtin_amdgcn_sched_barrier(0);
        if (second) {
            const mx_f4 rA0 = L.rA[lane];
            mx_f2 R[4];
            float lo4[4], hi4[4];
#pragma unroll
            for (int i = 0; i < 4; i++) {
                const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(rA0[i]), __float_as_uint(rc4[i]),
                                                                false, false);
                lo4[i] = __uint_as_float(r[0]);
                hi4[i] = __uint_as_float(r[1]);
            }
            R[0] = mx_f2{lo4[0], lo4[1]};
            R[1] = mx_f2{lo4[2], lo4[3]};
            R[2] = mx_f2{hi4[0], hi4[1]};
            R[3] = mx_f2{hi4[2], hi4[3]};
            mx_column_r<kSt420C>(R, mx_w(tb, 2, j), limc2, tb, 2, j, za, fl, 1);
        } else {
            L.rA[lane] = rc4;
        }
        mx_wave_sync();
        if (__builtin_expect(__ballot(fl != 0) != 0, 0)) {
            {   /* clamped MCUs past the launch's end: no tasks */
                if (ms + (gq >> 1) >= h.tm) fl &= ~0xffu;
                if (m0 + mx420_pm(gq) >= h.tm) fl &= ~0xff00u;
            }
            mx420_exact_inline(L, sp, fl, m0, g, h, T);
        }
        /* stores: the Y store; on the second step also the pair's chroma */
        if (simple) {
            const mx_u4 vy = *(const mx_u4 *)(L.stage + ro);
            __builtin_nontemporal_store(vy, (mx_u4 *)((const uint8_t *)(cc.ydst + 256u * k) + soy));
            if (second) {
                const mx_u4 vc = *(const mx_u4 *)(L.stage + rc);
                __builtin_nontemporal_store(vc, (mx_u4 *)((const uint8_t *)cc.cdst + soc));
            }
        } else {
            const unsigned l = mx_lane();
            {
                const unsigned jb = (l >> 3) & 3u, mm = ms + (jb >> 1);
                const unsigned mc = mm < h.tm ? mm : h.tm - 1u;
                const unsigned yb = mx420_yblock(g, h, mc - (jb >> 1), l >> 5, jb);
                const unsigned f = yb / g.nb, bi = yb - f * g.nb;
                const mx_u4 vy = *(const mx_u4 *)(L.stage + (l >> 3) * kBS + (l & 7u) * 16u);
                if (mm < h.tm)
                    __builtin_nontemporal_store(
                        vy, (mx_u4 *)(g.out + (long long)f * g.ofstride + (long long)bi * 64 + (l & 7u) * 8));
            }
            if (second) {
                const unsigned pm = (l >> 3) & 3u, mm = m0 + pm;
                const unsigned mc = mm < h.tm ? mm : h.tm - 1u;
                unsigned f, mi, my, mx;
                mx420_mcu(h, mc, f, mi, my, mx);
                const mx_u4 vc = *(const mx_u4 *)(L.stage + kSt420C + kBS * (4u * (l >> 5) + mx420_pm(pm)) +
                                                   (l & 7u) * 16u);
                if (mm < h.tm)
                    __builtin_nontemporal_store(
                        vc, (mx_u4 *)(g.out + (long long)f * g.ofstride +
                                      ((long long)g.nb + (l >> 5) * h.nmcu + mi) * 64 + (l & 7u) * 8));
            }
        }
        mx_wave_sync();
    };
    step(std::integral_constant<unsigned, 0>{});
    step(std::integral_constant<unsigned, 1>{});
}

int mx_rc(hipError_t e) { return e == hipSuccess ? JPGX_OK : JPGX_EHIP; }

constexpr int kMaxDev = 64;
std::once_flag g_mx_once[kMaxDev];
int g_mx_rc[kMaxDev];
int g_mx_waves[kMaxDev];

/* a float <= lim^2 (-1 where lim < 0: every coefficient flagged) */
float mx_lsq(float lim)
{
    if (!(lim > 0.0f)) return -1.0f;
    const double l2 = (double)lim * (double)lim;
    float s = (float)l2;
    if ((double)s > l2) s = nextafterf(s, 0.0f);
    return s;
}

/* the fast exact decision's R = fl(K / Q), K = fl((1/4 a(u)) a(v)) as the device computes it
 * (mx_exact_sum; dct.c:54, quantise.c:58) */
static void mx_fill_recip(jx_mxtab &t)
{
    const double qa0 = 0.25 * JX_ALPHA0;
    for (int c = 0; c < 2; c++)
        for (int u = 0; u < 8; u++)
            for (int v = 0; v < 8; v++) {
                const double K = (u == 0 ? qa0 : 0.25) * (v == 0 ? JX_ALPHA0 : 1.0);
                t.r[c][u * 8 + v] = K / (double)t.q[c][u * 8 + v];
            }
}

int mx_tables_for_current_device(int *waves)
{
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDev) return JPGX_ENODEV;
    std::call_once(g_mx_once[dev], [dev]() {
        std::vector<jx_mxtab> tab(2 * (JX_MAXQ + 1));
        memset(tab.data(), 0, tab.size() * sizeof(jx_mxtab));
        int rc = JPGX_OK;
        for (int q = 1; q <= JX_MAXQ && !rc; q++) {
            float w[24][8], lim[24][8];
            int16_t qq[2][64];
            rc = jx_plan_tables_mx(q, w, lim, qq);
            for (int f = 0; f < 2; f++) {
                jx_mxtab &t = tab[f * (JX_MAXQ + 1) + q];
                memcpy(t.q, qq, sizeof qq);
                mx_fill_recip(t);
                for (int n = 0; n < 24; n++)
                    for (int v = 0; v < 8; v++) {
                        t.w[n][v] = w[n][v] * kRScale;
                        t.lsq[n][v] = f ? -1.0f : mx_lsq(lim[n][v]);
                    }
            }
        }
        std::unique_ptr<uint16_t[][64][8]> opsp(new uint16_t[3 * JX_MX_PARTS][64][8]);   /* heap: reentrant */
        auto ops = opsp.get();
        if (!rc) rc = jx_mx_operands(ops);
        if (!rc) rc = mx_rc(hipMemcpyToSymbol(HIP_SYMBOL(g_mxtab), tab.data(),
                                              tab.size() * sizeof(jx_mxtab)));
        if (!rc) rc = mx_rc(hipMemcpyToSymbol(HIP_SYMBOL(g_mxB), ops, sizeof(uint16_t) * 3 * JX_MX_PARTS * 64 * 8));
        if (!rc) {
            /* k_mxs's workgroup images: B operands, the LDS table as k_mx's wave 0 lays it out, and
             * the hot-path limits mx_limc computes from it */
            std::vector<MxsImg> img(2 * (JX_MAXQ + 1));
            memset(img.data(), 0, img.size() * sizeof(MxsImg));
            for (int f = 0; f < 2; f++)
                for (int q = 1; q <= JX_MAXQ; q++) {
                    MxsImg &I = img[f * (JX_MAXQ + 1) + q];
                    const jx_mxtab &t = tab[f * (JX_MAXQ + 1) + q];
                    memcpy(I.B, ops, sizeof I.B);
                    static const double cosx[8][8] = JX_COS_INIT;
                    memcpy(I.ex.cosx_, cosx, sizeof cosx);
                    memcpy(I.ex.q_, t.q, sizeof t.q);
                    MxTab full;                            /* k_mx's layout; compacted below */
                    for (unsigned tt = 0; tt < 4; tt++)
                        for (unsigned jp = 0; jp < 16; jp++) {
                            const unsigned n = tt < 2 ? jp : 16u + (jp & 7u);
                            float x[8];
                            for (int pp = 0; pp < 4; pp++)
                                for (int h = 0; h < 2; h++) {
                                    const int v = jx_pk_k(pp, h);
                                    x[2 * pp + h] = (tt & 1u) ? t.lsq[n][v] : t.w[n][v];
                                }
                            full.wl[tt][0][jp] = mx_f4{x[0], x[1], x[2], x[3]};
                            full.wl[tt][1][jp] = mx_f4{x[4], x[5], x[6], x[7]};
                        }
                    for (unsigned jp = 0; jp < 16; jp++) {
                        I.limc[0][jp] = mx_limc(full, 1, jp);
                        I.limc[1][jp] = mx_limc(full, 3, jp);
                        for (int tt = 0; tt < 2; tt++)
                            for (int h = 0; h < 2; h++) {
                                I.tab.yc[tt][h][jp] = full.wl[tt][h][jp];
                                if (jp < 8) I.tab.cr[tt][h][jp] = full.wl[2 + tt][h][jp];
                            }
                    }
                    static const int scan[8][8] = JX_SCAN_ORDER_INIT;
                    for (int uu = 0; uu < 8; uu++)
                        for (int v = 0; v < 8; v++) I.scan_t[uu][v] = (uint8_t)scan[v][uu];
                }
            rc = mx_rc(hipMemcpyToSymbol(HIP_SYMBOL(g_mxs_img), img.data(), img.size() * sizeof(MxsImg)));
            std::vector<MxsImg1> img1(img.size());
            memset(img1.data(), 0, img1.size() * sizeof(MxsImg1));
            for (size_t i = 0; i < img.size(); i++) {
                for (int h = 0; h < 2; h++)
                    for (int jp = 0; jp < 16; jp++) {
                        img1[i].sc.w[0][h][jp] = img[i].tab.yc[0][h][jp];
                        img1[i].sc.w[1][h][jp] = img[i].tab.cr[0][h][jp & 7];
                    }
                memcpy(img1[i].limc, img[i].limc, sizeof img1[i].limc);
                memcpy(img1[i].scan_t, img[i].scan_t, sizeof img1[i].scan_t);
            }
            if (!rc)
                rc = mx_rc(hipMemcpyToSymbol(HIP_SYMBOL(g_mxs_img1), img1.data(), img1.size() * sizeof(MxsImg1)));
        }
        int cus = 0, per_cu = 0;
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
            cus = 256;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_mx, 256, JX_MX_DYNLDS) != hipSuccess ||
            per_cu < 1)
            per_cu = 2;
        g_mx_waves[dev] = cus * per_cu * 4;
        g_mx_rc[dev] = rc;
    });
    if (waves) *waves = g_mx_waves[dev];
    return g_mx_rc[dev];
}

std::once_flag g_mx422_once[kMaxDev];
int g_mx422_rc[kMaxDev];
int g_mx422_waves[kMaxDev];

int mx422_tables_for_current_device(int *waves)
{
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDev) return JPGX_ENODEV;
    std::call_once(g_mx422_once[dev], [dev]() {
        std::vector<jx_mxtab> tab(2 * (JX_MAXQ + 1));
        memset(tab.data(), 0, tab.size() * sizeof(jx_mxtab));
        int rc = JPGX_OK;
        for (int q = 1; q <= JX_MAXQ && !rc; q++) {
            float w[24][8], lim[24][8];
            int16_t qq[2][64];
            rc = jx_plan_tables_mx422(q, w, lim, qq);
            for (int f = 0; f < 2; f++) {
                jx_mxtab &t = tab[f * (JX_MAXQ + 1) + q];
                memcpy(t.q, qq, sizeof qq);
                mx_fill_recip(t);
                for (int n = 0; n < 24; n++)
                    for (int v = 0; v < 8; v++) {
                        t.w[n][v] = w[n][v] * kRScale;
                        t.lsq[n][v] = f ? -1.0f : mx_lsq(lim[n][v]);
                    }
            }
        }
        std::unique_ptr<uint16_t[][4][64][8]> opsp(new uint16_t[JX_MX_PARTS][4][64][8]);   /* heap: reentrant */
        auto ops = opsp.get();
        if (!rc) rc = jx_mx422_operands(ops);
        if (!rc) rc = mx_rc(hipMemcpyToSymbol(HIP_SYMBOL(g_mx422tab), tab.data(),
                                              tab.size() * sizeof(jx_mxtab)));
        if (!rc) rc = mx_rc(hipMemcpyToSymbol(HIP_SYMBOL(g_mx422B), ops, sizeof(uint16_t) * JX_MX_PARTS * 4 * 64 * 8));
        if (!rc) {
            /* k_mxs422's images: the B operands and k_mx422's LDS table (wave 0's layout: Y scales
             * / limits at plan column j % 8, chroma at 8 + j), the per-wave scales, limits, scan */
            std::vector<MxsImg422> img(2 * (JX_MAXQ + 1));
            std::vector<MxsImg1> img1(img.size());
            memset(img.data(), 0, img.size() * sizeof(MxsImg422));
            memset(img1.data(), 0, img1.size() * sizeof(MxsImg1));
            static const int scan[8][8] = JX_SCAN_ORDER_INIT;
            for (size_t i = 0; i < img.size(); i++) {
                const jx_mxtab &t = tab[i];
                memcpy(img[i].B, ops, sizeof img[i].B);
                for (unsigned tt = 0; tt < 4; tt++)
                    for (unsigned jp = 0; jp < 16; jp++) {
                        const unsigned n = tt < 2 ? (jp & 7u) : 8u + jp;
                        float x[8];
                        for (int pp = 0; pp < 4; pp++)
                            for (int h = 0; h < 2; h++) {
                                const int v = jx_pk_k(pp, h);
                                x[2 * pp + h] = (tt & 1u) ? t.lsq[n][v] : t.w[n][v];
                            }
                        img[i].tab.wl[tt][0][jp] = mx_f4{x[0], x[1], x[2], x[3]};
                        img[i].tab.wl[tt][1][jp] = mx_f4{x[4], x[5], x[6], x[7]};
                    }
                for (int h = 0; h < 2; h++)
                    for (int jp = 0; jp < 16; jp++) {
                        img1[i].sc.w[0][h][jp] = img[i].tab.wl[0][h][jp];
                        img1[i].sc.w[1][h][jp] = img[i].tab.wl[2][h][jp];
                    }
                for (unsigned jp = 0; jp < 16; jp++) {
                    img1[i].limc[0][jp] = mx_limc(img[i].tab, 1, jp);
                    img1[i].limc[1][jp] = mx_limc(img[i].tab, 3, jp);
                }
                for (int uu = 0; uu < 8; uu++)
                    for (int v = 0; v < 8; v++) img1[i].scan_t[uu][v] = (uint8_t)scan[v][uu];
            }
            rc = mx_rc(hipMemcpyToSymbol(HIP_SYMBOL(g_mxs422_img), img.data(), img.size() * sizeof(MxsImg422)));
            if (!rc)
                rc = mx_rc(hipMemcpyToSymbol(HIP_SYMBOL(g_mxs422_img1), img1.data(), img1.size() * sizeof(MxsImg1)));
            if (!rc) {
                std::vector<MxsImg422w> imgw(img.size());
                for (size_t i = 0; i < img.size(); i++) {
                    memcpy(imgw[i].B, img[i].B, sizeof imgw[i].B);
                    imgw[i].s = img1[i];
                }
                rc = mx_rc(hipMemcpyToSymbol(HIP_SYMBOL(g_mxs422_imgw), imgw.data(), imgw.size() * sizeof(MxsImg422w)));
            }
        }
        int cus = 0, per_cu = 0;
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
            cus = 256;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_mx422, 256, JX_MX_DYNLDS) != hipSuccess ||
            per_cu < 1)
            per_cu = 2;
        g_mx422_waves[dev] = cus * per_cu * 4;
        g_mx422_rc[dev] = rc;
    });
    if (waves) *waves = g_mx422_waves[dev];
    return g_mx422_rc[dev];
}

std::once_flag g_mx420_once[kMaxDev];
int g_mx420_rc[kMaxDev];
int g_mx420_waves[kMaxDev];

int mx420_tables_for_current_device(int *waves)
{
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDev) return JPGX_ENODEV;
    std::call_once(g_mx420_once[dev], [dev]() {
        std::vector<jx_mxtab> tab(2 * (JX_MAXQ + 1));
        memset(tab.data(), 0, tab.size() * sizeof(jx_mxtab));
        int rc = JPGX_OK;
        for (int q = 1; q <= JX_MAXQ && !rc; q++) {
            float w[24][8], lim[24][8];
            int16_t qq[2][64];
            rc = jx_plan_tables_mx420(q, w, lim, qq);
            for (int f = 0; f < 2; f++) {
                jx_mxtab &t = tab[f * (JX_MAXQ + 1) + q];
                memcpy(t.q, qq, sizeof qq);
                mx_fill_recip(t);
                for (int n = 0; n < 24; n++)
                    for (int v = 0; v < 8; v++) {
                        t.w[n][v] = w[n][v] * kRScale;
                        t.lsq[n][v] = f ? -1.0f : mx_lsq(lim[n][v]);
                    }
            }
        }
        std::unique_ptr<uint16_t[][5][64][8]> opsp(new uint16_t[JX_MX_PARTS][5][64][8]);   /* heap: reentrant */
        auto ops = opsp.get();
        if (!rc) rc = jx_mx420_operands(ops);
        if (!rc) rc = mx_rc(hipMemcpyToSymbol(HIP_SYMBOL(g_mx420tab), tab.data(),
                                              tab.size() * sizeof(jx_mxtab)));
        if (!rc) rc = mx_rc(hipMemcpyToSymbol(HIP_SYMBOL(g_mx420B), ops, sizeof(uint16_t) * JX_MX_PARTS * 5 * 64 * 8));
        if (!rc) {
            /* k_mxs420's images (k_mx420's table layout, as k_mxs422's) */
            std::vector<MxsImg420> img(2 * (JX_MAXQ + 1));
            std::vector<MxsImg1> img1(img.size());
            memset(img.data(), 0, img.size() * sizeof(MxsImg420));
            memset(img1.data(), 0, img1.size() * sizeof(MxsImg1));
            static const int scan[8][8] = JX_SCAN_ORDER_INIT;
            for (size_t i = 0; i < img.size(); i++) {
                const jx_mxtab &t = tab[i];
                memcpy(img[i].B, ops, sizeof img[i].B);
                for (unsigned tt = 0; tt < 4; tt++)
                    for (unsigned jp = 0; jp < 16; jp++) {
                        const unsigned n = tt < 2 ? (jp & 7u) : 8u + jp;
                        float x[8];
                        for (int pp = 0; pp < 4; pp++)
                            for (int hh = 0; hh < 2; hh++) {
                                const int v = jx_pk_k(pp, hh);
                                x[2 * pp + hh] = (tt & 1u) ? t.lsq[n][v] : t.w[n][v];
                            }
                        img[i].tab.wl[tt][0][jp] = mx_f4{x[0], x[1], x[2], x[3]};
                        img[i].tab.wl[tt][1][jp] = mx_f4{x[4], x[5], x[6], x[7]};
                    }
                for (int hh = 0; hh < 2; hh++)
                    for (int jp = 0; jp < 16; jp++) {
                        img1[i].sc.w[0][hh][jp] = img[i].tab.wl[0][hh][jp];
                        img1[i].sc.w[1][hh][jp] = img[i].tab.wl[2][hh][jp];
                    }
                for (unsigned jp = 0; jp < 16; jp++) {
                    img1[i].limc[0][jp] = mx_limc(img[i].tab, 1, jp);
                    img1[i].limc[1][jp] = mx_limc(img[i].tab, 3, jp);
                }
                for (int uu = 0; uu < 8; uu++)
                    for (int v = 0; v < 8; v++) img1[i].scan_t[uu][v] = (uint8_t)scan[v][uu];
                memcpy(img[i].limc, img1[i].limc, sizeof img[i].limc);
                memcpy(img[i].scan_t, img1[i].scan_t, sizeof img[i].scan_t);
            }
            rc = mx_rc(hipMemcpyToSymbol(HIP_SYMBOL(g_mxs420_img), img.data(), img.size() * sizeof(MxsImg420)));
            if (!rc)
                rc = mx_rc(hipMemcpyToSymbol(HIP_SYMBOL(g_mxs420_img1), img1.data(), img1.size() * sizeof(MxsImg1)));
        }
        int cus = 0, per_cu = 0;
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
            cus = 256;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_mx420, 256, JX_MX_DYNLDS) != hipSuccess ||
            per_cu < 1)
            per_cu = 2;
        g_mx420_waves[dev] = cus * per_cu * 4;
        g_mx420_rc[dev] = rc;
    });
    if (waves) *waves = g_mx420_waves[dev];
    return g_mx420_rc[dev];
}

}  // namespace


/* k_mx420 over every frame of the stripe (true 4:2:0: Y [nb][64], Cb and Cr [nb / 4][64] per
 * frame, the stripe an even number of block rows); no workspace. */
extern "C" int jx_launch_mx420(const jx_xform_args *xa, void *stream)
{
    int waves = 0;
    const int rc = mx420_tables_for_current_device(&waves);
    if (rc) return rc;
    const size_t mcus = (size_t)xa->g.nb / 4 * (size_t)xa->g.nframes;
#ifndef JX_MX420_SHORT
#define JX_MX420_SHORT 1                /* 1: k_mxs420 (a step pair per one-wave workgroup), 0: k_mx420 */
#endif
    if (JX_MX420_SHORT) {
        const size_t waves = (mcus + 3) / 4;
        hipLaunchKernelGGL(k_mxs420, dim3((unsigned)((waves + kMxs420WPG - 1) / kMxs420WPG)), dim3(64 * kMxs420WPG), 0,
                           (hipStream_t)stream, *xa);
        return mx_rc(hipGetLastError());
    }
    const size_t chunks = (mcus + kCM420 - 1) / kCM420;
    const size_t w = std::min<size_t>(chunks, (size_t)std::max(waves, 4));
    const unsigned grid = (unsigned)((w + 3) / 4);
    hipLaunchKernelGGL(k_mx420, dim3(grid), dim3(256), JX_MX_DYNLDS, (hipStream_t)stream, *xa);
    return mx_rc(hipGetLastError());
}


/* k_mx422 over every frame of the stripe (true 4:2:2: Y [nb][64], Cb and Cr [nb / 2][64] per
 * frame); no workspace. */
extern "C" int jx_launch_mx422(const jx_xform_args *xa, void *stream)
{
    int waves = 0;
    const int rc = mx422_tables_for_current_device(&waves);
    if (rc) return rc;
    const size_t total = (size_t)xa->g.nb * (size_t)xa->g.nframes;
    const size_t nsteps = (total + 7) / 8;
#ifndef JX_MX422_SHORT
#define JX_MX422_SHORT 1                /* 1: k_mxs422 (short one-wave workgroups), 0: k_mx422 */
#endif
    if (JX_MX422_SHORT) {
        const size_t waves = (nsteps + kMxs422C - 1) / kMxs422C;
        hipLaunchKernelGGL(k_mxs422, dim3((unsigned)((waves + kMxs422WPG - 1) / kMxs422WPG)), dim3(64 * kMxs422WPG), 0,
                           (hipStream_t)stream, *xa);
        return mx_rc(hipGetLastError());
    }
    const size_t w = std::min<size_t>(nsteps, (size_t)std::max(waves, 4));
    const unsigned grid = (unsigned)((w + 3) / 4);
    hipLaunchKernelGGL(k_mx422, dim3(grid), dim3(256), JX_MX_DYNLDS, (hipStream_t)stream, *xa);
    return mx_rc(hipGetLastError());
}


/* k_mx over every frame of the stripe (4:4:4 / reference-parity output); no workspace. */
#ifdef JX_MXS_STAMP
extern "C" int jx_mxs_stamps(unsigned long long *host, size_t n)
{
    return mx_rc(hipMemcpyFromSymbol(host, HIP_SYMBOL(g_mxs_ts), std::min<size_t>(n, 1u << 20) * 8));
}
#endif

extern "C" int jx_launch_mx(const jx_xform_args *xa, void *stream)
{
    int waves = 0;
    const int rc = mx_tables_for_current_device(&waves);
    if (rc) return rc;
    const size_t total = (size_t)xa->g.nb * (size_t)xa->g.nframes;
    const size_t nsteps = (total + 7) / 8;
#ifndef JX_MX_NP
#define JX_MX_NP 0
#endif
#ifndef JX_MX_SHORT
#define JX_MX_SHORT 1                   /* 1: k_mxs (short waves), 0: the persistent k_mx */
#endif
    if (JX_MX_SHORT) {
        const size_t w = (nsteps + kMxsC - 1) / kMxsC;
        hipLaunchKernelGGL(k_mxs, dim3((unsigned)((w + kMxsWPG - 1) / kMxsWPG)), dim3(64 * kMxsWPG), JX_MX_DYNLDS,
                           (hipStream_t)stream, *xa);
        return mx_rc(hipGetLastError());
    }
    const size_t w = JX_MX_NP ? (nsteps + JX_MX_NP - 1) / (JX_MX_NP ? JX_MX_NP : 1)
                              : std::min<size_t>(nsteps, (size_t)std::max(waves, 4));
    const unsigned grid = (unsigned)((w + 3) / 4);
    hipLaunchKernelGGL(k_mx, dim3(grid), dim3(256), JX_MX_DYNLDS, (hipStream_t)stream, *xa);
    return mx_rc(hipGetLastError());
}

/* the kernel a launch of this build runs for sample ratio 0 (4:4:4), 1 (true 4:2:2), 2 (4:2:0):
 * bench.py and the profiles name the kernel they time with it */
extern "C" const char *jx_mx_kernel_name(int sr)
{
    if (sr == 1) return JX_MX422_SHORT ? "k_mxs422" : "k_mx422";
    if (sr == 2) return JX_MX420_SHORT ? "k_mxs420" : "k_mx420";
    return JX_MX_SHORT ? "k_mxs" : "k_mx";
}
