/*
 * jpgx_mx.hip -- the gfx950 block-transform kernels of libjpgx.so: colour conversion and the row
 * DCT on the matrix cores (v_mfma_f32_16x16x32_f16), the column DCT, quantiser, guard band and
 * zig-zag in scalar fp32 VALU, and the exact-order fp64 pass for guard-band
 * coefficients inline, from the pixels already in LDS.
 *
 *   k_mxs     4:4:4 / reference-parity output (sample ratio 0, and 1 / 2 without
 *             JPGX_FLAG_SUBSAMPLE: the reference does not subsample, src/downsample.c:24-32)
 *   k_mxs422  true 4:2:2 (extension, JPGX_FLAG_SUBSAMPLE, sample ratio 1)
 *   k_mxs420  true 4:2:0 (extension, JPGX_FLAG_SUBSAMPLE, sample ratio 2)
 *
 * Reference path: preprocess.c:160-162,186-188 (colour + level shift) -> dct.c:36-59 ->
 * quantise.c:52-72 (transposed divisor, round()) -> zig_zag.c:48-58; output = the three
 * JpgData.zig_zag_* arrays, [frame][Y|Cb|Cr][nb][64] int16.
 *
 * Work unit: a "step" of 8 consecutive blocks (launch-global block index, frames concatenated).
 * Short-lived waves: one wave = three steps (k_mxs, k_mxs422) or one step pair (k_mxs420), one
 * workgroup of four waves sharing an LDS image of the B operands and tables; a wave issues the
 * DMA of all its steps up front and exits after its last store.
 *   Input   the step's 8 pixel rows x 8 blocks x 24 B land in a 1.5-KiB LDS slot ([y][24 jb + k])
 *           by LDS-DMA (16-byte pieces).
 *   Rows    set s (blocks 4s..4s+3), half h (pixel rows 4h..4h+3): a 16 x 32 f16 A operand,
 *           row m = 4 jb + y, k = byte k of the pixel row (zero-extended: the f16 b 2^-24,
 *           exact, one v_perm per two bytes; k = 24 the bias 1.0).  One product with B = colour x
 *           cosine gives, in C row m, column j, the row transform of channel j/8 (Y, Cb),
 *           frequency u = j%8.  Cr: the two sets' K halves as independent products summed by
 *           one VALU add (B zero outside its set's columns), so column j of the Cr tile is set
 *           j/8's Cr at u = j%8.  B = Bh + Bl (two f16 parts); acc_h = A Bh is EXACT in any
 *           summation order (jpgx_plan.cpp); R = acc_h + acc_l (Bl encoded at Bh's scale).
 *   Columns every lane then holds three whole columns (8 rows, registers 0..3 of the two
 *           halves): (set 0, c = j/8, u), (set 1, same), (Cr, set j/8, u).  Each runs jx_fdct8
 *           in scalar fp32 (the FOps code the band is derived for; no packed-fp32 instruction in
 *           these kernels, mx_unpack8), the quantiser tm = F w + 1.5 2^23 (low 16 bits = the
 *           rounded int16), the int16 to the LDS stage at its zig-zag position, and the band test d^2 - lsq >= 0 (d = F w - rint,
 *           exact) folded into a running max.
 *   Exact   (rare) a column whose max says "some coefficient in the band" records its flagged
 *           v's; the step recomputes them from the pixels still in its LDS slot into the stage
 *           before the store (mx_exact_inline).  Eight tasks at a time, eight lanes each: lane x
 *           forms (X(x,y) c_u[x]) c_v[y] in fp64, the sum runs x-outer / y-inner (dct.c:46-50)
 *           (or a tree order whose result is proven to round the same, mx_exact_sum),
 *           F = ((1/4 a(u)) a(v)) s, round(F / Q).
 *   Output  channel c's 8 blocks x 128 B leave as one 1-KiB nontemporal store.
 * The round-3 persistent kernels (k_mx, k_mx422, k_mx420) and the timing / diagnostic build knobs
 * (round-4b A/Bs and the round-5 fault probes) live in tools/probes/jpgx_mx_r5_knobs.patch, removed from
 * the tree in round 6: `git show 63924df:tools/probes/jpgx_mx_r5_knobs.patch | patch -p1` at that commit restores them.
 */
#include <hip/hip_ext.h>
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
typedef uint32_t mx_u4 __attribute__((ext_vector_type(4)));
typedef uint32_t mx_u2 __attribute__((ext_vector_type(2)));

constexpr float kMagic = 12582912.0f;   /* 1.5 * 2^23: x + kMagic rounds x to an integer     */
constexpr int kParts = JX_MX_PARTS;     /* f16 parts of B: hi (exact products) + lo [+ lo2]  */
constexpr unsigned kSlot = 1536;        /* one step's pixels: [y][8 blocks x 24 B]           */
constexpr int kWPE = 4;                 /* waves per SIMD the register allocation targets    */

/* LDS stage: 128 B per block in zig-zag order (rounds 2-5 padded each block to 144 B; round 6
 * XOR-swizzles the 16-byte pieces instead, mxs_coef / mx2_coef below).  k_mxs's block (c, jb) sits in
 * slot mx_pos(c, jb): Y 0..7, Cr 0..3 at 8..11, Cb at 12..19, Cr 4..7 at 20..23 -- so that a lane's
 * three columns, (c = j / 8, gq), (c = j / 8, 4 + gq) and (Cr, 4 (j / 8) + gq), lie at one lane
 * address plus 4 and 8 slots (one set of address registers with immediate offsets). */
__host__ __device__ constexpr unsigned mx_pos(unsigned c, unsigned jb)
{
    return c == 0 ? jb : (c == 1 ? 12u + jb : (jb < 4 ? 8u + jb : 16u + jb));
}
/* k_mxs's stage (round 6): 128-B blocks with no padding, the eight 16-byte pieces of the block in
 * slot s XOR-swizzled by mxs_h(s).  A ds_write_b16 of the column pass puts, per 32-lane half, the
 * coefficients (v, u = 0..7) of four blocks -- slots {s, s + 1, s + 12, s + 13} (+ 4 or 8 for the
 * other columns), whose swizzles are {0, 5, 2, 7} -- on the 32 banks: every one of the 24 writes of
 * a step is at most 2-way (the minimum: rows v = 1..6 use three or four pieces in one dword
 * position, 12-16 dwords for the 8 banks of that position), 36 extra bank cycles per step against
 * 60 (with three-way writes) for the 144-B padded slots of rounds 2-5; the 16-byte stage reads
 * (ro, rcb, rr: piece l & 7 of block l >> 3) stay conflict-free (the padded slots: 12 extra cycles).
 * A lane's three blocks (s, s + 4, s + 8) share one swizzle, so one set of addresses serves them. */
constexpr unsigned kBSs = 128;
__host__ __device__ constexpr unsigned mxs_h(unsigned s)
{
    return ((s & 1u) ? 5u : 0u) ^ (s >= 12u ? 2u : 0u);
}
__host__ __device__ constexpr unsigned mxs_piece(unsigned s, unsigned p)
{
    return kBSs * s + 16u * (p ^ mxs_h(s));
}
__host__ __device__ constexpr unsigned mxs_coef(unsigned s, unsigned z)
{
    return mxs_piece(s, z >> 3) + 2u * (z & 7u);
}
static_assert(mxs_h(0) == mxs_h(4) && mxs_h(0) == mxs_h(8) && mxs_h(1) == mxs_h(9) && mxs_h(12) == mxs_h(16) &&
                  mxs_h(12) == mxs_h(20) && mxs_h(13) == mxs_h(21),
              "a lane's three column blocks share a swizzle");
/* The 4:2:x kernels' stage (round 6): 16 unpadded 128-B blocks, Y in slots 0..7 and chroma in 8..15
 * (a lane's chroma column 8 slots after its Y column), pieces XOR-swizzled by mx2_h(s).  A column
 * write's 32-lane half covers slots {s, s + 1, s + 4, s + 5} (swizzles {0, 5, 2, 7}, the minimum 2-way
 * of the 4:4:4 stage above) and the 16-byte stage reads stay conflict-free. */
constexpr unsigned kBS2 = 128;
__host__ __device__ constexpr unsigned mx2_h(unsigned s)
{
    return ((s & 1u) ? 5u : 0u) ^ ((s & 4u) ? 2u : 0u);
}
__host__ __device__ constexpr unsigned mx2_piece(unsigned s, unsigned p)
{
    return kBS2 * s + 16u * (p ^ mx2_h(s));
}
__host__ __device__ constexpr unsigned mx2_coef(unsigned s, unsigned z)
{
    return mx2_piece(s, z >> 3) + 2u * (z & 7u);
}
static_assert(mx2_h(0) == mx2_h(8) && mx2_h(5) == mx2_h(13), "a lane's Y and chroma columns share a swizzle");
/* the stage reads of the stores (lane l: piece l & 7 of block l >> 3) in closed form -- a few bit
 * operations, so that the per-step re-derivation the register allocator chooses stays cheap:
 * 16 mx?_h(s) for s = l >> 3 is (l & 8) * 10 (bits 0 and 2 of the piece) ^ (l & 32) (bit 1) */
__host__ __device__ constexpr unsigned mx_ro(unsigned l) { return (l << 4) ^ ((l & 8u) * 10u); }
__host__ __device__ constexpr unsigned mx2_ro(unsigned l) { return mx_ro(l) ^ (l & 32u); }
__host__ __device__ constexpr bool mx_ro_ok()
{
    for (unsigned l = 0; l < 64; l++) {
        const unsigned s = l >> 3, p = l & 7u;
        if (mx_ro(l) != mxs_piece(s, p) || mx_ro(l) + 1536u - (mx_ro(l) & 32u) + (~mx_ro(l) & 32u) != mxs_piece(12u + s, p))
            return false;
        if ((mx_ro(l) ^ (l & 32u)) + 1024u + ((l & 32u) << 5) != mxs_piece(s + (s < 4 ? 8u : 16u), p))
            return false;
        if (mx2_ro(l) != mx2_piece(s, p) || mx2_ro(l) + 1024u != mx2_piece(8u + s, p)) return false;
    }
    return true;
}
static_assert(mx_ro_ok(), "closed forms of the stage read addresses");
/* per-lane scales / band limits, shared by the workgroup: table t, half h (pairs 2h, 2h + 1 in
 * jx_pk_k order), profile j = lane & 15 -- a column's read of one (t, h) by the wave touches 16
 * consecutive 16-byte entries, every bank once.  4:4:4 (compacted to MxsTab below): t = Wy|b, Ly|b
 * (plan column j), Wr, Lr (16 + j % 8); 4:2:2 / 4:2:0: Wy, Ly (j % 8), Wc, Lc (8 + j). */
struct MxTab {
    mx_f4 wl[4][2][16];
};


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
 * Fast decision (round 4b): the reference's 64-term sum runs sequentially
 * (dct.c:46-50), but only round(F / Q) is kept.  Each lane sums its 8 products in order, the 8
 * partial sums meet in a 3-level butterfly (every lane ends with the same total, a + b == b + a):
 * every term passes at most 10 additions.  Terms: |X| <= 171 (the Cb quirk, preprocess.c:161:
 * 128 - (0.168736 r - 0.331264 g + 0.5 b) spans [-170.6, 84.5]; Y, Cr and the 4:2:x averages stay
 * inside), |c| <= 1, so sum |t| <= 64 * 171 (1 + u)^2 <= 10944.01 (u = 2^-53).  Recursive
 * summation (Higham, Thm 4.4): |s_seq - s| <= g63 sum|t|, |s_par - s| <= g10 sum|t| (g_n = n u /
 * (1 - n u)), so |s_seq - s_par| <= 73.01 u 10944.01 < 8.9e-11.  The reference's t = fl(fl(K s) /
 * Q) (K = (1/4 a(u)) a(v) in (0, 0.25], Q >= 1, |t| <= 2736) and the fast t' = fl(s_par R), R =
 * fl(K / Q) (MxExLds::recip, the host's jx_mxtab.r), differ by at most 0.25 * 8.9e-11 + 4.01 u 2736 < 2.4e-11.
 * So when t' is more than 2^-33 (1.16e-10) away from every half-integer (|t' - rint(t')| < 1/2 -
 * 2^-33; the difference is exact), no half-integer lies between t' and the reference's t, and
 * round(t) == rint(t').  Otherwise (near-ties: flat blocks, exact DC halves) the whole batch takes
 * the sequential sum -- wave-uniform, rare.
 * Valid in lane x == 7 (fast path: every lane).
 */
template <bool FAST, class XT>
__device__ __forceinline__ int mx_exact_sum(const double (&prod)[8], unsigned ch, unsigned u, unsigned v,
                                            unsigned x, const XT &xt)
{
    const unsigned c = ch == 0 ? 0u : 1u;
    if constexpr (FAST) {
        double p = prod[0];
#pragma unroll
        for (int y = 1; y < 8; y++) p += prod[y];
        p += mx_dpp64<0xB1>(p);                  /* quad_perm [1,0,3,2]: lane x ^ 1 */
        p += mx_dpp64<0x4E>(p);                  /* quad_perm [2,3,0,1]: lane x ^ 2 */
        p += mx_dpp64<0x141>(p);                 /* row_half_mirror: lane 7 - x      */
        const double t = p * xt.recip(c, u * 8 + v), r = __builtin_rint(t);
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
    return (int)round(xt.kfac(u * 8 + v) * sum / xt.div(c, u * 8 + v));
}

/* where the exact pass's constants come from: the workgroup's LDS image and literals (MxExLds;
 * every kernel since round 5).  Round 4b: a global read in the exact pass waits, through the
 * in-order vmcnt, for every older VMEM operation of the wave -- the later steps' pixel DMA -- so it
 * costs the wave microseconds under full HBM load. */
struct alignas(16) MxExTab {
    double cosx_[8][8];                 /* the glibc cosines (JX_COS_INIT, jx_consts.h)  */
    double r_[2][64];                   /* jx_mxtab.r: fl(K / Q), the fast decision's R   */
    int16_t q_[2][64];                  /* jx_mxtab.q of the workgroup's quality     */
};
struct MxExLds {
    const MxExTab &X;
    const uint8_t (&scan_t)[8][8];
    __device__ double cosx(unsigned k, unsigned i) const { return X.cosx_[k][i]; }
    /* per channel the reference's colour constants, as literals (i is a compile-time constant at
     * every use): t = (k0 r + k1 g) + k2 b (the signs of its subtractions folded into k1, k2:
     * a - b*k == a + b*(-k) exactly), then (A + S t) - 128 with (A, S) = (0, 1) Y, (128, -1) Cb,
     * (128, 1) Cr */
    __device__ double colour(unsigned ch, unsigned i) const
    {
        const double y[5] = {0.299, 0.587, 0.114, 0.0, 1.0}, b[5] = {0.168736, -0.331264, 0.5, 128.0, -1.0},
                     r[5] = {0.5, -0.418688, -0.081312, 128.0, 1.0};
        return ch == 0 ? y[i] : (ch == 1 ? b[i] : r[i]);
    }
    /* K = fl((1/4 a(u)) a(v)) of dct.c:54 (0.25 a(u) is exact in a double), i = 8 u + v */
    __device__ double kfac(unsigned i) const
    {
        return ((i >> 3) == 0 ? 0.25 * JX_ALPHA0 : 0.25) * ((i & 7u) == 0 ? JX_ALPHA0 : 1.0);
    }
    /* the transposed divisor Q of quantise.c:58 (channel class c: 0 luminance, 1 chrominance) */
    __device__ double div(unsigned c, unsigned i) const { return (double)X.q_[c][i]; }
    /* jx_mxtab.r: fl(K / Q), computed on the host (mx_fill_recip) */
    __device__ double recip(unsigned c, unsigned i) const { return X.r_[c][i]; }
    __device__ unsigned scan(unsigned u, unsigned v) const { return scan_t[u][v]; }
};

/* the level-shifted channel ch of the pixel at p, in the reference's double colour arithmetic and
 * operation order (preprocess.c:160-162,186-188): (A + S ((k0 r + k1 g) + k2 b)) - 128 */
template <class P, class XT>
__device__ __forceinline__ double mx_ls(const P *p, unsigned ch, const XT &xt)
{
    const double t = (xt.colour(ch, 0) * (double)p[0] + xt.colour(ch, 1) * (double)p[1]) +
                     xt.colour(ch, 2) * (double)p[2];
    return (xt.colour(ch, 3) + xt.colour(ch, 4) * t) - 128.0;
}

/* The exact pass's samples X(x, y) of one block-channel (functors over the pixels):
 *   MxSmp1  4:4:4 and every Y block: the pixel (x, y), rows rs bytes apart;
 *   MxSmp2  4:2:2 chroma: (ls(2x, y) + ls(2x + 1, y)) 0.5 (oracle/cpu_ref.c cpuref_chroma_sample);
 *           the right half (x >= 4) from its own base -- a row-last MCU's true rows (L.qtrue);
 *   MxSmp4  4:2:0 chroma: ((ls(2x, 2y) + ls(2x+1, 2y)) + (ls(2x, 2y+1) + ls(2x+1, 2y+1))) 0.25,
 *           pixel rows rs bytes apart (LDS slots, or global memory for a general pair). */
struct MxSmp1 {
    const lds_u8 *p0;
    unsigned rs;
    template <class XT>
    __device__ double operator()(unsigned x, unsigned y, unsigned ch, const XT &xt) const
    {
        return mx_ls(p0 + rs * y + 3u * x, ch, xt);
    }
};
struct MxSmp2 {
    const lds_u8 *pl, *pr;
    unsigned rl, rr;
    template <class XT>
    __device__ double operator()(unsigned x, unsigned y, unsigned ch, const XT &xt) const
    {
        const lds_u8 *p = x >= 4 ? pr + rr * y + 6u * (x - 4u) : pl + rl * y + 6u * x;
        return (mx_ls(p, ch, xt) + mx_ls(p + 3, ch, xt)) * 0.5;
    }
};
template <class P, class S>
struct MxSmp4 {
    const P *p0;
    S rs;
    template <class XT>
    __device__ double operator()(unsigned x, unsigned y, unsigned ch, const XT &xt) const
    {
        const P *p = p0 + (S)(2u * y) * rs + 6u * x, *q = p + rs;
        return ((mx_ls(p, ch, xt) + mx_ls(p + 3, ch, xt)) + (mx_ls(q, ch, xt) + mx_ls(q + 3, ch, xt))) * 0.25;
    }
};

/* one exact coefficient per 8-lane group (lane 8 i + x): lane x forms the products
 * (X(x, y) c_u[x]) c_v[y] (dct.c:48-50), mx_exact_sum sums them and rounds.  Valid in lane x == 7. */
template <bool FAST, class SMP, class XT>
__device__ __forceinline__ int mx_exact_coef(const SMP &smp, unsigned ch, unsigned u, unsigned v, unsigned x,
                                             const XT &xt)
{
    const double cu = xt.cosx(u, x);
    double prod[8];
#pragma unroll
    for (int y = 0; y < 8; y++) prod[y] = smp(x, (unsigned)y, ch, xt) * cu * xt.cosx(v, y);
    return mx_exact_sum<FAST>(prod, ch, u, v, x, xt);
}

__device__ __forceinline__ lds_u8 *mx_lds(void *p) { return (lds_u8 *)p; }

/* s of the lane in the other 16-lane row of the pair (W = 16) or the other 32-lane half (W = 32),
 * added to s: v_permlane16_swap / v_permlane32_swap with both operands s give one register with
 * the even rows' values and one with the odd rows' (or the halves'), summed in the same order in
 * every lane */
template <int W>
__device__ __forceinline__ double mx_xsum64(double s)
{
    const uint64_t b = __builtin_bit_cast(uint64_t, s);
    const uint32_t lo = (uint32_t)b, hi = (uint32_t)(b >> 32);
    if constexpr (W == 16) {
        const auto l = __builtin_amdgcn_permlane16_swap(lo, lo, false, false);
        const auto h = __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
        return __builtin_bit_cast(double, (uint64_t)l[0] | ((uint64_t)h[0] << 32)) +
               __builtin_bit_cast(double, (uint64_t)l[1] | ((uint64_t)h[1] << 32));
    } else {
        const auto l = __builtin_amdgcn_permlane32_swap(lo, lo, false, false);
        const auto h = __builtin_amdgcn_permlane32_swap(hi, hi, false, false);
        return __builtin_bit_cast(double, (uint64_t)l[0] | ((uint64_t)h[0] << 32)) +
               __builtin_bit_cast(double, (uint64_t)l[1] | ((uint64_t)h[1] << 32));
    }
}

/* the sum of s over the wave, in every lane: the 8-lane butterfly of mx_exact_sum, row_mirror
 * (16 lanes), then the row pairs and the halves -- every term passes at most 6 additions */
__device__ __forceinline__ double mx_wave_sum64(double s)
{
    s += mx_dpp64<0xB1>(s);                      /* lane x ^ 1 */
    s += mx_dpp64<0x4E>(s);                      /* lane x ^ 2 */
    s += mx_dpp64<0x141>(s);                     /* row_half_mirror: the other 4 of the 8 */
    s += mx_dpp64<0x140>(s);                     /* row_mirror: the other 8 of the 16 */
    s = mx_xsum64<16>(s);
    return mx_xsum64<32>(s);
}

/*
 * A step whose flagged set is ONE coefficient (the common case: at q90 on random data ~0.13
 * flagged coefficients per step, so ~94 % of flagged steps hold one): the whole wave computes it.
 * Lane l = 8 y + x forms the reference's product (X(x,y) c_u[x]) c_v[y] (preprocess.c:160-162,
 * 186-188; dct.c:48-50) in its operation order; the 64 products meet in mx_wave_sum64 -- every term
 * through at most 6 additions, fewer than the 10 mx_exact_sum's bound allows, so that bound and its
 * 2^-33 margin hold unchanged -- and t' = s R decides as mx_exact_sum's fast path.  Every lane holds
 * the same t'; returns false on a near-tie (the caller then takes the sequential 8-lane path).
 * Round 5: one instruction stream for the wave instead of eight 8-lane groups of which seven idle.
 */
template <class SMP, class XT>
__device__ __forceinline__ bool mx_exact_one(const SMP &smp, unsigned ch, unsigned u, unsigned v, const XT &xt,
                                             int &val)
{
    const unsigned l = mx_lane(), x = l & 7u, y = l >> 3;
    const double sum = mx_wave_sum64(smp(x, y, ch, xt) * xt.cosx(u, x) * xt.cosx(v, y));
    const double t = sum * xt.recip(ch == 0 ? 0 : 1, u * 8 + v), r = __builtin_rint(t);
    val = (int)r;
    return 0.5 - __builtin_fabs(t - r) > 0x1p-33;                          /* t - r: exact */
}

/* The single-coefficient case of an inline exact pass: when exactly one lane holds exactly one
 * flag, one(sl, bit) computes it with the whole wave (mx_exact_one) and, unless it was a near-tie,
 * writes it from lane 0 and returns true; the flag is then cleared. */
template <class F>
__device__ __forceinline__ void mx_exact_single(uint32_t &bits, F &&one)
{
    const uint64_t act = __ballot(bits != 0);
    if (__popcll(act) == 1) {
        const unsigned sl = __builtin_amdgcn_readfirstlane((unsigned)__builtin_ctzll(act));
        const uint32_t b1 = (uint32_t)__builtin_amdgcn_readlane((int)bits, (int)sl);
        if (__popc(b1) == 1 && one(sl, (unsigned)__builtin_ctz(b1))) bits = 0;
    }
}

/* lane 0 writes a whole-wave result into the stage (byte offset off) */
__device__ __forceinline__ bool mx_put_one(const void *stage, unsigned off, bool ok, int val)
{
    if (!__builtin_amdgcn_readfirstlane((int)ok)) return false;
    if (mx_lane() == 0) *(__attribute__((address_space(3))) int16_t *)(mx_lds((void *)stage) + off) = (int16_t)val;
    return true;
}

/* the step's block jb and channel of a lane's column k (k_mxs column layout) */
__device__ __forceinline__ unsigned mx_col_block(unsigned k, unsigned sl)
{
    const unsigned gg = sl >> 4, jj = sl & 15u;
    return k == 0 ? gg : (k == 1 ? 4u + gg : (jj < 8 ? gg : 4u + gg));
}

/* Inline exact pass of one step: every flagged coefficient (bit 8 col + v of a lane's `bits`),
 * the single-coefficient case on the whole wave, otherwise eight at a time, patching the stage.
 * (Round 4b ended it with lgkmcnt(0) against a fault that round 5 traced to packed fp32, DESIGN.md
 * 4.3f; the wait is gone.) */
template <class Lds, class XT>
__device__ __forceinline__ void mx_exact_inline(Lds &L, const uint8_t *slot, uint32_t bits,
                                                const XT &xt)
{
    const unsigned lane = mx_lane();
    mx_wave_sync();
    mx_exact_single(bits, [&](unsigned sl, unsigned bt) __attribute__((always_inline)) {
        const unsigned k = bt >> 3, v = bt & 7u;
        const unsigned jj = sl & 15u, u = jj & 7u, ch = k < 2 ? (jj >> 3) : 2u;
        const unsigned jb = mx_col_block(k, sl);
        int val;
        const bool ok = mx_exact_one(MxSmp1{mx_lds((void *)slot) + 24u * jb, 192u}, ch, u, v, xt, val);
        return mx_put_one(L.stage, mxs_coef(mx_pos(ch, jb), xt.scan(u, v)), ok, val);
    });
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
        const int val = mx_exact_coef<true>(MxSmp1{mx_lds((void *)slot) + 24u * jb, 192u}, ch, u, v, x, xt);
        if (live && x == 7)
            *(__attribute__((address_space(3))) int16_t *)(mx_lds(L.stage) + mxs_coef(mx_pos(ch, jb), xt.scan(u, v))) =
                (int16_t)val;
        mx_wave_sync();
    }
}

/*
 * The column pass computes in SCALAR fp32 (v_add_f32 / v_fma_f32): no packed-fp32 VALU instruction
 * (v_pk_add_f32, v_pk_mul_f32, v_pk_fma_f32) is allowed in these kernels.  Round 5 found the cause
 * of the rows-12..15 fault: on gfx950, a packed-fp32 instruction of a wave that
 * also issues MFMAs intermittently writes wrong values in lanes 48..63 -- reproduced in isolation
 * (tools/probes/pk_hazard4.hip: the packed 8-point DCT wrong in 1.7e-4 of its runs when the wave's
 * own v_mfma_f32_16x16x32_f16 precede it, never without; tools/probes/pk_hazard5.hip: an op_sel
 * swap of a source's halves suffices).  Lanes 48..63 of the column pass are blocks 3 and 7 of a
 * step, i.e. the C rows 12..15 seen since round 3.  The scalar code is the very FOps sequence the
 * guard band is derived for (xform_math.h), so the output is bit-identical; tools/mfma_war_check.py
 * --no-pk rejects any packed-fp32 arithmetic in the built ISA (tests/test_isa.py).
 */
/* F[k] -> scale of output k of jx_fdct8 from the table's [half][4] layout (jx_pk_k order) */
__device__ __forceinline__ void mx_unpack8(const mx_f4 &a, const mx_f4 &b, float (&o)[8])
{
    o[0] = a.x, o[4] = a.y, o[2] = a.z, o[6] = a.w;
    o[1] = b.x, o[3] = b.y, o[5] = b.z, o[7] = b.w;
}

/* rare: the flagged v's of one column (the same arithmetic as mx_column_r) */
__device__ __forceinline__ uint32_t mx_flags(const float (&F)[8], const float (&W)[8], const float (&Lq)[8])
{
    uint32_t m = 0;
#pragma unroll
    for (int k = 0; k < 8; k++) {
        const float tm = __builtin_fmaf(F[k], W[k], kMagic);
        const float rr = tm - kMagic;
        const float d = __builtin_fmaf(F[k], W[k], -rr);
        const float e = __builtin_fmaf(d, d, -Lq[k]);
        m |= (e >= 0.0f ? 1u : 0u) << k;
    }
    return m;
}

/* R rows 0..7 of one column from the lo (rows 0..3) and hi (rows 4..7) tiles: the lo B part is
 * encoded at the hi part's scale (JX_MX_LOEXP = 0), so R = fl(acc_h + acc_l) */
static_assert(JX_MX_LOEXP == 0, "the kernels take R = acc_h + acc_l");
__device__ __forceinline__ void mx_combine(mx_f4 hl, mx_f4 ll, mx_f4 hh, mx_f4 lh, float (&R)[8])
{
    R[0] = ll.x + hl.x, R[1] = ll.y + hl.y, R[2] = ll.z + hl.z, R[3] = ll.w + hl.w;
    R[4] = lh.x + hh.x, R[5] = lh.y + hh.y, R[6] = lh.z + hh.z, R[7] = lh.w + hh.w;
}

/* a column's scales from the workgroup table; t0 = 0 (4:4:4: Y|Cb, 4:2:x: Y) or 2 (4:4:4: Cr,
 * 4:2:x: chroma); its squared band limits are table t0 + 1 */
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
__device__ __forceinline__ void mx_keep(const mx_f4 (&x)[4])
{
    asm volatile("" ::"v"(x[0]), "v"(x[1]), "v"(x[2]), "v"(x[3]));
}
/* the A / B operands of the products too: a product queued behind a chained one reads its
 * operands late, pass by pass */
template <class T>
__device__ __forceinline__ int mx_keep1(const T &x)
{
    asm volatile("" ::"v"(x));
    return 0;
}
template <class... T>
__device__ __forceinline__ void mx_keep_ops(const T &...x)
{
    const int k[] = {mx_keep1(x)...};
    (void)k;
}

/* Column pass of one column (R rows), quantiser, stage writes at za[v] + OFF, band flags (rare
 * path: the exact per-coefficient test with the limits of table t0 + 1, after mx_fence(*fence)
 * when an MFMA may be in flight) into fl.  Scalar fp32 throughout (see mx_unpack8). */
template <unsigned OFF, class TB>
__device__ __forceinline__ void mx_column_r(const float (&R)[8], const MxW &t, float limc, const TB &tb,
                                             unsigned t0, unsigned j, const uint32_t (&za)[8], uint32_t &fl, int kc,
                                             const mx_f4 *fence = nullptr)
{
    float F[8], W[8];
    jx_fdct8<FOps>(R, F);
    mx_unpack8(t.w01, t.w23, W);
    typedef __attribute__((address_space(3))) uint16_t l16;
    float em = 0.0f;
#pragma unroll
    for (int p = 0; p < 4; p++) {
        const int k0 = jx_pk_k(p, 0), k1 = jx_pk_k(p, 1);
        const float t0v = __builtin_fmaf(F[k0], W[k0], kMagic), t1v = __builtin_fmaf(F[k1], W[k1], kMagic);
        *(l16 *)(uintptr_t)(za[k0] + OFF) = (uint16_t)__float_as_uint(t0v);
        *(l16 *)(uintptr_t)(za[k1] + OFF) = (uint16_t)__float_as_uint(t1v);
        const float d0 = __builtin_fmaf(F[k0], W[k0], -(t0v - kMagic));
        const float d1 = __builtin_fmaf(F[k1], W[k1], -(t1v - kMagic));
        em = __builtin_fmaxf(__builtin_fmaxf(em, __builtin_fabsf(d0)), __builtin_fabsf(d1));
    }
    if (__builtin_expect(__ballot(em >= limc) != 0, 0)) {
        if (fence) mx_fence(*fence);
        const MxW lw = mx_l(tb, t0, j);
        float Lq[8];
        mx_unpack8(lw.w01, lw.w23, Lq);
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
    float R[8];
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

/* ==== k_mxs: 4:4:4 in short-lived waves (round 4) ============================================
 *
 * Wave w of the grid computes the three consecutive steps 3w .. 3w + 2 (24 blocks) and exits, so
 * the hardware dispatcher hands the chip one compact, advancing window of the batch (a persistent
 * grid-stride layout drifts: instruction arbitration favours older waves,
 * profiles/r03_skeleton_wgrank.txt; the memory skeleton reads 0.72-0.76 non-persistent vs
 * 0.67-0.70 persistent, profiles/r04_*).  What a short wave needs is a cheap start:
 *   - its B operands (6 KiB, quality-independent, g_mxs_B) come from global memory (L2) into
 *     registers, then its pixel DMA for all three steps is issued (step k lives in slot k);
 *   - this quality's scale / limit table with the hot-path band limits, the zig-zag positions and
 *     the exact pass's tables are one pre-laid-out image (g_mxs_img) that the workgroup's four
 *     waves copy into LDS with LDS-DMA (16-byte pieces), one s_barrier;
 *   - the exact pass runs inline per step on the stage (no cross-step queue, no side buffer).
 * vmcnt bookkeeping: every step issues exactly two DMA operations up front (padding operations
 * for general / absent steps) and three stores, so step k waits with vmcnt(2 (2 - k) + 3 k).
 */
constexpr unsigned kMxsC = 3;           /* steps per wave = LDS input slots (4: not faster, round 6) */
constexpr unsigned kMxsWPG = 4;         /* waves per workgroup (one LDS image) */
struct alignas(16) MxsLds {
    uint8_t ring[kMxsC][kSlot];         /* pixels, [y][24 jb + k]                       */
    uint8_t stage[24 * kBSs];           /* zig-zag stage (mx_pos, mxs_coef)             */
    uint16_t task[8];                   /* inline exact batch                           */
};
static_assert(sizeof(MxsLds) % 16 == 0, "16-byte aligned LDS regions");
/* the B operands (round 6): read by each wave from global memory (L2) into registers at its start,
 * [part * 3 + which] = Y|Cb, Cr set 0, Cr set 1 (zero in columns 8..15 / 0..7) -- no zeroing VALU
 * per step, no reload after an exact pass, and a 4-KiB smaller workgroup image (rounds 4b-5 kept
 * them in the image: 105.1 vs 106.0 us per launch on one box, profiles/r06_b_operands.txt; round 4b's
 * wrong C rows 12..15 with B from global memory were the packed-fp32 fault of DESIGN.md 4.3f) */
/* the workgroup image: scale / limit table, hot-path limits (mx_limc) per lane profile and column
 * kind, zig-zag positions, the exact pass's tables */
__device__ mx_u4 g_mxs_B[3 * JX_MX_PARTS][64];
struct alignas(16) MxsImg {
    MxsTab tab;
    float limc[2][16];
    uint8_t scan_t[8][8];               /* zig-zag position of (v, u) at [u][v] */
    MxExTab ex;                         /* the exact pass's tables                      */
};
constexpr unsigned kMxsPieces = sizeof(MxsImg) / 16;
static_assert(sizeof(MxsImg) % 16 == 0 && kMxsPieces <= 768, "three 16-byte pieces per thread");
static_assert(sizeof(MxsLds) * kMxsWPG + sizeof(MxsImg) <= 40 * 1024, "4 workgroups of 4 waves per CU");
__device__ MxsImg g_mxs_img[2][JX_MAXQ + 1];     /* [force][quality] */

template <unsigned N>
__device__ __forceinline__ void mx_wait_vm()
{
    static_assert(N < 64, "vmcnt is 6 bits");
    __builtin_amdgcn_s_waitcnt((int)((N & 15u) | ((N >> 4) << 14) | 0xF70u));
}

/* LDS-DMA of 16 (or 4) bytes per lane to lds_base + 16 (4) lane.  The builtin (not inline asm:
 * the compiler then drains vmcnt(0) before the next LDS read of the wave, since it cannot tell
 * which LDS bytes the DMA writes -- which costs nothing here, all DMA being issued together; an
 * asm form measured 2-4 % slower, profiles/r03_dma_pipelining.txt) */
template <int SIZE>
__device__ __forceinline__ void mxs_dma(const void *g, void *lds)
{
    static_assert(SIZE == 16 || SIZE == 4, "dwordx4 or dword pieces");
    if constexpr (SIZE == 16)
        __builtin_amdgcn_global_load_lds((mx_gp)g, (mx_lp)lds, 16, 0, 0);
    else
        __builtin_amdgcn_global_load_lds((mx_gp)g, (mx_lp)lds, 4, 0, 0);
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

__global__ __launch_bounds__(64 * kMxsWPG, kWPE) void k_mxs(const jx_xform_args a)
{
    __shared__ __attribute__((aligned(16))) MxsLds s_lds[kMxsWPG];
    __shared__ __attribute__((aligned(16))) MxsImg s_img;
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
    const unsigned wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    MxsLds &L = s_lds[wave];
    mx_u4 B[kParts][3];                          /* older than every DMA of the wave */
#pragma unroll
    for (int p = 0; p < kParts; p++)
#pragma unroll
        for (int w = 0; w < 3; w++) B[p][w] = g_mxs_B[3 * p + w][lane];
    /* the image into LDS (LDS-DMA: piece p of thread t lands at 16 p) */
    {
        const uint8_t *img = (const uint8_t *)&g_mxs_img[g.force ? 1 : 0][g.quality];
#pragma unroll
        for (unsigned i = 0; i < (kMxsPieces + 64u * kMxsWPG - 1u) / (64u * kMxsWPG); i++) {
            const unsigned piece = 64u * kMxsWPG * i + threadIdx.x;
            if (64u * kMxsWPG * i + 64u * wave < kMxsPieces && piece < kMxsPieces)
                mxs_dma<16>(img + 16u * piece, (uint8_t *)&s_img + 16u * (64u * kMxsWPG * i + 64u * wave));
        }
    }
    /* this wave's steps' DMA */
    const unsigned wv = blockIdx.x * kMxsWPG + wave;
    const uint32_t off0 = (uint32_t)((lane / 12u) * (unsigned)g.pitch + 16u * (lane % 12u));
    const uint32_t off1 = (uint32_t)(((64u + lane) / 12u) * (unsigned)g.pitch + 16u * ((64u + lane) % 12u));
    MxsCur iss;                                  /* issue cursor */
    mxs_at(iss, g, 8u * kMxsC * wv);
    MxsCur cmp = iss;                            /* compute cursor */
#pragma unroll
    for (unsigned k = 0; k < kMxsC; k++) {
        mxs_issue(iss, g, L.ring[k], off0, off1, lane);
        mxs_next(iss, g);
    }

    /* lane constants */
    const unsigned m = lane & 15u, q = lane >> 4;
    /* lanes 48..63 (the bias / zero rows k = 24..31) use no pixel byte: they read lanes 32..47's
     * addresses, an LDS broadcast (round 6: their own addresses made every A read 2-way in the
     * upper half of the wave) */
    const uint32_t aoff = 192u * (m & 3u) + 24u * (m >> 2) + 8u * (q < 3 ? q : 2u);
    const uint32_t s0 = q < 3 ? kSelLo : kSelOne;
    const uint32_t s1 = q < 3 ? kSelHi : kSelZero;
    const uint32_t s2 = q < 3 ? kSelLo : kSelZero;
    const uint32_t so0 = lane * 16u, so1 = so0 + g.nb * 128u, so2 = so1 + g.nb * 128u;
    const uint32_t ro = mx_ro(lane);                          /* mxs_piece(lane >> 3, lane & 7) */
    const uint32_t rr = (ro ^ (lane & 32u)) + 1024u + ((lane & 32u) << 5);   /* Cr: slots 8..11, 20..23 */
    const uint32_t rcb = (ro ^ 32u) + 1536u;                  /* Cb: slots 12..19 */
    const unsigned gq = lane >> 4, j = lane & 15u, u = j & 7u;
    const MxExLds xt{s_img.ex, s_img.scan_t};

    /* the image has landed (it is older than the prologue's pixel operations), in every wave */
    mx_wait_vm<2u * kMxsC>();
    __builtin_amdgcn_s_barrier();
    mx_wave_sync();
    if (cmp.b >= g.total) {
        mx_wait_vm<0>();                                /* no LDS-DMA outlives the wave */
        return;
    }
    /* stage addresses of this lane's column at v = 0..7: the zig-zag positions from the image (no
     * global load: its wait would drain the pixel DMA too) */
    uint32_t za[8];
    {
        const unsigned s = mx_pos(j >> 3, gq);
        const uint32_t base = (uint32_t)(uintptr_t)mx_lds(L.stage) + kBSs * s, hs = mxs_h(s);
        const mx_u2 sc = *(const mx_u2 *)&s_img.scan_t[u][0];
#pragma unroll
        for (int v = 0; v < 8; v++) {
            const uint32_t z = (v < 4 ? sc.x : sc.y) >> (8 * (v & 3)) & 0xffu;
            za[v] = base + 16u * ((z >> 3) ^ hs) + 2u * (z & 7u);
        }
    }
    const float limc0 = s_img.limc[0][j], limc2 = s_img.limc[1][j];
    const MxsTab &tb = s_img.tab;

    /* one step from `sp` (its DMA has landed): transform, inline exact pass, three stores */
    const auto body = [&](const MxsCur &S, uint8_t *sp) __attribute__((always_inline)) {
        if (!S.simple) {
            MxCur P;
            mx_seek(P, g, S.b);
            mx_issue(g, P, S.b, false, off0, off1, sp);      /* register path; waits vmcnt(0) */
        }
        mx_wave_sync();
        const mx_u2 d00 = *(const mx_u2 *)(sp + aoff);
        const mx_u2 d01 = *(const mx_u2 *)(sp + aoff + 768u);
        const mx_u2 d10 = *(const mx_u2 *)(sp + aoff + 96u);
        const mx_u2 d11 = *(const mx_u2 *)(sp + aoff + 864u);
        const MxW w0 = mx_w(tb, 0, j);
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
        };
        mma_set(acc[0], A00, A01);
        __builtin_amdgcn_sched_barrier(0);
        mma_set(acc[1], A10, A11);
        __builtin_amdgcn_sched_barrier(0);
        mx_column_t<0>(acc[0], w0, limc0, tb, 0, j, za, fl, 0);
        __builtin_amdgcn_sched_barrier(0);
        /* the Cr tile: the two sets' K halves as eight independent products and one VALU add per
         * element, cr[0] + cr[1] -- bit-identical to a chained form, since in every column one of
         * the two halves is an exact zero (B1 is zero in columns 8..15, B2 in 0..7) -- so no
         * product of k_mxs waits in the matrix pipe for another; the products
         * are issued in source order (cr[1][3] last: the fence) */
        mx_f4 cr[2][4];
        cr[0][0] = mx_mma(A00, B[0][1], z);
        __builtin_amdgcn_sched_barrier(0);
        cr[0][2] = mx_mma(A01, B[0][1], z);
        __builtin_amdgcn_sched_barrier(0);
        cr[0][1] = mx_mma(A00, B[1][1], z);
        __builtin_amdgcn_sched_barrier(0);
        cr[0][3] = mx_mma(A01, B[1][1], z);
        __builtin_amdgcn_sched_barrier(0);
        cr[1][0] = mx_mma(A10, B[0][2], z);
        __builtin_amdgcn_sched_barrier(0);
        cr[1][2] = mx_mma(A11, B[0][2], z);
        __builtin_amdgcn_sched_barrier(0);
        cr[1][1] = mx_mma(A10, B[1][2], z);
        __builtin_amdgcn_sched_barrier(0);
        cr[1][3] = mx_mma(A11, B[1][2], z);
        __builtin_amdgcn_sched_barrier(0);
        mx_column_t<4 * kBSs>(acc[1], w0, limc0, tb, 0, j, za, fl, 1, &cr[1][3]);
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
            const mx_u4 val = *(const mx_u4 *)(L.stage + mxs_piece(mx_pos((unsigned)c, l >> 3), l & 7u));
            if (bl < g.total)
                __builtin_nontemporal_store(
                    val, (mx_u4 *)(g.out + (long long)f * g.ofstride + ((long long)c * g.nb + bi) * 64 + (l & 7u) * 8));
        };
        const bool early = S.simple && __ballot((fl & 0xffffu) != 0) == 0;
        if (early) {
            mx_fence(cr[1][3]);                        /* the Cr products are done (operand rule) */
            mx_wave_sync();
            const mx_u4 v0 = *(const mx_u4 *)(L.stage + ro);
            const mx_u4 v1 = *(const mx_u4 *)(L.stage + rcb);
            __builtin_nontemporal_store(v0, (mx_u4 *)(ob + so0));
            __builtin_nontemporal_store(v1, (mx_u4 *)(ob + so1));
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int i = 0; i < 4; i++)                    /* scalar adds (no packed fp32, mx_unpack8) */
            acc[2][i] = mx_f4{cr[0][i].x + cr[1][i].x, cr[0][i].y + cr[1][i].y, cr[0][i].z + cr[1][i].z,
                              cr[0][i].w + cr[1][i].w};
        mx_column_t<8 * kBSs, true>(acc[2], w0, limc2, tb, 2, j, za, fl, 2);
        mx_wave_sync();
        if (__builtin_expect(__ballot(fl != 0) != 0, 0)) {
            clamp(fl);
            mx_exact_inline(L, sp, fl, xt);
        }
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

    /* step k waits for its DMA: younger are 2 - k steps' two DMA operations and k steps' three
     * stores */
    const auto step = [&](auto kc) __attribute__((always_inline)) {
        constexpr unsigned k = decltype(kc)::value;
        if (cmp.b >= g.total) {
            mx_wait_vm<0>();                            /* no LDS-DMA outlives the wave */
            return;
        }
        mx_wait_vm<2 * (kMxsC - 1 - k) + 3 * k>();
        body(cmp, L.ring[k]);
        mxs_next(cmp, g);
    };
    step(std::integral_constant<unsigned, 0>{});
    step(std::integral_constant<unsigned, 1>{});
    step(std::integral_constant<unsigned, 2>{});
}

/* ==== k_mxs422: true 4:2:2 (extension, JPGX_FLAG_SUBSAMPLE, sample_ratio 1), round 4 ========
 *
 * k_mxs's scheme (three steps per wave, their DMA up front, step k in slot k, four waves per
 * workgroup sharing an LDS image, the exact pass inline on the stage) around a 4:2:2 step: 8 Y
 * blocks = 4 MCUs (chroma block cb of the step = Y blocks 2 cb, 2 cb + 1: W is a multiple of 16
 * and steps start at multiples of 8, so an MCU never straddles a step or a block-row).
 *   Y       k_mxs's Y row transform with the two sets concatenated along K (B_Y0 zero in columns
 *           8..15, B_Y1 in 0..7): column j of the C tile is set j / 8's Y at u = j % 8.
 *   Chroma  A row m = chroma block m >> 2, pixel row m & 3 of the half, K = the 48 bytes of the
 *           MCU's pixel row over two K = 32 products; B (jpgx_plan.cpp jx_mx422_operands) holds
 *           0.5 a[c][p] cos((2 floor(x/2) + 1) u pi/16), so column j is the row transform of the
 *           pair-averaged level-shifted chroma: Cb (j < 8) or Cr of chroma block gq at u = j % 8.
 *           Same encoding, split and rigorous band as 4:4:4 (jx_plan_tables_mx422: 65 fp32
 *           additions per lo part instead of 33).
 *   Columns each lane holds two, Y block (j / 8) 4 + gq and chroma block (channel j / 8, gq):
 *           16 MFMAs and 2 x 8 column DCTs per step (4:4:4: 16 and 3 x 8); 1 KiB Y + 512 B Cb +
 *           512 B Cr leave in two stores (lanes 0..31 Cb, 32..63 Cr): step k waits with
 *           vmcnt(2 (2 - k) + 2 k).  Stage: Y block jb at 144 jb, chroma (c, cb) at 1152 +
 *           144 (4 c + cb), so the chroma column's address is the Y column's plus a constant.
 *   Quirk   the x0 = -8 quirk shifts a row-last Y block's rows by one (Y only); a general step
 *           holding such a block loads the block's true rows into L.qtrue for its chroma block.
 *   Exact   inline: a chroma task follows the oracle's definition (oracle/cpu_ref.c
 *           cpuref_chroma_sample, dct_coef): X = (ls(2X) + ls(2X+1)) * 0.5, ls = the level-shifted
 *           chroma in preprocess.c's operation order.
 */
constexpr unsigned kSt422C = 8 * kBS2;        /* chroma (c, cb) in slot 8 + 4 c + cb (mx2_coef) */

/* Y block of a lane's columns (lane (gq, j): set j / 8); also the chroma column's stage slot */
__device__ __forceinline__ unsigned mx422_yblock(unsigned sl)
{
    return (sl & 15u) < 8 ? (sl >> 4) : 4u + (sl >> 4);
}

/* the samples of chroma block cb of a step (MCU cb: pixels 16 cb .. 16 cb + 15 of the slot's rows);
 * the right Y block's rows come from L.qtrue when it is a row-last block (bit cb of qmask) */
template <class Lds>
__device__ __forceinline__ MxSmp2 mx422_smp(Lds &L, const uint8_t *sp, uint32_t qmask, unsigned cb)
{
    const bool q = (qmask >> cb) & 1u;
    const lds_u8 *pl = mx_lds((void *)sp) + 48u * cb;
    return MxSmp2{pl, q ? mx_lds(L.qtrue[cb]) : pl + 24u, 192u, q ? 24u : 192u};
}

/* Inline exact pass of one step: bit 8 col + v of a lane's bits (col 0 Y, 1 chroma); the single-
 * coefficient case on the whole wave, then eight tasks at a time (8 lanes each) */
template <class Lds, class XT>
__device__ __forceinline__ void mx422_exact_inline(Lds &L, const uint8_t *sp, uint32_t qmask,
                                                   uint32_t bits, const XT &xt)
{
    const unsigned lane = mx_lane();
    mx_wave_sync();
    mx_exact_single(bits, [&](unsigned sl, unsigned bt) __attribute__((always_inline)) {
        const unsigned k = bt >> 3, v = bt & 7u, jj = sl & 15u, u = jj & 7u;
        const unsigned slot = mx422_yblock(sl);
        int val;
        bool ok;
        if (k == 0)
            ok = mx_exact_one(MxSmp1{mx_lds((void *)sp) + 24u * slot, 192u}, 0u, u, v, xt, val);
        else
            ok = mx_exact_one(mx422_smp(L, sp, qmask, sl >> 4), 1u + (jj >> 3), u, v, xt, val);
        return mx_put_one(L.stage, mx2_coef(slot + (k ? 8u : 0u), xt.scan(u, v)), ok, val);
    });
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
        int val;
        if (k == 0)
            val = mx_exact_coef<true>(MxSmp1{mx_lds((void *)sp) + 24u * slot, 192u}, 0u, u, v, x, xt);
        else
            val = mx_exact_coef<true>(mx422_smp(L, sp, qmask, sl >> 4), 1u + (jj >> 3), u, v, x, xt);
        if (live && x == 7)
            *(__attribute__((address_space(3))) int16_t *)(mx_lds(L.stage) + mx2_coef(slot + (k ? 8u : 0u), xt.scan(u, v))) =
                (int16_t)val;
        mx_wave_sync();
    }
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

constexpr unsigned kMxs422C = 3;
constexpr unsigned kMxs422WPG = 4;
struct alignas(16) Mxs422Lds {
    uint8_t ring[kMxs422C][kSlot];
    uint8_t stage[16 * kBS2];
    uint8_t qtrue[4][192];
    uint16_t task[8];
};
/* the LDS image: B operands [part * 3 + which][lane] (which 0: the two Y sets' operands merged --
 * B_Y0 is zero in columns 8..15, B_Y1 in 0..7, so lane l keeps set (l & 15) / 8's and the kernel
 * rebuilds the zeros; 1, 2: chroma), the scale / limit table (round 5: the band limits of the rare
 * path too, no global read there), the hot-path limits, the zig-zag positions and the exact pass's
 * tables */
struct alignas(16) MxsImg422 {
    mx_u4 B[JX_MX_PARTS * 3][64];
    MxTab tab;
    float limc[2][16];
    uint8_t scan_t[8][8];
    MxExTab ex;
};
constexpr unsigned kMxs422Pieces = sizeof(MxsImg422) / 16;
static_assert(sizeof(Mxs422Lds) % 16 == 0 && sizeof(Mxs422Lds) * kMxs422WPG + sizeof(MxsImg422) <= 40 * 1024,
              "4 workgroups of 4 waves per CU");
__device__ MxsImg422 g_mxs422_img[2][JX_MAXQ + 1];

__global__ __launch_bounds__(64 * kMxs422WPG, kWPE) void k_mxs422(const jx_xform_args a)
{
    __shared__ __attribute__((aligned(16))) Mxs422Lds s_lds[kMxs422WPG];
    __shared__ __attribute__((aligned(16))) MxsImg422 s_img;
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
    const unsigned wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    Mxs422Lds &L = s_lds[wave];
    {
        const uint8_t *img = (const uint8_t *)&g_mxs422_img[g.force ? 1 : 0][g.quality];
#pragma unroll
        for (unsigned i = 0; i < (kMxs422Pieces + 64u * kMxs422WPG - 1u) / (64u * kMxs422WPG); i++) {
            const unsigned piece = 64u * kMxs422WPG * i + threadIdx.x;
            if (64u * kMxs422WPG * i + 64u * wave < kMxs422Pieces && piece < kMxs422Pieces)
                mxs_dma<16>(img + 16u * piece, (uint8_t *)&s_img + 16u * (64u * kMxs422WPG * i + 64u * wave));
        }
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

    /* lane constants */
    const unsigned m = lane & 15u, q = lane >> 4;
    const uint32_t aoff = 192u * (m & 3u) + 24u * (m >> 2) + 8u * (q < 3 ? q : 2u);
    const uint32_t s0 = q < 3 ? kSelLo : kSelOne;
    const uint32_t s1 = q < 3 ? kSelHi : kSelZero;
    const uint32_t s2 = q < 3 ? kSelLo : kSelZero;
    const uint32_t coff0 = 192u * (m & 3u) + 48u * (m >> 2) + 8u * q;
    const uint32_t coff1 = 192u * (m & 3u) + 48u * (m >> 2) + 32u + 8u * (q < 2 ? q : 0u);
    const uint32_t t0 = q < 2 ? kSelLo : (q == 2 ? kSelOne : kSelZero);
    const uint32_t t1 = q < 2 ? kSelHi : kSelZero;
    const uint32_t t2 = q < 2 ? kSelLo : kSelZero;
    const unsigned gq = lane >> 4, j = lane & 15u, u = j & 7u;

    mx_wait_vm<2u * kMxs422C>();                    /* the image (older than the pixel DMA) */
    __builtin_amdgcn_s_barrier();
    mx_wave_sync();
    if (cmp.b >= g.total) {
        mx_wait_vm<0>();                                /* no LDS-DMA outlives the wave */
        return;
    }
    uint32_t za[8];
    {
        const unsigned s = (j >> 3) * 4u + gq;
        const uint32_t base = (uint32_t)(uintptr_t)mx_lds(L.stage) + kBS2 * s, hs = mx2_h(s);
        const mx_u2 sc = *(const mx_u2 *)&s_img.scan_t[u][0];
#pragma unroll
        for (int v = 0; v < 8; v++) {
            const uint32_t zz = (v < 4 ? sc.x : sc.y) >> (8 * (v & 3)) & 0xffu;
            za[v] = base + 16u * ((zz >> 3) ^ hs) + 2u * (zz & 7u);
        }
    }
    /* the B operands; reloaded after an exact pass, so that their registers are free during it */
    mx_u4 B[kParts][4];
    const auto load_b = [&](unsigned l) __attribute__((always_inline)) {
#pragma unroll
        for (int p = 0; p < kParts; p++) {
            const mx_u4 by = s_img.B[3 * p][l], zero = {};
            B[p][0] = (l & 15u) < 8 ? by : zero;
            B[p][1] = (l & 15u) < 8 ? zero : by;
            B[p][2] = s_img.B[3 * p + 1][l];
            B[p][3] = s_img.B[3 * p + 2][l];
        }
    };
    load_b(lane);
    const float limc0 = s_img.limc[0][j], limc2 = s_img.limc[1][j];
    const MxTab &tb = s_img.tab;
    const MxExLds xt{s_img.ex, s_img.scan_t};

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
            mx422_exact_inline(L, sp, qmask, fl, xt);
            load_b(mx_lane());
        }
        /* always two store instructions (the vmcnt accounting counts on it) */
        if (S.simple) {
            /* the store's lane offsets, re-derived here (no VGPRs held across the step for them) */
            const unsigned l = mx_lane();
            const uint32_t soy = l * 16u, soc = (l & 31u) * 16u + (l >> 5) * (g.nb / 2u) * 128u;
            const mx_u4 vy = *(const mx_u4 *)(L.stage + mx2_ro(l));
            const mx_u4 vc = *(const mx_u4 *)(L.stage + mx2_ro(l) + kSt422C);
            __builtin_nontemporal_store(vy, (mx_u4 *)((const uint8_t *)S.dst + soy));
            __builtin_nontemporal_store(vc, (mx_u4 *)((const uint8_t *)S.cdst + soc));
        } else {
            const unsigned l = mx_lane();
            const unsigned by = S.b + (l >> 3), bc = S.b + 2u * ((l >> 3) & 3u);
            const unsigned yb = by < g.total ? by : g.total - 1u, cbk = bc < g.total ? bc : g.total - 1u;
            const unsigned fy = yb / g.nb, biy = yb - fy * g.nb;
            const unsigned fc = cbk / g.nb, bic = cbk - fc * g.nb;
            const mx_u4 vy = *(const mx_u4 *)(L.stage + mx2_ro(l));
            const mx_u4 vc = *(const mx_u4 *)(L.stage + mx2_ro(l) + kSt422C);
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
        if (cmp.b >= g.total) {
            mx_wait_vm<0>();                            /* no LDS-DMA outlives the wave */
            return;
        }
        mx_wait_vm<2 * (kMxs422C - 1 - k) + 2 * k>();
        body(cmp, L.ring[k]);
        mxs_next(cmp, g);
    };
    step(std::integral_constant<unsigned, 0>{});
    step(std::integral_constant<unsigned, 1>{});
    step(std::integral_constant<unsigned, 2>{});
}

/* ==== k_mxs420: true 4:2:0 (extension, JPGX_FLAG_SUBSAMPLE, sample_ratio 2), round 4 ========
 *
 * One wave = one step pair: a step is two consecutive MCUs (MCU-linear launch-global index, frames
 * concatenated), their 16 pixel rows x 96 bytes (8 Y blocks: the top block row of the two MCUs is
 * set 0, the bottom one set 1) in a 1.5-KiB LDS slot by the same LDS-DMA as k_mxs; both steps' DMA
 * up front (slots 0 and 1); four waves per workgroup sharing the LDS image.
 *   Y       k_mxs422's Y: the two sets K-concatenated, column j = set j / 8 at u = j % 8.
 *   Chroma  A row m = (MCU cb = m >> 3, chroma row Y' = m & 7), K = the 96 bytes of the MCU's
 *           pixel rows 2Y', 2Y'+1 over three K = 32 products; B (jpgx_plan.cpp
 *           jx_mx420_operands) holds 0.25 a[c][p] cos((2 floor(x/2) + 1) u pi/16): column j of
 *           the one C tile is the row transform of the quad-averaged chroma, Cb (j < 8) or Cr, at
 *           rows 4gq..4gq+3 of the tile.  After the pair's second step, one v_permlane16_swap per
 *           row value gives every lane a whole column of one of the pair's four MCUs (lane gq: MCU
 *           (gq & 1) 2 + (gq >> 1) of the pair), so the chroma column DCTs run once per pair on
 *           all 64 lanes: 1.5 column passes per step; step 0's chroma R tile waits in LDS (rA).
 *   Output  per step 8 Y blocks in one store (lanes 0..31 the top row, 32..63 the bottom row, bpr
 *           blocks further); the pair's 4 Cb + 4 Cr blocks leave with step 1: step 0 waits
 *           vmcnt(2), step 1 vmcnt(1).
 *   Quirk   a general step whose MCU's right block column is a row's last loads that column's
 *           true pixel rows into L.qtrue (inside the chroma stage region, which the chroma column
 *           only writes after the A operands are read).
 *   Exact   inline: Y tasks from the slot; chroma tasks read their MCU's pixels from global
 *           memory, in the oracle's order: ((ls(p00) + ls(p01)) + (ls(p10) + ls(p11))) * 0.25.
 */
constexpr unsigned kSt420C = 8 * kBS2;        /* chroma (c, lane group gq) in slot 8 + 4 c + gq (mx2_coef) */

/* MCU geometry of the launch */
struct Mx420G {
    unsigned mpr, nmcu, tm, rows;       /* MCUs per row, per frame, in the launch; MCU rows per frame */
    jx_udiv dmpr, dnmcu;                /* division by mpr, nmcu (jx_geom) */
};

struct Mx420Chunk {
    unsigned m0, f, mi, my, mx;         /* first MCU (launch-global), frame, MCU in frame, row, col */
    const uint8_t *src;                 /* pixel (16 mx, 16 my) of frame f */
    int16_t *ydst, *cdst;               /* Y block (2my, 2mx), chroma block mi (Cb) of frame f */
};

__device__ __forceinline__ void mx420_ptrs(Mx420Chunk &C, const MxG &g, const Mx420G &h)
{
    C.src = g.rgb + (long long)C.f * g.fstride + 16ll * C.my * g.pitch + 48ll * C.mx;
    C.ydst = g.out + (long long)C.f * g.ofstride + 64ll * (2ull * C.my * g.bpr + 2u * C.mx);
    C.cdst = g.out + (long long)C.f * g.ofstride + 64ll * (g.nb + C.mi);
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

/* the MCU's pixel (0, 0) */
__device__ __forceinline__ const uint8_t *mx420_mcu_src(const MxG &g, const Mx420G &h, unsigned m)
{
    unsigned f, mi, my, mx;
    mx420_mcu(h, m, f, mi, my, mx);
    return g.rgb + (long long)f * g.fstride + 16ll * my * g.pitch + 48ll * mx;
}

/* pair-MCU of a chroma-column lane group (the permlane16 swap's order) */
__device__ __forceinline__ unsigned mx420_pm(unsigned gq) { return (gq & 1u) * 2u + (gq >> 1); }

/* Inline exact pass: Y bits (col 0) of this step and chroma bits (col 1, pair base mp).  A chroma
 * task's MCU pm of the pair lies in slot pm / 2 (bytes 48 (pm & 1) of each of its 16 pixel rows) of
 * a simple pair (both slots intact after step 1's rows); a general pair's MCUs (quirk rows, frame
 * or launch ends) read their pixels from global memory. */
template <class Lds, class XT>
__device__ __forceinline__ void mx420_exact_inline(Lds &L, const uint8_t *sp, uint32_t bits, unsigned mp,
                                                   bool simple, const uint8_t *ps0, const uint8_t *ps1,
                                                   const MxG &g, const Mx420G &h, const XT &xt)
{
    const unsigned lane = mx_lane();
    mx_wave_sync();
    const auto chroma = [&](unsigned gq, auto &&fn) __attribute__((always_inline)) {
        const unsigned pm = mx420_pm(gq);
        if (simple)
            return fn(MxSmp4<lds_u8, unsigned>{mx_lds((void *)((pm >> 1) ? ps1 : ps0)) + 48u * (pm & 1u), 96u});
        unsigned m = mp + pm;
        m = m < h.tm ? m : h.tm - 1u;
        return fn(MxSmp4<uint8_t, long long>{mx420_mcu_src(g, h, m), g.pitch});
    };
    mx_exact_single(bits, [&](unsigned sl, unsigned bt) __attribute__((always_inline)) {
        const unsigned k = bt >> 3, v = bt & 7u, jj = sl & 15u, u = jj & 7u, gq = sl >> 4;
        const unsigned slot = 4u * (jj >> 3) + gq;
        int val;
        bool ok;
        if (k == 0)
            ok = mx_exact_one(MxSmp1{mx_lds((void *)sp) + 768u * (jj >> 3) + 24u * gq, 96u}, 0u, u, v, xt, val);
        else
            ok = chroma(gq, [&](const auto &smp) __attribute__((always_inline)) {
                return mx_exact_one(smp, 1u + (jj >> 3), u, v, xt, val);
            });
        return mx_put_one(L.stage, mx2_coef(slot + (k ? 8u : 0u), xt.scan(u, v)), ok, val);
    });
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
        if (k == 0)
            val = mx_exact_coef<true>(MxSmp1{mx_lds((void *)sp) + 768u * (jj >> 3) + 24u * gq, 96u}, 0u, u, v, x, xt);
        else
            val = chroma(gq, [&](const auto &smp) __attribute__((always_inline)) {
                return mx_exact_coef<true>(smp, 1u + (jj >> 3), u, v, x, xt);
            });
        if (live && x == 7)
            *(__attribute__((address_space(3))) int16_t *)(mx_lds(L.stage) + mx2_coef(slot + (k ? 8u : 0u), xt.scan(u, v))) =
                (int16_t)val;
        mx_wave_sync();
    }
}

/* Y block (launch-global, frame-concatenated) of step m0's block (set, jb) */
__device__ __forceinline__ unsigned mx420_yblock(const MxG &g, const Mx420G &h, unsigned m0, unsigned set,
                                                 unsigned jb)
{
    unsigned f, mi, my, mx;
    mx420_mcu(h, m0 + (jb >> 1), f, mi, my, mx);
    return f * g.nb + (2u * my + set) * g.bpr + 2u * mx + (jb & 1u);
}

struct alignas(16) Mxs420Lds {
    uint8_t ring[3][kSlot];             /* [y 0..15][4 blocks x 24 B]: steps 0, 1, 2; step 3 reuses slot 0 */
    union {
        uint8_t stage[16 * kBS2];
        struct {                        /* general step: MCU's right column, true rows [16][24]; read
                                           for the A operands before the Y column writes here */
            uint8_t qtrue[2][384];
            uint8_t y_[kSt420C - 2 * 384];
            mx_f4 rA[64];               /* a pair's first chroma R tile, in the chroma stage (written
                                           at the end of the pair's first step, read before the
                                           pair's chroma column writes there) */
        };
    };
    uint16_t task[8];
};
static_assert(2 * 384 <= kSt420C && 64 * 16 <= 16 * kBS2 - kSt420C, "qtrue in the Y stage, rA in the chroma stage");
constexpr unsigned kMxs420WPG = 4;
struct alignas(16) MxsImg420 {
    mx_u4 B[JX_MX_PARTS * 4][64];       /* [part * 4 + which]: the two Y sets merged (as k_mxs422), chroma K steps */
    MxTab tab;
    float limc[2][16];
    uint8_t scan_t[8][8];
    MxExTab ex;
};
constexpr unsigned kMxs420Pieces = sizeof(MxsImg420) / 16;
static_assert(sizeof(MxsImg420) % 16 == 0 && kMxs420Pieces <= 1024, "four 16-byte pieces per thread");
static_assert(sizeof(Mxs420Lds) % 16 == 0 && sizeof(Mxs420Lds) * kMxs420WPG + sizeof(MxsImg420) <= 40 * 1024,
              "4 workgroups of 4 waves per CU");
__device__ MxsImg420 g_mxs420_img[2][JX_MAXQ + 1];

__global__ __launch_bounds__(64 * kMxs420WPG, kWPE) void k_mxs420(const jx_xform_args a)
{
    __shared__ __attribute__((aligned(16))) Mxs420Lds s_lds[kMxs420WPG];
    __shared__ __attribute__((aligned(16))) MxsImg420 s_img;
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
    const unsigned wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    Mxs420Lds &L = s_lds[wave];
    {
        const uint8_t *img = (const uint8_t *)&g_mxs420_img[g.force ? 1 : 0][g.quality];
#pragma unroll
        for (unsigned i = 0; i < (kMxs420Pieces + 64u * kMxs420WPG - 1u) / (64u * kMxs420WPG); i++) {
            const unsigned piece = 64u * kMxs420WPG * i + threadIdx.x;
            if (64u * kMxs420WPG * i + 64u * wave < kMxs420Pieces && piece < kMxs420Pieces)
                mxs_dma<16>(img + 16u * piece, (uint8_t *)&s_img + 16u * (64u * kMxs420WPG * i + 64u * wave));
        }
    }
    /* two pairs: MCUs m0 .. m0 + 3 and m0 + 4 .. m0 + 7; simple = one MCU row of one frame, no
     * row-last MCU, in range (per pair) */
    const unsigned m0 = 8u * (blockIdx.x * kMxs420WPG + wave);
    const uint32_t off0 = (uint32_t)((lane / 6u) * (unsigned)g.pitch + 16u * (lane % 6u));
    const uint32_t off1 = (uint32_t)(((64u + lane) / 6u) * (unsigned)g.pitch + 16u * ((64u + lane) % 6u));
    /* the current pair's cursor; of pair 1 only its pixel pointer is kept until its steps (SGPRs) */
    Mx420Chunk cc;
    bool simple[2] = {false, false};
    const uint8_t *src1 = g.rgb;
#pragma unroll
    for (unsigned pp = 0; pp < 2; pp++) {
        const unsigned mp = m0 + 4u * pp;
        if (mp < h.tm) {
            mx420_at(cc, g, h, mp);
            simple[pp] = mp + 4u <= h.tm && cc.mx + 4u < h.mpr && g.lin_store;
            if (pp == 1) src1 = cc.src;
        }
    }
    if (m0 < h.tm) mx420_at(cc, g, h, m0);
    /* steps 0, 1 (pair 0) and 2 (pair 1's first) into slots 0..2 now; step 3 into slot 0 after
     * pair 0 is done (mx420_dma3) */
#pragma unroll
    for (unsigned k = 0; k < 3; k++) {
        const unsigned pp = k >> 1, ks = k & 1u;
        const uint8_t *src = pp ? src1 : cc.src;
        if (simple[pp]) {
            mxs_dma<16>(src + 96u * ks + off0, L.ring[k]);
            if (lane < 32) mxs_dma<16>(src + 96u * ks + off1, L.ring[k] + 1024u);
        } else {
            mxs_dma<4>(g.rgb, L.ring[k]);                   /* padding: filled at compute time */
            mxs_dma<4>(g.rgb, L.ring[k]);
        }
    }

    /* lane constants */
    const unsigned m = lane & 15u, q = lane >> 4;
    const uint32_t aoff = 96u * (m & 3u) + 24u * (m >> 2) + 8u * (q < 3 ? q : 2u);
    const uint32_t s0 = q < 3 ? kSelLo : kSelOne;
    const uint32_t s1 = q < 3 ? kSelHi : kSelZero;
    const uint32_t s2 = q < 3 ? kSelLo : kSelZero;
    const uint32_t cof0 = 192u * (m & 7u) + 48u * (m >> 3) + 8u * q;
    const uint32_t cof1 = cof0 + (q < 2 ? 32u : 80u);
    const uint32_t soy = (lane & 31u) * 16u + (lane >> 5) * g.bpr * 128u;
    const uint32_t soc = (lane & 31u) * 16u + (lane >> 5) * h.nmcu * 128u;
    const uint32_t ro = mx2_ro(lane);                         /* mx2_piece(lane >> 3, lane & 7) */
    const uint32_t rc = mx2_piece(8u + 4u * (lane >> 5) + mx420_pm((lane >> 3) & 3u), lane & 7u);
    const unsigned gq = lane >> 4, j = lane & 15u, u = j & 7u;

    mx_wait_vm<6>();                                    /* the image (older than the pixel DMA) */
    __builtin_amdgcn_s_barrier();
    mx_wave_sync();
    if (m0 >= h.tm) {
        mx_wait_vm<0>();                                /* no LDS-DMA outlives the wave */
        return;
    }
    uint32_t za[8];
    {
        const unsigned s = 4u * (j >> 3) + gq;
        const uint32_t base = (uint32_t)(uintptr_t)mx_lds(L.stage) + kBS2 * s, hs = mx2_h(s);
        const mx_u2 sc = *(const mx_u2 *)&s_img.scan_t[u][0];
#pragma unroll
        for (int v = 0; v < 8; v++) {
            const uint32_t zz = (v < 4 ? sc.x : sc.y) >> (8 * (v & 3)) & 0xffu;
            za[v] = base + 16u * ((zz >> 3) ^ hs) + 2u * (zz & 7u);
        }
    }
    /* the B operands; reloaded after an exact pass, so that their registers are free during it */
    mx_u4 B[kParts][5];
    const auto load_b = [&](unsigned l) __attribute__((always_inline)) {
#pragma unroll
        for (int p = 0; p < kParts; p++) {
            const mx_u4 by = s_img.B[4 * p][l], zero = {};
            B[p][0] = (l & 15u) < 8 ? by : zero;
            B[p][1] = (l & 15u) < 8 ? zero : by;
#pragma unroll
            for (int w = 2; w < 5; w++) B[p][w] = s_img.B[4 * p + w - 1][l];
        }
    };
    load_b(lane);
    const float limc0 = s_img.limc[0][j], limc2 = s_img.limc[1][j];
    const MxTab &tb = s_img.tab;
    const MxExLds xt{s_img.ex, s_img.scan_t};

    const auto step = [&](auto kc) __attribute__((always_inline)) {
        constexpr unsigned k = decltype(kc)::value;
        constexpr unsigned pp = k >> 1, slot = k == 3 ? 0u : k;
        constexpr bool second = (k & 1u) != 0;
        const unsigned mp = m0 + 4u * pp;               /* the pair's first MCU */
        const unsigned ms = mp + 2u * (k & 1u);         /* the step's first MCU */
        if (mp >= h.tm) {
            mx_wait_vm<0>();
            return;
        }
        /* the step's DMA has landed: younger are 4 / 2 + 1 / 1 + 2 + 2 / 1 operations */
        if (k == 0)
            mx_wait_vm<4>();
        else if (k == 1)
            mx_wait_vm<3>();
        else if (k == 2)
            mx_wait_vm<5>();
        else
            mx_wait_vm<1>();
        const bool simp = simple[pp];
        if (k == 2) mx420_at(cc, g, h, mp);             /* pair 1's cursor */
        uint8_t *const sp = L.ring[slot];
        if (!simp) mx420_issue_general(g, h, ms, sp);      /* register path; waits vmcnt(0) */
        const uint32_t qmask = simp ? 0u : mx420_true_rows(L, g, h, ms);
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
            if (kParts == 3) {
                accC[1] = mx_mma(C0, B[kParts - 1][2], accC[1]);
                accC[1] = mx_mma(C1, B[kParts - 1][3], accC[1]);
                accC[1] = mx_mma(C2, B[kParts - 1][4], accC[1]);
            }
        }
        __builtin_amdgcn_sched_barrier(0);
        mx_fence_all(accC);
        mx_keep(midC);
        mx_keep_ops(C1, C2);
        __builtin_amdgcn_sched_barrier(0);
        mx_column_t<0, true>(accY, MxW{}, limc0, tb, 0, j, za, fl, 0);
        __builtin_amdgcn_sched_barrier(0);
        const mx_f4 rc4 = {accC[1].x + accC[0].x, accC[1].y + accC[0].y, accC[1].z + accC[0].z,
                           accC[1].w + accC[0].w};   /* scalar adds (no packed fp32, mx_unpack8) */
        __builtin_amdgcn_sched_barrier(0);
        if (second) {
            const mx_f4 rA0 = L.rA[lane];
            float lo4[4], hi4[4];
#pragma unroll
            for (int i = 0; i < 4; i++) {
                const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(rA0[i]), __float_as_uint(rc4[i]),
                                                                false, false);
                lo4[i] = __uint_as_float(r[0]);
                hi4[i] = __uint_as_float(r[1]);
            }
            const float R[8] = {lo4[0], lo4[1], lo4[2], lo4[3], hi4[0], hi4[1], hi4[2], hi4[3]};
            mx_column_r<kSt420C>(R, mx_w(tb, 2, j), limc2, tb, 2, j, za, fl, 1);
        } else {
            L.rA[lane] = rc4;
        }
        mx_wave_sync();
        if (__builtin_expect(__ballot(fl != 0) != 0, 0)) {
            {   /* clamped MCUs past the launch's end: no tasks */
                if (ms + (gq >> 1) >= h.tm) fl &= ~0xffu;
                if (mp + mx420_pm(gq) >= h.tm) fl &= ~0xff00u;
            }
            mx420_exact_inline(L, sp, fl, mp, simp, L.ring[pp ? 2 : 0], L.ring[pp ? 0 : 1], g, h, xt);
            if (k < 3) load_b(mx_lane());
        }
        /* stores: the Y store; on the second step also the pair's chroma */
        if (simp) {
            const mx_u4 vy = *(const mx_u4 *)(L.stage + ro);
            __builtin_nontemporal_store(vy, (mx_u4 *)((const uint8_t *)(cc.ydst + 256u * (k & 1u)) + soy));
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
                const mx_u4 vy = *(const mx_u4 *)(L.stage + mx2_ro(l));
                if (mm < h.tm)
                    __builtin_nontemporal_store(
                        vy, (mx_u4 *)(g.out + (long long)f * g.ofstride + (long long)bi * 64 + (l & 7u) * 8));
            }
            if (second) {
                const unsigned pm = (l >> 3) & 3u, mm = mp + pm;
                const unsigned mc = mm < h.tm ? mm : h.tm - 1u;
                unsigned f, mi, my, mx;
                mx420_mcu(h, mc, f, mi, my, mx);
                const mx_u4 vc = *(const mx_u4 *)(L.stage + mx2_piece(8u + 4u * (l >> 5) + mx420_pm(pm), l & 7u));
                if (mm < h.tm)
                    __builtin_nontemporal_store(
                        vc, (mx_u4 *)(g.out + (long long)f * g.ofstride +
                                      ((long long)g.nb + (l >> 5) * h.nmcu + mi) * 64 + (l & 7u) * 8));
            }
        }
        mx_wave_sync();
        if (k == 1) {
            /* pair 0 is done with slot 0 (its chroma exact pass read it): step 3's pixels into it,
             * from inline asm so that the compiler does not drain vmcnt before step 2's LDS reads
             * (it does after a builtin LDS-DMA, not knowing which bytes it writes).  The asm sets
             * M0, which the compiler treats as reserved: no instruction of the kernel after this
             * point reads M0 (the builtin LDS-DMAs are all in the prologue; checked in the ISA by
             * tests/test_isa.py). */
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"
            const uint32_t l0 = (uint32_t)(uintptr_t)mx_lds(L.ring[0]);
            if (m0 + 4u < h.tm && simple[1]) {
                const uint8_t *src = src1 + 96u + off0;
                asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(src), "s"(l0)
                             : "memory", "m0");
                const uint8_t *srcb = src1 + 96u + off1;
                const uint32_t l1 = l0 + 1024u;
                if (lane < 32)
                    asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(srcb), "s"(l1)
                                 : "memory", "m0");
            } else {
                asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dword %0, off" ::"v"(g.rgb), "s"(l0)
                             : "memory", "m0");
                asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dword %0, off" ::"v"(g.rgb), "s"(l0)
                             : "memory", "m0");
            }
#pragma clang diagnostic pop
        }
    };
    step(std::integral_constant<unsigned, 0>{});
    step(std::integral_constant<unsigned, 1>{});
    step(std::integral_constant<unsigned, 2>{});
    step(std::integral_constant<unsigned, 3>{});
}

int mx_rc(hipError_t e) { return e == hipSuccess ? JPGX_OK : JPGX_EHIP; }

constexpr int kMaxDev = 64;

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

/* the per-quality tables of one kernel family ([force][quality]): scales w (2^9 folded, kRScale),
 * squared band limits (all -1 under FORCE_EXACT), divisors and the fast decision's reciprocals */
template <class Plan>
int mx_plan_tabs(std::vector<jx_mxtab> &tab, Plan plan)
{
    tab.assign(2 * (JX_MAXQ + 1), jx_mxtab{});
    for (int q = 1; q <= JX_MAXQ; q++) {
        float w[24][8], lim[24][8];
        int16_t qq[2][64];
        const int rc = plan(q, w, lim, qq);
        if (rc) return rc;
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
    return JPGX_OK;
}

/* table tt (0 scales, 1 squared limits of the plan columns n0 + jp ..., 2 / 3 of the chroma
 * columns) of one MxTab in the [t][half][profile] layout; ncol(tt, jp) = the plan column */
template <class Col>
void mx_layout_tab(MxTab &o, const jx_mxtab &t, Col ncol)
{
    for (unsigned tt = 0; tt < 4; tt++)
        for (unsigned jp = 0; jp < 16; jp++) {
            const unsigned n = ncol(tt, jp);
            float x[8];
            for (int pp = 0; pp < 4; pp++)
                for (int h = 0; h < 2; h++) {
                    const int v = jx_pk_k(pp, h);
                    x[2 * pp + h] = (tt & 1u) ? t.lsq[n][v] : t.w[n][v];
                }
            o.wl[tt][0][jp] = mx_f4{x[0], x[1], x[2], x[3]};
            o.wl[tt][1][jp] = mx_f4{x[4], x[5], x[6], x[7]};
        }
}

/* zig-zag position of (v, u) at [u][v] (zig_zag.c:6-15) */
void mx_scan_t(uint8_t (&st)[8][8])
{
    static const int scan[8][8] = JX_SCAN_ORDER_INIT;
    for (int uu = 0; uu < 8; uu++)
        for (int v = 0; v < 8; v++) st[uu][v] = (uint8_t)scan[v][uu];
}

/* the exact pass's LDS tables: the glibc cosines and this quality's divisors */
void mx_ex_tab(MxExTab &x, const jx_mxtab &t)
{
    static const double cosx[8][8] = JX_COS_INIT;
    memcpy(x.cosx_, cosx, sizeof cosx);
    memcpy(x.q_, t.q, sizeof t.q);
    memcpy(x.r_, t.r, sizeof t.r);
}

std::once_flag g_mx_once[kMaxDev];
int g_mx_rc[kMaxDev];

int mx_tables_for_current_device()
{
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDev) return JPGX_ENODEV;
    std::call_once(g_mx_once[dev], [dev]() {
        std::vector<jx_mxtab> tab;
        int rc = mx_plan_tabs(tab, jx_plan_tables_mx);
        std::unique_ptr<uint16_t[][64][8]> opsp(new uint16_t[3 * JX_MX_PARTS][64][8]);   /* heap: reentrant */
        auto ops = opsp.get();
        if (!rc) rc = jx_mx_operands(ops);
        if (!rc) {
            /* k_mxs's workgroup images: B operands, the scale / limit table (Y|Cb at 16 lane
             * profiles, Cr compacted to 8), the hot-path limits mx_limc computes from the full
             * table, the zig-zag positions and the exact pass's tables */
            std::vector<MxsImg> img(2 * (JX_MAXQ + 1));
            memset(img.data(), 0, img.size() * sizeof(MxsImg));
            for (int f = 0; f < 2; f++)
                for (int q = 1; q <= JX_MAXQ; q++) {
                    MxsImg &I = img[f * (JX_MAXQ + 1) + q];
                    const jx_mxtab &t = tab[f * (JX_MAXQ + 1) + q];
                    mx_ex_tab(I.ex, t);
                    MxTab full;
                    mx_layout_tab(full, t, [](unsigned tt, unsigned jp) { return tt < 2 ? jp : 16u + (jp & 7u); });
                    for (unsigned jp = 0; jp < 16; jp++) {
                        I.limc[0][jp] = mx_limc(full, 1, jp);
                        I.limc[1][jp] = mx_limc(full, 3, jp);
                        for (int tt = 0; tt < 2; tt++)
                            for (int h = 0; h < 2; h++) {
                                I.tab.yc[tt][h][jp] = full.wl[tt][h][jp];
                                if (jp < 8) I.tab.cr[tt][h][jp] = full.wl[2 + tt][h][jp];
                            }
                    }
                    mx_scan_t(I.scan_t);
                }
            if (!rc) rc = mx_rc(hipMemcpyToSymbol(HIP_SYMBOL(g_mxs_img), img.data(), img.size() * sizeof(MxsImg)));
            /* the Cr sets' operands are zero in opposite column halves (B1 in 8..15, B2 in 0..7):
             * the kernel's Cr sum cr[0] + cr[1] is exact because of it */
            for (int p = 0; p < JX_MX_PARTS; p++)
                for (unsigned l = 0; l < 64; l++)
                    for (int e = 0; e < 8; e++)
                        if (ops[3 * p + ((l & 15u) < 8 ? 2 : 1)][l][e]) rc = JPGX_EARG;
            if (!rc) rc = mx_rc(hipMemcpyToSymbol(HIP_SYMBOL(g_mxs_B), ops, sizeof(uint16_t) * 3 * JX_MX_PARTS * 64 * 8));
        }
        g_mx_rc[dev] = rc;
    });
    return g_mx_rc[dev];
}

std::once_flag g_mx422_once[kMaxDev];
int g_mx422_rc[kMaxDev];

int mx422_tables_for_current_device()
{
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDev) return JPGX_ENODEV;
    std::call_once(g_mx422_once[dev], [dev]() {
        std::vector<jx_mxtab> tab;
        int rc = mx_plan_tabs(tab, jx_plan_tables_mx422);
        std::unique_ptr<uint16_t[][4][64][8]> opsp(new uint16_t[JX_MX_PARTS][4][64][8]);   /* heap: reentrant */
        auto ops = opsp.get();
        if (!rc) rc = jx_mx422_operands(ops);
        if (!rc) {
            /* k_mxs422's image: B operands, the scale / limit table (Y at plan column j % 8,
             * chroma at 8 + j), hot-path limits, zig-zag positions, the exact pass's tables */
            std::vector<MxsImg422> img(2 * (JX_MAXQ + 1));
            memset(img.data(), 0, img.size() * sizeof(MxsImg422));
            for (size_t i = 0; i < img.size(); i++) {
                mx_layout_tab(img[i].tab, tab[i], [](unsigned tt, unsigned jp) { return tt < 2 ? (jp & 7u) : 8u + jp; });
                for (int p = 0; p < JX_MX_PARTS; p++)
                    for (unsigned l = 0; l < 64; l++) {
                        const bool set0 = (l & 15u) < 8;
                        const uint16_t *keep = ops[p][set0 ? 0 : 1][l], *zero = ops[p][set0 ? 1 : 0][l];
                        for (int e = 0; e < 8; e++)
                            if (zero[e]) rc = JPGX_EARG;      /* the merge needs the zero halves (as jpgx_plan.cpp) */
                        memcpy(&img[i].B[3 * p][l], keep, 16);
                        memcpy(&img[i].B[3 * p + 1][l], ops[p][2][l], 16);
                        memcpy(&img[i].B[3 * p + 2][l], ops[p][3][l], 16);
                    }
                for (unsigned jp = 0; jp < 16; jp++) {
                    img[i].limc[0][jp] = mx_limc(img[i].tab, 1, jp);
                    img[i].limc[1][jp] = mx_limc(img[i].tab, 3, jp);
                }
                mx_scan_t(img[i].scan_t);
                mx_ex_tab(img[i].ex, tab[i]);
            }
            if (!rc) rc = mx_rc(hipMemcpyToSymbol(HIP_SYMBOL(g_mxs422_img), img.data(), img.size() * sizeof(MxsImg422)));
        }
        g_mx422_rc[dev] = rc;
    });
    return g_mx422_rc[dev];
}

std::once_flag g_mx420_once[kMaxDev];
int g_mx420_rc[kMaxDev];

int mx420_tables_for_current_device()
{
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDev) return JPGX_ENODEV;
    std::call_once(g_mx420_once[dev], [dev]() {
        std::vector<jx_mxtab> tab;
        int rc = mx_plan_tabs(tab, jx_plan_tables_mx420);
        std::unique_ptr<uint16_t[][5][64][8]> opsp(new uint16_t[JX_MX_PARTS][5][64][8]);   /* heap: reentrant */
        auto ops = opsp.get();
        if (!rc) rc = jx_mx420_operands(ops);
        if (!rc) {
            /* k_mxs420's image (the 4:2:2 table layout) */
            std::vector<MxsImg420> img(2 * (JX_MAXQ + 1));
            memset(img.data(), 0, img.size() * sizeof(MxsImg420));
            for (size_t i = 0; i < img.size(); i++) {
                for (int p = 0; p < JX_MX_PARTS; p++)
                    for (unsigned l = 0; l < 64; l++) {
                        const bool set0 = (l & 15u) < 8;   /* the Y sets' zero halves (as k_mxs422) */
                        const uint16_t *keep = ops[p][set0 ? 0 : 1][l], *zero = ops[p][set0 ? 1 : 0][l];
                        for (int e = 0; e < 8; e++)
                            if (zero[e]) rc = JPGX_EARG;
                        memcpy(&img[i].B[4 * p][l], keep, 16);
                        for (int w = 2; w < 5; w++) memcpy(&img[i].B[4 * p + w - 1][l], ops[p][w][l], 16);
                    }
                mx_layout_tab(img[i].tab, tab[i], [](unsigned tt, unsigned jp) { return tt < 2 ? (jp & 7u) : 8u + jp; });
                for (unsigned jp = 0; jp < 16; jp++) {
                    img[i].limc[0][jp] = mx_limc(img[i].tab, 1, jp);
                    img[i].limc[1][jp] = mx_limc(img[i].tab, 3, jp);
                }
                mx_scan_t(img[i].scan_t);
                mx_ex_tab(img[i].ex, tab[i]);
            }
            if (!rc) rc = mx_rc(hipMemcpyToSymbol(HIP_SYMBOL(g_mxs420_img), img.data(), img.size() * sizeof(MxsImg420)));
        }
        g_mx420_rc[dev] = rc;
    });
    return g_mx420_rc[dev];
}

}  // namespace

/* a launch on `stream`; with ev_start / ev_stop (hipEvent_t, both or neither) through
 * hipExtLaunchKernel, whose events carry the kernel's own begin / end timestamps -- the interval a
 * rocprofv3 kernel trace reports, without the queue gap before the dispatch (bench.py) */
template <class K>
void mx_launch_k(K kernel, dim3 grid, dim3 block, hipStream_t s, void *ev_start, void *ev_stop, const jx_xform_args &a)
{
    if (ev_start && ev_stop)
        hipExtLaunchKernelGGL(kernel, grid, block, 0, s, (hipEvent_t)ev_start, (hipEvent_t)ev_stop, 0, a);
    else
        hipLaunchKernelGGL(kernel, grid, block, 0, s, a);
}

/* k_mxs420 over every frame of the stripe (true 4:2:0: Y [nb][64], Cb and Cr [nb / 4][64] per
 * frame, the stripe an even number of block rows); no workspace. */
extern "C" int jx_launch_mx420(const jx_xform_args *xa, void *stream, void *ev_start, void *ev_stop)
{
    const int rc = mx420_tables_for_current_device();
    if (rc) return rc;
    const size_t mcus = (size_t)xa->g.nb / 4 * (size_t)xa->g.nframes;
    const size_t waves = (mcus + 7) / 8;
    mx_launch_k(k_mxs420, dim3((unsigned)((waves + kMxs420WPG - 1) / kMxs420WPG)), dim3(64 * kMxs420WPG), (hipStream_t)stream,
                ev_start, ev_stop, *xa);
    return mx_rc(hipGetLastError());
}

/* k_mxs422 over every frame of the stripe (true 4:2:2: Y [nb][64], Cb and Cr [nb / 2][64] per
 * frame); no workspace. */
extern "C" int jx_launch_mx422(const jx_xform_args *xa, void *stream, void *ev_start, void *ev_stop)
{
    const int rc = mx422_tables_for_current_device();
    if (rc) return rc;
    const size_t nsteps = ((size_t)xa->g.nb * (size_t)xa->g.nframes + 7) / 8;
    const size_t waves = (nsteps + kMxs422C - 1) / kMxs422C;
    mx_launch_k(k_mxs422, dim3((unsigned)((waves + kMxs422WPG - 1) / kMxs422WPG)), dim3(64 * kMxs422WPG), (hipStream_t)stream,
                ev_start, ev_stop, *xa);
    return mx_rc(hipGetLastError());
}

/* k_mxs over every frame of the stripe (4:4:4 / reference-parity output); no workspace. */
extern "C" int jx_launch_mx(const jx_xform_args *xa, void *stream, void *ev_start, void *ev_stop)
{
    const int rc = mx_tables_for_current_device();
    if (rc) return rc;
    const size_t nsteps = ((size_t)xa->g.nb * (size_t)xa->g.nframes + 7) / 8;
    const size_t waves = (nsteps + kMxsC - 1) / kMxsC;
    mx_launch_k(k_mxs, dim3((unsigned)((waves + kMxsWPG - 1) / kMxsWPG)), dim3(64 * kMxsWPG), (hipStream_t)stream,
                ev_start, ev_stop, *xa);
    return mx_rc(hipGetLastError());
}

/* the kernel a launch runs for sample ratio 0 (4:4:4), 1 (true 4:2:2), 2 (4:2:0): bench.py and
 * the profiles name the kernel they time with it */
extern "C" const char *jx_mx_kernel_name(int sr)
{
    if (sr == 1) return "k_mxs422";
    if (sr == 2) return "k_mxs420";
    return "k_mxs";
}
