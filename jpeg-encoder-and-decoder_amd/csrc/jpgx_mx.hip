/*
 * jpgx_mx.hip -- k_mx, the gfx950 block-transform kernel with the colour conversion and the
 * row DCT on the matrix cores (v_mfma_f32_32x32x16_f16), the column DCT, quantiser, guard
 * band and zig-zag in VALU, and the exact-order fp64 pass for guard-band coefficients inside
 * the same waves.
 *
 * Reference path: preprocess.c:160-162,186-188 (colour + level shift) -> dct.c:36-59 ->
 * quantise.c:52-72 (transposed divisor, round()) -> zig_zag.c:48-58; output = the three
 * JpgData.zig_zag_* arrays, [frame][Y|Cb|Cr][nb][64] int16.
 *
 * Work unit.  Each wave walks a contiguous range of "steps" of 8 consecutive blocks
 * (launch-global block index, frames concatenated); a step is two MFMA groups of 4 blocks.
 * Per group, lane l loads ONE 16-byte piece: pixel row y of block blk (the A-operand row
 * m = l & 31 of the group) at byte offset 8 hA, hA = l >> 5 (jpgx_plan.cpp: K layout), issued
 * a step ahead.  MFMA row m = 8i + 4hh + j <-> block blk = 2hh + (i >> 1)... precisely:
 *     i = (m & 3) + 4 (m >> 3),  blk = 2 ((m >> 2) & 1) + (i & 1),  y = i >> 1,
 * so that in the 32x32 result (column n = lane & 31 = 8c + u, rows (r & 3) + 8 (r >> 2) +
 * 4 (lane >> 5) in register r) lane half h holds all 8 pixel rows of blocks 2h, 2h + 1 as the
 * aligned register pairs (2y, 2y + 1):
 *     A[m][k]  = b_k - 128 (exact in f16; bytes -> f16 by v_perm + v_pk_add_f16),
 *                the bias slot A = 1.0 (k-step 1, lane half 0, element 0)
 *     R[m][n]  = (A Bh) + 2^-12 (A Bl [+ A Bm])    (acc_h exact: jpgx_plan.cpp)
 * = the colour-converted, level-shifted row transform of all three channels, 2 * JX_MX_PARTS
 * MFMAs per 4 blocks.  Each lane then runs the column DCT of its column for its two blocks in
 * lock-step (jx_fdct8 over v_pk_* pairs: lane by lane the FOps code the guard band is derived
 * for), quantises with the per-lane (c,u) scales (tm = F w + 1.5 2^23: the low 16 bits are the
 * rounded int16), writes each int16 to the wave's LDS stage at its zig-zag position, and folds
 * the guard-band test d^2 - lim^2 >= 0 (d = F w - rint, exact) into one running max.  After each
 * step, the 8 blocks x 3 channels x 128 B leave as three 1-KiB nontemporal stores.
 *
 * Exactness.  A group whose running max says "some coefficient inside the
 * band" (rare: wave-uniform branch) re-tests its coefficients, copies the flagged blocks'
 * pixel rows (already in registers) into an LDS slot and queues one task per flagged
 * coefficient.  A full queue, and the end of the wave's range, run the exact pass: eight tasks
 * at a time, eight lanes each -- lane x forms (X(x,y) c_u[x]) c_v[y] in fp64 for y = 0..7
 * with X in the reference's double colour arithmetic, the 64-term sum runs x-outer / y-inner
 * (dct.c:46-50) through lanes x = 0..7 in turn, then F = ((1/4 a(u)) a(v)) s and round(F / Q)
 * with the transposed divisor.  The exact value patches the LDS stage if its block belongs to
 * the step being built, else global memory (after the wave's earlier stores have landed).
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
typedef float mx_f2 __attribute__((ext_vector_type(2)));

constexpr float kMagic = 12582912.0f;   /* 1.5 * 2^23: x + kMagic rounds x to an integer   */
constexpr int kParts = JX_MX_PARTS;
constexpr int kSlots = 10;              /* LDS pixel slots (one block each) for exact tasks */
constexpr int kRecs = 4;                /* flagged-group records per wave                   */
#ifndef JX_MX_WPE
#define JX_MX_WPE 4                     /* waves per SIMD the register allocation targets  */
#endif

/* LDS stage: channel c at mx_stage_base(c), 8 blocks x 128 B each, blocks in step order,
 * zig-zag order inside a block.  The bases put the three channels' 16-bit zig-zag writes of one
 * instruction on different banks (bank = dword % 32: shifts 0, 4, 16 dwords; at most 3-way,
 * about 2-way on average over the 8 rows v) and keep every 16-byte store chunk aligned.  The
 * MFMA's padding columns 24..31 compute Y's columns again (jx_mx_operands), so those lanes
 * write the very values lanes 0..7 write to the same addresses: no dummy area, no exec mask. */
__host__ __device__ constexpr unsigned mx_stage_base(unsigned c)
{
    return 1152u * c + 16u * (c + 2u * (c >> 1));
}
constexpr unsigned kStageBytes = mx_stage_base(2) + 1024;

struct MxLds {
    uint8_t stage[kStageBytes];
    mx_u4 in[2][2][64];                 /* [step & 1][group][lane]: the A-operand pieces, landed
                                           by LDS-DMA one step ahead                         */
    uint8_t pix[kSlots][8][24];         /* exact tasks: the flagged blocks' 8 pixel rows    */
    uint16_t rbits[kRecs][64];          /* flagged-group record: per lane, bit 2v + j = its
                                           coefficient (u, v) of block 2h + j is in the band */
    uint32_t rblk[kRecs];               /* the group's first launch-global block            */
    uint8_t rslot[kRecs][4];            /* pixel slot of each of its 4 blocks               */
    uint32_t tblk[8];                   /* one exact batch: launch-global block             */
    uint16_t tcode[8];                  /*                  slot << 9 | c << 6 | v << 3 | u  */
};
static_assert(kStageBytes % 16 == 0, "LDS-DMA pieces must stay 16-byte aligned");

__device__ mx_u4 g_mxB[2 * kParts][64];          /* B operands: (part, kstep) x lane      */
__device__ jx_mxtab g_mxtab[2][JX_MAXQ + 1];     /* [force][quality]                      */
__constant__ double kMxCos[8][8] = JX_COS_INIT;
__constant__ int kMxScan[8][8] = JX_SCAN_ORDER_INIT;
constexpr double kMxAlpha0 = JX_ALPHA0;
/* per channel the reference's colour constants as the exact pass uses them: t = (k0 r + k1 g)
 * + k2 b (the signs of its subtractions folded into k1, k2: a - b*k == a + b*(-k) exactly),
 * then (A + S t) - 128 with (A, S) = (0, 1) Y, (128, -1) Cb, (128, 1) Cr */
__constant__ double kMxQuarterAlpha[8] = {0.25 * JX_ALPHA0, 0.25, 0.25, 0.25, 0.25, 0.25, 0.25, 0.25};
__constant__ double kMxAlpha[8] = {JX_ALPHA0, 1.0, 1.0, 1.0, 1.0, 1.0, 1.0, 1.0};
__constant__ double kMxColour[3][5] = {{0.299, 0.587, 0.114, 0.0, 1.0},
                                       {0.168736, -0.331264, 0.5, 128.0, -1.0},
                                       {0.5, -0.418688, -0.081312, 128.0, 1.0}};

/* Order this wave's LDS accesses across lanes: a wave's LDS instructions execute in program
 * order, so only the compiler must be kept from moving memory operations across this point
 * (no fence: a wavefront-scope fence makes the compiler drain the vector memory counter). */
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

/* The lane id, recomputed where it is used by the rare paths: an opaque (volatile) value
 * cannot be hoisted, so the rare paths' lane-derived constants do not occupy registers
 * across the tile loop. */
__device__ __forceinline__ unsigned mx_lane()
{
    unsigned l;
    asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
    return l;
}

/* four pixel bytes of dword d -> two f16 b - 128: perm makes 0x64bb (= 1024 + b) from each
 * byte (K = 0x64646481: byte 5 is 0x64, byte 4 is 0x81 = 129, which the bias selector of
 * lane half 0 picks to make 1153 - 1152 = 1.0), then one packed subtraction, exact. */
__device__ __forceinline__ uint32_t mx_cvt2(uint32_t K, uint32_t d, uint32_t sel)
{
    const mx_h2 v = __builtin_bit_cast(mx_h2, __builtin_amdgcn_perm(K, d, sel)) -
                    (mx_h2){(_Float16)1152.0f, (_Float16)1152.0f};
    return __builtin_bit_cast(uint32_t, v);
}

/* The launch geometry as plain values (references into the kernel-argument struct, or indexed
 * reads of its arrays, make the compiler copy it to scratch) */
struct MxG {
    const uint8_t *rgb;
    int16_t *out;
    long long pitch, fstride, ofstride;
    unsigned bpr, nb, total;
    int row0, quality, force;
    uint32_t u[6];                      /* the underflow pixel row (jx_geom.under) */
};

typedef const mx_u4 __attribute__((address_space(1))) *mx_gp;   /* global (not flat) loads */

/*
 * Address of the 16 bytes of pixel row y of block b (launch-global, clamped into range) at
 * offset 8 hA, with the reference's addressing: blockToCoords (preprocess.c:199-211) gives
 * x0 = -8 for the last block of a block-row, i.e. pixel row 8r+y-1, columns W-8..W-1; at frame
 * block-row 0, y = 0 those are the bytes in front of the planes (the underflow row): *under is
 * set and the address points at a readable row (the value is replaced at its use).
 */
__device__ __forceinline__ const uint8_t *mx_addr_general(const MxG &g, unsigned b, unsigned y,
                                                         unsigned hA, bool *under)
{
    b = b < g.total ? b : g.total - 1u;
    const unsigned f = b / g.nb, bi = b - f * g.nb;
    const unsigned r = bi / g.bpr, c = bi - r * g.bpr;
    const bool last = c == g.bpr - 1u;
    *under = last && y == 0 && g.row0 + (int)r == 0;
    const long long pr = *under ? 0 : 8ll * r + y - (last ? 1 : 0);
    return g.rgb + (long long)f * g.fstride + pr * g.pitch + 24ll * c + 8 * hA;
}

/* position of a step's first block: frame f, block bi in the frame, block-row r, column c */
struct MxPos {
    unsigned f, bi, r, c;
};

__device__ __forceinline__ void mx_advance(MxPos &p, const MxG &g)
{
    p.bi += 8u;
    p.c += 8u;
    while (p.c >= g.bpr) {
        p.c -= g.bpr;
        p.r++;
    }
    while (p.bi >= g.nb) {          /* next frame (frames smaller than a step: several) */
        p.bi -= g.nb;
        p.f++;
        p.r = p.bi / g.bpr;
        p.c = p.bi - p.r * g.bpr;
    }
}

/* the step's 8 blocks lie in one block-row of one frame, none is the row's last block, and
 * all are in range: the fast (one-add) load and store addressing applies */
__device__ __forceinline__ bool mx_simple(const MxPos &p, const MxG &g, unsigned b0)
{
    return p.c + 8u < g.bpr && b0 + 8u <= g.total;
}

/* The two group loads of the step at position P (first block b0), by LDS-DMA into dst[q]
 * (lane l's 16 bytes land at dst[q][l]): one global_load_lds_dwordx4 per group on every path
 * (the general path only computes other addresses; bit q of the return value marks a lane
 * whose group-q piece is the underflow row, replaced at its use). */
__device__ __forceinline__ uint32_t mx_issue(const MxG &g, const MxPos &P, unsigned b0,
                                             bool simple, uint32_t laneoff, mx_u4 (*dst)[64])
{
    const uint8_t *p[2];
    uint32_t un = 0;
    if (simple) {
        const uint8_t *base = g.rgb + (long long)P.f * g.fstride + 8ll * P.r * g.pitch +
                              24ll * P.c + laneoff;
        p[0] = base;
        p[1] = base + 96;
    } else {
        const unsigned lane = mx_lane(), m = lane & 31u, hA = lane >> 5;
        const unsigned iA = (m & 3u) + 4u * (m >> 3);
        const unsigned blkA = 2u * ((m >> 2) & 1u) + (iA & 1u), yA = iA >> 1;
#pragma unroll
        for (int q = 0; q < 2; q++) {
            bool uq;
            p[q] = mx_addr_general(g, b0 + 4u * q + blkA, yA, hA, &uq);
            un |= (uq ? 1u : 0u) << q;
        }
    }
#ifdef JX_MX_DBG_NOLOAD        /* timing experiments only: no pixel loads (pieces set once) */
    if (un != 0xdeadbeefu) {
        const unsigned l = mx_lane();
#pragma unroll
        for (int q = 0; q < 2; q++) {
            const uint32_t h = (l * 2654435761u) ^ (q * 0x9e3779b9u) ^ b0;
            dst[q][l] = mx_u4{h, h * 747796405u + 1u, h ^ 0x5bd1e995u, h * 3u + 7u};
        }
        return un;
    }
#endif
#pragma unroll
    for (int q = 0; q < 2; q++)
        __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *)p[q],
                                         (__attribute__((address_space(3))) void *)&dst[q][0],
                                         16, 0, 0);
    return un;
}

/*
 * One exact batch of n <= 8 tasks (L.tblk / L.tcode), eight lanes each: lane x of task i forms
 * the products (X(x,y) c_u[x]) c_v[y], y = 0..7 (dct.c:48-50, X in the reference's double
 * colour arithmetic, preprocess.c:160-162,186-188), and the sum runs x-outer / y-inner
 * (dct.c:46-47) through lanes x = 0..7 in turn; F = ((1/4 a(u)) a(v)) s (dct.c:54) and
 * round(F / Q) with the transposed divisor (quantise.c:58).  Blocks >= step_b0 (the step whose
 * stage is being built) patch the stage; the others global memory (the caller has waited for
 * the wave's stores).
 */
__device__ __forceinline__ void mx_batch(MxLds &L, int nt, const MxG &g, unsigned step_b0)
{
    const unsigned lane = mx_lane();
    const jx_mxtab &T = g_mxtab[0][g.quality];
    const unsigned i = lane >> 3, x = lane & 7u;
    const bool live = (int)i < nt;
    const unsigned blk = L.tblk[live ? i : 0u];
    const unsigned code = L.tcode[live ? i : 0u];
    const int slot = (int)(code >> 9), ch = (int)((code >> 6) & 7u), v = (int)((code >> 3) & 7u),
              u = (int)(code & 7u);
    const double cu = kMxCos[u][x];
    const double k0c = kMxColour[ch][0], k1c = kMxColour[ch][1], k2c = kMxColour[ch][2];
    const double Ac = kMxColour[ch][3], Sc = kMxColour[ch][4];
    double prod[8];
#pragma unroll
    for (int y = 0; y < 8; y++) {
        const uint8_t *px = &L.pix[slot][y][3 * x];
        const double rr = (double)px[0], gg = (double)px[1], bb = (double)px[2];
        const double tt = (k0c * rr + k1c * gg) + k2c * bb;
        const double X = (Ac + Sc * tt) - 128.0;
        prod[y] = X * cu * kMxCos[v][y];
    }
    double sum = 0.0;
#pragma unroll
    for (int xx = 0; xx < 8; xx++) {
        if ((int)x == xx) {
#pragma unroll
            for (int y = 0; y < 8; y++) sum += prod[y];
        }
        sum = __shfl(sum, (int)((lane & ~7u) | (unsigned)xx), 64);
    }
    if (live && x == 0) {
        /* ((0.25 * a(u)) * a(v)) * s, dct.c:54 (0.25 * a(u) is exact in the table) */
        const double F = kMxQuarterAlpha[u] * kMxAlpha[v] * sum;
        const int q = T.q[ch == 0 ? 0 : 1][u * 8 + v];
        const int16_t val = (int16_t)(int)round(F / (double)q);
        const int z = kMxScan[v][u];
        if (blk >= step_b0) {
            *(int16_t *)(L.stage + mx_stage_base((unsigned)ch) + (blk - step_b0) * 128u + 2u * z) = val;
        } else {
            const unsigned f = blk / g.nb, bi = blk - f * g.nb;
            g.out[(long long)f * g.ofstride + ((long long)ch * g.nb + bi) * 64 + z] = val;
        }
    }
    mx_wave_sync();                                    /* batch buffer reused */
}

/* Exact pass over every recorded flagged group: tasks eight at a time (the records are
 * expanded lane by lane, lowest bit first). */
__device__ __forceinline__ void mx_drain(MxLds &L, int nrec, const MxG &g, unsigned step_b0)
{
    const unsigned lane = mx_lane();
#ifdef JX_MX_EXPERIMENT_NODRAIN
    return;
#endif
    const unsigned n = lane & 31u, h = lane >> 5, c = n >> 3, u = n & 7u;
    __builtin_amdgcn_s_waitcnt(0xF70);                 /* vmcnt(0): the wave's stores landed */
    mx_wave_sync();
    int nt = 0;
    for (int r = 0; r < nrec; r++) {
        uint32_t bits = L.rbits[r][lane];
        const unsigned gb0 = L.rblk[r];
        for (;;) {
            const uint64_t act = __ballot(bits != 0);
            if (!act) break;
            const int room = 8 - nt, rk = mx_rank(act);
            if (bits != 0 && rk < room) {
                const int k = __builtin_ctz(bits);
                bits &= bits - 1u;
                const unsigned v = (unsigned)k >> 1, blk = 2u * h + ((unsigned)k & 1u);
                L.tblk[nt + rk] = gb0 + blk;
                L.tcode[nt + rk] = (uint16_t)((unsigned)L.rslot[r][blk] << 9 | c << 6 | v << 3 | u);
            }
            nt += std::min((int)__popcll(act), room);
            mx_wave_sync();
            if (nt == 8) {
                mx_batch(L, 8, g, step_b0);
                nt = 0;
            }
        }
    }
    if (nt) mx_batch(L, nt, g, step_b0);
    /* nothing of the exact pass stays in flight: the tile loop's wait accounting (and the
     * compiler's, which would otherwise drain the counter at every reuse of these registers)
     * starts clean */
    __builtin_amdgcn_s_waitcnt(0xF70);
}

/*
 * Rare path of one group (some lane's running max says a coefficient is inside the band):
 * re-test every coefficient (the fast path's arithmetic exactly) and record the flagged ones
 * with the flagged blocks' pixel rows (already in registers) copied to LDS slots; the caller
 * guarantees room for one record and four slots.
 */
__device__ __forceinline__ void mx_record(MxLds &L, int &nrec, int &nslot, const mx_f2 (&F)[8],
                                          const float (&w)[8], const float (&lsq)[8], mx_u4 ld,
                                          unsigned gb0)
{
    const unsigned lane = mx_lane();
    const unsigned n = lane & 31u;
    const unsigned m = lane & 31u, hA = lane >> 5;
    const unsigned iA = (m & 3u) + 4u * (m >> 3);
    const unsigned blkA = 2u * ((m >> 2) & 1u) + (iA & 1u), yA = iA >> 1;
    uint32_t bits = 0;
#pragma unroll
    for (int v = 7; v >= 0; v--) {
        const float t0 = __builtin_fmaf(F[v].x, w[v], kMagic);
        const float t1 = __builtin_fmaf(F[v].y, w[v], kMagic);
        const float d0 = __builtin_fmaf(F[v].x, w[v], -(t0 - kMagic));
        const float d1 = __builtin_fmaf(F[v].y, w[v], -(t1 - kMagic));
        const float e0 = __builtin_fmaf(d0, d0, -lsq[v]);
        const float e1 = __builtin_fmaf(d1, d1, -lsq[v]);
        bits = (bits << 2) | (e1 >= 0.0f ? 2u : 0u) | (e0 >= 0.0f ? 1u : 0u);
    }
    if (n >= 24) bits = 0;
    /* flagged blocks of the group: bit (2h + j) */
    const uint64_t m0 = __ballot((bits & 0x5555u) != 0), m1 = __ballot((bits & 0xaaaau) != 0);
    const unsigned blkmask = ((uint32_t)m0 ? 1u : 0u) | ((uint32_t)m1 ? 2u : 0u) |
                             ((m0 >> 32) ? 4u : 0u) | ((m1 >> 32) ? 8u : 0u);
    if (!blkmask) return;
    const int r = nrec;
    L.rbits[r][lane] = (uint16_t)bits;
    if (lane == 0) L.rblk[r] = gb0;
    if (lane < 4) {
        const bool fl = (blkmask >> lane) & 1u;
        L.rslot[r][lane] = fl ? (uint8_t)(nslot + __builtin_popcount(blkmask & ((1u << lane) - 1u))) : 0;
    }
    if ((blkmask >> blkA) & 1u) {
        const int sl = nslot + __builtin_popcount(blkmask & ((1u << blkA) - 1u));
        uint8_t *row = &L.pix[sl][yA][8 * hA];
        *(uint32_t *)(row + 0) = ld.x;
        *(uint32_t *)(row + 4) = ld.y;
        *(uint32_t *)(row + 8) = ld.z;
        *(uint32_t *)(row + 12) = ld.w;
    }
    nrec++;
    nslot += __builtin_popcount(blkmask);
}

/* Colour conversion + row DCT of one group of 4 blocks through the matrix cores: R[y] =
 * (block 2h, block 2h + 1) at pixel row y for this lane's column n. */
__device__ __forceinline__ void mx_rows(mx_u4 ld, uint32_t K, uint32_t selb, const mx_h8 (&B)[2 * kParts],
                                        mx_f2 (&R)[8])
{
    const uint32_t s0 = 0x05010500u, s1 = 0x05030502u;
    const mx_u4 a0 = {mx_cvt2(K, ld.x, s0), mx_cvt2(K, ld.x, s1), mx_cvt2(K, ld.y, s0),
                      mx_cvt2(K, ld.y, s1)};
    const mx_u4 a1 = {mx_cvt2(K, ld.z, selb), mx_cvt2(K, ld.z, s1), mx_cvt2(K, ld.w, s0),
                      mx_cvt2(K, ld.w, s1)};
    const mx_h8 A0 = __builtin_bit_cast(mx_h8, a0), A1 = __builtin_bit_cast(mx_h8, a1);
    const mx_f16 zero = {};
    mx_f16 ah = __builtin_amdgcn_mfma_f32_32x32x16_f16(A0, B[0], zero, 0, 0, 0);
    mx_f16 al = __builtin_amdgcn_mfma_f32_32x32x16_f16(A0, B[2], zero, 0, 0, 0);
    ah = __builtin_amdgcn_mfma_f32_32x32x16_f16(A1, B[1], ah, 0, 0, 0);
    al = __builtin_amdgcn_mfma_f32_32x32x16_f16(A1, B[3], al, 0, 0, 0);
    if (kParts == 3) {
        al = __builtin_amdgcn_mfma_f32_32x32x16_f16(A0, B[4 % (2 * kParts)], al, 0, 0, 0);
        al = __builtin_amdgcn_mfma_f32_32x32x16_f16(A1, B[5 % (2 * kParts)], al, 0, 0, 0);
    }
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
#pragma unroll
    for (int k = 0; k < 6; k++) g.u[k] = a.g.under[k];

    const unsigned lane = threadIdx.x & 63u;
    MxLds &L = s_lds[threadIdx.x >> 6];
    /* each wave walks a contiguous range of steps */
    const unsigned nsteps = (g.total + 7u) / 8u;
    const unsigned nw = gridDim.x * 4u;
    const unsigned wv = __builtin_amdgcn_readfirstlane(blockIdx.x * 4u + (threadIdx.x >> 6));
    const unsigned s_end = (unsigned)(((unsigned long long)nsteps * (wv + 1)) / nw);
    unsigned s = (unsigned)(((unsigned long long)nsteps * wv) / nw);
    if (s >= s_end) return;

    /* A-operand row of this lane (both groups): block blkA of the group, pixel row yA */
    const unsigned hA = lane >> 5, m = lane & 31u;
    const unsigned iA = (m & 3u) + 4u * (m >> 3);
    const unsigned blkA = 2u * ((m >> 2) & 1u) + (iA & 1u), yA = iA >> 1;
    const uint32_t laneoff = (uint32_t)(yA * (unsigned)g.pitch + 24u * blkA + 8u * hA);
    const uint32_t K = 0x64646481u;
    const uint32_t selb = hA ? 0x05010500u : 0x05010504u;

    /* output column n = 8c + u of this lane; C-layout lane half h = blocks 2h, 2h + 1 */
    const unsigned n = lane & 31u, h = lane >> 5;
    const unsigned cz = (n >> 3) % 3u, uz = n & 7u;     /* padding columns 24..31 = Y again */
    const jx_mxtab &T = g_mxtab[g.force ? 1 : 0][g.quality];
    float w[8], lsq[8];
    uint32_t zo[8];
#pragma unroll
    for (int v = 0; v < 8; v++) {
        w[v] = T.w[n][v];
        lsq[v] = T.lsq[n][v];
        zo[v] = mx_stage_base(cz) + 256u * h + 2u * (unsigned)kMxScan[v][uz];
    }
    mx_h8 B[2 * kParts];
#pragma unroll
    for (int i = 0; i < 2 * kParts; i++) B[i] = __builtin_bit_cast(mx_h8, g_mxB[i][lane]);

    int nrec = 0, nslot = 0;               /* flagged-group records, pixel slots in use */
    MxPos P;
    {
        const unsigned b0 = 8u * s;
        P.f = b0 / g.nb;
        P.bi = b0 - P.f * g.nb;
        P.r = P.bi / g.bpr;
        P.c = P.bi - P.r * g.bpr;
    }
    /* the loads of the wave's first step; every later step issues the next step's loads
     * right after waiting for its own (vmcnt counts loads, LDS-DMA and stores in issue order:
     * younger than this step's DMA are only the previous step's three stores) */
    uint32_t un = mx_issue(g, P, 8u * s, mx_simple(P, g, 8u * s), laneoff, L.in[s & 1u]);
    __builtin_amdgcn_s_waitcnt(0xF70);           /* vmcnt(0): tables, operands, first step */
    bool first = true;
    for (; s < s_end; s++) {
        const unsigned b0 = 8u * s;
        const MxPos PC = P;
        if (!first) __builtin_amdgcn_s_waitcnt(0xF73);   /* vmcnt(3) */
        first = false;
        mx_wave_sync();
        const uint32_t uc = un;
        mx_advance(P, g);
        if (s + 1u < s_end)
            un = mx_issue(g, P, b0 + 8u, mx_simple(P, g, b0 + 8u), laneoff, L.in[(s + 1u) & 1u]);
        const bool underrow = !mx_simple(PC, g, b0) && __ballot(uc != 0) != 0;
#pragma unroll
        for (int q = 0; q < 2; q++) {
            mx_u4 ld = L.in[s & 1u][q][lane];
            if (underrow && ((uc >> q) & 1u))       /* rare: the underflow row */
                ld = hA ? mx_u4{g.u[2], g.u[3], g.u[4], g.u[5]} : mx_u4{g.u[0], g.u[1], g.u[2], g.u[3]};
            mx_f2 R[8], F[8];
#if defined(JX_MX_DBG_NOCOMPUTE)  /* timing experiments only: the stage writes, no transform */
#pragma unroll
            for (int v = 0; v < 8; v++) {
                *(uint16_t *)(L.stage + zo[v] + 512u * q) = (uint16_t)(ld[v & 3] >> (v & 16));
                *(uint16_t *)(L.stage + zo[v] + 512u * q + 128u) = (uint16_t)(ld[(v + 1) & 3]);
            }
            if (ld.x == 0xdeadbeefu)
#endif
            {
#ifdef JX_MX_DBG_NOMFMA          /* timing experiments only: R by VALU from the bytes */
#pragma unroll
            for (int y = 0; y < 8; y++)
                R[y] = mx_f2{(float)((ld[y & 3] >> (8 * (y >> 2))) & 0xffu) - 128.0f,
                             (float)((ld[(y + 1) & 3] >> 8) & 0xffu) - 128.0f} * 7.0f;
#else
            mx_rows(ld, K, selb, B, R);
#endif
            jx_fdct8<PairOps<MxPair>>(R, F);
            }
            float emax = -1.0f;
#if defined(JX_MX_DBG_NOCOMPUTE)
            if (ld.x == 0xdeadbeefu)
#endif
#pragma unroll
            for (int v = 0; v < 8; v++) {
                /* quant_coef: tm = F w + 1.5 2^23 (low 16 bits = the rounded int16), d = F w -
                 * rint (exact); band test d*d - lsq >= 0 folded into a running max */
                const float t0 = __builtin_fmaf(F[v].x, w[v], kMagic);
                const float t1 = __builtin_fmaf(F[v].y, w[v], kMagic);
#ifndef JX_MX_DBG_NOSTAGE        /* timing experiments only: no zig-zag LDS writes */
                *(uint16_t *)(L.stage + zo[v] + 512u * q) = (uint16_t)__float_as_uint(t0);
                *(uint16_t *)(L.stage + zo[v] + 512u * q + 128u) = (uint16_t)__float_as_uint(t1);
#else
                emax += __uint_as_float(__float_as_uint(t0) ^ __float_as_uint(t1)) * 1e-30f;
#endif
                const float d0 = __builtin_fmaf(F[v].x, w[v], -(t0 - kMagic));
                const float d1 = __builtin_fmaf(F[v].y, w[v], -(t1 - kMagic));
                const float e0 = __builtin_fmaf(d0, d0, -lsq[v]);
                const float e1 = __builtin_fmaf(d1, d1, -lsq[v]);
                emax = __builtin_fmaxf(emax, __builtin_fmaxf(e0, e1));
            }
#ifdef JX_MX_DBG_NORARE           /* timing experiments only: no exact pass */
            if (emax == 12345.0f)
#else
            if (__ballot(emax >= 0.0f))              /* rare: some coefficient in the band */
#endif
                mx_record(L, nrec, nslot, F, w, lsq, ld, b0 + 4u * q);
            __builtin_amdgcn_sched_barrier(0);
        }
        mx_wave_sync();
        /* exact pass when the next step might not find room (rarely before the wave's end) */
        if (nrec > kRecs - 2 || nslot > kSlots - 8) {
            mx_drain(L, nrec, g, b0);
            nrec = 0;
            nslot = 0;
        }
        /* stores: channel c's 8 blocks x 128 B are contiguous, 16 B per lane; always three
         * store instructions (the vmcnt(3) above counts on it) */
#ifdef JX_MX_DBG_NOSTORE        /* timing experiments only: no coefficient stores */
        if (b0 == 0xdeadbeefu)
#endif
        if (mx_simple(PC, g, b0)) {
            int16_t *ob = g.out + (long long)PC.f * g.ofstride + (long long)PC.bi * 64 + lane * 8;
#pragma unroll
            for (int c = 0; c < 3; c++) {
                const mx_u4 val = *(const mx_u4 *)(L.stage + mx_stage_base(c) + lane * 16);
                __builtin_nontemporal_store(val, (mx_u4 *)(ob + (long long)c * g.nb * 64));
            }
        } else {
            /* lanes past the end rewrite the last block's chunk with its own bytes */
            const unsigned lane = mx_lane();
            const unsigned bl = b0 + (lane >> 3), b = bl < g.total ? bl : g.total - 1u;
            const unsigned f = b / g.nb, bi = b - f * g.nb;
            const unsigned src = bl < g.total ? lane : ((g.total - 1u - b0) << 3) | (lane & 7u);
#pragma unroll
            for (int c = 0; c < 3; c++) {
                const mx_u4 val = *(const mx_u4 *)(L.stage + mx_stage_base(c) + src * 16);
                __builtin_nontemporal_store(
                    val, (mx_u4 *)(g.out + (long long)f * g.ofstride +
                                   ((long long)c * g.nb + bi) * 64 + (lane & 7u) * 8));
            }
        }
        mx_wave_sync();
    }
    if (nrec) mx_drain(L, nrec, g, 0xffffffffu);
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
                for (int n = 0; n < 32; n++)        /* columns 24..31 repeat Y's 0..7 */
                    for (int v = 0; v < 8; v++) {
                        t.w[n][v] = w[n % 24][v];
                        t.lsq[n][v] = f ? -1.0f : mx_lsq(lim[n % 24][v]);
                    }
            }
        }
        uint16_t ops[2 * kParts][64][8];
        if (!rc) rc = jx_mx_operands(ops);
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

/* k_mx over every frame of the stripe (4:4:4 / reference-parity output); no workspace. */
extern "C" int jx_launch_mx(const jx_xform_args *xa, void *stream)
{
    int waves = 0;
    const int rc = mx_tables_for_current_device(&waves);
    if (rc) return rc;
    const size_t total = (size_t)xa->g.nb * (size_t)xa->g.nframes;
    const size_t nsteps = (total + 7) / 8;
    const size_t w = std::min<size_t>(nsteps, (size_t)std::max(waves, 4));
    const unsigned grid = (unsigned)((w + 3) / 4);
    hipLaunchKernelGGL(k_mx, dim3(grid), dim3(256), 0, (hipStream_t)stream, *xa);
    return mx_rc(hipGetLastError());
}
