/*
 * jpgx_internal.h -- launch-argument layouts shared by the host plan (jpgx_plan.cpp) and
 * the gfx950 kernels (jpgx_kernels.hip).  Passed by value as kernel arguments so the
 * per-coefficient tables are read with scalar loads (wave-uniform).
 */
#ifndef JPGX_INTERNAL_H
#define JPGX_INTERNAL_H

#include <stddef.h>
#include <stdint.h>

#include "../../include/jpgx.h"

#define JX_WG 256           /* threads per workgroup for the transform (4 waves)           */

/* unsigned 32-bit division by a launch constant d >= 1 as a multiply-high (Granlund and
 * Montgomery's round-up method): q = (t + ((n - t) >> s1)) >> s2, t = mulhi(m, n); exact for
 * every 32-bit n.  Lets a wave find its position with a few scalar operations instead of the
 * ~35-instruction software division. */
struct jx_udiv {
    uint32_t m, s1, s2;
};
static inline struct jx_udiv jx_udiv_make(uint32_t d)
{
    unsigned l = 0;
    while (l < 32 && (1ull << l) < (unsigned long long)d) l++;
    struct jx_udiv r;
    r.m = (uint32_t)(((1ull << 32) * ((1ull << l) - d)) / d + 1);
    r.s1 = l ? 1u : 0u;
    r.s2 = l ? l - 1u : 0u;
    return r;
}

struct jx_geom {
    const uint8_t *rgb;     /* pixel (0, 8*row_begin) of frame 0                          */
    int16_t *out;           /* frame 0 output [3][nb][64]                                 */
    long long in_pitch;     /* bytes                                                      */
    long long in_fstride;   /* bytes                                                      */
    long long out_fstride;  /* int16 elements                                             */
    int bpr;                /* blocks per block-row (width/8)                             */
    int nb;                 /* blocks per frame in this stripe                            */
    int nframes;
    int row0;               /* frame block-row of stripe row 0 (underflow only at row 0)  */
    uint32_t under[6];      /* the underflow pixel row, interleaved (u0 u0 u0 u1 u1 u1..)  */
    struct jx_udiv dnb, dbpr;   /* division by nb and by bpr                              */
    uint32_t mpr, nmcu;         /* true 4:2:0: MCUs per MCU row, per frame (16x16 MCUs)       */
    struct jx_udiv dmpr, dnmcu; /* division by them                                       */
};

/* Per-quality tables, device resident (one copy per quality 1..97, built once per device).
 * Column-major ([ch][u][v]) so one column's 8 entries are one scalar load. */
struct jx_qtab {
    float w[3][8][8];       /* [ch][u][v]: fp32 scale of coefficient (u,v), 1/Q folded    */
    int16_t q[2][64];       /* scaled tables, q[t][u*8+v] = Qs[u][v] as the reference
                               indexes them (src/quantise.c:58)                           */
};

/* guard band: |t - rint(t)| >= lim -> exact path.  [0] = rigorous band, [1] = FORCE_EXACT
 * (every entry -1: every coefficient takes the exact path) */
struct jx_limtab {
    float lim[3][8][8];     /* [ch][u][v] */
};

#define JX_MAXQ 97

/* k_mx (csrc/jpgx_mx.hip): the colour conversion + row DCT of each pixel row is one f16 MFMA
 * product with B split into JX_MX_PARTS f16 parts (hi exact, lo parts scaled by 2^12).  Per
 * quality, plan column n = 8c + u holds the scales and guard band of coefficients (c, u,
 * v = 0..7). */
#ifndef JX_MX_PARTS
#define JX_MX_PARTS 2       /* 2: hi + one lo part (band 1.28x that of 3 parts, 16 MFMAs per
                               8 blocks instead of 24: jpgx_plan.cpp's bound covers either) */
#endif
/* scale of the lo f16 parts of B (exponent): 0 stores them at the hi parts' scale, so R = acc_h +
 * acc_l is one add (round 4); 12 stores them x 2^12 (R = fma(acc_l, 2^-12, acc_h), rounds 2-3).
 * Either way R = fl(acc_h + acc_l) bit for bit. */
#ifndef JX_MX_LOEXP
#define JX_MX_LOEXP 0
#endif
struct jx_mxtab {
    float w[24][8];         /* 1/4 a(u) a(v) k(v) / Q[u][v] (row transform uses exact cosines) */
    float lsq[24][8];       /* a float <= lim^2 of the rigorous band (flag: d*d - lsq >= 0);
                               -1 with FORCE_EXACT                                            */
    int16_t q[2][64];       /* scaled tables, q[t][u*8+v] = Qs[u][v] (src/quantise.c:58)       */
    double r[2][64];        /* fl(fl(1/4 a(u) a(v)) / q[t][u*8+v]): the exact pass's fast decision */
};

struct jx_xform_args {
    jx_geom g;
    int quality;            /* index into the device table                                */
    int force_exact;        /* JPGX_FLAG_FORCE_EXACT: flag every coefficient              */
    int luma_only;          /* k_xform: channel 0 only (chroma from k_chroma)             */
    int sub;                /* k_chroma: 1 = true 4:2:2, 2 = true 4:2:0                   */
};


#ifdef __cplusplus
extern "C" {
#endif
/* host plan (jpgx_plan.cpp) */
int jx_plan_tables(int quality, float w[3][64], float lim[3][64], int16_t q[2][64]);
/* the same for true chroma subsampling: sub 1 = 4:2:2 averages, 2 = 4:2:0 (chroma bounds) */
int jx_plan_tables_mode(int quality, int sub, float w[3][64], float lim[3][64], int16_t q[2][64]);
void jx_under_dwords(const uint8_t under[3][8], uint32_t out[6]);
/* packed-pair vs scalar transform, bit for bit (host; returns the mismatch count) */
long long jx_selftest_pk(long long nblocks, unsigned long long seed);
int jx_mx_parts(void);
int jx_mx_loexp(void);
/* k_mx: tables and f16 B operands (host plan), launch (device side) */
int jx_plan_tables_mx(int quality, float w[24][8], float lim[24][8], int16_t q[2][64]);
int jx_mx_operands(uint16_t ops[3 * JX_MX_PARTS][64][8]);
long long jx_selftest_mx(long long nblocks, unsigned long long seed, int quality,
                         long long *flagged, double *ratio);
int jx_launch_mx(const struct jx_xform_args *xa, void *stream, void *ev_start, void *ev_stop);
/* k_mx422 (true 4:2:2 on the matrix cores): operands [part][which][lane], tables, launch */
int jx_mx422_operands(uint16_t ops[JX_MX_PARTS][4][64][8]);
int jx_plan_tables_mx422(int quality, float w[24][8], float lim[24][8], int16_t q[2][64]);
long long jx_selftest_mx422(long long nblocks, unsigned long long seed, int quality,
                            long long *flagged, double *ratio);
int jx_launch_mx422(const struct jx_xform_args *xa, void *stream, void *ev_start, void *ev_stop);
/* k_mx420 (true 4:2:0 on the matrix cores): operands [part][which][lane], tables, launch */
int jx_mx420_operands(uint16_t ops[JX_MX_PARTS][5][64][8]);
int jx_plan_tables_mx420(int quality, float w[24][8], float lim[24][8], int16_t q[2][64]);
long long jx_selftest_mx420(long long nblocks, unsigned long long seed, int quality,
                            long long *flagged, double *ratio);
int jx_launch_mx420(const struct jx_xform_args *xa, void *stream, void *ev_start, void *ev_stop);
#ifdef __cplusplus
}
#endif

#endif
