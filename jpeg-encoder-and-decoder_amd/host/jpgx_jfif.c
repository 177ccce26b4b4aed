/*
 * jpgx_jfif.c -- baseline JFIF writer for the block transform's output (host C99).
 *
 * The reference never writes a file: its huffman_encode() does not terminate and only counts
 * symbols (src/huffman.c:23-235), and its dpcm() is an alternating-sign
 * recurrence, not a DC prediction (src/dpcm.c:10-20).  This is the build's own entropy stage
 * (parity unpinned): baseline sequential DCT, 8-bit, one interleaved scan, 4:4:4
 * (the reference's output for every sample_ratio), the standard Huffman tables of ITU-T T.81
 * Annex K.3, true DC prediction per component.
 *
 * The coefficients are the reference's, quirks included, and the file describes them
 * faithfully: the DQT entries are the divisors the reference actually applied, i.e. the scaled
 * table transposed (src/quantise.c:58); when one exceeds 255 (q <= 23) the tables are 16-bit
 * and the frame is extended sequential (SOF1) instead of baseline.  A standard decoder therefore reproduces the
 * reference's pipeline output -- including the effects of its Cb sign error
 * (src/preprocess.c:161) and of the x0 = -8 last-column quirk.  AC magnitudes above 1023
 * (possible only for chroma at q >= 93 with the sign error) are clamped to the baseline range.
 */
#define _POSIX_C_SOURCE 200809L
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>
#ifdef __SSE2__
#include <emmintrin.h>
#endif

#include "../../include/jpgx_compat.h"
#include "../csrc/jx_consts.h"

/* ITU-T T.81 Annex K.3, Tables K.3-K.6: code-length counts and symbol values */
static const uint8_t kDcLumBits[16] = {0, 1, 5, 1, 1, 1, 1, 1, 1, 0, 0, 0, 0, 0, 0, 0};
static const uint8_t kDcChrBits[16] = {0, 3, 1, 1, 1, 1, 1, 1, 1, 1, 1, 0, 0, 0, 0, 0};
static const uint8_t kDcVals[12] = {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11};
static const uint8_t kAcLumBits[16] = {0, 2, 1, 3, 3, 2, 4, 3, 5, 5, 4, 4, 0, 0, 1, 0x7d};
static const uint8_t kAcLumVals[162] = {
    0x01, 0x02, 0x03, 0x00, 0x04, 0x11, 0x05, 0x12, 0x21, 0x31, 0x41, 0x06, 0x13, 0x51, 0x61,
    0x07, 0x22, 0x71, 0x14, 0x32, 0x81, 0x91, 0xa1, 0x08, 0x23, 0x42, 0xb1, 0xc1, 0x15, 0x52,
    0xd1, 0xf0, 0x24, 0x33, 0x62, 0x72, 0x82, 0x09, 0x0a, 0x16, 0x17, 0x18, 0x19, 0x1a, 0x25,
    0x26, 0x27, 0x28, 0x29, 0x2a, 0x34, 0x35, 0x36, 0x37, 0x38, 0x39, 0x3a, 0x43, 0x44, 0x45,
    0x46, 0x47, 0x48, 0x49, 0x4a, 0x53, 0x54, 0x55, 0x56, 0x57, 0x58, 0x59, 0x5a, 0x63, 0x64,
    0x65, 0x66, 0x67, 0x68, 0x69, 0x6a, 0x73, 0x74, 0x75, 0x76, 0x77, 0x78, 0x79, 0x7a, 0x83,
    0x84, 0x85, 0x86, 0x87, 0x88, 0x89, 0x8a, 0x92, 0x93, 0x94, 0x95, 0x96, 0x97, 0x98, 0x99,
    0x9a, 0xa2, 0xa3, 0xa4, 0xa5, 0xa6, 0xa7, 0xa8, 0xa9, 0xaa, 0xb2, 0xb3, 0xb4, 0xb5, 0xb6,
    0xb7, 0xb8, 0xb9, 0xba, 0xc2, 0xc3, 0xc4, 0xc5, 0xc6, 0xc7, 0xc8, 0xc9, 0xca, 0xd2, 0xd3,
    0xd4, 0xd5, 0xd6, 0xd7, 0xd8, 0xd9, 0xda, 0xe1, 0xe2, 0xe3, 0xe4, 0xe5, 0xe6, 0xe7, 0xe8,
    0xe9, 0xea, 0xf1, 0xf2, 0xf3, 0xf4, 0xf5, 0xf6, 0xf7, 0xf8, 0xf9, 0xfa};
static const uint8_t kAcChrBits[16] = {0, 2, 1, 2, 4, 4, 3, 4, 7, 5, 4, 4, 0, 1, 2, 0x77};
static const uint8_t kAcChrVals[162] = {
    0x00, 0x01, 0x02, 0x03, 0x11, 0x04, 0x05, 0x21, 0x31, 0x06, 0x12, 0x41, 0x51, 0x07, 0x61,
    0x71, 0x13, 0x22, 0x32, 0x81, 0x08, 0x14, 0x42, 0x91, 0xa1, 0xb1, 0xc1, 0x09, 0x23, 0x33,
    0x52, 0xf0, 0x15, 0x62, 0x72, 0xd1, 0x0a, 0x16, 0x24, 0x34, 0xe1, 0x25, 0xf1, 0x17, 0x18,
    0x19, 0x1a, 0x26, 0x27, 0x28, 0x29, 0x2a, 0x35, 0x36, 0x37, 0x38, 0x39, 0x3a, 0x43, 0x44,
    0x45, 0x46, 0x47, 0x48, 0x49, 0x4a, 0x53, 0x54, 0x55, 0x56, 0x57, 0x58, 0x59, 0x5a, 0x63,
    0x64, 0x65, 0x66, 0x67, 0x68, 0x69, 0x6a, 0x73, 0x74, 0x75, 0x76, 0x77, 0x78, 0x79, 0x7a,
    0x82, 0x83, 0x84, 0x85, 0x86, 0x87, 0x88, 0x89, 0x8a, 0x92, 0x93, 0x94, 0x95, 0x96, 0x97,
    0x98, 0x99, 0x9a, 0xa2, 0xa3, 0xa4, 0xa5, 0xa6, 0xa7, 0xa8, 0xa9, 0xaa, 0xb2, 0xb3, 0xb4,
    0xb5, 0xb6, 0xb7, 0xb8, 0xb9, 0xba, 0xc2, 0xc3, 0xc4, 0xc5, 0xc6, 0xc7, 0xc8, 0xc9, 0xca,
    0xd2, 0xd3, 0xd4, 0xd5, 0xd6, 0xd7, 0xd8, 0xd9, 0xda, 0xe2, 0xe3, 0xe4, 0xe5, 0xe6, 0xe7,
    0xe8, 0xe9, 0xea, 0xf2, 0xf3, 0xf4, 0xf5, 0xf6, 0xf7, 0xf8, 0xf9, 0xfa};

/* ---- header bytes (fixed-size segments before the scan) ------------------------------------ */
typedef struct {
    uint8_t *p;
    size_t n, cap;
    int overflow;
} Out;

static void put_byte(Out *o, uint8_t b)
{
    if (o->n < o->cap) o->p[o->n] = b;
    else o->overflow = 1;
    o->n++;
}

static void put_u16(Out *o, unsigned v)
{
    put_byte(o, (uint8_t)(v >> 8));
    put_byte(o, (uint8_t)v);
}

static void put_dht(Out *o, int cls_id, const uint8_t bits[16], const uint8_t *vals)
{
    int n = 0;
    for (int i = 0; i < 16; i++) n += bits[i];
    put_u16(o, 0xffc4);
    put_u16(o, (unsigned)(2 + 1 + 16 + n));
    put_byte(o, (uint8_t)cls_id);
    for (int i = 0; i < 16; i++) put_byte(o, bits[i]);
    for (int i = 0; i < n; i++) put_byte(o, vals[i]);
}

/* ---- entropy-coded data: a word-at-a-time bit writer into a growable buffer ---------------
 * Bits accumulate MSB first in a 64-bit register; every 32 bits leave as four bytes at once
 * unless one of them is 0xFF (then byte by byte with the 0x00 stuffing of T.81 F.1.2.3). */
typedef struct {
    uint8_t *p;
    size_t n, cap;
    uint64_t acc;     /* the low nacc bits are pending */
    int nacc;
    int oom;
} BW;

static int bw_reserve(BW *w, size_t more)
{
    if (w->n + more <= w->cap) return 1;
    size_t nc = w->cap ? w->cap : 1u << 16;
    while (nc < w->n + more) nc *= 2;
    uint8_t *q = (uint8_t *)realloc(w->p, nc);
    if (!q) {
        w->oom = 1;
        return 0;
    }
    w->p = q;
    w->cap = nc;
    return 1;
}

static inline void bw_byte(BW *w, uint8_t b)
{
    w->p[w->n++] = b;
    if (b == 0xff) w->p[w->n++] = 0x00;
}

/* v < 2^nb, nb <= 32 (a Huffman code and its additional bits in one call); the caller has
 * reserved room (bw_reserve) */
static inline void bw_bits(BW *w, uint32_t v, int nb)
{
    w->acc = (w->acc << nb) | v;
    w->nacc += nb;
    if (w->nacc >= 32) {
        w->nacc -= 32;
        const uint32_t x = (uint32_t)(w->acc >> w->nacc);
        if (((~x - 0x01010101u) & x & 0x80808080u) == 0) {       /* no 0xFF byte in x */
            uint8_t *d = w->p + w->n;
            d[0] = (uint8_t)(x >> 24);
            d[1] = (uint8_t)(x >> 16);
            d[2] = (uint8_t)(x >> 8);
            d[3] = (uint8_t)x;
            w->n += 4;
        } else {
            bw_byte(w, (uint8_t)(x >> 24));
            bw_byte(w, (uint8_t)(x >> 16));
            bw_byte(w, (uint8_t)(x >> 8));
            bw_byte(w, (uint8_t)x);
        }
    }
}

/* pad to a byte boundary with 1-bits and emit the pending bytes */
static void bw_flush(BW *w)
{
    const int pad = (8 - (w->nacc & 7)) & 7;
    if (pad) {
        w->acc = (w->acc << pad) | ((1u << pad) - 1u);
        w->nacc += pad;
    }
    while (w->nacc >= 8) {
        w->nacc -= 8;
        bw_byte(w, (uint8_t)(w->acc >> w->nacc));
    }
}

/* magnitude category and the value's additional bits (T.81 F.1.2.1) */
static inline int category(int v, uint32_t *extra)
{
    const unsigned a = (unsigned)(v < 0 ? -v : v);
    const int s = a ? 32 - __builtin_clz(a) : 0;
    *extra = (uint32_t)(v < 0 ? v + (1 << s) - 1 : v) & ((1u << s) - 1u);
    return s;
}

/* canonical Huffman codes (T.81 Annex C) indexed by symbol, packed: code << 8 | length */
typedef struct {
    uint32_t cl[256];
} HuffCodes;

static void build_codes(const uint8_t bits[16], const uint8_t *vals, HuffCodes *h)
{
    memset(h, 0, sizeof(*h));
    unsigned code = 0, k = 0;
    for (int l = 1; l <= 16; l++) {
        for (int i = 0; i < bits[l - 1]; i++, k++) h->cl[vals[k]] = (code++) << 8 | (unsigned)l;
        code <<= 1;
    }
}

/* worst-case coded bytes of one block, stuffing included */
#define JX_BLOCK_MAX (2 * (22 + 63 * 26 + 11 + 8) / 8 + 16)

/* bit k set: z[k] != 0 */
static inline uint64_t nonzero_mask(const int16_t *z)
{
#ifdef __SSE2__
    const __m128i zero = _mm_setzero_si128();
    uint64_t m = 0;
    for (int i = 0; i < 4; i++) {
        const __m128i a = _mm_loadu_si128((const __m128i *)(z + 16 * i));
        const __m128i b = _mm_loadu_si128((const __m128i *)(z + 16 * i + 8));
        const __m128i e = _mm_packs_epi16(_mm_cmpeq_epi16(a, zero), _mm_cmpeq_epi16(b, zero));
        m |= (uint64_t)(uint16_t)~_mm_movemask_epi8(e) << (16 * i);
    }
    return m;
#else
    uint64_t m = 0;
    for (int k = 0; k < 64; k++) m |= (uint64_t)(z[k] != 0) << k;
    return m;
#endif
}

/* one block's Huffman-coded data (T.81 F.1.2): DC difference against *pred, AC run/size */
static void encode_block(BW *w, const int16_t *z, int *pred, const HuffCodes *dc, const HuffCodes *ac)
{
    uint32_t extra;
    int diff = z[0] - *pred;                       /* true DC prediction */
    if (diff > 2047) diff = 2047;                  /* (never reached: |DC| <= 1364) */
    if (diff < -2047) diff = -2047;
    *pred = z[0];
    int s = category(diff, &extra);
    uint32_t c = dc->cl[s];
    bw_bits(w, (c >> 8) << s | extra, (int)(c & 0xff) + s);
    uint64_t nz = nonzero_mask(z) & ~1ull;         /* the nonzero AC coefficients */
    int prev = 0;
    while (nz) {
        const int k = __builtin_ctzll(nz);
        nz &= nz - 1;
        int run = k - prev - 1;
        prev = k;
        int v = z[k];
        if (v > 1023) v = 1023;
        if (v < -1023) v = -1023;
        while (run > 15) {                         /* ZRL */
            c = ac->cl[0xf0];
            bw_bits(w, c >> 8, (int)(c & 0xff));
            run -= 16;
        }
        s = category(v, &extra);
        c = ac->cl[run << 4 | s];
        bw_bits(w, (c >> 8) << s | extra, (int)(c & 0xff) + s);
    }
    if (prev < 63) {                               /* EOB */
        c = ac->cl[0x00];
        bw_bits(w, c >> 8, (int)(c & 0xff));
    }
}

size_t jpgx_jfif_bound(int width, int height)
{
    if (width <= 0 || height <= 0) return 0;
    /* headers + a per-block maximum with margin -- DC code + magnitude <= 16 + 16 bits, 63 AC
     * codes + magnitudes <= 63 x (16 + 16) bits, EOB <= 16 bits -- doubled for 0xFF stuffing,
     * plus per restart interval (at most one per MCU row) the padding byte, its possible stuffing
     * byte and RSTm: 4 bytes */
    const size_t blocks = (size_t)(width / 8 + 1) * (height / 8 + 1) * 3;
    return 1024 + blocks * 2 * (32 + 63 * 32 + 16) / 8 + 4 * (size_t)(height / 8 + 1);
}

/* The scan's geometry and tables, shared by the coding threads */
typedef struct {
    const int16_t *coef;
    int hs, vs;
    size_t bpr, nb, cpr, nbc, mrows;
    size_t rows_per_interval, nintervals;
    HuffCodes dc[2], ac[2];
} Scan;

/* restart intervals [i0, i1) into w: DC predictors reset at each, RSTm after each but the
 * scan's last (T.81 F.1.2.1.3, B.2.4.4) */
static void code_intervals(const Scan *S, size_t i0, size_t i1, BW *w)
{
    for (size_t iv = i0; iv < i1 && !w->oom; iv++) {
        int pred[3] = {0, 0, 0};
        const size_t r0 = iv * S->rows_per_interval;
        size_t r1 = r0 + S->rows_per_interval;
        if (r1 > S->mrows) r1 = S->mrows;
        for (size_t my = r0; my < r1; my++) {
            if (!bw_reserve(w, S->cpr * (size_t)(S->hs * S->vs + 2) * JX_BLOCK_MAX)) return;
            for (size_t mx = 0; mx < S->cpr; mx++) {
                /* MCU: hs x vs luma blocks (raster within the MCU), then Cb, then Cr (T.81 A.2.3) */
                for (int dy = 0; dy < S->vs; dy++)
                    for (int dx = 0; dx < S->hs; dx++) {
                        const size_t yb = (my * S->vs + dy) * S->bpr + mx * S->hs + dx;
                        encode_block(w, S->coef + yb * 64, &pred[0], &S->dc[0], &S->ac[0]);
                    }
                const size_t cb = my * S->cpr + mx;
                encode_block(w, S->coef + (S->nb + cb) * 64, &pred[1], &S->dc[1], &S->ac[1]);
                encode_block(w, S->coef + (S->nb + S->nbc + cb) * 64, &pred[2], &S->dc[1], &S->ac[1]);
            }
        }
        if (!bw_reserve(w, 16)) return;
        bw_flush(w);
        if (iv + 1 < S->nintervals) {
            w->p[w->n++] = 0xff;
            w->p[w->n++] = (uint8_t)(0xd0 + (iv & 7));
        }
    }
}

typedef struct {
    const Scan *S;
    size_t i0, i1;
    BW w;
} Job;

static void *job_main(void *arg)
{
    Job *j = (Job *)arg;
    code_intervals(j->S, j->i0, j->i1, &j->w);
    return NULL;
}

int jpgx_write_jfif(const int16_t *coef, int width, int height, int quality, uint8_t *out,
                    size_t cap, size_t *len)
{
    return jpgx_write_jfif_ex(coef, width, height, quality, 0, 0, 1, out, cap, len);
}

int jpgx_write_jfif_sub(const int16_t *coef, int width, int height, int quality,
                        int sample_ratio, uint8_t *out, size_t cap, size_t *len)
{
    return jpgx_write_jfif_ex(coef, width, height, quality, sample_ratio, 0, 1, out, cap, len);
}

int jpgx_write_jfif_ex(const int16_t *coef, int width, int height, int quality, int sample_ratio,
                       int restart_rows, int nthreads, uint8_t *out, size_t cap, size_t *len)
{
    if (!coef || !out || width <= 0 || height <= 0 || width % 8 || height % 8 ||
        width > 65535 || height > 65535 || sample_ratio < 0 || sample_ratio > 2 ||
        restart_rows < -1 || nthreads < 0)
        return JPGX_EARG;
    const int hs = sample_ratio ? 2 : 1, vs = sample_ratio == 2 ? 2 : 1;   /* Y sampling */
    if (width % (8 * hs) || height % (8 * vs)) return JPGX_EGEOMETRY;
    int qs[2][8][8];
    if (jpgx_scale_table(0, quality, qs[0]) || jpgx_scale_table(1, quality, qs[1]))
        return JPGX_EQUALITY;
    static const int scan[8][8] = JX_SCAN_ORDER_INIT;

    Scan S;
    S.coef = coef;
    S.hs = hs;
    S.vs = vs;
    S.bpr = (size_t)(width / 8);
    S.nb = S.bpr * (size_t)(height / 8);
    S.cpr = S.bpr / (size_t)hs;
    S.mrows = (size_t)(height / 8 / vs);
    S.nbc = S.cpr * S.mrows;                               /* chroma planes' blocks */
    long T = nthreads;
    if (T == 0) {
        T = sysconf(_SC_NPROCESSORS_ONLN);
        if (T < 1) T = 1;
        if (T > 64) T = 64;
    }
    /* restart interval: rows of MCUs, Ri = rows x MCUs per row (a 16-bit field) */
    const size_t maxrows = 65535 / S.cpr;
    size_t rr = 0;
    if (restart_rows > 0) {
        rr = (size_t)restart_rows;
        if (rr > maxrows) return JPGX_EARG;
    } else if (restart_rows == -1) {                       /* auto: ~4 intervals per thread */
        rr = (S.mrows + 4 * (size_t)T - 1) / (4 * (size_t)T);
        if (rr > maxrows) rr = maxrows;
        if (rr < 1) rr = 1;
    }
    S.rows_per_interval = rr ? rr : S.mrows;
    S.nintervals = (S.mrows + S.rows_per_interval - 1) / S.rows_per_interval;
    if ((size_t)T > S.nintervals) T = (long)S.nintervals;
    build_codes(kDcLumBits, kDcVals, &S.dc[0]);
    build_codes(kDcChrBits, kDcVals, &S.dc[1]);
    build_codes(kAcLumBits, kAcLumVals, &S.ac[0]);
    build_codes(kAcChrBits, kAcChrVals, &S.ac[1]);

    /* headers */
    Out o = {out, 0, cap, 0};
    put_u16(&o, 0xffd8);                                   /* SOI */
    put_u16(&o, 0xffe0);                                   /* APP0 JFIF 1.01 */
    put_u16(&o, 16);
    put_byte(&o, 'J'); put_byte(&o, 'F'); put_byte(&o, 'I'); put_byte(&o, 'F'); put_byte(&o, 0);
    put_u16(&o, 0x0101);
    put_byte(&o, 0);
    put_u16(&o, 1);
    put_u16(&o, 1);
    put_byte(&o, 0); put_byte(&o, 0);
    /* DQT: the divisors applied.  For q <= 23 some exceed 255 (q = 1: 6050); baseline allows
     * only 8-bit tables, so then both tables are written with 16-bit precision (Pq = 1) and
     * the frame is extended sequential (SOF1, same Huffman coding), as libjpeg does. */
    int wide = 0;
    for (int t = 0; t < 2; t++)
        for (int i = 0; i < 64; i++)
            if (qs[t][i / 8][i % 8] > 255) wide = 1;
    for (int t = 0; t < 2; t++) {
        int zz[64];
        for (int v = 0; v < 8; v++)
            for (int u = 0; u < 8; u++) {
                const int q = qs[t][u][v];                 /* coefficient (row v, col u) was
                                                              divided by Qs[u][v] */
                zz[scan[v][u]] = q < 1 ? 1 : q;
            }
        put_u16(&o, 0xffdb);
        put_u16(&o, (unsigned)(2 + 1 + 64 * (wide ? 2 : 1)));
        put_byte(&o, (uint8_t)(wide << 4 | t));
        for (int k = 0; k < 64; k++) {
            if (wide) put_u16(&o, (unsigned)zz[k]);
            else put_byte(&o, (uint8_t)zz[k]);
        }
    }
    put_u16(&o, wide ? 0xffc1 : 0xffc0);                   /* SOF1 / SOF0 */
    put_u16(&o, 8 + 3 * 3);
    put_byte(&o, 8);
    put_u16(&o, (unsigned)height);
    put_u16(&o, (unsigned)width);
    put_byte(&o, 3);
    for (int c = 0; c < 3; c++) {
        put_byte(&o, (uint8_t)(c + 1));
        put_byte(&o, (uint8_t)(c ? 0x11 : (hs << 4 | vs)));   /* 0x11, 0x21 or 0x22 */
        put_byte(&o, (uint8_t)(c ? 1 : 0));
    }
    put_dht(&o, 0x00, kDcLumBits, kDcVals);
    put_dht(&o, 0x10, kAcLumBits, kAcLumVals);
    put_dht(&o, 0x01, kDcChrBits, kDcVals);
    put_dht(&o, 0x11, kAcChrBits, kAcChrVals);
    if (rr) {                                              /* DRI (T.81 B.2.4.4) */
        put_u16(&o, 0xffdd);
        put_u16(&o, 4);
        put_u16(&o, (unsigned)(rr * S.cpr));
    }
    put_u16(&o, 0xffda);                                   /* SOS */
    put_u16(&o, 6 + 2 * 3);
    put_byte(&o, 3);
    for (int c = 0; c < 3; c++) {
        put_byte(&o, (uint8_t)(c + 1));
        put_byte(&o, (uint8_t)(c ? 0x11 : 0x00));
    }
    put_byte(&o, 0);
    put_byte(&o, 63);
    put_byte(&o, 0);

    /* the scan: thread t codes intervals [t NI / T, (t + 1) NI / T) into its own buffer */
    Job *jobs = (Job *)calloc((size_t)T, sizeof(Job));
    pthread_t *tid = (pthread_t *)calloc((size_t)T, sizeof(pthread_t));
    int rc = (jobs && tid) ? JPGX_OK : JPGX_ENOMEM;
    long nthr = T;                                         /* jobs 1 .. nthr - 1 run on threads */
    for (long t = 0; t < T && !rc; t++) {
        jobs[t].S = &S;
        jobs[t].i0 = (size_t)t * S.nintervals / (size_t)T;
        jobs[t].i1 = (size_t)(t + 1) * S.nintervals / (size_t)T;
        if (t == 0 || t >= nthr) continue;                 /* the calling thread codes job 0 */
        if (pthread_create(&tid[t], NULL, job_main, &jobs[t])) nthr = t;   /* no thread: code it here */
    }
    if (!rc) {
        job_main(&jobs[0]);
        for (long t = nthr; t < T; t++) job_main(&jobs[t]);   /* the jobs no thread took */
    }
    for (long t = 1; t < nthr; t++) pthread_join(tid[t], NULL);
    for (long t = 0; t < T && !rc; t++)
        if (jobs[t].w.oom) rc = JPGX_ENOMEM;
    if (!rc) {
        for (long t = 0; t < T; t++) {
            if (o.n + jobs[t].w.n <= o.cap) memcpy(o.p + o.n, jobs[t].w.p, jobs[t].w.n);
            else o.overflow = 1;
            o.n += jobs[t].w.n;
        }
        put_u16(&o, 0xffd9);                               /* EOI */
        if (len) *len = o.n;
        if (o.overflow) rc = JPGX_EARG;
    }
    if (jobs)
        for (long t = 0; t < T; t++) free(jobs[t].w.p);
    free(jobs);
    free(tid);
    return rc;
}

int jpgx_encode_rgb_to_jpeg(const uint8_t *rgb, int width, int height, size_t pitch,
                            const char *output, int quality, int sample_ratio, unsigned flags,
                            int device)
{
    if (!rgb || !output) return JPGX_EARG;
    jpgx_params p;
    jpgx_default_params(&p, width, height, quality, sample_ratio);
    /* true subsampling needs a ratio; with sample_ratio 0 the flag means plain 4:4:4 (as in
     * jpgx_encode_bmp_to_jpeg_ex) */
    const int sub = (flags & JPGX_FLAG_SUBSAMPLE) && sample_ratio != 0;
    p.flags = sub ? JPGX_FLAG_SUBSAMPLE : 0u;
    int rc = jpgx_validate(width, height, &p);
    if (rc) return rc;
    const size_t nb = (size_t)(width / 8) * (height / 8);
    const size_t nbc = jpgx_chroma_blocks(width, 0, height / 8, sample_ratio, p.flags);
    int16_t *coef = (int16_t *)malloc((nb + 2 * nbc) * 64 * sizeof(int16_t));
    const size_t cap = jpgx_jfif_bound(width, height);
    uint8_t *buf = (uint8_t *)malloc(cap);
    size_t len = 0;
    rc = (coef && buf) ? JPGX_OK : JPGX_ENOMEM;
    if (!rc) rc = jpgx_blocks(rgb, width, height, pitch, &p, coef, device);
    if (!rc)
        rc = sub ? jpgx_write_jfif_sub(coef, width, height, quality, sample_ratio, buf, cap, &len)
                 : jpgx_write_jfif(coef, width, height, quality, buf, cap, &len);
    if (!rc) {
        FILE *f = fopen(output, "wb");
        if (!f || fwrite(buf, 1, len, f) != len) rc = JPGX_EARG;
        if (f && fclose(f)) rc = JPGX_EARG;
    }
    free(coef);
    free(buf);
    return rc;
}

int jpgx_encode_bmp_to_jpeg_ex(const char *input, const char *output, int quality,
                               int sample_ratio, unsigned flags, int device)
{
    if (!input || !output) return JPGX_EARG;
    if (!(flags & JPGX_FLAG_SUBSAMPLE) || sample_ratio == 0)
        return jpgx_encode_bmp_to_jpeg(input, output, quality, sample_ratio);
    int W = 0, H = 0;
    uint8_t *rgb = NULL;
    size_t fsize = 0;
    int rc = jpgx_bmp_read(input, &rgb, &W, &H, &fsize);
    if (rc) return rc;
    jpgx_params p;
    jpgx_default_params(&p, W, H, quality, sample_ratio);
    p.flags = flags;
    const size_t nb = (size_t)(W / 8) * (H / 8);
    const size_t nbc = jpgx_chroma_blocks(W, 0, H / 8, sample_ratio, flags);
    int16_t *coef = (int16_t *)malloc((nb + 2 * nbc) * 64 * sizeof(int16_t));
    const size_t cap = jpgx_jfif_bound(W, H);
    uint8_t *buf = (uint8_t *)malloc(cap);
    size_t len = 0;
    rc = (coef && buf) ? JPGX_OK : JPGX_EARG;
    if (!rc) rc = jpgx_blocks(rgb, W, H, (size_t)W * 3, &p, coef, device);
    if (!rc) rc = jpgx_write_jfif_sub(coef, W, H, quality, sample_ratio, buf, cap, &len);
    if (!rc) {
        FILE *f = fopen(output, "wb");
        if (!f || fwrite(buf, 1, len, f) != len) rc = JPGX_EARG;
        if (f && fclose(f)) rc = JPGX_EARG;
    }
    jpgx_free(rgb);
    free(coef);
    free(buf);
    return rc;
}

int jpgx_encode_bmp_to_jpeg(const char *input, const char *output, int quality,
                            int sample_ratio)
{
    if (!input || !output) return JPGX_EARG;
    jpgx_jpeg_data j;
    memset(&j, 0, sizeof j);
    int rc = jpgx_encode_bmp(input, quality, sample_ratio, 0, 0, &j);
    if (rc) return rc;
    const size_t nb = (size_t)j.num_blocks_Y;
    int16_t *coef = (int16_t *)malloc(nb * 3 * 64 * sizeof(int16_t));
    const size_t cap = jpgx_jfif_bound(j.width, j.height);
    uint8_t *buf = (uint8_t *)malloc(cap);
    size_t len = 0;
    rc = (coef && buf) ? JPGX_OK : JPGX_EARG;
    if (!rc) {
        int **zz[3] = {j.zig_zag_Y, j.zig_zag_Cb, j.zig_zag_Cr};
        for (int c = 0; c < 3; c++)
            for (size_t i = 0; i < nb; i++)
                for (int k = 0; k < 64; k++) coef[((size_t)c * nb + i) * 64 + k] = (int16_t)zz[c][i][k];
        rc = jpgx_write_jfif(coef, j.width, j.height, quality, buf, cap, &len);
    }
    if (!rc) {
        FILE *f = fopen(output, "wb");
        if (!f || fwrite(buf, 1, len, f) != len) rc = JPGX_EARG;
        if (f && fclose(f)) rc = JPGX_EARG;
    }
    jpgx_free_jpgdata(&j);
    free(coef);
    free(buf);
    return rc;
}
