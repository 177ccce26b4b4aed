/*
 * jfif_dec.c -- TEST INFRASTRUCTURE: an independent baseline-JPEG entropy decoder, written from
 * ITU-T T.81 (B.2 markers, C canonical codes, F.2.2 decoding, F.1.2.3 stuffing, F.2.2.5 restart),
 * used to check jpgx_write_jfif_ex on frames too large for tests/jfif_decode.py (16384^2).
 * It knows only what the writer is asked to produce: 8-bit SOF0/SOF1, three components (Y
 * sampled 1x1, 2x1 or 2x2, chroma 1x1), one interleaved scan, optional DRI.  Restart intervals
 * are found by their RSTm markers and decoded on host threads.
 *
 *   int jfd_decode(const uint8_t *data, size_t len, int16_t *coef, size_t coef_elems,
 *                  int nthreads, int info[6]);
 * coef: Y [nb][64] | Cb [nbc][64] | Cr [nbc][64] (zig-zag order, the writer's input layout);
 * info: width, height, hs, vs, restart interval (MCUs), number of RST markers.  Returns 0 or a
 * negative line number of the check that failed.
 */
#define _POSIX_C_SOURCE 200809L
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define FAIL() return -__LINE__
#define CHECK(c) do { if (!(c)) FAIL(); } while (0)

typedef struct {              /* decoding table (T.81 F.2.2.3, with a 9-bit lookup) */
    int32_t maxcode[18];
    int32_t valptr[17];
    int32_t mincode[17];
    uint8_t vals[256];
    uint16_t look[512];       /* (length << 8 | symbol) for codes of <= 9 bits, else 0 */
    int present;
} Huff;

static void huff_build(Huff *h, const uint8_t bits[16], const uint8_t *vals, int n)
{
    memset(h, 0, sizeof *h);
    memcpy(h->vals, vals, (size_t)n);
    int code = 0, k = 0;
    for (int l = 1; l <= 16; l++) {
        h->valptr[l] = k;
        h->mincode[l] = code;
        for (int i = 0; i < bits[l - 1]; i++, k++, code++)
            if (l <= 9)
                for (int f = 0; f < (1 << (9 - l)); f++)
                    h->look[(code << (9 - l)) | f] = (uint16_t)(l << 8 | vals[k]);
        h->maxcode[l] = bits[l - 1] ? code - 1 : -1;
        code <<= 1;
    }
    h->maxcode[17] = 0x7fffffff;
    h->present = 1;
}

typedef struct {              /* bit reader over one restart interval's bytes */
    const uint8_t *p, *end;
    uint64_t acc;
    int n;
} Bits;

static void fill(Bits *b)
{
    while (b->n <= 56) {
        uint8_t x = 0;
        if (b->p < b->end) {
            x = *b->p++;
            if (x == 0xff) {
                if (b->p < b->end && *b->p == 0x00) b->p++;     /* stuffed byte */
                else x = 0, b->p = b->end;                       /* a marker: stop */
            }
        }
        b->acc |= (uint64_t)x << (56 - b->n);
        b->n += 8;
    }
}

static int getbits(Bits *b, int k)
{
    if (!k) return 0;
    if (b->n < k) fill(b);
    const int v = (int)(b->acc >> (64 - k));
    b->acc <<= k;
    b->n -= k;
    return v;
}

static int decode_sym(Bits *b, const Huff *h)
{
    if (b->n < 16) fill(b);
    const unsigned top = (unsigned)(b->acc >> 55);
    const unsigned e = h->look[top];
    if (e) {
        b->acc <<= (e >> 8);
        b->n -= (int)(e >> 8);
        return (int)(e & 0xff);
    }
    int code = 0, l = 0;
    while (l < 16) {
        code = (code << 1) | getbits(b, 1);
        l++;
        if (code <= h->maxcode[l]) return h->vals[h->valptr[l] + code - h->mincode[l]];
    }
    return -1;
}

static int extend(int v, int s) { return (s && v < (1 << (s - 1))) ? v - (1 << s) + 1 : v; }

typedef struct {
    Huff dc[4], ac[4];
    int td[3], ta[3];
    int hs, vs, ri;
    size_t bpr, nb, cpr, nbc, mrows, nmcu;
    int16_t *coef;
} Dec;

static int decode_block(const Dec *D, Bits *b, int c, int *pred, int16_t *dst)
{
    const int s = decode_sym(b, &D->dc[D->td[c]]);
    if (s < 0 || s > 11) FAIL();
    *pred += extend(getbits(b, s), s);
    memset(dst, 0, 64 * sizeof(int16_t));
    dst[0] = (int16_t)*pred;
    for (int k = 1; k < 64;) {
        const int rs = decode_sym(b, &D->ac[D->ta[c]]);
        if (rs < 0) FAIL();
        const int r = rs >> 4, sz = rs & 15;
        if (sz == 0) {
            if (r != 15) break;                  /* EOB */
            k += 16;
            continue;
        }
        k += r;
        if (k > 63) FAIL();
        dst[k++] = (int16_t)extend(getbits(b, sz), sz);
    }
    return 0;
}

/* MCUs [m0, m1) from the interval's bytes */
static int decode_mcus(const Dec *D, const uint8_t *p, const uint8_t *end, size_t m0, size_t m1)
{
    Bits b = {p, end, 0, 0};
    int pred[3] = {0, 0, 0};
    for (size_t m = m0; m < m1; m++) {
        const size_t my = m / D->cpr, mx = m % D->cpr;
        for (int dy = 0; dy < D->vs; dy++)
            for (int dx = 0; dx < D->hs; dx++) {
                const size_t yb = (my * D->vs + dy) * D->bpr + mx * D->hs + dx;
                const int rc = decode_block(D, &b, 0, &pred[0], D->coef + yb * 64);
                if (rc) return rc;
            }
        for (int c = 1; c < 3; c++) {
            const size_t cb = (c == 1 ? D->nb : D->nb + D->nbc) + m;
            const int rc = decode_block(D, &b, c, &pred[c], D->coef + cb * 64);
            if (rc) return rc;
        }
    }
    return 0;
}

typedef struct {
    const Dec *D;
    const uint8_t **start, **stop;
    size_t i0, i1;
    int rc;
} Job;

static void *job(void *arg)
{
    Job *j = (Job *)arg;
    for (size_t i = j->i0; i < j->i1 && !j->rc; i++) {
        const size_t m0 = i * (size_t)(j->D->ri ? j->D->ri : (int)j->D->nmcu);
        size_t m1 = m0 + (size_t)(j->D->ri ? j->D->ri : (int)j->D->nmcu);
        if (m1 > j->D->nmcu) m1 = j->D->nmcu;
        j->rc = decode_mcus(j->D, j->start[i], j->stop[i], m0, m1);
    }
    return NULL;
}

static unsigned u16(const uint8_t *p) { return (unsigned)p[0] << 8 | p[1]; }

int jfd_decode(const uint8_t *data, size_t len, int16_t *coef, size_t coef_elems, int nthreads,
               int info[6])
{
    Dec *D = (Dec *)calloc(1, sizeof(Dec));
    CHECK(D);
    size_t i = 2;
    int W = 0, H = 0, rc = 0;
    if (len < 4 || data[0] != 0xff || data[1] != 0xd8) { free(D); FAIL(); }
    for (;;) {
        if (i + 4 > len || data[i] != 0xff) { free(D); FAIL(); }
        const unsigned m = data[i + 1], ln = u16(data + i + 2);
        const uint8_t *seg = data + i + 4;
        if (i + 2 + ln > len) { free(D); FAIL(); }
        if (m == 0xc4) {
            size_t j = 0;
            while (j < ln - 2) {
                const int tc = seg[j] >> 4, th = seg[j] & 15;
                int n = 0;
                for (int k = 0; k < 16; k++) n += seg[j + 1 + k];
                huff_build(tc ? &D->ac[th & 3] : &D->dc[th & 3], seg + j + 1, seg + j + 17, n);
                j += 17 + (size_t)n;
            }
        } else if (m == 0xc0 || m == 0xc1) {
            if (seg[0] != 8 || seg[5] != 3) { free(D); FAIL(); }
            H = (int)u16(seg + 1);
            W = (int)u16(seg + 3);
            D->hs = seg[7] >> 4;
            D->vs = seg[7] & 15;
            if (seg[10] != 0x11 || seg[13] != 0x11) { free(D); FAIL(); }
        } else if (m == 0xdd) {
            D->ri = (int)u16(seg);
        } else if (m == 0xda) {
            if (seg[0] != 3) { free(D); FAIL(); }
            for (int c = 0; c < 3; c++) {
                D->td[c] = (seg[2 + 2 * c] >> 4) & 3;
                D->ta[c] = seg[2 + 2 * c] & 3;
            }
            i += 2 + ln;
            break;
        }
        i += 2 + ln;
    }
    if (!W || !H || D->hs < 1 || D->vs < 1) { free(D); FAIL(); }
    D->bpr = (size_t)W / 8;
    D->nb = D->bpr * ((size_t)H / 8);
    D->cpr = D->bpr / (size_t)D->hs;
    D->mrows = (size_t)H / 8 / (size_t)D->vs;
    D->nbc = D->cpr * D->mrows;
    D->nmcu = D->nbc;
    D->coef = coef;
    if (coef_elems < (D->nb + 2 * D->nbc) * 64) { free(D); FAIL(); }
    /* the intervals: split the entropy data at RSTm markers (never inside it: stuffing) */
    const size_t nint = D->ri ? (D->nmcu + (size_t)D->ri - 1) / (size_t)D->ri : 1;
    const uint8_t **start = (const uint8_t **)calloc(nint, sizeof(*start));
    const uint8_t **stop = (const uint8_t **)calloc(nint, sizeof(*stop));
    if (!start || !stop) { free(D); free(start); free(stop); FAIL(); }
    size_t k = 0, nrst = 0;
    start[0] = data + i;
    for (size_t p = i; p + 1 < len; p++) {
        if (data[p] != 0xff || data[p + 1] == 0x00) continue;
        const unsigned mk = data[p + 1];
        if (mk >= 0xd0 && mk <= 0xd7) {
            if (mk != 0xd0 + (nrst & 7) || k + 1 >= nint) { rc = -__LINE__; break; }
            stop[k++] = data + p;
            start[k] = data + p + 2;
            nrst++;
            p++;
        } else if (mk == 0xd9) {
            stop[k] = data + p;
            break;
        } else {
            rc = -__LINE__;
            break;
        }
    }
    if (!rc && (k + 1 != nint || !stop[k])) rc = -__LINE__;
    if (!rc) {
        int T = nthreads < 1 ? 1 : nthreads;
        if ((size_t)T > nint) T = (int)nint;
        Job *jobs = (Job *)calloc((size_t)T, sizeof(Job));
        pthread_t *tid = (pthread_t *)calloc((size_t)T, sizeof(pthread_t));
        if (!jobs || !tid) rc = -__LINE__;
        for (int t = 0; t < T && !rc; t++) {
            jobs[t] = (Job){D, start, stop, (size_t)t * nint / (size_t)T, (size_t)(t + 1) * nint / (size_t)T, 0};
            if (t && pthread_create(&tid[t], NULL, job, &jobs[t])) rc = -__LINE__;
        }
        if (!rc) {
            job(&jobs[0]);
            for (int t = 1; t < T; t++) pthread_join(tid[t], NULL);
            for (int t = 0; t < T; t++)
                if (jobs[t].rc) rc = jobs[t].rc;
        }
        free(jobs);
        free(tid);
    }
    if (info) {
        info[0] = W;
        info[1] = H;
        info[2] = D->hs;
        info[3] = D->vs;
        info[4] = D->ri;
        info[5] = (int)nrst;
    }
    free(start);
    free(stop);
    free(D);
    return rc;
}
