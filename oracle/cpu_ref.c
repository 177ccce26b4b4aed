/*
 * cpu_ref.c -- CPU restatement (ORACLE) of the reference hot path.  TEST INFRASTRUCTURE ONLY:
 * see cpu_ref.h for the rules and the reference file:line map.  Compiled with
 * -std=c99 -ffp-contract=off so every double operation rounds exactly as the reference's
 * gcc -std=c99 build does on x86-64 (no FMA contraction).
 */
#include "cpu_ref.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

#ifdef _OPENMP
#include <omp.h>
#endif

/* dct.c:9-11 defines M_PI itself under -std=c99; same double. */
#define REF_PI (3.14159265358979323846)

const int cpuref_q_lum[8][8] = {           /* quantise.c:8-15 */
    {16, 11, 10, 16, 24, 40, 51, 61},   {12, 12, 14, 19, 26, 58, 60, 55},
    {14, 13, 16, 24, 40, 57, 69, 56},   {14, 17, 22, 29, 51, 87, 80, 62},
    {18, 22, 37, 56, 68, 109, 103, 77}, {24, 35, 55, 64, 81, 104, 113, 92},
    {49, 64, 78, 87, 103, 121, 120, 101}, {72, 92, 95, 98, 112, 100, 103, 99}};

const int cpuref_q_chr[8][8] = {           /* quantise.c:18-25 */
    {17, 18, 24, 47, 99, 99, 99, 99}, {18, 21, 26, 66, 99, 99, 99, 99},
    {24, 26, 56, 99, 99, 99, 99, 99}, {47, 66, 99, 99, 99, 99, 99, 99},
    {99, 99, 99, 99, 99, 99, 99, 99}, {99, 99, 99, 99, 99, 99, 99, 99},
    {99, 99, 99, 99, 99, 99, 99, 99}, {99, 99, 99, 99, 99, 99, 99, 99}};

const int cpuref_scan_order[8][8] = {      /* zig_zag.c:6-15 (the standard JPEG scan) */
    {0, 1, 5, 6, 14, 15, 27, 28},     {2, 4, 7, 13, 16, 26, 29, 42},
    {3, 8, 12, 17, 25, 30, 41, 43},   {9, 11, 18, 24, 31, 40, 44, 53},
    {10, 19, 23, 32, 39, 45, 52, 54}, {20, 22, 33, 38, 46, 51, 55, 60},
    {21, 34, 37, 47, 50, 56, 59, 61}, {35, 36, 48, 49, 57, 58, 62, 63}};

void cpuref_scale_table(const int base[8][8], int quality, int out[8][8])
{
    /* quantise.c:81-83: s depends on quality only; integer division, floor of an int. */
    int s = (quality < 50) ? 5000 / quality : 200 - 2 * quality;
    for (int i = 0; i < 8; i++)
        for (int j = 0; j < 8; j++)
            out[i][j] = (s * base[i][j] + 50) / 100;
}

/* ---- cosine table: the exact doubles glibc returns for the reference's expression ---- */
static double g_cos[8][8];
static int g_cos_ready = 0;

static double ref_cos(int k, int i)
{
    /* dct.c:49-50: cos(((2*x + 1) * u * M_PI) / 16), int product first */
    return cos(((2 * i + 1) * k * REF_PI) / 16);
}

static void cos_init(void)
{
    if (g_cos_ready) return;
    for (int k = 0; k < 8; k++)
        for (int i = 0; i < 8; i++) g_cos[k][i] = ref_cos(k, i);
    g_cos_ready = 1;
}

/* dct.c:13: ALPHA(x) (x == 0 ? 1/sqrt(2) : 1) */
static double alpha(int k) { return k == 0 ? 1 / sqrt(2) : 1; }

/* One coefficient, exact order: s accumulates (X*c_u[x])*c_v[y], x outer, y inner. */
static double dct_coef(const double X[64], int u, int v, int mode)
{
    double s = 0.0;
    if (mode == CPUREF_MODE_REFCOST) {
        for (int x = 0; x < 8; x++)
            for (int y = 0; y < 8; y++) s += X[y * 8 + x] * ref_cos(u, x) * ref_cos(v, y);
    } else {
        const double *cu = g_cos[u], *cv = g_cos[v];
        for (int x = 0; x < 8; x++)
            for (int y = 0; y < 8; y++) s += X[y * 8 + x] * cu[x] * cv[y];
    }
    return 0.25 * alpha(u) * alpha(v) * s;   /* ((0.25*a_u)*a_v)*s, dct.c:54 */
}

void cpuref_dct_block(double v[64], int mode)
{
    double X[64];
    cos_init();
    memcpy(X, v, sizeof X);
    for (int u = 0; u < 8; u++)
        for (int vv = 0; vv < 8; vv++) v[vv * 8 + u] = dct_coef(X, u, vv, mode);
}

void cpuref_quantise_block(double v[64], const int table[8][8])
{
    /* quantise.c:56-58: value at (x=i, y=j) i.e. v[j*8+i], divided by table[i][j]. */
    for (int i = 0; i < 8; i++)
        for (int j = 0; j < 8; j++) v[j * 8 + i] = round(v[j * 8 + i] / table[i][j]);
}

void cpuref_zigzag_block(const double v[64], int zz[64])
{
    for (int i = 0; i < 8; i++)
        for (int j = 0; j < 8; j++) zz[cpuref_scan_order[i][j]] = (int)v[i * 8 + j];
}

/* ---- underflow bytes --------------------------------------------------- */
static unsigned long long req2size(unsigned long long n)
{
    unsigned long long s = (n + 8 + 15) & ~15ULL;
    return s < 32 ? 32 : s;
}

void cpuref_glibc_underflow(long long n_pixels, long long file_size, uint8_t out[8])
{
    /* The planes r_new/g_new/b_new (preprocess.c:127-129) are brk chunks unless the mmap
     * threshold was left at its 128 KiB default; the earlier free of the file-sized buffer
     * (bitmap.c:151) raises it to that chunk's size when that chunk is <= 32 MiB. */
    const unsigned long long page = 4096, thr0 = 128 * 1024, thr_max = 32ULL << 20;
    unsigned long long n = (unsigned long long)n_pixels, fs = (unsigned long long)file_size;
    unsigned long long thr = thr0;
    unsigned long long fchunk = req2size(fs);
    if (fchunk >= thr0) {                                  /* file buffer was mmapped */
        unsigned long long mm = (fchunk + 8 + page - 1) & ~(page - 1);
        if (mm > thr && mm <= thr_max) thr = mm;
    }
    unsigned long long nb = req2size(n), size;
    if (nb >= thr) size = ((nb + 8 + page - 1) & ~(page - 1)) | 2ULL; /* IS_MMAPPED */
    else size = nb | 1ULL;                                             /* PREV_INUSE */
    for (int k = 0; k < 8; k++) out[k] = (uint8_t)(size >> (8 * k));
}

/* ---- whole hot path ----------------------------------------------------------------- */
static int validate(int W, int H, int quality, int sample_ratio)
{
    if (sample_ratio < 0 || sample_ratio > 2) return -3;
    if (quality < 1 || quality > 97) return -2;
    int wm = sample_ratio == 0 ? 8 : 16, hm = sample_ratio == 2 ? 16 : 8;
    if (W <= 0 || H <= 0 || W % wm || H % hm) return -1;
    return 0;
}

/* Reference pixel fetch through blockToCoords (preprocess.c:155-163, 199-211). */
static void fetch_block_rgb(const uint8_t *rgb, int W, size_t pitch, long bn,
                            const uint8_t underflow[3][8], int px[64][3])
{
    unsigned int w = (unsigned int)W, tw = 8u * (unsigned int)bn;
    long y0 = (long)(tw / w) * 8;
    if (tw % w == 0) y0 -= 8;
    long x0 = (long)(tw % w) - 8;
    for (int y = 0; y < 8; y++)
        for (int x = 0; x < 8; x++) {
            long off = (y + y0) * (long)W + (x0 + x);
            for (int k = 0; k < 3; k++) {
                if (off < 0) px[y * 8 + x][k] = underflow[k][off + 8];
                else
                    px[y * 8 + x][k] = rgb[(size_t)(off / W) * pitch + (size_t)(off % W) * 3 + k];
            }
        }
}

int cpuref_blocks_rows(const uint8_t *rgb, int W, int H, size_t pitch, int quality,
                       int sample_ratio, const uint8_t underflow[3][8], int mode, int nthreads,
                       int row_begin, int row_end, int16_t *out)
{
    int err = validate(W, H, quality, sample_ratio);
    if (err) return err;
    if (row_begin < 0 || row_end > H / 8 || row_begin > row_end) return -1;
    int qt[2][8][8];
    cpuref_scale_table(cpuref_q_lum, quality, qt[0]);
    cpuref_scale_table(cpuref_q_chr, quality, qt[1]);
    cos_init();
    const long bpr = W / 8;
    const long nb_out = (long)(row_end - row_begin) * bpr;
    const long first = (long)row_begin * bpr;
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel for schedule(dynamic, 64) if (nthreads != 1)
#endif
    for (long i = 0; i < nb_out; i++) {
        int px[64][3];
        double X[3][64];
        fetch_block_rgb(rgb, W, pitch, first + i + 1, underflow, px);
        for (int p = 0; p < 64; p++) {
            int r = px[p][0], g = px[p][1], b = px[p][2];
            double yv = 0.299 * r + 0.587 * g + 0.114 * b;              /* :160 */
            double cb = 128 - (0.168736 * r - 0.331264 * g + 0.5 * b);  /* :161 */
            double cr = 128 + (0.5 * r - 0.418688 * g - 0.081312 * b);  /* :162 */
            X[0][p] = yv - 128;                                         /* :186-188 */
            X[1][p] = cb - 128;
            X[2][p] = cr - 128;
        }
        for (int ch = 0; ch < 3; ch++) {
            const int (*q)[8] = qt[ch == 0 ? 0 : 1];
            int16_t *o = out + ((long)ch * nb_out + i) * 64;
            for (int u = 0; u < 8; u++)
                for (int v = 0; v < 8; v++) {
                    double F = dct_coef(X[ch], u, v, mode);
                    o[cpuref_scan_order[v][u]] = (int16_t)(int)round(F / q[u][v]);
                }
        }
    }
    return 0;
}

/* ---- true chroma subsampling (extension; the reference's stubs print only) ------------- */
/* Level-shifted chroma of one pixel, the reference's double arithmetic (preprocess.c:161-162,
 * 186-188). */
static double chroma_ls(int ch, const uint8_t *p)
{
    const int r = p[0], g = p[1], b = p[2];
    if (ch == 1) {
        const double cb = 128 - (0.168736 * r - 0.331264 * g + 0.5 * b);
        return cb - 128;
    }
    const double cr = 128 + (0.5 * r - 0.418688 * g - 0.081312 * b);
    return cr - 128;
}

/* Chroma sample (X, Y) of the subsampled plane: the level-shifted values (Notes: "level shift
 * before chroma subsample") averaged as (p0 + p1) * 0.5 over the horizontal pair (4:2:2) or
 * ((p00 + p01) + (p10 + p11)) * 0.25 over the 2x2 quad (4:2:0), in double. */
double cpuref_chroma_sample(const uint8_t *rgb, size_t pitch, int sample_ratio, int ch, long X,
                            long Y)
{
    if (sample_ratio == 1) {
        const uint8_t *p = rgb + (size_t)Y * pitch + (size_t)(2 * X) * 3;
        return (chroma_ls(ch, p) + chroma_ls(ch, p + 3)) * 0.5;
    }
    const uint8_t *p = rgb + (size_t)(2 * Y) * pitch + (size_t)(2 * X) * 3;
    const uint8_t *q = p + pitch;
    return ((chroma_ls(ch, p) + chroma_ls(ch, p + 3)) + (chroma_ls(ch, q) + chroma_ls(ch, q + 3))) *
           0.25;
}

int cpuref_chroma_sub_rows(const uint8_t *rgb, int W, int H, size_t pitch, int quality,
                           int sample_ratio, int mode, int nthreads, int crow_begin,
                           int crow_end, int16_t *out)
{
    if (sample_ratio != 1 && sample_ratio != 2) return -3;
    int err = validate(W, H, quality, sample_ratio);
    if (err) return err;
    const int Wc = W / 2, Hc = sample_ratio == 2 ? H / 2 : H;
    if (crow_begin < 0 || crow_end > Hc / 8 || crow_begin > crow_end) return -1;
    int qt[8][8];
    cpuref_scale_table(cpuref_q_chr, quality, qt);
    cos_init();
    const long bpr = Wc / 8;
    const long nb_out = (long)(crow_end - crow_begin) * bpr;
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel for schedule(dynamic, 64) if (nthreads != 1)
#endif
    for (long i = 0; i < nb_out; i++) {
        const long by = crow_begin + i / bpr, bx = i % bpr;
        for (int ch = 1; ch <= 2; ch++) {
            double X[64];
            for (int y = 0; y < 8; y++)
                for (int x = 0; x < 8; x++)
                    X[y * 8 + x] = cpuref_chroma_sample(rgb, pitch, sample_ratio, ch, 8 * bx + x,
                                                        8 * by + y);
            int16_t *o = out + ((long)(ch - 1) * nb_out + i) * 64;
            for (int u = 0; u < 8; u++)
                for (int v = 0; v < 8; v++) {
                    const double F = dct_coef(X, u, v, mode);
                    o[cpuref_scan_order[v][u]] = (int16_t)(int)round(F / qt[u][v]);
                }
        }
    }
    return 0;
}

/* ---- entropy-stage statistics (dpcm.c:6-21, huffman.c:23-44,182-235) ------------------- */
static int get_class(int value)             /* huffman.c:226-235 */
{
    int c = 0;
    value = abs(value);
    while (value > 0) {
        value >>= 1;
        c++;
    }
    return c;
}

static void freq_ac(int32_t *freq, const int *zz)   /* huffman.c:187-222, '|' quirk kept */
{
    int last = 0, zeros = 0;
    for (int i = 63; i > 0; i--)
        if (zz[i] != 0) {
            last = i;
            break;
        }
    for (int i = 1; i < 64; i++) {
        if (i == last + 1) {
            freq[0x00]++;                        /* EOB */
            break;
        }
        if (zz[i] == 0) {
            if (++zeros == 16) {
                freq[0xF0]++;                    /* ZRL */
                zeros = 0;
            }
        } else {
            freq[zeros | get_class(zz[i])]++;    /* the reference ORs, not (run << 4) */
            zeros = 0;
        }
    }
}

void cpuref_entropy_stats(const int16_t *coef, long nb_y, long nb_c, int32_t *dc,
                          int32_t hist[4][257])
{
    for (int t = 0; t < 4; t++) {                /* initialize_huffman, huffman.c:52-75 */
        for (int k = 0; k < 256; k++) hist[t][k] = 0;
        hist[t][256] = 1;
    }
    long off = 0;
    for (int ch = 0; ch < 3; ch++) {
        const long nb = ch == 0 ? nb_y : nb_c;
        int prev = 0;
        for (long i = 0; i < nb; i++) {
            int zz[64];
            for (int k = 0; k < 64; k++) zz[k] = coef[(off + i) * 64 + k];
            const int d = i == 0 ? zz[0] : zz[0] - prev;     /* dpcm.c:10-20, in place */
            prev = d;
            zz[0] = d;
            dc[off + i] = d;
            hist[ch == 0 ? 0 : 2][get_class(d)]++;           /* calculate_freq_block_DC */
            freq_ac(hist[ch == 0 ? 1 : 3], zz);               /* calculate_freq_block_AC */
        }
        off += nb;
    }
}

int cpuref_blocks(const uint8_t *rgb, int W, int H, size_t pitch, int quality,
                  int sample_ratio, const uint8_t underflow[3][8], int mode, int nthreads,
                  int16_t *out)
{
    return cpuref_blocks_rows(rgb, W, H, pitch, quality, sample_ratio, underflow, mode,
                              nthreads, 0, H > 0 ? H / 8 : 0, out);
}

void cpuref_dpcm_i32(int32_t *zz, long nb)
{
    for (long i = 1; i < nb; i++) zz[i * 64] = zz[i * 64] - zz[(i - 1) * 64];
}

/* ---- BMP loader semantics ------------------------------------------------------------- */
static int rd32(const uint8_t *p) { return (int)((uint32_t)p[0] | (uint32_t)p[1] << 8 |
                                                 (uint32_t)p[2] << 16 | (uint32_t)p[3] << 24); }

int cpuref_bmp_decode(const uint8_t *file, size_t fs, int *W, int *H, uint8_t *rgb)
{
    if (fs < 30) return -1;
    int w = rd32(file + 18), h = rd32(file + 22);
    int depth = (int)(int16_t)((uint16_t)file[28] | (uint16_t)file[29] << 8);
    if (w <= 0 || h <= 0 || depth != 24) return -1;
    *W = w;
    *H = h;
    if (!rgb) return 0;
    long row_bytes = (long)w * (depth / 8);
    for (long i = 1; i <= h; i++) {
        long off = (long)fs - i * row_bytes;   /* bitmap.c:130 */
        if (off < 0) return -1;
        memcpy(rgb + (size_t)(i - 1) * w * 3, file + off, (size_t)w * 3);
    }
    return 0;
}

/* ---- synthetic frames ---------------------------------------------------------------- */
void cpuref_gen_splitmix(uint64_t seed, int W, int H, uint8_t *rgb)
{
    size_t n = (size_t)W * H * 3;
    for (size_t k = 0; k < n; k++) {
        uint64_t z = seed + (uint64_t)(k + 1) * 0x9E3779B97F4A7C15ULL;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
        z ^= z >> 31;
        rgb[k] = (uint8_t)(z >> 56);
    }
}

void cpuref_gen_tie(int W, int H, uint8_t *rgb)
{
    int bpr = W / 8;
    for (int y = 0; y < H; y++)
        for (int x = 0; x < W; x++) {
            long bi = (long)(y / 8) * bpr + x / 8;
            uint8_t v = (uint8_t)(97 + 2 * (bi % 40));
            uint8_t *p = rgb + ((size_t)y * W + x) * 3;
            p[0] = p[1] = p[2] = v;
        }
}
