/*
 * sanitize.c -- TEST INFRASTRUCTURE: the host C/C++ layer under AddressSanitizer +
 * UndefinedBehaviorSanitizer (tests/c/Makefile `sanitize`, run by tests/test_sanitize.py).
 *
 * Built from host/ *.c, csrc/jpgx_plan.cpp and oracle/cpu_ref.c with -fsanitize=address,undefined
 * (no GPU: san_nogpu.c answers jpgx_blocks with JPGX_ENODEV).  Exercises:
 *   - jpgx_bmp_read on the bundled images and on hostile files (truncated, negative / zero /
 *     huge dimensions, W*H*3 beyond the file, wrong bit depth, empty, missing) -- the loader
 *     restates bitmap.c:41-152, which trusts its header;
 *   - validation, defaults, the glibc underflow model, scale tables, the guard-band planning
 *     (jpgx_plan.cpp, every quality, both kernels' tables) and stripes;
 *   - the oracle's whole hot path, including the modelled x0 = -8 underflow read
 *     (preprocess.c:159-160) at block-row 0 and inside stripes, the true 4:2:x
 *     definition, the entropy statistics and the BMP decode of hostile buffers;
 *   - the Block API, the JpgData adapter + dpcm, the DC recurrence, the JFIF writers (4:4:4
 *     and 4:2:x, with a too-small output buffer).
 * Every check that fails prints a line and makes the exit status non-zero; the sanitizers abort
 * on their first report.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "jpgx_compat.h"
#include "../../oracle/cpu_ref.h"

int jx_plan_tables(int quality, float w[3][64], float lim[3][64], int16_t q[2][64]);
int jx_plan_tables_mode(int quality, int sub, float w[3][64], float lim[3][64], int16_t q[2][64]);
int jx_plan_tables_mx(int quality, float w[24][8], float lim[24][8], int16_t q[2][64]);
int jx_mx_operands(uint16_t ops[3 * 2][64][8]);
int jx_mx_parts(void);
long long jx_selftest_pk(long long nblocks, unsigned long long seed);

static int g_fail;
#define CHECK(c)                                                                 \
    do {                                                                         \
        if (!(c)) {                                                              \
            fprintf(stderr, "FAIL %s:%d: %s\n", __FILE__, __LINE__, #c);        \
            g_fail = 1;                                                          \
        }                                                                        \
    } while (0)

static const char *g_tmp;

static void put32(uint8_t *p, int32_t v) { memcpy(p, &v, 4); }
static void put16(uint8_t *p, int16_t v) { memcpy(p, &v, 2); }

/* a BMP file of `fs` bytes whose header claims w x h at bpp bits */
static const char *write_bmp(const char *name, long fs, int32_t w, int32_t h, int16_t bpp)
{
    static char path[4096];
    snprintf(path, sizeof path, "%s/%s", g_tmp, name);
    uint8_t *b = (uint8_t *)calloc(1, fs > 0 ? (size_t)fs : 1);
    if (fs >= 30) {
        b[0] = 'B';
        b[1] = 'M';
        put32(b + 2, (int32_t)fs);
        put32(b + 10, 54);
        put32(b + 18, w);
        put32(b + 22, h);
        put16(b + 26, 1);
        put16(b + 28, bpp);
    }
    for (long i = 54; i < fs; i++) b[i] = (uint8_t)(i * 7);
    FILE *f = fopen(path, "wb");
    if (f) {
        if (fs > 0) fwrite(b, 1, (size_t)fs, f);
        fclose(f);
    }
    free(b);
    return path;
}

static void bmp_hostile(void)
{
    uint8_t *rgb;
    int w, h;
    size_t fs;
    /* a good one */
    CHECK(jpgx_bmp_read(write_bmp("ok.bmp", 54 + 16 * 8 * 3, 16, 8, 24), &rgb, &w, &h, &fs) == 0);
    CHECK(w == 16 && h == 8 && fs == 54 + 16 * 8 * 3);
    jpgx_free(rgb);
    /* hostile headers: every one must be refused without reading out of bounds */
    struct { const char *n; long fs; int32_t w, h; int16_t bpp; } bad[] = {
        {"trunc0.bmp", 0, 0, 0, 24},
        {"trunc20.bmp", 20, 16, 8, 24},
        {"trunc53.bmp", 53, 16, 8, 24},
        {"neg_h.bmp", 54 + 16 * 8 * 3, 16, -8, 24},
        {"neg_w.bmp", 54 + 16 * 8 * 3, -16, 8, 24},
        {"zero_w.bmp", 54 + 16 * 8 * 3, 0, 8, 24},
        {"big.bmp", 54 + 16 * 8 * 3, 16, 10, 24},         /* W*H*3 > file size */
        {"big1.bmp", 54 + 16 * 8 * 3, 439, 1, 24},
        {"huge.bmp", 54 + 16 * 8 * 3, 0x7fffffff, 0x7fffffff, 24},
        {"huge_h.bmp", 54 + 16 * 8 * 3, 1, 0x7fffffff, 24},
        {"bpp32.bmp", 54 + 16 * 8 * 4, 16, 8, 32},
        {"bpp8.bmp", 54 + 16 * 8, 16, 8, 8},
        {"min_neg.bmp", 54 + 16 * 8 * 3, 16, (int32_t)0x80000000, 24},
    };
    for (size_t i = 0; i < sizeof bad / sizeof bad[0]; i++) {
        rgb = (uint8_t *)0x1;
        const int rc = jpgx_bmp_read(write_bmp(bad[i].n, bad[i].fs, bad[i].w, bad[i].h, bad[i].bpp),
                                     &rgb, &w, &h, &fs);
        if (rc == 0) fprintf(stderr, "accepted %s\n", bad[i].n);
        CHECK(rc != 0 && rgb == NULL);
    }
    CHECK(jpgx_bmp_read("/nonexistent/x.bmp", &rgb, &w, &h, &fs) != 0);
    CHECK(jpgx_bmp_read(NULL, &rgb, &w, &h, &fs) != 0);
    /* a file exactly W*H*3 long (header overlapped by pixel rows, as the reference allows) */
    CHECK(jpgx_bmp_read(write_bmp("exact.bmp", 64 * 3, 8, 8, 24), &rgb, &w, &h, &fs) == 0);
    jpgx_free(rgb);
}

static void bmp_images(const char *dir)
{
    const char *names[] = {"cam.bmp", "tiger.bmp"};
    for (int i = 0; i < 2; i++) {
        char path[4096];
        snprintf(path, sizeof path, "%s/%s", dir, names[i]);
        uint8_t *rgb;
        int w, h;
        size_t fs;
        CHECK(jpgx_bmp_read(path, &rgb, &w, &h, &fs) == 0);
        /* the oracle's in-memory decode of the same file agrees */
        FILE *f = fopen(path, "rb");
        uint8_t *file = (uint8_t *)malloc(fs);
        CHECK(f && fread(file, 1, fs, f) == fs);
        if (f) fclose(f);
        int W2, H2;
        uint8_t *rgb2 = (uint8_t *)malloc((size_t)w * h * 3);
        CHECK(cpuref_bmp_decode(file, fs, &W2, &H2, rgb2) == 0 && W2 == w && H2 == h);
        CHECK(memcmp(rgb, rgb2, (size_t)w * h * 3) == 0);
        /* the hot path of the oracle over the image, with the glibc underflow model */
        uint8_t uf[3][8];
        jpgx_glibc_underflow((long long)w * h, (long long)fs, uf[0]);
        memcpy(uf[1], uf[0], 8);
        memcpy(uf[2], uf[0], 8);
        const size_t nb = (size_t)(w / 8) * (h / 8);
        int16_t *out = (int16_t *)malloc(3 * nb * 64 * sizeof(int16_t));
        CHECK(cpuref_blocks(rgb, w, h, (size_t)w * 3, 90, 0, (const uint8_t(*)[8])uf, 0, 1, out) == 0);
        free(out);
        free(rgb2);
        free(file);
        jpgx_free(rgb);
    }
    /* hostile in-memory buffers for the oracle's decoder */
    uint8_t small[60] = {'B', 'M'};
    int W, H;
    put32(small + 18, 100);
    put32(small + 22, 100);
    put16(small + 28, 24);
    uint8_t *px = (uint8_t *)malloc(100 * 100 * 3);
    CHECK(cpuref_bmp_decode(small, sizeof small, &W, &H, NULL) == 0);   /* header query only */
    CHECK(cpuref_bmp_decode(small, sizeof small, &W, &H, px) != 0);     /* rows outside the file */
    CHECK(cpuref_bmp_decode(small, 10, &W, &H, px) != 0);
    put32(small + 22, -100);
    CHECK(cpuref_bmp_decode(small, sizeof small, &W, &H, px) != 0);
    free(px);
}

static void planning(void)
{
    jpgx_params p;
    for (int q = -2; q <= 101; q++) {
        int t[8][8];
        const int rc = jpgx_scale_table(0, q, t);
        CHECK((q >= 1 && q <= 97) ? rc == 0 : 1);
        jpgx_default_params(&p, 64, 48, q, 0);
        const int v = jpgx_validate(64, 48, &p);
        CHECK((q >= 1 && q <= 97) == (v == 0));
        if (q < 1 || q > 97) continue;
        float s[3][64], lim[3][64];
        CHECK(jpgx_guard_band(q, s, lim) == 0);
        int16_t qq[2][64];
        for (int sub = 0; sub <= 2; sub++) CHECK(jx_plan_tables_mode(q, sub, s, lim, qq) == 0);
        float w[24][8], l2[24][8];
        CHECK(jx_plan_tables_mx(q, w, l2, qq) == 0);
    }
    uint16_t ops[3 * 2][64][8];
    if (jx_mx_parts() == 2) CHECK(jx_mx_operands(ops) == 0);
    CHECK(jx_selftest_pk(2000, 7) == 0);
    /* geometry edges */
    const int geo[][2] = {{0, 8}, {8, 0}, {-8, 8}, {12, 8}, {8, 12}, {8, 8}, {16, 16}, {1 << 20, 8}};
    for (size_t i = 0; i < sizeof geo / sizeof geo[0]; i++)
        for (int sr = -1; sr <= 3; sr++) {
            jpgx_default_params(&p, geo[i][0] > 0 ? geo[i][0] : 8, geo[i][1] > 0 ? geo[i][1] : 8, 50,
                                sr >= 0 && sr <= 2 ? sr : 0);
            p.sample_ratio = sr;
            (void)jpgx_validate(geo[i][0], geo[i][1], &p);
            p.flags = JPGX_FLAG_SUBSAMPLE;
            (void)jpgx_validate(geo[i][0], geo[i][1], &p);
            (void)jpgx_chroma_blocks(geo[i][0] > 0 ? geo[i][0] : 8, 0, 4, sr, p.flags);
        }
    for (long long n = 1; n < (1ll << 34); n = n * 3 + 1) {
        uint8_t u[8];
        jpgx_glibc_underflow(n, 54 + 3 * n, u);
        uint8_t u2[8];
        cpuref_glibc_underflow(n, 54 + 3 * n, u2);
        CHECK(memcmp(u, u2, 8) == 0);
    }
    for (int rows = 0; rows < 40; rows++)
        for (int n = 1; n <= 9; n++) {
            int prev = 0;
            for (int k = 0; k < n; k++) {
                int a, b;
                jpgx_stripe(rows, n, k, &a, &b);
                CHECK(a == prev && b >= a);
                prev = b;
            }
            CHECK(prev == rows);
        }
}

static void oracle_paths(void)
{
    const int geo[][2] = {{8, 8}, {24, 8}, {16, 16}, {64, 24}, {136, 40}, {32, 32}};
    uint8_t uf[3][8];
    for (int k = 0; k < 24; k++) uf[k / 8][k % 8] = (uint8_t)(k * 11 + 5);
    for (size_t g = 0; g < sizeof geo / sizeof geo[0]; g++) {
        const int W = geo[g][0], H = geo[g][1];
        /* exact-size heap buffer, so ASan sees any read outside the image */
        uint8_t *rgb = (uint8_t *)malloc((size_t)W * H * 3);
        cpuref_gen_splitmix(11 + g, W, H, rgb);
        const size_t nb = (size_t)(W / 8) * (H / 8);
        int16_t *out = (int16_t *)malloc(3 * nb * 64 * sizeof(int16_t));
        for (int mode = 0; mode < 2; mode++)
            CHECK(cpuref_blocks(rgb, W, H, (size_t)W * 3, 75, 0, (const uint8_t(*)[8])uf, mode, 1, out) == 0);
        /* stripes: rows [r0, r1) with the pointer at pixel row 8 r0 (the halo above is read) */
        for (int r0 = 0; r0 < H / 8; r0++) {
            int16_t *o = (int16_t *)malloc(3 * (size_t)(W / 8) * 64 * sizeof(int16_t));
            CHECK(cpuref_blocks_rows(rgb, W, H, (size_t)W * 3, 60, 0, (const uint8_t(*)[8])uf, 0, 1, r0,
                                     r0 + 1, o) == 0);
            free(o);
        }
        /* the entropy statistics and dpcm over the output */
        int32_t *dc = (int32_t *)malloc(3 * nb * sizeof(int32_t));
        int32_t hist[4][257];
        cpuref_entropy_stats(out, (long)nb, (long)nb, dc, hist);
        int32_t *dc2 = (int32_t *)malloc(3 * nb * sizeof(int32_t));
        CHECK(jpgx_dpcm_dc(out, nb, NULL, dc2) == 0);
        free(dc2);
        free(dc);
        /* true 4:2:x definition */
        for (int sr = 1; sr <= 2; sr++) {
            if (W % 16 || H % (sr == 2 ? 16 : 8)) continue;
            const int crows = sr == 2 ? H / 16 : H / 8;
            const size_t nbc = (size_t)crows * (W / 16);
            int16_t *oc = (int16_t *)malloc(2 * nbc * 64 * sizeof(int16_t));
            CHECK(cpuref_chroma_sub_rows(rgb, W, H, (size_t)W * 3, 75, sr, 0, 1, 0, crows, oc) == 0);
            /* JFIF writer over Y | Cb | Cr */
            int16_t *all = (int16_t *)malloc((nb + 2 * nbc) * 64 * sizeof(int16_t));
            memcpy(all, out, nb * 64 * sizeof(int16_t));
            memcpy(all + nb * 64, oc, 2 * nbc * 64 * sizeof(int16_t));
            const size_t cap = jpgx_jfif_bound(W, H);
            uint8_t *buf = (uint8_t *)malloc(cap);
            size_t len = 0;
            CHECK(jpgx_write_jfif_sub(all, W, H, 75, sr, buf, cap, &len) == 0 && len <= cap);
            CHECK(jpgx_write_jfif_sub(all, W, H, 75, sr, buf, 40, &len) != 0);
            free(buf);
            free(all);
            free(oc);
        }
        /* 4:4:4 JFIF, with the exact bound and a too-small buffer */
        const size_t cap = jpgx_jfif_bound(W, H);
        uint8_t *buf = (uint8_t *)malloc(cap);
        size_t len = 0;
        CHECK(jpgx_write_jfif(out, W, H, 75, buf, cap, &len) == 0 && len <= cap);
        uint8_t *exact = (uint8_t *)malloc(len);
        size_t len2 = 0;
        CHECK(jpgx_write_jfif(out, W, H, 75, exact, len, &len2) == 0 && len2 == len);
        CHECK(jpgx_write_jfif(out, W, H, 75, exact, len - 1, &len2) != 0);
        free(exact);
        free(buf);
        /* JpgData adapter + dpcm */
        jpgx_jpeg_data j;
        memset(&j, 0, sizeof j);
        j.width = W;
        j.height = H;
        CHECK(jpgx_fill_jpgdata(&j, out) == 0);
        jpgx_dpcm(&j);
        jpgx_free_jpgdata(&j);
        free(out);
        free(rgb);
    }
    /* the tie frame: every Y DC an exact .5 */
    uint8_t *t = (uint8_t *)malloc(64 * 64 * 3);
    cpuref_gen_tie(64, 64, t);
    int16_t *o = (int16_t *)malloc(3 * 64 * 64 * sizeof(int16_t));
    uint8_t uz[3][8] = {{0}};
    CHECK(cpuref_blocks(t, 64, 64, 64 * 3, 50, 0, (const uint8_t(*)[8])uz, 0, 1, o) == 0);
    free(o);
    free(t);
}

static void block_api(void)
{
    jpgx_Block b = jpgx_new_block();
    for (int y = 0; y < 8; y++)
        for (int x = 0; x < 8; x++) jpgx_set_value_block(b, x, y, (double)((x * 37 + y * 11) % 255) - 128.0);
    jpgx_Block c = jpgx_copy_block(b);
    jpgx_dct_block(c);
    int t[8][8];
    CHECK(jpgx_scale_table(0, 90, t) == 0);
    jpgx_quantise_block(c, (const int(*)[8])t);
    int zz[64];
    jpgx_zig_zag_block(c, zz);
    jpgx_Block d = jpgx_copy_block(b);
    jpgx_dct_block(d);
    jpgx_quantise_lum(d);
    jpgx_quantise_chr(d);
    jpgx_scale_table_inplace(jpgx_q_table_lum, 50);
    jpgx_destroy_block(d);
    jpgx_destroy_block(c);
    jpgx_destroy_block(b);
}

int main(int argc, char **argv)
{
    g_tmp = argc > 1 ? argv[1] : "/tmp";
    const char *images = argc > 2 ? argv[2] : ".";
    bmp_hostile();
    bmp_images(images);
    planning();
    oracle_paths();
    block_api();
    /* the GPU entry points answer ENODEV in this build; the drop-in wrapper propagates it */
    uint8_t rgb[8 * 8 * 3] = {0};
    char out[4096];
    snprintf(out, sizeof out, "%s/never.jpg", g_tmp);
    CHECK(jpgx_encode_rgb_to_jpeg(rgb, 8, 8, 24, out, 90, 0, JPGX_FLAG_SUBSAMPLE, 0) == JPGX_ENODEV);
    printf(g_fail ? "sanitize: FAILED\n" : "sanitize: clean\n");
    return g_fail;
}
