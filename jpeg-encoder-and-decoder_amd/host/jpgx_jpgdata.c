/*
 * jpgx_jpgdata.c -- JpgData adapter, DC recurrence, BMP reader and the encode stage sequence
 * (jpgx_compat.h parts 2-4), host C99.
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/jpgx_compat.h"

void jpgx_free(void *p) { free(p); }

static void free_rows(int **rows, int n)
{
    if (!rows) return;
    for (int i = 0; i < n; i++) free(rows[i]);
    free(rows);
}

void jpgx_free_jpgdata(jpgx_JpgData j)
{
    if (!j) return;
    free_rows(j->zig_zag_Y, j->num_blocks_Y);
    free_rows(j->zig_zag_Cb, j->num_blocks_Cb);
    free_rows(j->zig_zag_Cr, j->num_blocks_Cr);
    j->zig_zag_Y = j->zig_zag_Cb = j->zig_zag_Cr = NULL;
}

int jpgx_fill_jpgdata(jpgx_JpgData j, const int16_t *coef)
{
    if (!j || !coef || j->width <= 0 || j->height <= 0 || j->width % 8 || j->height % 8)
        return JPGX_EARG;
    if (j->zig_zag_Y || j->zig_zag_Cb || j->zig_zag_Cr) return JPGX_EARG;  /* would leak */
    const int nb = (j->width / 8) * (j->height / 8);  /* preprocess.c:45-47, every ratio */
    int **zz[3] = {NULL, NULL, NULL};
    for (int c = 0; c < 3; c++) {                     /* zig_zag.c:24-32                */
        zz[c] = (int **)calloc((size_t)nb, sizeof(int *));
        if (!zz[c]) goto oom;
        for (int i = 0; i < nb; i++) {
            int *row = (int *)malloc(64 * sizeof(int));
            if (!row) goto oom;
            const int16_t *src = coef + ((size_t)c * nb + i) * 64;
            for (int k = 0; k < 64; k++) row[k] = src[k];
            zz[c][i] = row;
        }
    }
    j->zig_zag_Y = zz[0];
    j->zig_zag_Cb = zz[1];
    j->zig_zag_Cr = zz[2];
    j->num_blocks_Y = j->num_blocks_Cb = j->num_blocks_Cr = nb;   /* only once all exist */
    return JPGX_OK;
oom:                                                  /* rows not yet allocated are NULL */
    for (int c = 0; c < 3; c++) free_rows(zz[c], nb);
    return JPGX_ENOMEM;
}

void jpgx_dpcm(jpgx_JpgData j)
{
    int **zz[3] = {j->zig_zag_Y, j->zig_zag_Cb, j->zig_zag_Cr};
    const int n[3] = {j->num_blocks_Y, j->num_blocks_Cb, j->num_blocks_Cr};
    for (int c = 0; c < 3; c++)                       /* dpcm.c:10-20                   */
        for (int i = 1; i < n[c]; i++) zz[c][i][0] = zz[c][i][0] - zz[c][i - 1][0];
}

int jpgx_dpcm_dc(const int16_t *coef, size_t nb, const int32_t carry[3], int32_t *dc)
{
    if (!coef || !dc) return JPGX_EARG;
    for (int c = 0; c < 3; c++) {
        int32_t prev = carry ? carry[c] : 0;
        for (size_t i = 0; i < nb; i++) {
            const int32_t d = (int32_t)coef[((size_t)c * nb + i) * 64] - prev;
            dc[(size_t)c * nb + i] = d;
            prev = d;
        }
    }
    return JPGX_OK;
}

int jpgx_bmp_read(const char *path, uint8_t **rgb, int *width, int *height, size_t *file_size)
{
    if (!path || !rgb || !width || !height) return JPGX_EARG;
    *rgb = NULL;
    FILE *fp = fopen(path, "rb");
    if (!fp) return JPGX_EARG;
    uint8_t *buf = NULL;
    long fs = -1;
    if (fseek(fp, 0, SEEK_END) == 0) fs = ftell(fp);
    if (fs >= 54 && fseek(fp, 0, SEEK_SET) == 0) {
        buf = (uint8_t *)malloc((size_t)fs);
        if (buf && fread(buf, 1, (size_t)fs, fp) != (size_t)fs) {
            free(buf);
            buf = NULL;
        }
    }
    fclose(fp);
    if (!buf) return JPGX_EARG;
    int32_t w, h;
    int16_t bpp;
    memcpy(&w, buf + 18, 4);                          /* bitmap.c:73-80 header fields   */
    memcpy(&h, buf + 22, 4);
    memcpy(&bpp, buf + 28, 2);
    /* the reference reads 3 bytes per pixel at a row stride of W*(bpp/8): only 24-bit
     * files are meaningful; rows are taken backwards from the end of the file
     * (bitmap.c:127-137) and must lie inside it */
    /* W*H*3 <= fs, tested without forming a product that can overflow (hostile headers) */
    if (bpp != 24 || w <= 0 || h <= 0 || (long long)w > fs / 3 || (long long)h > fs / 3 / w) {
        free(buf);
        return JPGX_EARG;
    }
    uint8_t *out = (uint8_t *)malloc((size_t)w * h * 3);
    if (!out) {
        free(buf);
        return JPGX_EARG;
    }
    const size_t row = (size_t)w * 3;
    for (int i = 0; i < h; i++)                       /* top-down row i                 */
        memcpy(out + (size_t)i * row, buf + (size_t)fs - (size_t)(i + 1) * row, row);
    free(buf);
    *rgb = out;
    *width = w;
    *height = h;
    if (file_size) *file_size = (size_t)fs;
    return JPGX_OK;
}

int jpgx_encode_bmp(const char *path, int quality, int sample_ratio, int device, int do_dpcm,
                    jpgx_JpgData j)
{
    if (!j) return JPGX_EARG;
    uint8_t *rgb = NULL;
    int w = 0, h = 0;
    size_t fs = 0;
    int rc = jpgx_bmp_read(path, &rgb, &w, &h, &fs);
    if (rc) return rc;
    jpgx_params p;
    jpgx_default_params(&p, w, h, quality, sample_ratio);
    uint8_t under[8];
    jpgx_glibc_underflow((long long)w * h, (long long)fs, under);
    for (int c = 0; c < 3; c++) memcpy(p.underflow[c], under, 8);
    rc = jpgx_validate(w, h, &p);
    int16_t *coef = NULL;
    if (!rc) {
        coef = (int16_t *)malloc((size_t)w * h * 3 * sizeof(int16_t));
        rc = coef ? jpgx_blocks(rgb, w, h, (size_t)w * 3, &p, coef, device) : JPGX_ENOMEM;
    }
    free(rgb);
    if (!rc) {
        j->width = w;                                  /* preprocess.c:38-39            */
        j->height = h;
        j->quality = quality;
        j->sample_ratio = sample_ratio;
        j->input_filename = (char *)path;
        rc = jpgx_fill_jpgdata(j, coef);
        if (!rc && do_dpcm) jpgx_dpcm(j);
    }
    free(coef);
    return rc;
}
