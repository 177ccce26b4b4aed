/*
 * jpgx_block.c -- the reference's per-block API (jpgx_compat.h part 1), host C99.
 *
 * Same arithmetic as the reference, one block at a time: IEEE double, the reference's
 * operation order, FP contraction off (Makefile: -ffp-contract=off), the glibc cosine doubles
 * from a table instead of two cos() calls per term (same values, jx_consts.h).
 */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/jpgx_compat.h"
#include "../csrc/jx_consts.h"

static const double kCos[8][8] = JX_COS_INIT;
static const int kScan[8][8] = JX_SCAN_ORDER_INIT;

int jpgx_q_table_lum[8][8] = JX_Q_LUM_INIT;
int jpgx_q_table_chr[8][8] = JX_Q_CHR_INIT;

jpgx_Block jpgx_new_block(void) { return (jpgx_Block)malloc(sizeof(jpgx_block)); }

double jpgx_get_value_block(jpgx_Block b, int x, int y) { return b->values[y * 8 + x]; }

void jpgx_set_value_block(jpgx_Block b, int x, int y, double v) { b->values[y * 8 + x] = v; }

jpgx_Block jpgx_copy_block(jpgx_Block b)
{
    jpgx_Block c = jpgx_new_block();
    if (c) memcpy(c, b, sizeof(*c));
    return c;
}

void jpgx_show_block(jpgx_Block b)
{
    /* block.c:50-62: a newline before every row, "%8.2f " per value, a final newline */
    for (int i = 0; i < 64; i++) {
        if (i % 8 == 0) printf("\n");
        printf("%8.2f ", b->values[i]);
    }
    printf("\n");
    fflush(stdout);
}

void jpgx_destroy_block(jpgx_Block b) { free(b); }

void jpgx_dct_block(jpgx_Block b)
{
    double in[64];
    memcpy(in, b->values, sizeof(in));                 /* dct.c:41 works on a copy      */
    for (int u = 0; u < 8; u++)
        for (int v = 0; v < 8; v++) {
            double s = 0.0;
            for (int x = 0; x < 8; x++)                /* x outer, y inner (dct.c:46-47) */
                for (int y = 0; y < 8; y++) s += in[y * 8 + x] * kCos[u][x] * kCos[v][y];
            const double au = u == 0 ? JX_ALPHA0 : 1.0, av = v == 0 ? JX_ALPHA0 : 1.0;
            b->values[v * 8 + u] = 0.25 * au * av * s; /* dct.c:54, left to right        */
        }
}

void jpgx_quantise_block(jpgx_Block b, const int table[8][8])
{
    for (int i = 0; i < 8; i++)
        for (int j = 0; j < 8; j++)                    /* get(b,i,j) = values[j*8+i]     */
            b->values[j * 8 + i] = round(b->values[j * 8 + i] / table[i][j]);
}

void jpgx_quantise_lum(jpgx_Block b) { jpgx_quantise_block(b, (const int(*)[8])jpgx_q_table_lum); }

void jpgx_quantise_chr(jpgx_Block b) { jpgx_quantise_block(b, (const int(*)[8])jpgx_q_table_chr); }

void jpgx_scale_table_inplace(int table[8][8], int quality)
{
    if (quality == 0) return;                          /* reference divides by zero here */
    const int s = quality < 50 ? 5000 / quality : 200 - 2 * quality;
    for (int i = 0; i < 8; i++)
        for (int j = 0; j < 8; j++) table[i][j] = (s * table[i][j] + 50) / 100;
}

void jpgx_zig_zag_block(jpgx_Block b, int *zz)
{
    for (int i = 0; i < 8; i++)
        for (int j = 0; j < 8; j++) zz[kScan[i][j]] = (int)b->values[i * 8 + j];
}
