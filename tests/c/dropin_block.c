/*
 * dropin_block.c -- a translation unit written against the reference's Block API names
 * (src/headers/block.h, dct.h, quantise.h, zig_zag.h), compiled with include/jpgx_refnames.h
 * and linked only against libjpgx.so: the reference's call sites, unchanged, on libjpgx.
 *
 * stdin: 64 pixel values (row y, column x order), an optional quality (0 = the unscaled base
 * table, as the reference's test_dct() in src/jpg_driver.c:54-150 uses it).
 * stdout: the 64 DCT values (%.17g), then the 64 zig-zag integers.
 */
#include <stdio.h>
#include <stdlib.h>

#include "jpgx_refnames.h"

int main(void)
{
    double v[64];
    for (int i = 0; i < 64; i++)
        if (scanf("%lf", &v[i]) != 1) return 2;
    int quality = 0;
    if (scanf("%d", &quality) != 1) quality = 0;

    Block b = new_block();
    for (int y = 0; y < 8; y++)
        for (int x = 0; x < 8; x++) set_value_block(b, x, y, v[y * 8 + x]);
    dct_block(b);
    for (int y = 0; y < 8; y++)
        for (int x = 0; x < 8; x++) printf("%.17g%c", get_value_block(b, x, y), x == 7 ? '\n' : ' ');
    if (quality > 0) scale_table(q_table_lum, quality);
    quantise_lum(b);
    int zz[64];
    zig_zag_block(b, zz);
    for (int i = 0; i < 64; i++) printf("%d%c", zz[i], i % 16 == 15 ? '\n' : ' ');
    destroy_block(b);
    return 0;
}
