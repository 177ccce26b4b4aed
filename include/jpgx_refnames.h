/*
 * jpgx_refnames.h -- the reference's unprefixed per-block API names mapped onto libjpgx.
 *
 * Include this instead of src/headers/block.h, dct.h, quantise.h and zig_zag.h in a
 * translation unit written against matthewT53/JPEG-Encoder-and-Decoder's Block API; the call
 * sites stay unchanged and link against libjpgx.so:
 *   new_block / get_value_block / set_value_block / copy_block / show_block / destroy_block
 *                                          src/headers/block.h:15-40, src/block.c:20-67
 *   dct_block                              src/headers/dct.h:10,      src/dct.c:36-59
 *   quantise_lum / quantise_chr            src/headers/quantise.h:9-10, src/quantise.c:52-72
 *   zig_zag_block                          src/headers/zig_zag.h:11,  src/zig_zag.c:48-58
 * Block is the reference's pointer-to-struct _block (one double[8][8]).  quantise_lum/chr read
 * the legacy global tables jpgx_q_table_lum/chr (the reference's q_table_lum/chr, rescaled in
 * place by scale_table), not reentrant by the reference's design (src/quantise.c:34-35).
 * tests/c/dropin_block.c compiles against this header (tests/test_dropin.py).
 */
#ifndef JPGX_REFNAMES_H
#define JPGX_REFNAMES_H

#include "jpgx_compat.h"

typedef jpgx_Block Block;

#define new_block jpgx_new_block
#define get_value_block jpgx_get_value_block
#define set_value_block jpgx_set_value_block
#define copy_block jpgx_copy_block
#define show_block jpgx_show_block
#define destroy_block jpgx_destroy_block
#define dct_block jpgx_dct_block
#define quantise_lum jpgx_quantise_lum
#define quantise_chr jpgx_quantise_chr
#define scale_table jpgx_scale_table_inplace
#define q_table_lum jpgx_q_table_lum
#define q_table_chr jpgx_q_table_chr
#define zig_zag_block jpgx_zig_zag_block

#endif
