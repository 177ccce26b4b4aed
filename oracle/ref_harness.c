/*
 * ref_harness.c -- TEST INFRASTRUCTURE ONLY (this container; never shipped to the GPU box).
 *
 * Drives the REAL reference stage functions, compiled in place from /root/reference/src by
 * oracle/Makefile into oracle/_ref/, and dumps their output:
 *     ref_dump <in.bmp> <out.bin> <quality> <sample_ratio> [dpcm [stats.bin]]
 * writes int32 zig_zag_Y | zig_zag_Cb | zig_zag_Cr (each [nb][64]) after
 * preprocess_jpeg -> chroma_subsample -> dct -> quantise -> zig_zag (jpg_encode.c:32-44),
 * optionally followed by dpcm (jpg_encode.c:47).  huffman_encode is not called: it never
 * terminates -- in construct_huffman_table; with stats.bin the harness runs
 * its terminating first half instead: initialize_huffman and the per-block
 * calculate_freq_block_DC / _AC calls of huffman.c:23-44, and writes the four int32 freq[257]
 * tables lum_DC | lum_AC | chrom_DC | chrom_AC.  The stages print one line per block to
 * stdout; redirect it.
 *
 * Allocation discipline: nothing large is malloc'd before preprocess_jpeg so that the heap
 * history (which decides the bytes read by the x0 = -8 underflow, preprocess.c:159-160)
 * matches a plain encode_bmp_to_jpeg() call.
 */
#include <stdio.h>
#include <stdlib.h>

#include "headers/jpg_encode.h"
#include "headers/preprocess.h"
#include "headers/downsample.h"
#include "headers/dct.h"
#include "headers/quantise.h"
#include "headers/zig_zag.h"
#include "headers/dpcm.h"
#include "headers/huffman.h"

/* huffman.c's own (non-static) helpers, declared there, not in its header */
void initialize_huffman(JpgData j_data);
void calculate_freq_block_DC(HuffmanData *huffman_data, int *image_data);
void calculate_freq_block_AC(HuffmanData *huffman_data, int *image_data);

/* Linked with -Wl,--wrap=malloc: records the 8 bytes in front of every allocation so the
 * underflow model can be checked against what glibc really left there.
 * No allocation happens in here, so the heap history is unchanged. */
void *__real_malloc(size_t n);
static size_t g_watch = 0;
static unsigned char g_seen[16][8];
static int g_nseen = 0;
void *__wrap_malloc(size_t n)
{
    unsigned char *p = __real_malloc(n);
    if (p && g_watch && n == g_watch && g_nseen < 16) {
        for (int k = 0; k < 8; k++) g_seen[g_nseen][k] = p[k - 8];
        g_nseen++;
    }
    return p;
}

int main(int argc, char **argv)
{
    if (argc < 5) {
        fprintf(stderr, "usage: %s in.bmp out.bin quality sample_ratio [dpcm]\n", argv[0]);
        return 2;
    }
    JpgData j = calloc(1, sizeof(JpegData));
    j->input_filename = argv[1];
    j->output_filename = argv[2];
    j->quality = atoi(argv[3]);
    j->sample_ratio = atoi(argv[4]);
    if (getenv("REF_WATCH_PIXELS")) g_watch = (size_t)atol(getenv("REF_WATCH_PIXELS"));

    preprocess_jpeg(j);
    if (getenv("REF_STOP_AFTER_PREPROCESS")) {
        /* only the underflow bytes (recorded during preprocess_jpeg's r_new/g_new/b_new
         * mallocs, preprocess.c:127-129): seconds instead of the DCT's minutes */
        fprintf(stderr, "W=%d H=%d nb=%d\n", j->width, j->height, j->num_blocks_Y);
        for (int i = 0; i < g_nseen; i++) {
            fprintf(stderr, "pre[%d]=", i);
            for (int k = 0; k < 8; k++) fprintf(stderr, "%02x", g_seen[i][k]);
            fprintf(stderr, "\n");
        }
        return 0;
    }
    chroma_subsample(j);
    dct(j);
    quantise(j);
    zig_zag(j);
    if (argc > 5) dpcm(j);

    FILE *f = fopen(argv[2], "wb");
    if (!f) return 1;
    int **zz[3] = {j->zig_zag_Y, j->zig_zag_Cb, j->zig_zag_Cr};
    int nbs[3] = {j->num_blocks_Y, j->num_blocks_Cb, j->num_blocks_Cr};
    for (int c = 0; c < 3; c++)
        for (int i = 0; i < nbs[c]; i++) fwrite(zz[c][i], sizeof(int), 64, f);
    fclose(f);
    if (argc > 6) {
        /* huffman.c:23-44 up to (not including) construct_huffman_table */
        initialize_huffman(j);
        for (int i = 0; i < j->num_blocks_Y; i++) {
            calculate_freq_block_DC(&j->lum_DC, j->zig_zag_Y[i]);
            calculate_freq_block_AC(&j->lum_AC, j->zig_zag_Y[i]);
        }
        for (int i = 0; i < j->num_blocks_Cb; i++) {
            calculate_freq_block_DC(&j->chrom_DC, j->zig_zag_Cb[i]);
            calculate_freq_block_AC(&j->chrom_AC, j->zig_zag_Cb[i]);
        }
        for (int i = 0; i < j->num_blocks_Cr; i++) {
            calculate_freq_block_DC(&j->chrom_DC, j->zig_zag_Cr[i]);
            calculate_freq_block_AC(&j->chrom_AC, j->zig_zag_Cr[i]);
        }
        FILE *g = fopen(argv[6], "wb");
        if (!g) return 1;
        const HuffmanData *hd[4] = {&j->lum_DC, &j->lum_AC, &j->chrom_DC, &j->chrom_AC};
        for (int t = 0; t < 4; t++) fwrite(hd[t]->freq, sizeof(int), 257, g);
        fclose(g);
    }
    fprintf(stderr, "W=%d H=%d nb=%d\n", j->width, j->height, j->num_blocks_Y);
    /* allocations of exactly w*h bytes, in order: bitmap.c:116-118 planes, then
     * preprocess.c:127-129 r_new/g_new/b_new (the ones the underflow reads) */
    for (int i = 0; i < g_nseen; i++) {
        fprintf(stderr, "pre[%d]=", i);
        for (int k = 0; k < 8; k++) fprintf(stderr, "%02x", g_seen[i][k]);
        fprintf(stderr, "\n");
    }
    return 0;
}
