/*
 * dropin_entropy.c -- the drop-in proven at the C level: a JpgData filled by libjpgx is handed
 * to the reference's OWN, unchanged entropy front end.
 *
 * Compiled against the reference's headers (src/headers/jpg_encode.h: JpgData, HuffmanData)
 * where they lie, linked with the reference's own dpcm.o and huffman.o (compiled from
 * src/dpcm.c and src/huffman.c by `make -C oracle ref` into oracle/_ref/) and libjpgx.so.
 *   coef mode:  dropin_entropy coef <coef.bin> <W> <H> <dc.bin> <hist.bin>
 *               coef.bin = int16 [3][nb][64] zig-zag coefficients (what jpgx_blocks_gpu writes)
 *   bmp mode:   dropin_entropy bmp <in.bmp> <quality> <dc.bin> <hist.bin>
 *               jpgx_encode_bmp on GPU 0 (replacing src/jpg_encode.c:32-44)
 * then, on the same JpgData: dpcm() (src/dpcm.c:6-21) and the frequency half of
 * huffman_encode() (src/huffman.c:23-44: initialize_huffman, calculate_freq_block_DC/AC per
 * block; construct_huffman_table never terminates in the reference and is not called).
 * Writes the post-dpcm DC values (int32, Y then Cb then Cr) and the four freq[257] tables.
 */
#include <stdio.h>
#include <stdlib.h>

#include "headers/dpcm.h"
#include "headers/jpg_encode.h"
#include "jpgx_compat.h"

/* src/huffman.c (non-static, declared only there) */
void initialize_huffman(JpgData j_data);
void calculate_freq_block_DC(HuffmanData *huffman_data, int *image_data);
void calculate_freq_block_AC(HuffmanData *huffman_data, int *image_data);

_Static_assert(sizeof(JpegData) == sizeof(jpgx_jpeg_data), "JpgData layout");

int main(int argc, char **argv)
{
    if (argc < 2) return 2;
    JpgData j = (JpgData)calloc(1, sizeof(JpegData));
    const char *dcp, *hp;
    int rc;
    if (argv[1][0] == 'c' && argc == 7) {
        j->width = atoi(argv[3]);
        j->height = atoi(argv[4]);
        const size_t nb = (size_t)(j->width / 8) * (j->height / 8);
        int16_t *coef = (int16_t *)malloc(nb * 3 * 64 * sizeof(int16_t));
        FILE *f = fopen(argv[2], "rb");
        if (!f || fread(coef, sizeof(int16_t), nb * 3 * 64, f) != nb * 3 * 64) return 3;
        fclose(f);
        rc = jpgx_fill_jpgdata((jpgx_JpgData)j, coef);
        free(coef);
        dcp = argv[5];
        hp = argv[6];
    } else if (argv[1][0] == 'b' && argc == 6) {
        rc = jpgx_encode_bmp(argv[2], atoi(argv[3]), NO_CHROMA_SUBSAMPLING, 0, 0, (jpgx_JpgData)j);
        dcp = argv[4];
        hp = argv[5];
    } else {
        return 2;
    }
    if (rc) {
        fprintf(stderr, "jpgx error %d\n", rc);
        return 4;
    }

    dpcm(j);                                                  /* the reference's own */
    initialize_huffman(j);                                    /* src/huffman.c:23-44 */
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

    FILE *fd = fopen(dcp, "wb"), *fh = fopen(hp, "wb");
    if (!fd || !fh) return 5;
    int **zz[3] = {j->zig_zag_Y, j->zig_zag_Cb, j->zig_zag_Cr};
    const int n[3] = {j->num_blocks_Y, j->num_blocks_Cb, j->num_blocks_Cr};
    for (int c = 0; c < 3; c++)
        for (int i = 0; i < n[c]; i++) fwrite(&zz[c][i][0], sizeof(int), 1, fd);
    const HuffmanData *h[4] = {&j->lum_DC, &j->lum_AC, &j->chrom_DC, &j->chrom_AC};
    for (int k = 0; k < 4; k++) fwrite(h[k]->freq, sizeof(int), 257, fh);
    fclose(fd);
    fclose(fh);
    jpgx_free_jpgdata((jpgx_JpgData)j);
    free(j);
    return 0;
}
