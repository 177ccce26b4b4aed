/*
 * jpgx_compat.h -- the reference-compatible host API of libjpgx.so (C99, host code).
 *
 * The drop-in surface a user of matthewT53/JPEG-Encoder-and-Decoder keeps while the batched
 * hot path runs on the GPU (jpgx.h):
 *
 *   1. Block API with the reference's semantics, one 8x8 block of doubles at a time
 *      (src/headers/block.h:10-40, src/block.c:15-67; src/dct.c:36-59; src/quantise.c:52-86;
 *      src/zig_zag.c:48-58).  jpgx_block has the reference's struct _block layout, so the
 *      pointers are interchangeable.  These are per-block CPU calls for API compatibility and
 *      small jobs -- the throughput path is jpgx_blocks_gpu().
 *   2. A JpgData adapter: struct jpgx_jpeg_data has the field order and types of the
 *      reference's JpegData (src/headers/jpg_encode.h:21-70), and jpgx_fill_jpgdata() widens
 *      the GPU's int16 [3][nb][64] output into its zig_zag_Y/Cb/Cr int** arrays exactly as
 *      zig_zag() allocates them (src/zig_zag.c:24-32), so an unmodified dpcm()-style consumer
 *      (src/dpcm.c:6-21) works on it.
 *   3. Host stitch of the DC recurrence (src/dpcm.c:6-21) over the int16 layout, with a
 *      carry so that block-row stripes computed on different GPUs stitch exactly.
 *   4. The BMP reader (src/bitmap.c:41-152 semantics) and the stage sequence of
 *      encode_bmp_to_jpeg() up to the entropy stage (src/jpg_encode.c:19-47).
 *
 * Differences from the reference, all deliberate: functions report errors through return
 * codes (the reference returns void); zig-zag does not print one line per block
 * (src/zig_zag.c:21,50); nothing leaks (the reference never frees JpgData).
 */
#ifndef JPGX_COMPAT_H
#define JPGX_COMPAT_H

#include <stddef.h>
#include <stdint.h>

#include "jpgx.h"

#ifdef __cplusplus
extern "C" {
#endif

/* ---- 1. Block API ------------------------------------------------------------------------ */

/* src/block.c:15-17: 64 doubles, index y*8+x */
typedef struct jpgx_block {
    double values[64];
} jpgx_block;
typedef jpgx_block *jpgx_Block;

jpgx_Block jpgx_new_block(void);                                /* block.c:20-23   */
double jpgx_get_value_block(jpgx_Block b, int x, int y);       /* block.c:25-28   */
void jpgx_set_value_block(jpgx_Block b, int x, int y, double v); /* block.c:30-33 */
jpgx_Block jpgx_copy_block(jpgx_Block b);                       /* block.c:35-48   */
void jpgx_show_block(jpgx_Block b);                             /* block.c:50-62   */
void jpgx_destroy_block(jpgx_Block b);                          /* block.c:64-67   */

/* In-place forward DCT-II, the reference's exact operation order and double arithmetic
 * (dct.c:36-59): F(u,v) stored at get(b,u,v) = values[v*8+u]. */
void jpgx_dct_block(jpgx_Block b);

/* values[j*8+i] = round(values[j*8+i] / table[i][j]) -- the reference's transposed use of the
 * table (quantise.c:52-72), with an explicit table (reentrant). */
void jpgx_quantise_block(jpgx_Block b, const int table[8][8]);

/* Legacy global-table variants (quantise.c:8-26,52-72): they read jpgx_q_table_lum/chr, which
 * start as the base tables and are rescaled in place by jpgx_scale_table_inplace(), as the
 * reference's quantise() does (quantise.c:34-35; a second call rescales again).  Not
 * reentrant, by the reference's design; prefer jpgx_quantise_block(). */
extern int jpgx_q_table_lum[8][8];
extern int jpgx_q_table_chr[8][8];
void jpgx_quantise_lum(jpgx_Block b);
void jpgx_quantise_chr(jpgx_Block b);
/* quantise.c:74-86, in place, no validation (q outside [1,97] gives the reference's zeros) */
void jpgx_scale_table_inplace(int table[8][8], int quality);

/* zz[scan_order[i][j]] = (int) get(b, j, i)  (zig_zag.c:48-58) */
void jpgx_zig_zag_block(jpgx_Block b, int *zz);

/* ---- 2. JpgData adapter ------------------------------------------------------------------ */

/* src/headers/jpg_encode.h:21-34 */
typedef struct jpgx_huffman_data {
    int freq[257];
    int code_len[257];
    int others[257];
    int bits[32];
    int huffval[256];
} jpgx_huffman_data;

/* src/headers/jpg_encode.h:36-70, field for field */
typedef struct jpgx_jpeg_data {
    char *output_filename;
    char *input_filename;
    int width;
    int height;
    int sample_ratio;
    int quality;
    int num_blocks_Y;
    int num_blocks_Cb;
    int num_blocks_Cr;
    jpgx_Block *Y;
    jpgx_Block *Cb;
    jpgx_Block *Cr;
    int **zig_zag_Y;
    int **zig_zag_Cb;
    int **zig_zag_Cr;
    jpgx_huffman_data lum_DC;
    jpgx_huffman_data lum_AC;
    jpgx_huffman_data chrom_DC;
    jpgx_huffman_data chrom_AC;
} jpgx_jpeg_data;
typedef jpgx_jpeg_data *jpgx_JpgData;

/* j->width, j->height must be set (multiples of 8) and zig_zag_Y/Cb/Cr must be NULL (a filled
 * JpgData is released with jpgx_free_jpgdata first).  Allocates zig_zag_* as zig_zag() does
 * (an int* array of int[64], zig_zag.c:24-32), widens coef [3][nb][64] into it and then sets
 * num_blocks_* = (W/8)(H/8) (preprocess.c:45-47).  Returns 0, JPGX_EARG, or JPGX_ENOMEM
 * (then j is unchanged). */
int jpgx_fill_jpgdata(jpgx_JpgData j, const int16_t *coef);
/* frees what jpgx_fill_jpgdata allocated (zig_zag_*), leaves the rest */
void jpgx_free_jpgdata(jpgx_JpgData j);
/* dpcm.c:6-21 on j->zig_zag_*, in place */
void jpgx_dpcm(jpgx_JpgData j);

/* ---- 3. DC recurrence over the int16 layout ---------------------------------------------- */

/* dc[c][i] for channel c, block i of a run of nb blocks of coef [3][nb][64]:
 *   dc[c][0] = coef[c][0][0] - carry[c],  dc[c][i] = coef[c][i][0] - dc[c][i-1]
 * i.e. dpcm.c:10-20 (which reads the already-updated previous entry).  For a whole frame
 * carry = 0 and dc[c][0] = coef[c][0][0] (the reference leaves block 0 as is); for the
 * stripe starting at block s, carry = the previous stripe's last dc.  int32 output: the
 * recurrence is an alternating sum and can leave the int16 range.  Returns 0 / JPGX_EARG. */
int jpgx_dpcm_dc(const int16_t *coef, size_t nb, const int32_t carry[3], int32_t *dc);

/* ---- 4. BMP input and the encode stage sequence ------------------------------------------ */

/* Reads a BMP with the reference loader's semantics (bitmap.c:41-152): width/height/bit depth
 * from header offsets 18/22/28; pixel row i (top-down) taken from file offset
 * fs - (i+1)*W*(bpp/8) (the file is read backwards from its end, offsetRGB and row padding
 * ignored); stored byte order kept (byte 0 of a triple is the reference's "red").
 * Output: *rgb = malloc'd interleaved top-down W*H*3 bytes (free with jpgx_free), *file_size
 * = the file size (it sets the underflow bytes, jpgx_glibc_underflow).
 * Returns 0, JPGX_EARG (unreadable / not 24-bit / too short). */
int jpgx_bmp_read(const char *path, uint8_t **rgb, int *width, int *height, size_t *file_size);
void jpgx_free(void *p);

/* encode_bmp_to_jpeg() up to the entropy stage (jpg_encode.c:19-47): read the BMP, run the
 * block transform on GPU `device`, widen into *j (jpgx_fill_jpgdata) and, if do_dpcm, apply
 * dpcm.  Fills width/height/sample_ratio/quality.  Geometry rules as jpgx_validate(); the
 * underflow bytes follow the glibc model for this file (jpgx_glibc_underflow). */
int jpgx_encode_bmp(const char *path, int quality, int sample_ratio, int device, int do_dpcm,
                    jpgx_JpgData j);

/* ---- 5. Entropy stage: a baseline JFIF writer (the build's own; the reference's Huffman stage
 *         never terminates, src/huffman.c:23-235, so this has no reference to match) --------- */

/* Upper bound of the file size jpgx_write_jfif can produce for a width x height image. */
size_t jpgx_jfif_bound(int width, int height);

/* Baseline sequential JFIF (8-bit, one interleaved scan, 4:4:4, ITU-T T.81 Annex K.3 Huffman
 * tables, true DC prediction) of coef [3][nb][64] (zig-zag, raster blocks).  The DQT holds the
 * divisors the reference applied (its scaled tables, transposed: src/quantise.c:58), so a
 * standard decoder reproduces the reference's coefficients' image.  Returns 0, JPGX_EARG
 * (geometry, or cap too small: *len is then the size needed), JPGX_EQUALITY. */
int jpgx_write_jfif(const int16_t *coef, int width, int height, int quality, uint8_t *out,
                    size_t cap, size_t *len);

/* The same for coef = Y [nb][64] | Cb [nbc][64] | Cr [nbc][64] with sample_ratio 1 (true 4:2:2,
 * Y sampled 2x1, MCU = 2 Y + Cb + Cr) or 2 (true 4:2:0, 2x2, MCU = 4 Y + Cb + Cr), the layout
 * JPGX_FLAG_SUBSAMPLE produces; sample_ratio 0 is jpgx_write_jfif. */
int jpgx_write_jfif_sub(const int16_t *coef, int width, int height, int quality,
                        int sample_ratio, uint8_t *out, size_t cap, size_t *len);

/* The same with restart intervals, coded on host threads: `restart_rows` MCU rows per interval
 * (0: none, the single-interval stream of jpgx_write_jfif_sub; -1: about four intervals per
 * thread; the interval, rows x MCUs per row, must fit DRI's 16 bits), a DRI segment, DC
 * predictors reset and an RSTm marker at every interval boundary (T.81 F.1.2.1.3, B.2.4.4);
 * `nthreads` threads (0: one per online CPU, at most 64) code contiguous runs of intervals
 * into their own buffers, concatenated in order -- e.g. the 8 GPU stripes of a 16384^2 frame.
 * Returns as jpgx_write_jfif_sub, or JPGX_ENOMEM. */
int jpgx_write_jfif_ex(const int16_t *coef, int width, int height, int quality, int sample_ratio,
                       int restart_rows, int nthreads, uint8_t *out, size_t cap, size_t *len);

/* encode_bmp_to_jpeg with flags: JPGX_FLAG_SUBSAMPLE and sample_ratio 1/2 write a truly
 * subsampled JFIF (extension); otherwise exactly jpgx_encode_bmp_to_jpeg.  GPU `device`. */
int jpgx_encode_bmp_to_jpeg_ex(const char *input, const char *output, int quality,
                               int sample_ratio, unsigned flags, int device);

/* The reference's declared in-memory entry point (src/headers/jpg_encode.h:99,
 * encode_rgb_to_jpeg(Byte *colours, output, quality, sample_ratio); declared, never defined
 * there, and without the image size, which this one takes): interleaved top-down RGB rows
 * `pitch` bytes apart -> the block transform on GPU `device` -> a JFIF file at `output`
 * (truly subsampled with JPGX_FLAG_SUBSAMPLE and sample_ratio 1/2).  The x0 = -8 underflow
 * bytes are jpgx_default_params's (those of a 54-byte-header BMP of this size).  Returns 0 or a
 * JPGX_E* code. */
int jpgx_encode_rgb_to_jpeg(const uint8_t *rgb, int width, int height, size_t pitch,
                            const char *output, int quality, int sample_ratio, unsigned flags,
                            int device);

/* The reference's public entry point (src/headers/jpg_encode.h:85): BMP in, JPEG file out --
 * the block transform on GPU 0, then jpgx_write_jfif.  Returns 0 or a JPGX_E* code. */
int jpgx_encode_bmp_to_jpeg(const char *input, const char *output, int quality,
                            int sample_ratio);

#ifdef __cplusplus
}
#endif

#endif
