/*
 * jpgx.h -- C ABI of the MI355X-native JPEG block-transform hot path (libjpgx.so).
 *
 * Replaces, for device-resident (or host) RGB frames, the per-8x8-block stage sequence of
 * matthewT53/JPEG-Encoder-and-Decoder that encode_bmp_to_jpeg() runs between loading the
 * bitmap and the entropy stage (reference src/jpg_encode.c:32-44):
 *
 *     preprocess_jpeg   src/preprocess.c:25-70   RGB -> YCbCr, level shift, 8x8 tiling
 *     chroma_subsample  src/downsample.c:9-32    (a print-only no-op in the reference)
 *     dct               src/dct.c:19-59          forward DCT-II per block
 *     quantise          src/quantise.c:30-86     quality-scaled tables, applied transposed
 *     zig_zag           src/zig_zag.c:17-58      scan order; result in JpgData.zig_zag_*
 *
 * Output contract (bit-exact to the reference on the same input, quirks included):
 *   int16 coefficients laid out [channel Y,Cb,Cr][block n, raster order][64 zig-zag], i.e. the
 *   reference's JpgData.zig_zag_Y[n][k], zig_zag_Cb[n][k], zig_zag_Cr[n][k]
 *   (src/headers/jpg_encode.h:60-62) narrowed to int16 (|coef| <= 2728 always fits).
 *
 * Input contract: interleaved, top-down pixels; byte k of each pixel is what the reference
 * loader calls plane k ("red", "green", "blue": src/bitmap.c:129-137).
 *
 * Conventions (unlike the reference, whose stages return void and mutate globals):
 *   - every entry point returns 0 or a negative JPGX_E* code;
 *   - callers own every buffer; the device path keeps no global mutable state (reentrant);
 *     the host-buffer path keeps its device buffers, streams and pinned staging in explicit
 *     contexts (jpgx_host_*), which jpgx_blocks / jpgx_blocks_multi take from a thread-safe
 *     process-wide pool (jpgx_host_release frees it).  One jpgx_host_ctx serves ONE caller at
 *     a time: its shards' buffers are reused call to call, so two threads must not call
 *     jpgx_host_blocks on the same context concurrently (use one context per thread, or the
 *     pooled jpgx_blocks, which hands each concurrent call its own context);
 *   - quantisation tables are rebuilt from the pristine base tables on every call
 *     (the reference rescales its globals in place, src/quantise.c:34-35).
 */
#ifndef JPGX_H
#define JPGX_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define JPGX_OK 0
#define JPGX_EGEOMETRY (-1)  /* width/height not a multiple of 8 (16 for 4:2:2 / 4:2:0)   */
#define JPGX_EQUALITY (-2)   /* quality outside [1, 97] (q >= 98 divides by zero, q <= 0
                                divides by zero: src/quantise.c:81-82)                     */
#define JPGX_ESAMPLE (-3)    /* sample_ratio not 0, 1 or 2                                 */
#define JPGX_EARG (-4)       /* null pointer, bad stripe, misaligned buffer or stride      */
#define JPGX_EHIP (-5)       /* HIP runtime error                                          */
#define JPGX_EWORKSPACE (-6) /* workspace smaller than jpgx_workspace_size()               */
#define JPGX_ENODEV (-7)     /* no usable GPU                                              */
#define JPGX_ENOMEM (-8)     /* host allocation failed                                     */

/* Chroma sampling constants, src/headers/jpg_encode.h:13-15.  The reference does not
 * actually subsample (src/downsample.c:24-32): 1 and 2 only tighten the geometry rule
 * (src/preprocess.c:87-95) and produce 4:4:4 output, which is what parity requires. */
#define JPGX_NO_CHROMA_SUBSAMPLING 0
#define JPGX_HORIZONTAL_SUBSAMPLING 1
#define JPGX_HORIZONTAL_VERTICAL_SUBSAMPLING 2

/* flags */
#define JPGX_FLAG_FORCE_EXACT 1u /* send every coefficient through the exact fp64 path     */
/* EXTENSION (no reference counterpart: src/downsample.c:24-32 only prints): with sample_ratio
 * 1 or 2, really subsample the chroma -- level-shifted Cb/Cr averaged over the horizontal pixel
 * pair (4:2:2) or the 2x2 quad (4:2:0), in that order; the (W/2) x H or (W/2) x (H/2) planes are
 * tiled in raster order (the x0 = -8 quirk stays a property of the 4:4:4 tiling only).  Y is
 * unchanged.  Frame output becomes Y [nb][64], Cb [nbc][64], Cr [nbc][64] contiguous, nbc =
 * jpgx_chroma_blocks(); for 4:2:0 stripes must start and end on even block rows. */
#define JPGX_FLAG_SUBSAMPLE 2u

typedef struct jpgx_params {
    int quality;              /* 1..97                                                    */
    int sample_ratio;         /* JPGX_*_SUBSAMPLING                                       */
    unsigned flags;           /* JPGX_FLAG_*                                              */
    uint8_t underflow[3][8];  /* [plane][x]: the 8 bytes the reference reads in front of
                                 each pixel plane r_new/g_new/b_new (src/preprocess.c:
                                 127-129) for the last block of block-row 0 (offset
                                 (y+y0)*W + x0 + x < 0 at :159, blockToCoords x0 = -8 at
                                 :199-211).  They are glibc's chunk-size words;
                                 jpgx_default_params fills the value a fresh
                                 encode_bmp_to_jpeg() process reads (all three equal). */
} jpgx_params;

/* A batch of frames, or one block-row stripe [row_begin, row_end) of each frame. */
typedef struct jpgx_frames {
    int width, height;        /* full-frame pixel geometry                                */
    int row_begin, row_end;   /* block rows processed; 0 and height/8 for whole frames    */
    int nframes;              /* frames in the batch (>= 1)                               */
    size_t in_pitch;          /* bytes between pixel rows (multiple of 8, at most 2^27)   */
    size_t in_frame_stride;   /* bytes between frames (multiple of 8)                     */
    size_t out_frame_stride;  /* int16 elements between frames' outputs                   */
} jpgx_frames;

/* Validation shared by every entry point. */
int jpgx_validate(int width, int height, const jpgx_params *p);

/* Defaults: the given quality/sample_ratio, no flags, glibc underflow bytes for a 24-bit
 * 54-byte-header BMP of this size (jpgx_glibc_underflow with file = 54 + 3*w*h). */
void jpgx_default_params(jpgx_params *p, int width, int height, int quality, int sample_ratio);

/* Chunk-size bytes glibc leaves in front of the reference's r_new/g_new/b_new planes
 * (src/preprocess.c:127-129) after its BMP loader freed a file-sized buffer
 * (src/bitmap.c:113,151), when the planes come from the top chunk or from mmap (every
 * image of 64x48 pixels or more in the fixtures; tiny images can reuse a freed chunk, then
 * pass the real bytes per plane).  n_pixels = w*h, bmp_file_size = size of the BMP file. */
void jpgx_glibc_underflow(long long n_pixels, long long bmp_file_size, uint8_t out[8]);

/* quantise.c:74-86 on a pristine base table: 0 = luminance, 1 = chrominance. */
int jpgx_scale_table(int which, int quality, int out[8][8]);

/* The guard band in use for `quality` (per channel, natural index v*8+u): a coefficient
 * whose fp32 quotient lies within lim of a rounding boundary is recomputed exactly.
 * Also returns the fp32 per-coefficient scale.  For tests and documentation. */
int jpgx_guard_band(int quality, float scale[3][64], float lim[3][64]);

/* Chroma blocks per channel of the stripe [row_begin, row_end) of a width-pixel frame: nb =
 * (row_end-row_begin)*width/8 without JPGX_FLAG_SUBSAMPLE (or sample_ratio 0), else
 * rows*width/16 (4:2:2) or rows/2*width/16 (4:2:0). */
size_t jpgx_chroma_blocks(int width, int row_begin, int row_end, int sample_ratio, unsigned flags);

/* ---- device path (pointers are device pointers; `stream` is a hipStream_t or NULL) ---- */

/* Bytes of device workspace one jpgx_blocks_gpu call on `fr` needs: 0 for every geometry
 * (both 4:4:4 kernels and k_chroma keep their exact-pass queues in LDS; d_workspace may then
 * be NULL).  Kept so callers stay source-compatible. */
size_t jpgx_workspace_size(const jpgx_frames *fr);

/* The fused hot path: RGB -> quantised zig-zag int16 for every block of fr's stripe of every
 * frame.  d_rgb points at pixel (0, 8*row_begin) of frame 0; when row_begin > 0 the pixel
 * row above it must be readable too (the x0 = -8 quirk reads the last 8 pixels of the
 * previous pixel row).  Frame f's output is [3][nb][64] at d_out + f*out_frame_stride,
 * nb = (row_end-row_begin)*width/8.  Asynchronous on `stream`. */
int jpgx_blocks_gpu(const jpgx_frames *fr, const jpgx_params *p, const uint8_t *d_rgb,
                    int16_t *d_out, void *d_workspace, size_t workspace_bytes, void *stream);

/* Same, and records hipEvent_t `event_between` (if non-NULL) on `stream` right after the
 * transform kernel (for timing the kernel alone against an event recorded before the call). */
int jpgx_blocks_gpu_ev(const jpgx_frames *fr, const jpgx_params *p, const uint8_t *d_rgb,
                       int16_t *d_out, void *d_workspace, size_t workspace_bytes, void *stream,
                       void *event_between);

/* Same as jpgx_blocks_gpu, and times the transform kernel itself: the 4:4:4 / true-4:2:x kernels
 * are launched through hipExtLaunchKernel with hipEvent_t ev_start / ev_stop (both required,
 * created by the caller), so hipEventElapsedTime(ev_start, ev_stop) is the kernel's execution
 * interval -- the one a rocprofv3 kernel trace reports, without the queue gap before the dispatch
 * that events recorded around the call include (bench.py's roofline).  The test-only library
 * records them around its kernels instead. */
int jpgx_blocks_gpu_timed(const jpgx_frames *fr, const jpgx_params *p, const uint8_t *d_rgb,
                          int16_t *d_out, void *d_workspace, size_t workspace_bytes, void *stream,
                          void *ev_start, void *ev_stop);

/* Entropy-stage statistics on the device: over one image's coefficients
 * d_coef = Y [nb_y][64] | Cb [nb_c][64] | Cr [nb_c][64] (what jpgx_blocks_gpu writes; nb_c =
 * nb_y unless JPGX_FLAG_SUBSAMPLE), the reference's in-place DC recurrence (src/dpcm.c:6-21)
 * into d_dc[nb_y + 2 nb_c] (int32), and huffman_encode's frequency pass (src/huffman.c:23-44,
 * 182-235; construct_huffman_table excluded) into d_hist[4][257] (uint32: lum_DC, lum_AC,
 * chrom_DC, chrom_AC; freq[256] = 1 as initialize_huffman reserves it; AC symbols keep the
 * reference's `run | size`).  carry (host, may be NULL = image start): per channel the last
 * dpcm'd DC of the blocks before these (jpgx_dpcm_dc semantics), for stripes.  Workspace:
 * jpgx_entropy_workspace_size() bytes, 8-byte aligned.  Asynchronous on `stream`. */
size_t jpgx_entropy_workspace_size(size_t nb_y, size_t nb_c);
int jpgx_entropy_stats_gpu(const int16_t *d_coef, size_t nb_y, size_t nb_c, const int32_t *carry,
                           int32_t *d_dc, uint32_t *d_hist, void *d_workspace,
                           size_t workspace_bytes, void *stream);
/* The same over a batch of nframes independent images of one size in one set of launches (what
 * jpgx_blocks_gpu writes for a frame batch: frame f's coefficients at d_coef + f *
 * coef_frame_stride int16 elements, a multiple of 64 and >= (nb_y + 2 nb_c) 64): d_dc
 * [nframes][nb_y + 2 nb_c], d_hist [nframes][4][257]; every frame starts its recurrence at the
 * image start (carry must be NULL unless nframes == 1).  Per-image launches leave the chip mostly
 * idle at 4K.  Workspace: jpgx_entropy_workspace_size_batch() bytes. */
size_t jpgx_entropy_workspace_size_batch(size_t nb_y, size_t nb_c, size_t nframes);
int jpgx_entropy_stats_gpu_batch(const int16_t *d_coef, size_t coef_frame_stride, size_t nframes, size_t nb_y,
                                 size_t nb_c, const int32_t *carry, int32_t *d_dc, uint32_t *d_hist,
                                 void *d_workspace, size_t workspace_bytes, void *stream);

/* Synthetic frames, generated directly in device memory (SURVEY.md 8c generator G: byte k
 * of the buffer = splitmix64(seed + (k+1)*0x9E3779B97F4A7C15) >> 56). */
int jpgx_gen_splitmix_gpu(uint8_t *d_dst, size_t nbytes, uint64_t seed, void *stream);
/* Tie frame T: flat gray 8x8 blocks, v = 97 + 2*(block_index % 40), R=G=B. */
int jpgx_gen_tie_gpu(uint8_t *d_dst, int width, int height, void *stream);

/* ---- host-buffer path (synchronous; csrc/jpgx_host.cpp) ------------------------------ */

/* A host-buffer context: the image is cut into `nshards` balanced block-row shards
 * (jpgx_stripe; MCU-row pairs for true 4:2:0), shard k runs on GPU devices[k] (NULL: k modulo
 * the device count; several shards may name the same GPU), one host thread per shard, no
 * communication between shards (each reads the pixel row above its first block row as halo and
 * writes a disjoint range of the output).  A shard streams its rows through the device in
 * chunks of `chunk_rows` block rows (0: about 4 MB of RGB per chunk), two chunks in flight on
 * two streams, so one chunk's H2D overlaps the previous chunk's D2H.  Device chunk buffers,
 * streams, events and pinned staging buffers are allocated on first use, grown when an image
 * needs more, and kept until jpgx_host_destroy.  Pageable caller buffers are staged through
 * the pinned buffers (host copies overlapped with the DMA); page-locked ones (hipHostMalloc,
 * jpgx_host_register) are copied directly.  A context is used by one call at a time. */
typedef struct jpgx_host_ctx jpgx_host_ctx;
int jpgx_host_create(jpgx_host_ctx **ctx, int nshards, const int *devices, int chunk_rows);
void jpgx_host_destroy(jpgx_host_ctx *ctx);

/* Whole image in host memory (pixel rows `pitch` bytes apart) -> host int16 output laid out as
 * jpgx_blocks_gpu's frame output ([3][nb][64], or Y | Cb | Cr with JPGX_FLAG_SUBSAMPLE). */
int jpgx_host_blocks(jpgx_host_ctx *ctx, const uint8_t *rgb, int width, int height, size_t pitch,
                     const jpgx_params *p, int16_t *out);

/* Page-lock (hipHostRegister, portable) / release a caller buffer so that jpgx_host_blocks
 * DMAs it directly. */
int jpgx_host_register(void *ptr, size_t bytes);
int jpgx_host_unregister(void *ptr);

/* Frees the pooled contexts behind jpgx_blocks / jpgx_blocks_multi. */
void jpgx_host_release(void);

/* Whole image on GPU `device` (a pooled one-shard context). */
int jpgx_blocks(const uint8_t *rgb, int width, int height, size_t pitch, const jpgx_params *p,
                int16_t *out, int device);

/* Same, sharded into ngpus block-row stripes on GPUs 0..ngpus-1 (a pooled context). */
int jpgx_blocks_multi(const uint8_t *rgb, int width, int height, size_t pitch,
                      const jpgx_params *p, int16_t *out, int ngpus);

/* Block-row stripe bounds of shard k of n (balanced, contiguous). */
void jpgx_stripe(int block_rows, int nshards, int k, int *row_begin, int *row_end);

/* Number of visible GPUs (0 if none). */
int jpgx_device_count(void);

/* Library version string. */
const char *jpgx_version(void);

#ifdef __cplusplus
}
#endif
#endif
