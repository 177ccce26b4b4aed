/*
 * jx_consts.h -- constant tables of the reference's arithmetic, shared (as initialiser
 * macros) by the gfx950 kernels, the host plan and the host C compatibility layer, so every
 * copy in the library is the same one.  Plain C: included from C99, C++ and HIP.
 */
#ifndef JX_CONSTS_H
#define JX_CONSTS_H

/* Base quantisation tables, src/quantise.c:8-25 (row index = first subscript). */
#define JX_Q_LUM_INIT                                                                   \
    {{16, 11, 10, 16, 24, 40, 51, 61},   {12, 12, 14, 19, 26, 58, 60, 55},              \
     {14, 13, 16, 24, 40, 57, 69, 56},   {14, 17, 22, 29, 51, 87, 80, 62},              \
     {18, 22, 37, 56, 68, 109, 103, 77}, {24, 35, 55, 64, 81, 104, 113, 92},            \
     {49, 64, 78, 87, 103, 121, 120, 101}, {72, 92, 95, 98, 112, 100, 103, 99}}
#define JX_Q_CHR_INIT                                                                   \
    {{17, 18, 24, 47, 99, 99, 99, 99}, {18, 21, 26, 66, 99, 99, 99, 99},                \
     {24, 26, 56, 99, 99, 99, 99, 99}, {47, 66, 99, 99, 99, 99, 99, 99},                \
     {99, 99, 99, 99, 99, 99, 99, 99}, {99, 99, 99, 99, 99, 99, 99, 99},                \
     {99, 99, 99, 99, 99, 99, 99, 99}, {99, 99, 99, 99, 99, 99, 99, 99}}

/* Scan position of natural (row i, column j), src/zig_zag.c:6-15. */
#define JX_SCAN_ORDER_INIT                                                              \
    {{0, 1, 5, 6, 14, 15, 27, 28},     {2, 4, 7, 13, 16, 26, 29, 42},                   \
     {3, 8, 12, 17, 25, 30, 41, 43},   {9, 11, 18, 24, 31, 40, 44, 53},                 \
     {10, 19, 23, 32, 39, 45, 52, 54}, {20, 22, 33, 38, 46, 51, 55, 60},                \
     {21, 34, 37, 47, 50, 56, 59, 61}, {35, 36, 48, 49, 57, 58, 62, 63}}

/* cos(((2x+1)*u*M_PI)/16) exactly as glibc returns it for the reference (src/dct.c:49-50;
 * SURVEY.md Appendix B; tests/test_host.py re-derives it from the host libm).  [u][x]. */
#define JX_COS_INIT                                                                     \
    {{0x1p+0, 0x1p+0, 0x1p+0, 0x1p+0, 0x1p+0, 0x1p+0, 0x1p+0, 0x1p+0},                  \
     {0x1.f6297cff75cbp-1, 0x1.a9b66290ea1a3p-1, 0x1.1c73b39ae68c9p-1,                  \
      0x1.8f8b83c69a60dp-3, -0x1.8f8b83c69a608p-3, -0x1.1c73b39ae68c6p-1,               \
      -0x1.a9b66290ea1a4p-1, -0x1.f6297cff75cbp-1},                                     \
     {0x1.d906bcf328d46p-1, 0x1.87de2a6aea964p-2, -0x1.87de2a6aea962p-2,                \
      -0x1.d906bcf328d46p-1, -0x1.d906bcf328d47p-1, -0x1.87de2a6aea96dp-2,              \
      0x1.87de2a6aea967p-2, 0x1.d906bcf328d44p-1},                                      \
     {0x1.a9b66290ea1a3p-1, -0x1.8f8b83c69a608p-3, -0x1.f6297cff75cbp-1,                \
      -0x1.1c73b39ae68c8p-1, 0x1.1c73b39ae68c5p-1, 0x1.f6297cff75cbp-1,                 \
      0x1.8f8b83c69a61dp-3, -0x1.a9b66290ea1a2p-1},                                     \
     {0x1.6a09e667f3bcdp-1, -0x1.6a09e667f3bccp-1, -0x1.6a09e667f3bcep-1,              \
      0x1.6a09e667f3bcbp-1, 0x1.6a09e667f3bcep-1, -0x1.6a09e667f3bc5p-1,               \
      -0x1.6a09e667f3bc9p-1, 0x1.6a09e667f3bc4p-1},                                     \
     {0x1.1c73b39ae68c9p-1, -0x1.f6297cff75cbp-1, 0x1.8f8b83c69a60cp-3,                 \
      0x1.a9b66290ea1a5p-1, -0x1.a9b66290ea1a2p-1, -0x1.8f8b83c69a602p-3,               \
      0x1.f6297cff75cb2p-1, -0x1.1c73b39ae68c2p-1},                                     \
     {0x1.87de2a6aea964p-2, -0x1.d906bcf328d47p-1, 0x1.d906bcf328d44p-1,                \
      -0x1.87de2a6aea965p-2, -0x1.87de2a6aea971p-2, 0x1.d906bcf328d46p-1,               \
      -0x1.d906bcf328d43p-1, 0x1.87de2a6aea95fp-2},                                     \
     {0x1.8f8b83c69a60dp-3, -0x1.1c73b39ae68c8p-1, 0x1.a9b66290ea1a5p-1,                \
      -0x1.f6297cff75cb2p-1, 0x1.f6297cff75cbp-1, -0x1.a9b66290ea1a1p-1,                \
      0x1.1c73b39ae68c2p-1, -0x1.8f8b83c69a616p-3}}

/* src/dct.c:13 ALPHA(0) = 1/sqrt(2) as the reference's double */
#define JX_ALPHA0 0x1.6a09e667f3bccp-1

#endif
