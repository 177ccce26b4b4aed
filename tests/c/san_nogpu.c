/* san_nogpu.c -- TEST INFRASTRUCTURE for the sanitizer build (tests/c/sanitize.c): the host
 * layer's only call into the HIP runtime (csrc/jpgx_host.cpp), answered as on a machine
 * without a GPU.  Never linked into libjpgx.so. */
#include "jpgx.h"

int jpgx_blocks(const uint8_t *rgb, int width, int height, size_t pitch, const jpgx_params *p,
                int16_t *out, int device)
{
    (void)rgb; (void)width; (void)height; (void)pitch; (void)p; (void)out; (void)device;
    return JPGX_ENODEV;
}
