/*
 * jpgx_host.cpp -- host-buffer runtime of libjpgx (include/jpgx.h "host-buffer path"): images
 * in host memory, split into block-row shards, each shard on a GPU (several shards may share
 * one), streamed through the device in chunks of block rows with the PCIe copies of
 * neighbouring chunks overlapped in both directions.
 *
 * The reference has no counterpart (it is single-threaded CPU code, src/jpg_encode.c:32-44):
 * this is the SURVEY.md 8(e) split -- independent block-row stripes, the one pixel row above a
 * stripe as halo (src/preprocess.c:199-211's x0 = -8 read), no data exchange between shards --
 * applied to host buffers.
 *
 * Per shard the context keeps, across calls: two HIP streams, two device input/output chunk
 * buffers, two pinned (hipHostMalloc) staging buffers per direction and two events.  Chunk i
 * uses slot i % 2.  Pageable caller memory is staged: the host thread packs chunk i+1 into
 * pinned memory while chunk i's H2D / kernel / D2H run, and unpacks chunk i-1's output.  When
 * the caller's buffers are already page-locked (hipHostMalloc'd or jpgx_host_register'ed) the
 * chunks are copied directly, with no host copy at all.
 */
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <mutex>
#include <thread>
#include <vector>

#include "jpgx.h"

namespace {

int hip_rc(hipError_t e) { return e == hipSuccess ? JPGX_OK : JPGX_EHIP; }

constexpr size_t kChunkInBytes = 4u << 20;   /* auto chunk: about 4 MB of RGB per chunk */

struct Shard {
    int dev = 0;
    hipStream_t st[2] = {nullptr, nullptr};
    hipEvent_t ev[2] = {nullptr, nullptr};
    uint8_t *d_in[2] = {nullptr, nullptr};
    int16_t *d_out[2] = {nullptr, nullptr};
    uint8_t *h_in[2] = {nullptr, nullptr};
    int16_t *h_out[2] = {nullptr, nullptr};
    size_t cap_in = 0, cap_out = 0;          /* bytes per slot */
    bool ready = false;
};

/* one chunk: block rows [c0, c1) of the image */
struct Chunk {
    int c0, c1, halo;
    size_t rows_px;                           /* pixel rows copied, halo included */
    size_t nb, nbc;                           /* Y and chroma blocks of the chunk */
    size_t y_dst, c_dst;                      /* block offsets of its Y / chroma in the image */
};

/* page-locked (pinned or registered) host range? */
bool host_locked(const void *p, size_t bytes)
{
    if (!p || !bytes) return false;
    const void *ends[2] = {p, (const uint8_t *)p + bytes - 1};
    for (const void *q : ends) {
        hipPointerAttribute_t a;
        if (hipPointerGetAttributes(&a, q) != hipSuccess) {
            (void)hipGetLastError();
            return false;
        }
        if (a.type != hipMemoryTypeHost) return false;
    }
    return true;
}

}  // namespace

struct jpgx_host_ctx {
    int nshards = 0;
    int chunk_rows = 0;                       /* 0: auto */
    std::vector<Shard> sh;
};

namespace {

void shard_free(Shard &s)
{
    if (!s.ready) return;
    (void)hipSetDevice(s.dev);
    for (int b = 0; b < 2; b++) {
        if (s.st[b]) (void)hipStreamDestroy(s.st[b]);
        if (s.ev[b]) (void)hipEventDestroy(s.ev[b]);
        if (s.d_in[b]) (void)hipFree(s.d_in[b]);
        if (s.d_out[b]) (void)hipFree(s.d_out[b]);
        if (s.h_in[b]) (void)hipHostFree(s.h_in[b]);
        if (s.h_out[b]) (void)hipHostFree(s.h_out[b]);
        s.st[b] = nullptr;
        s.ev[b] = nullptr;
        s.d_in[b] = nullptr;
        s.d_out[b] = nullptr;
        s.h_in[b] = nullptr;
        s.h_out[b] = nullptr;
    }
    s.cap_in = s.cap_out = 0;
    s.ready = false;
}

/* streams/events once; buffers grown to the chunk size (device + pinned staging) */
int shard_reserve(Shard &s, size_t in_bytes, size_t out_bytes, bool staged)
{
    int rc = hip_rc(hipSetDevice(s.dev));
    if (rc) return rc;
    if (!s.ready) {
        for (int b = 0; b < 2 && !rc; b++) {
            rc = hip_rc(hipStreamCreateWithFlags(&s.st[b], hipStreamNonBlocking));
            if (!rc) rc = hip_rc(hipEventCreateWithFlags(&s.ev[b], hipEventDisableTiming));
        }
        s.ready = true;                        /* partial creation is freed by shard_free */
        if (rc) return rc;
    }
    if (in_bytes > s.cap_in || out_bytes > s.cap_out) {
        for (int b = 0; b < 2; b++) {
            (void)hipFree(s.d_in[b]);
            (void)hipFree(s.d_out[b]);
            (void)hipHostFree(s.h_in[b]);
            (void)hipHostFree(s.h_out[b]);
            s.d_in[b] = nullptr;
            s.d_out[b] = nullptr;
            s.h_in[b] = nullptr;
            s.h_out[b] = nullptr;
        }
        s.cap_in = s.cap_out = 0;
        for (int b = 0; b < 2; b++) {
            if (hipMalloc(&s.d_in[b], in_bytes) != hipSuccess ||
                hipMalloc(&s.d_out[b], out_bytes) != hipSuccess)
                return JPGX_EHIP;
        }
        s.cap_in = in_bytes;
        s.cap_out = out_bytes;
    }
    if (staged && !(s.h_in[0] && s.h_in[1] && s.h_out[0] && s.h_out[1])) {
        bool ok = true;
        for (int b = 0; b < 2 && ok; b++) {
            if (!s.h_in[b] && hipHostMalloc(&s.h_in[b], s.cap_in, hipHostMallocDefault) != hipSuccess) {
                s.h_in[b] = nullptr;
                ok = false;
            }
            if (ok && !s.h_out[b] && hipHostMalloc(&s.h_out[b], s.cap_out, hipHostMallocDefault) != hipSuccess) {
                s.h_out[b] = nullptr;
                ok = false;
            }
        }
        if (!ok) {
            /* never leave a partial set behind: the next call re-allocates all four */
            for (int b = 0; b < 2; b++) {
                (void)hipHostFree(s.h_in[b]);
                (void)hipHostFree(s.h_out[b]);
                s.h_in[b] = nullptr;
                s.h_out[b] = nullptr;
            }
            return JPGX_EHIP;
        }
    }
    return JPGX_OK;
}

struct Image {
    const uint8_t *rgb;
    int width, height;
    size_t pitch;
    const jpgx_params *p;
    int16_t *out;
    size_t nb, nbc;                           /* whole-image blocks per Y / chroma channel */
    bool direct;                              /* caller buffers page-locked */
};

Chunk make_chunk(const Image &im, int c0, int c1)
{
    Chunk c;
    c.c0 = c0;
    c.c1 = c1;
    c.halo = c0 > 0 ? 1 : 0;
    c.rows_px = (size_t)(c1 - c0) * 8 + c.halo;
    c.nb = (size_t)(c1 - c0) * (im.width / 8);
    c.nbc = jpgx_chroma_blocks(im.width, c0, c1, im.p->sample_ratio, im.p->flags);
    c.y_dst = (size_t)c0 * (im.width / 8);
    c.c_dst = jpgx_chroma_blocks(im.width, 0, c0, im.p->sample_ratio, im.p->flags);
    return c;
}

/* the chunk's output [Y nb | Cb nbc | Cr nbc][64], from `src` (host), to the image planes */
void scatter_out(const Image &im, const Chunk &c, const int16_t *src)
{
    memcpy(im.out + c.y_dst * 64, src, c.nb * 64 * sizeof(int16_t));
    for (int ch = 1; ch < 3; ch++)
        memcpy(im.out + (im.nb + (size_t)(ch - 1) * im.nbc + c.c_dst) * 64,
               src + (c.nb + (size_t)(ch - 1) * c.nbc) * 64, c.nbc * 64 * sizeof(int16_t));
}

/* H2D, kernel, D2H of chunk c in slot b (all async on the slot's stream) */
int enqueue_chunk(Shard &s, const Image &im, const Chunk &c, int b, size_t dpitch)
{
    const size_t row_bytes = (size_t)im.width * 3;
    const uint8_t *src = im.rgb + ((size_t)c.c0 * 8 - c.halo) * im.pitch;
    int rc = im.direct
                 ? hip_rc(hipMemcpy2DAsync(s.d_in[b], dpitch, src, im.pitch, row_bytes, c.rows_px,
                                           hipMemcpyHostToDevice, s.st[b]))
                 : hip_rc(hipMemcpyAsync(s.d_in[b], s.h_in[b], dpitch * c.rows_px,
                                         hipMemcpyHostToDevice, s.st[b]));
    if (rc) return rc;
    jpgx_frames fr;
    memset(&fr, 0, sizeof fr);
    fr.width = im.width;
    fr.height = im.height;
    fr.row_begin = c.c0;
    fr.row_end = c.c1;
    fr.nframes = 1;
    fr.in_pitch = dpitch;
    fr.in_frame_stride = dpitch * c.rows_px;
    fr.out_frame_stride = (c.nb + 2 * c.nbc) * 64;
    rc = jpgx_blocks_gpu(&fr, im.p, s.d_in[b] + c.halo * dpitch, s.d_out[b], nullptr, 0, s.st[b]);
    if (rc) return rc;
    if (im.direct) {
        rc = hip_rc(hipMemcpyAsync(im.out + c.y_dst * 64, s.d_out[b], c.nb * 64 * sizeof(int16_t),
                                   hipMemcpyDeviceToHost, s.st[b]));
        for (int ch = 1; ch < 3 && !rc; ch++)
            rc = hip_rc(hipMemcpyAsync(im.out + (im.nb + (size_t)(ch - 1) * im.nbc + c.c_dst) * 64,
                                       s.d_out[b] + (c.nb + (size_t)(ch - 1) * c.nbc) * 64,
                                       c.nbc * 64 * sizeof(int16_t), hipMemcpyDeviceToHost,
                                       s.st[b]));
    } else {
        rc = hip_rc(hipMemcpyAsync(s.h_out[b], s.d_out[b], (c.nb + 2 * c.nbc) * 64 * sizeof(int16_t),
                                   hipMemcpyDeviceToHost, s.st[b]));
    }
    if (rc) return rc;
    return hip_rc(hipEventRecord(s.ev[b], s.st[b]));
}

/* shard k's block rows [r0, r1), chunk by chunk, two slots in flight */
int run_shard(Shard &s, const Image &im, int r0, int r1, int chunk_rows, int unit)
{
    if (r0 == r1) return JPGX_OK;
    const size_t row_bytes = (size_t)im.width * 3;
    const size_t dpitch = (row_bytes + 7) & ~(size_t)7;
    int cr = chunk_rows > 0 ? chunk_rows : (int)std::max<size_t>(1, kChunkInBytes / (8 * dpitch));
    cr = std::max(unit, cr / unit * unit);
    cr = std::min(cr, r1 - r0);
    const size_t in_bytes = ((size_t)cr * 8 + 1) * dpitch;
    const size_t out_bytes = (size_t)cr * (im.width / 8) * 3 * 64 * sizeof(int16_t);
    int rc = shard_reserve(s, in_bytes, out_bytes, !im.direct);
    if (rc) return rc;
    std::vector<Chunk> chunks;
    for (int c0 = r0; c0 < r1; c0 += cr) chunks.push_back(make_chunk(im, c0, std::min(r1, c0 + cr)));
    const size_t n = chunks.size();
    for (size_t i = 0; i < n + 2 && !rc; i++) {
        const int b = (int)(i & 1);
        if (i >= 2) {                          /* chunk i-2 done: its slot is free */
            rc = hip_rc(hipEventSynchronize(s.ev[b]));
            if (rc) break;
            if (!im.direct) scatter_out(im, chunks[i - 2], s.h_out[b]);
        }
        if (i >= n) continue;
        const Chunk &c = chunks[i];
        if (!im.direct) {
            const uint8_t *src = im.rgb + ((size_t)c.c0 * 8 - c.halo) * im.pitch;
            for (size_t y = 0; y < c.rows_px; y++)
                memcpy(s.h_in[b] + y * dpitch, src + y * im.pitch, row_bytes);
        }
        rc = enqueue_chunk(s, im, c, b, dpitch);
    }
    if (rc) {                                  /* drain before the buffers can be reused */
        (void)hipStreamSynchronize(s.st[0]);
        (void)hipStreamSynchronize(s.st[1]);
    }
    return rc;
}

/* process-wide pool behind jpgx_blocks / jpgx_blocks_multi: contexts are reused across calls
 * (taken out of the pool for the duration of a call, so concurrent calls never share one) */
std::mutex g_pool_mu;
std::vector<jpgx_host_ctx *> g_pool;

jpgx_host_ctx *pool_take(int nshards, const int *devices)
{
    {
        std::lock_guard<std::mutex> lk(g_pool_mu);
        for (size_t i = 0; i < g_pool.size(); i++) {
            jpgx_host_ctx *c = g_pool[i];
            bool same = c->nshards == nshards && c->chunk_rows == 0;
            for (int k = 0; same && k < nshards; k++) same = c->sh[k].dev == devices[k];
            if (same) {
                g_pool.erase(g_pool.begin() + i);
                return c;
            }
        }
    }
    jpgx_host_ctx *c = nullptr;
    return jpgx_host_create(&c, nshards, devices, 0) == JPGX_OK ? c : nullptr;
}

void pool_give(jpgx_host_ctx *c)
{
    std::lock_guard<std::mutex> lk(g_pool_mu);
    g_pool.push_back(c);
}

}  // namespace

extern "C" {

int jpgx_host_create(jpgx_host_ctx **ctx, int nshards, const int *devices, int chunk_rows)
{
    if (!ctx || nshards < 1 || chunk_rows < 0) return JPGX_EARG;
    *ctx = nullptr;
    const int ndev = jpgx_device_count();
    if (ndev < 1) return JPGX_ENODEV;
    for (int k = 0; devices && k < nshards; k++)
        if (devices[k] < 0 || devices[k] >= ndev) return JPGX_ENODEV;
    jpgx_host_ctx *c = new (std::nothrow) jpgx_host_ctx;
    if (!c) return JPGX_ENOMEM;
    c->nshards = nshards;
    c->chunk_rows = chunk_rows;
    c->sh.resize(nshards);
    for (int k = 0; k < nshards; k++) c->sh[k].dev = devices ? devices[k] : k % ndev;
    *ctx = c;
    return JPGX_OK;
}

void jpgx_host_destroy(jpgx_host_ctx *ctx)
{
    if (!ctx) return;
    for (auto &s : ctx->sh) shard_free(s);
    delete ctx;
}

int jpgx_host_blocks(jpgx_host_ctx *ctx, const uint8_t *rgb, int width, int height, size_t pitch,
                     const jpgx_params *p, int16_t *out)
{
    if (!ctx || !rgb || !out || !p) return JPGX_EARG;
    int rc = jpgx_validate(width, height, p);
    if (rc) return rc;
    if (pitch < (size_t)width * 3) return JPGX_EARG;
    const bool sub = (p->flags & JPGX_FLAG_SUBSAMPLE) != 0;
    if (sub && p->sample_ratio == 0) return JPGX_ESAMPLE;
    Image im;
    im.rgb = rgb;
    im.width = width;
    im.height = height;
    im.pitch = pitch;
    im.p = p;
    im.out = out;
    im.nb = (size_t)(height / 8) * (width / 8);
    im.nbc = jpgx_chroma_blocks(width, 0, height / 8, p->sample_ratio, p->flags);
    im.direct = host_locked(rgb, pitch * (size_t)(height - 1) + (size_t)width * 3) &&
                host_locked(out, (im.nb + 2 * im.nbc) * 64 * sizeof(int16_t));
    /* true 4:2:0 shards and chunks split MCU rows (pairs of block rows) */
    const int unit = sub && p->sample_ratio == 2 ? 2 : 1;
    const int n = ctx->nshards;
    int caller_dev = 0;
    if (hipGetDevice(&caller_dev) != hipSuccess) return JPGX_ENODEV;
    std::vector<int> rcs(n, JPGX_OK);
    const auto work = [&](int k) {
        int r0, r1;
        jpgx_stripe(height / 8 / unit, n, k, &r0, &r1);
        rcs[k] = run_shard(ctx->sh[k], im, r0 * unit, r1 * unit, ctx->chunk_rows, unit);
    };
    if (n == 1) {
        work(0);
        (void)hipSetDevice(caller_dev);        /* the caller's current device is left as found */
    } else {
        std::vector<std::thread> th;
        th.reserve(n);
        for (int k = 0; k < n; k++) th.emplace_back(work, k);
        for (auto &t : th) t.join();
    }
    for (int k = 0; k < n; k++)
        if (rcs[k]) return rcs[k];
    return JPGX_OK;
}

int jpgx_host_register(void *ptr, size_t bytes)
{
    if (!ptr || !bytes) return JPGX_EARG;
    if (jpgx_device_count() < 1) return JPGX_ENODEV;
    return hip_rc(hipHostRegister(ptr, bytes, hipHostRegisterPortable));
}

int jpgx_host_unregister(void *ptr)
{
    if (!ptr) return JPGX_EARG;
    return hip_rc(hipHostUnregister(ptr));
}

void jpgx_host_release(void)
{
    std::vector<jpgx_host_ctx *> all;
    {
        std::lock_guard<std::mutex> lk(g_pool_mu);
        all.swap(g_pool);
    }
    for (auto *c : all) jpgx_host_destroy(c);
}

int jpgx_blocks(const uint8_t *rgb, int width, int height, size_t pitch, const jpgx_params *p,
                int16_t *out, int device)
{
    if (!rgb || !out || !p) return JPGX_EARG;
    int rc = jpgx_validate(width, height, p);
    if (rc) return rc;
    if (device < 0 || device >= jpgx_device_count()) return JPGX_ENODEV;
    jpgx_host_ctx *c = pool_take(1, &device);
    if (!c) return JPGX_ENOMEM;
    rc = jpgx_host_blocks(c, rgb, width, height, pitch, p, out);
    pool_give(c);
    return rc;
}

int jpgx_blocks_multi(const uint8_t *rgb, int width, int height, size_t pitch,
                      const jpgx_params *p, int16_t *out, int ngpus)
{
    if (!rgb || !out || !p || ngpus < 1) return JPGX_EARG;
    int rc = jpgx_validate(width, height, p);
    if (rc) return rc;
    if (ngpus > jpgx_device_count()) return JPGX_ENODEV;
    std::vector<int> devs(ngpus);
    for (int k = 0; k < ngpus; k++) devs[k] = k;
    jpgx_host_ctx *c = pool_take(ngpus, devs.data());
    if (!c) return JPGX_ENOMEM;
    rc = jpgx_host_blocks(c, rgb, width, height, pitch, p, out);
    pool_give(c);
    return rc;
}

}  /* extern "C" */
