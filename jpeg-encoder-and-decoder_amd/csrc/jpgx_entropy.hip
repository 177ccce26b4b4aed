/*
 * jpgx_entropy.hip -- entropy-stage statistics on the device.
 *
 * What the reference's host runs on the hot path's output before it writes any bits:
 *   dpcm            src/dpcm.c:6-21        d_i = v_i - d_{i-1} over each channel's DCs, in place
 *   huffman_encode  src/huffman.c:23-44    frequency pass: per block calculate_freq_block_DC
 *                   (class of the dpcm'd DC, :182-185) and calculate_freq_block_AC (run/size
 *                   symbols, ZRL, EOB, :187-222, with the reference's `run | size`), into
 *                   lum_DC, lum_AC, chrom_DC (Cb and Cr), chrom_AC; freq[256] = 1 (:55).
 * (construct_huffman_table, which never terminates, is not part of this.)
 *
 * The recurrence is sequential; it is an alternating prefix sum:
 *     d_l = (-1)^l (P_l - c),  P_l = sum_{k<=l} (-1)^k v_k,  c = the DC carried in
 * so three launches per image, (A) over chunks of 512 blocks of one channel (4 waves, one
 * workgroup):
 *   (A) k_ent_ac: every block's AC symbols into count bins, the chunk's sum of (-1)^k v_k, and the
 *       DC words compacted (2 bytes per block) into the workspace.  A wave's 16 coalesced 1-KiB
 *       loads (128 blocks) pass through an LDS tile so that each lane walks two whole blocks in
 *       zig-zag order (round 6, below): a nonzero AC coefficient at position i after the previous
 *       nonzero p (the DC position 0 if none) is the reference's symbol ((i - p - 1) & 15) | class
 *       after (i - p - 1) >> 4 ZRLs; a block ends in EOB iff its coefficient 63 is zero
 *       (huffman.c:193-221).  The workgroup sums its count columns at its end into per-chunk
 *       counts (plain stores).
 *   (B) k_ent_dc: the sum of the channel's earlier chunk sums (at most a few hundred, read from
 *       L2), the in-chunk scan over the compacted DC words, d_l, and the DC classes per chunk.
 *   (C) k_ent_hist: one workgroup per count row sums it over the luma / chroma chunks and writes
 *       the histogram -- every entry, so no memset and no global atomics (a few thousand
 *       device-scope atomics on the same few words cost more than the whole coefficient read).
 * HBM traffic: the coefficients once (128 B per block) plus 2 + 2 + 4 bytes per block of DC.
 * A call takes a batch of frames (jpgx_entropy_stats_gpu_batch): the chunks of every frame in one
 * grid, each frame's recurrence starting from its own carry-in -- one frame per launch leaves the
 * chip mostly idle (49.8 MB of 4K coefficients is ~10 us of HBM time against ~3 launches).
 */
#include <hip/hip_runtime.h>
#include <stdint.h>


#include "jpgx_internal.h"

namespace {

constexpr int kChunk = 256;            /* threads per workgroup (4 waves)                           */
constexpr int kLoads = 16;             /* k_ent_ac: 8-block loads per wave, all issued first        */
constexpr int kAcW = 4;                /* k_ent_ac: waves per workgroup (8: slower, r06_entropy)  */
constexpr int kAcT = 64 * kAcW;
constexpr int kCB = 8 * kAcW * kLoads; /* blocks per chunk: kAcW waves x kLoads x 8 blocks     */
constexpr int kSyms = 32;       /* AC symbols (zeros | class) 1..31; 0 = no symbol    */
constexpr int kRows = 66;       /* per-chunk count rows: AC 0..31 (row 0: EOB), ZRL 32, DC class 33..65 */

__device__ __forceinline__ int dc_class(int v)   /* huffman.c:226-235 get_class */
{
    const unsigned a = (unsigned)(v < 0 ? -v : v);
    return a ? 32 - __builtin_clz(a) : 0;
}

struct Chunks {
    const int16_t *coef;        /* frame f: Y [nb_y][64] | Cb [nb_c][64] | Cr [nb_c][64] at f fstride */
    int32_t *dc;                /* frame f: [nb_y + 2 nb_c] at f (nb_y + 2 nb_c)                 */
    uint32_t *hist;             /* [nframes][4][257]                                             */
    long long *part;            /* [nchunks] chunk sums of (-1)^k v_k (k local to channel)        */
    uint32_t *cnt;              /* [kRows][nchunks] per-chunk counts                             */
    int16_t *dcv;               /* [nframes][nb_y + 2 nb_c] the DC words, compacted              */
    unsigned long long fstride; /* coefficient blocks from one frame to the next                 */
    unsigned nchunks, nchf;     /* chunks in all, per frame                                      */
    unsigned ndcg;              /* DC workgroups per frame (k_ent_dc)                            */
    bool vec;                   /* k_ent_dc's 16-byte DC loads / stores are aligned              */
    unsigned nbf;               /* nb_y + 2 nb_c                                                 */
    unsigned nb[3];             /* blocks per channel                                            */
    unsigned first[3];          /* first chunk of each channel within a frame                    */
    unsigned off[3];            /* first block of each channel within a frame                    */
    int carry[3];               /* DC carried in per channel (0 at the image start)              */
};

/* chunk -> frame f, channel ch, first block k0 of the chunk in the channel */
__device__ __forceinline__ void chunk_of(const Chunks &c, unsigned chunk, unsigned &f, int &ch, unsigned &k0)
{
    f = chunk / c.nchf;
    const unsigned l = chunk - f * c.nchf;
    ch = l >= c.first[2] ? 2 : (l >= c.first[1] ? 1 : 0);
    k0 = (l - c.first[ch]) * kCB;
}

/*
 * Round 6: one lane per block.  The wave's 16 loads stay the coalesced 1-KiB loads (lane l: 16 bytes
 * of block l >> 3); each half of them (64 blocks) goes through a per-wave LDS tile so that lane b
 * then holds all 64 coefficients of block b, and walks them in zig-zag order with the previous
 * nonzero position in a register -- no cross-lane max-scan.  A lane walks its two blocks (one per
 * half) side by side (two independent chains).  Per coefficient: its class (frexp of the float, 0
 * for 0), the run since the previous nonzero, and ONE LDS add into a count bin:
 *   nonzero:  bin ((run & 15) | class), the reference's symbol (huffman.c:199-218, `run | size`);
 *   zero:     bin 32 + (run & 15) -- a zero whose run is 15 mod 16 completes a group of 16 zeros, so
 *             bin 47 counts the ZRLs (huffman.c:199-204: (run >> 4) ZRLs before a symbol), except
 *             for the groups in the block's trailing zeros (no ZRL: EOB, :219-221), floor((63 - L)
 *             / 16) for the last nonzero position L, subtracted per block.
 * Count columns are per lane & 31 and shared by the workgroup's waves (an LDS add is atomic across
 * waves, and lanes l, l + 32 are serviced in different LDS cycles), so the counters take 6 KiB and
 * four workgroups fit a CU.  The round-5 form (8 lanes per block, an 8-lane max-scan through
 * ds_bpermute, 8 SGPR masks per load that the compiler spilled into VGPR lanes, per-thread columns
 * of 32 KiB; in the git history at 63924df) issued ~1.8x the VALU per coefficient and ran 111 us
 * per 8 x 4K batch against 78.5 (profiles/r06_entropy.txt).
 */
constexpr int kBins = 48;                        /* AC symbols 0..31, zero coefficients 32 + (run & 15) */
typedef uint32_t ent_u4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) ent_u4 ent_l4;
typedef __attribute__((address_space(3))) uint32_t ent_l32;

/* a coefficient load: nontemporal (global_load_dwordx4 ... nt) -- each byte is read once; 69.4 vs
 * 78.8 us per 8 x 4K batch with the default policy (profiles/r06_entropy.txt) */
__device__ __forceinline__ uint4 ent_ld(const uint4 *p)
{
    const ent_u4 x = __builtin_nontemporal_load((const ent_u4 *)p);
    return uint4{x.x, x.y, x.z, x.w};
}

/* the transposition tile: block b (0..63) in 128 bytes at 128 b, its 16-byte pieces XOR-swizzled by
 * (b >> 1) & 7 -- the piece writes (8 contiguous lanes = one block) and the per-lane block reads (a
 * ds_read_b128 16-lane group: 16 distinct (b & 1, (b >> 1) & 7)) hit distinct banks */
__device__ __forceinline__ unsigned ent_tile(unsigned b, unsigned piece)
{
    return 128u * b + 16u * (piece ^ ((b >> 1) & 7u));
}

/* the 8 loads qh (64 blocks) through the tile into u: lane b's block b */
__device__ __forceinline__ void ent_transpose(const uint4 (&qh)[8], uint8_t *tile, unsigned lane, uint32_t (&u)[32])
{
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");     /* earlier tile reads first */
#pragma unroll
    for (int r = 0; r < 8; r++) {
        const uint32_t x = qh[r].x, y = qh[r].y, zz = qh[r].z, ww = qh[r].w;
        *(ent_l4 *)(tile + ent_tile(8u * r + (lane >> 3), lane & 7u)) = ent_u4{x, y, zz, ww};
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");     /* other lanes' writes first */
#pragma unroll
    for (int r = 0; r < 8; r++) {
        const ent_u4 x = *(const ent_l4 *)(tile + ent_tile(lane, (unsigned)r));
        u[4 * r] = x.x, u[4 * r + 1] = x.y, u[4 * r + 2] = x.z, u[4 * r + 3] = x.w;
    }
}

/* coefficient k of a block: its count bin (above) and the previous-nonzero update */
__device__ __forceinline__ void ent_coef(const uint32_t (&u)[32], int k, uint32_t &prev, uint32_t colb)
{
    const uint32_t word = u[k >> 1];
    const int v = (k & 1) ? (int)word >> 16 : (int)(int16_t)(word & 0xffffu);
    /* class = frexp exponent of the exact float (0 for 0), huffman.c:226-235 */
    const uint32_t cls = (uint32_t)__builtin_amdgcn_frexp_expf((float)v);
    const uint32_t run = (uint32_t)(k - 1) - prev;
    const bool nz = cls != 0;
    const uint32_t bin = (run & 15u) | (nz ? cls : 32u);
    __hip_atomic_fetch_add((ent_l32 *)(uintptr_t)(colb + bin * 128u), 1u, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_WORKGROUP);
    prev = nz ? (uint32_t)k : prev;
}

/* a block's end: EOB, DC word and chunk sum (live blocks), the trailing-zero ZRL correction (every
 * block: a dead block reads as zeros and fed bin 47 too) */
__device__ __forceinline__ void ent_block_end(const uint32_t (&u)[32], uint32_t prev, unsigned blk, unsigned n,
                                              uint32_t &eob, uint32_t &zcor, long long &w, const Chunks &c,
                                              unsigned f, int ch, unsigned k0)
{
    zcor += (63u - prev) >> 4;
    if (blk < n) {
        eob += (u[31] >> 16) == 0 ? 1u : 0u;          /* huffman.c:219-221 */
        const int v0 = (int)(int16_t)(u[0] & 0xffffu);
        c.dcv[f * c.nbf + c.off[ch] + k0 + blk] = (int16_t)v0;
        w += ((k0 + blk) & 1u) ? -(long long)v0 : (long long)v0;
    }
}

__global__ __launch_bounds__(kAcT, 16 / kAcW) void k_ent_ac(const Chunks c)
{
    __shared__ uint32_t cnt[kBins][32];              /* [bin][lane & 31], shared by the 4 waves */
    __shared__ __attribute__((aligned(16))) uint8_t tile[kAcW][64 * 128];
    __shared__ long long wsum[kAcW];
    __shared__ uint32_t wez[kAcW][2];
    unsigned f, k0;
    int ch;
    chunk_of(c, blockIdx.x, f, ch, k0);
    const unsigned t = threadIdx.x, lane = t & 63u, wave = t >> 6;
    const unsigned n = min(c.nb[ch] - k0, (unsigned)kCB);
    const int16_t *z = c.coef + (f * c.fstride + c.off[ch] + k0) * 64;
    static_assert(kLoads == 16, "two halves of 64 blocks per wave");
    uint4 qa[8], qb[8];                               /* all 16 loads in flight at once */
#pragma unroll
    for (int it = 0; it < 8; it++) {
        const unsigned blk = 8u * kLoads * wave + 8u * (unsigned)it + (lane >> 3);
        qa[it] = ent_ld((const uint4 *)(z + (size_t)(blk < n ? blk : 0u) * 64 + 8u * (lane & 7u)));
    }
#pragma unroll
    for (int it = 0; it < 8; it++) {
        const unsigned blk = 8u * kLoads * wave + 64u + 8u * (unsigned)it + (lane >> 3);
        qb[it] = ent_ld((const uint4 *)(z + (size_t)(blk < n ? blk : 0u) * 64 + 8u * (lane & 7u)));
    }
    for (unsigned i = t; i < (unsigned)kBins * 32u; i += kAcT) (&cnt[0][0])[i] = 0;   /* under the loads */
    const unsigned ba = 8u * kLoads * wave + lane, bb = ba + 64u;      /* this lane's two blocks */
    uint32_t eob = 0, zcor = 0;
    long long w = 0;
    const uint32_t colb = (uint32_t)(uintptr_t)(ent_l32 *)&cnt[0][lane & 31u];
    uint32_t ua[32], ub[32];
    ent_transpose(qa, tile[wave], lane, ua);
    ent_transpose(qb, tile[wave], lane, ub);
    if (n < (unsigned)kCB) {                          /* the channel's last chunk: dead blocks read as zeros */
        const uint32_t la = ba < n ? ~0u : 0u, lb = bb < n ? ~0u : 0u;
#pragma unroll
        for (int i = 0; i < 32; i++) ua[i] &= la, ub[i] &= lb;
    }
    __syncthreads();                                  /* the counters are zeroed */
    uint32_t pa = 0, pb = 0;                          /* previous nonzero: the DC position */
#pragma unroll
    for (int k = 1; k < 64; k++) {
        ent_coef(ua, k, pa, colb);
        ent_coef(ub, k, pb, colb);
    }
    ent_block_end(ua, pa, ba, n, eob, zcor, w, c, f, ch, k0);
    ent_block_end(ub, pb, bb, n, eob, zcor, w, c, f, ch, k0);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        w += __shfl_xor(w, o, 64);
        eob += __shfl_xor(eob, o, 64);
        zcor += __shfl_xor(zcor, o, 64);
    }
    if (lane == 0) {
        wsum[wave] = w;
        wez[wave][0] = eob;
        wez[wave][1] = zcor;
    }
    __syncthreads();
    {   /* the count rows: symbol r = t / 8 (r 1..31; r 0 stands for bin 47, the ZRL row), eight
         * threads per row summing four columns each (rotated by the row: distinct banks), then a
         * three-step shuffle; row 0 is EOB (wez), ZRL = bin 47 minus the trailing-zero groups */
        static_assert(kAcT == 8 * kSyms, "eight threads per count row");
        const unsigned r = t >> 3, e = t & 7u, bin = r ? r : 47u;
        uint32_t sum = 0;
#pragma unroll
        for (unsigned j = 0; j < 4; j++) sum += cnt[bin][(4u * e + j + r) & 31u];
        sum += __shfl_xor(sum, 1, 8);
        sum += __shfl_xor(sum, 2, 8);
        sum += __shfl_xor(sum, 4, 8);
        if (e == 0) {
            if (r == 0) {
                uint32_t eobs = 0, zc = 0;
#pragma unroll
                for (int i = 0; i < kAcW; i++) eobs += wez[i][0], zc += wez[i][1];
                c.cnt[blockIdx.x] = eobs;                                        /* row 0: EOB */
                c.cnt[(size_t)kSyms * c.nchunks + blockIdx.x] = sum - zc;         /* row 32: ZRL */
            } else {
                c.cnt[(size_t)r * c.nchunks + blockIdx.x] = sum;
            }
        } else if (t == 1) {
            long long ws = 0;
#pragma unroll
            for (int i = 0; i < kAcW; i++) ws += wsum[i];
            c.part[blockIdx.x] = ws;
        }
    }
}

/* DC pass over kDcChunks consecutive chunks of one channel (8 blocks per thread): the channel's
 * earlier chunk sums, the scan, d_l and the classes; its class counts go to column blockIdx.x of
 * the DC count rows (frame f's DC workgroups are f dc_groups() .. + dc_groups() - 1, luma first). */
constexpr int kDcChunks = 2048 / kCB;   /* 2,048 blocks per DC workgroup */
static_assert(kCB <= 2048 && 2048 % kCB == 0, "DC workgroups tile whole chunks");
__global__ __launch_bounds__(kChunk) void k_ent_dc(const Chunks c)
{
    __shared__ uint32_t cnt[16][kChunk];              /* [class / 2][thread], 16-bit halves: classes 0..31 */
    __shared__ uint32_t red[kChunk / 16][32];
    __shared__ uint32_t top[kChunk / 64];             /* class 32 (d = INT_MIN) per wave */
    __shared__ int wtot[kChunk / 64];
    __shared__ long long wbase[kChunk / 64];
    /* workgroup g: chunks kDcChunks g' .. of channel ch of frame f (g' counts per channel) */
    const unsigned per[3] = {(c.first[1] - c.first[0] + kDcChunks - 1) / kDcChunks,
                             (c.first[2] - c.first[1] + kDcChunks - 1) / kDcChunks,
                             (c.nchf - c.first[2] + kDcChunks - 1) / kDcChunks};
    const unsigned pf = per[0] + per[1] + per[2];
    const unsigned f = blockIdx.x / pf;
    unsigned l = blockIdx.x - f * pf;
    const int ch = l >= per[0] + per[1] ? 2 : (l >= per[0] ? 1 : 0);
    l -= ch == 0 ? 0u : (ch == 1 ? per[0] : per[0] + per[1]);
    const unsigned chunk0 = f * c.nchf + c.first[ch] + kDcChunks * l;      /* first chunk */
    const unsigned b0 = kDcChunks * kCB * l;                              /* first block */
    const unsigned t = threadIdx.x, lane = t & 63u, wave = t >> 6;
#pragma unroll
    for (int b = 0; b < 16; b++) cnt[b][t] = 0;      /* own column: no barrier before use */
    const unsigned k = b0 + 8u * t;                   /* this thread's 8 blocks */
    const size_t at = (size_t)f * c.nbf + c.off[ch] + k;
    const bool vec = c.vec && k + 8u <= c.nb[ch];    /* 16-byte loads / stores */
    int v[8];
    if (vec) {
        const uint4 q = *(const uint4 *)(c.dcv + at);
        const uint32_t u[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
        for (int j = 0; j < 4; j++) v[2 * j] = (int)(int16_t)(u[j] & 0xffffu), v[2 * j + 1] = (int)u[j] >> 16;
    } else {
#pragma unroll
        for (int i = 0; i < 8; i++) v[i] = k + i < c.nb[ch] ? (int)c.dcv[at + i] : 0;
    }
    long long e = 0;                                  /* the channel's earlier chunks */
    {
        const unsigned i0 = f * c.nchf + c.first[ch] + t;
        long long pp[4];                              /* up to 1024 earlier chunks, loads together */
#pragma unroll
        for (int r = 0; r < 4; r++) pp[r] = i0 + r * kChunk < chunk0 ? c.part[i0 + r * kChunk] : 0;
        for (unsigned i = i0 + 4 * kChunk; i < chunk0; i += kChunk) e += c.part[i];
#pragma unroll
        for (int r = 0; r < 4; r++) e += pp[r];
    }
    int run = 0;                                      /* k is even: (-1)^(k+i) = (-1)^i */
#pragma unroll
    for (int i = 0; i < 8; i++) run += (i & 1) ? -v[i] : v[i];
    int p32 = run;                                    /* inclusive scan of the thread totals: */
#pragma unroll                                        /* |.| <= 2048 * 32768, 32-bit          */
    for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(p32, o, 64);
        if (lane >= (unsigned)o) p32 += y;
        e += __shfl_xor(e, o, 64);
    }
    if (lane == 63) wtot[wave] = p32;
    if (lane == 0) wbase[wave] = e;
    __syncthreads();
    long long p = p32 - run;                          /* exclusive */
#pragma unroll
    for (unsigned wv = 0; wv < kChunk / 64; wv++) {
        p += wbase[wv];
        if (wv < wave) p += wtot[wv];
    }
    uint32_t n32 = 0;
    int dv[8];
#pragma unroll
    for (int i = 0; i < 8; i++) {
        p += (i & 1) ? -v[i] : v[i];
        const long long d = (i & 1) ? -(p - c.carry[ch]) : (p - c.carry[ch]);
        dv[i] = (int)d;                               /* the reference's int */
        if (k + i < c.nb[ch]) {
            const int cl = dc_class(dv[i]);
            if (cl < 32) atomicAdd(&cnt[cl >> 1][t], 1u << ((cl & 1) << 4));
            else n32++;
        }
    }
    if (vec) {
        *(int4 *)(c.dc + at) = make_int4(dv[0], dv[1], dv[2], dv[3]);
        *(int4 *)(c.dc + at + 4) = make_int4(dv[4], dv[5], dv[6], dv[7]);
    } else {
#pragma unroll
        for (int i = 0; i < 8; i++)
            if (k + i < c.nb[ch]) c.dc[at + i] = dv[i];
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) n32 += __shfl_xor(n32, o, 64);
    if (lane == 0) top[wave] = n32;
    __syncthreads();
    {   /* column sums: word b (classes 2b, 2b + 1) of 16 columns; 64 distinct banks per wave */
        const unsigned b = t & 15u, r = t >> 4;
        uint32_t lo = 0, hi = 0;
#pragma unroll
        for (unsigned j = 0; j < 16; j++) {
            const uint32_t x = cnt[b][16u * r + ((j + b) & 15u)];
            lo += x & 0xffffu, hi += x >> 16;
        }
        red[r][2 * b] = lo;
        red[r][2 * b + 1] = hi;
    }
    __syncthreads();
    if (t <= 32) {
        uint32_t tot = 0;
        if (t < 32) {
#pragma unroll
            for (int r = 0; r < kChunk / 16; r++) tot += red[r][t];
        } else {
#pragma unroll
            for (int r = 0; r < kChunk / 64; r++) tot += top[r];
        }
        c.cnt[(size_t)(kSyms + 1 + t) * c.nchunks + blockIdx.x] = tot;
    }
}

/* the DC workgroups of one frame */
unsigned dc_groups(const Chunks &c)
{
    return (c.first[1] - c.first[0] + kDcChunks - 1) / kDcChunks + (c.first[2] - c.first[1] + kDcChunks - 1) / kDcChunks +
           (c.nchf - c.first[2] + kDcChunks - 1) / kDcChunks;
}

/* the histograms from the per-chunk count rows: workgroup (r, f) sums row r over frame f's luma
 * chunks and over its chroma chunks; workgroup (0, f) also writes every entry no row maps to (0,
 * and the reserved freq[256] = 1 of initialize_huffman, huffman.c:55) */
__global__ __launch_bounds__(kChunk) void k_ent_hist(const Chunks c)
{
    __shared__ uint32_t part[2][kChunk / 64];
    const unsigned r = blockIdx.x, f = blockIdx.y, t = threadIdx.x, lane = t & 63u, wave = t >> 6;
    const bool dcrow = r > (unsigned)kSyms;
    const unsigned ny = dcrow ? (c.first[1] + kDcChunks - 1) / kDcChunks : c.first[1];   /* luma columns */
    const unsigned ncol = dcrow ? c.ndcg : c.nchf;                                  /* columns per frame */
    const uint32_t *row = c.cnt + (size_t)r * c.nchunks + (size_t)f * ncol;
    uint32_t *hist = c.hist + (size_t)f * 4 * 257;
    uint32_t sy = 0, sc = 0;
    for (unsigned i0 = t; i0 < ncol; i0 += 8 * kChunk) {     /* eight loads in flight */
        uint32_t x[8];
#pragma unroll
        for (int r = 0; r < 8; r++) x[r] = i0 + r * kChunk < ncol ? row[i0 + r * kChunk] : 0u;
#pragma unroll
        for (int r = 0; r < 8; r++) (i0 + r * kChunk < ny ? sy : sc) += x[r];
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        sy += __shfl_xor(sy, o, 64);
        sc += __shfl_xor(sc, o, 64);
    }
    if (lane == 0) part[0][wave] = sy, part[1][wave] = sc;
    __syncthreads();
    if (t == 0) {
        uint32_t y = 0, ch = 0;
#pragma unroll
        for (int w = 0; w < kChunk / 64; w++) y += part[0][w], ch += part[1][w];
        if (r <= (unsigned)kSyms) {                   /* AC: symbol r, or ZRL */
            const unsigned e = r < (unsigned)kSyms ? r : 0xF0u;
            hist[1 * 257 + e] = y;
            hist[3 * 257 + e] = ch;
        } else {                                      /* DC class r - 33 */
            hist[0 * 257 + r - kSyms - 1] = y;
            hist[2 * 257 + r - kSyms - 1] = ch;
        }
    }
    if (r == 0) {
        for (unsigned e = t; e < 4u * 257u; e += kChunk) {
            const unsigned k = e / 257u, i = e - 257u * k;
            const bool ac = k & 1u;
            const bool mapped = ac ? (i < (unsigned)kSyms || i == 0xF0u) : i <= 32u;
            if (!mapped) hist[e] = i == 256u ? 1u : 0u;
        }
    }
}

int hip_rc2(hipError_t e) { return e == hipSuccess ? JPGX_OK : JPGX_EHIP; }

size_t nchunks_of(size_t nb_y, size_t nb_c)
{
    return (nb_y + kCB - 1) / kCB + 2 * ((nb_c + kCB - 1) / kCB);
}

size_t round8(size_t x) { return (x + 7) / 8 * 8; }

}  // namespace

extern "C" {

size_t jpgx_entropy_workspace_size_batch(size_t nb_y, size_t nb_c, size_t nframes)
{
    const size_t nch = nchunks_of(nb_y, nb_c) * nframes;
    return nch * sizeof(long long) + round8(kRows * nch * sizeof(uint32_t)) +
           round8(nframes * (nb_y + 2 * nb_c) * sizeof(int16_t));
}

size_t jpgx_entropy_workspace_size(size_t nb_y, size_t nb_c)
{
    return jpgx_entropy_workspace_size_batch(nb_y, nb_c, 1);
}

int jpgx_entropy_stats_gpu_batch(const int16_t *d_coef, size_t coef_frame_stride, size_t nframes, size_t nb_y,
                                 size_t nb_c, const int32_t *carry, int32_t *d_dc, uint32_t *d_hist,
                                 void *d_workspace, size_t workspace_bytes, void *stream)
{
    const size_t nbf = nb_y + 2 * nb_c;
    if (!d_coef || !d_dc || !d_hist || ((uintptr_t)d_coef & 15) || nb_y == 0 || nframes == 0 ||
        coef_frame_stride < nbf * 64 || coef_frame_stride % 64 || nbf >= (1ull << 31) ||
        nframes * nbf >= (1ull << 31) || nframes > 65535 || (carry && nframes != 1))
        return JPGX_EARG;
    const size_t nchf = nchunks_of(nb_y, nb_c), nch = nchf * nframes;
    if (nch >= (1ull << 31))
        return JPGX_EARG;
    if (!d_workspace || workspace_bytes < jpgx_entropy_workspace_size_batch(nb_y, nb_c, nframes) ||
        ((uintptr_t)d_workspace & 7))
        return JPGX_EWORKSPACE;
    Chunks c;
    c.coef = d_coef;
    c.dc = d_dc;
    c.hist = d_hist;
    c.part = (long long *)d_workspace;
    c.cnt = (uint32_t *)((char *)d_workspace + nch * sizeof(long long));
    c.dcv = (int16_t *)((char *)c.cnt + round8(kRows * nch * sizeof(uint32_t)));
    c.fstride = coef_frame_stride / 64;
    c.nchunks = (unsigned)nch;
    c.nchf = (unsigned)nchf;
    c.nbf = (unsigned)nbf;
    c.nb[0] = (unsigned)nb_y;
    c.nb[1] = c.nb[2] = (unsigned)nb_c;
    c.first[0] = 0;
    c.first[1] = (unsigned)((nb_y + kCB - 1) / kCB);
    c.first[2] = c.first[1] + (unsigned)((nb_c + kCB - 1) / kCB);
    c.off[0] = 0;
    c.off[1] = (unsigned)nb_y;
    c.off[2] = (unsigned)(nb_y + nb_c);
    for (int k = 0; k < 3; k++) c.carry[k] = carry ? carry[k] : 0;
    hipStream_t s = (hipStream_t)stream;
    hipLaunchKernelGGL(k_ent_ac, dim3((unsigned)nch), dim3(kAcT), 0, s, c);
    c.ndcg = dc_groups(c);
    c.vec = nbf % 8 == 0 && nb_y % 8 == 0 && nb_c % 8 == 0 && ((uintptr_t)c.dcv & 15) == 0 &&
            ((uintptr_t)d_dc & 15) == 0;
    hipLaunchKernelGGL(k_ent_dc, dim3(c.ndcg * (unsigned)nframes), dim3(kChunk), 0, s, c);
    hipLaunchKernelGGL(k_ent_hist, dim3(kRows, (unsigned)nframes), dim3(kChunk), 0, s, c);
    return hip_rc2(hipGetLastError());
}

int jpgx_entropy_stats_gpu(const int16_t *d_coef, size_t nb_y, size_t nb_c, const int32_t *carry,
                           int32_t *d_dc, uint32_t *d_hist, void *d_workspace,
                           size_t workspace_bytes, void *stream)
{
    return jpgx_entropy_stats_gpu_batch(d_coef, (nb_y + 2 * nb_c) * 64, 1, nb_y, nb_c, carry, d_dc, d_hist,
                                        d_workspace, workspace_bytes, stream);
}

}  /* extern "C" */
