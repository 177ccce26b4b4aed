// membench3.hip -- the memory skeleton of k_mx with synthetic compute (not product code).
// 8 x 4K frames, fresh input (two input sets alternating launch by launch), 9 B/px.
// Per wave-step (8 blocks): 2 LDS-DMA pieces of the step's 8 pixel rows x 192 B issued DIST
// steps ahead into a ring, one constant vmcnt wait, NV synthetic VALU instructions (v_pk_fma
// chains), NM MFMAs, NL ds_write_b16 to a stage, then 3 x (ds_read_b128 + 1 KiB nt store) to the
// Y/Cb/Cr planes.  Chunks of CH steps come from a static grid-stride (QM 0), one atomic counter
// (QM 1), or static rounds then the counter (QM 3).  Occupancy is pinned by dynamic LDS.
// Build: hipcc --offload-arch=gfx950 -O3 tools/membench3.hip -o tools/membench3
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <algorithm>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

typedef uint32_t u4 __attribute__((ext_vector_type(4)));
typedef float f2 __attribute__((ext_vector_type(2)));
typedef float f4 __attribute__((ext_vector_type(4)));
typedef _Float16 h8 __attribute__((ext_vector_type(8)));

constexpr unsigned kW = 3840, kH = 2160, kPitch = kW * 3;
constexpr unsigned kStepsPerRow = kW / 64;                 /* 60 */
constexpr unsigned kNb = (kW / 8) * (kH / 8);               /* blocks per frame */
constexpr unsigned kStepsPerFrame = kNb / 8;
constexpr unsigned kSlot = 1536, kStage = 3 * 1152;

typedef __attribute__((address_space(3))) void *lp;
typedef const __attribute__((address_space(1))) void *gp;

struct Args {
    const uint8_t *in;
    int16_t *out;
    unsigned nsteps;
    unsigned *ctr;                 /* dynamic queue counter, monotonically increasing         */
    unsigned base;                 /* this launch's first counter value                       */
    unsigned long long *ts;        /* per-wave {start, end} s_memrealtime, or null            */
    unsigned nstatic;              /* QM 3: chunks handed out statically before the queue     */
};

template <int DIST>
__device__ __forceinline__ constexpr int wait_imm()
{
    return (int)(((5 * DIST - 2) & 15) | (((5 * DIST - 2) >> 4) << 14) | 0xF70);
}

/* the chunk source; fetch() starts a request whose value take() returns later.  QM 4: the
 * workgroup's chunk sequence is super-chunks blockIdx.x, blockIdx.x + gridDim.x, ... of
 * a.nstatic chunks each; its waves take the next one from an LDS counter */
template <int QM>
struct Q {
    unsigned nw, wv, round, pend;
    unsigned *lq;
    __device__ __forceinline__ void fetch(const Args &a)
    {
        if (QM == 0 || QM == 6 || QM == 8 || QM == 9) { pend = wv + nw * (round++); return; }
        if (QM == 4 || QM == 10) {
            unsigned t0 = 0;
            if ((threadIdx.x & 63u) == 0) t0 = atomicAdd(lq, 1u);
            const unsigned t = __builtin_amdgcn_readfirstlane(t0);
            if (QM == 10) {
                /* the workgroup's t-th chunk: round r = t / W, m = t % W; the W chunks of a round
                 * spread like W/4 four-wave workgroups' (groups of 4 consecutive chunks, 4 G apart) */
                const unsigned W = nw / gridDim.x, r = t / W, mm = t - r * W;
                pend = r * nw + (mm >> 2) * (4u * gridDim.x) + 4u * blockIdx.x + (mm & 3u);
                return;
            }
            const unsigned sc = a.nstatic, r = t / sc;
            pend = (blockIdx.x + gridDim.x * r) * sc + (t - r * sc);
            return;
        }
        if (QM == 3 || QM == 7) {
            const unsigned k = wv + nw * round;
            if (k < a.nstatic) { round++; pend = k; return; }
        }
        if (QM == 7) {
            const unsigned x = (unsigned)__builtin_amdgcn_s_getreg((2 << 11) | 20) & 7u;
            unsigned v7 = 0;
            if ((threadIdx.x & 63u) == 0) v7 = 0x80000000u | atomicAdd(a.ctr + 32 * x, 1u);
            pend = v7;                              /* bit 31: a dynamic ticket */
            return;
        }
        unsigned v = 0;
        if (QM == 5) {
            const unsigned x = (unsigned)__builtin_amdgcn_s_getreg((2 << 11) | 20) & 7u;
            if ((threadIdx.x & 63u) == 0) v = atomicAdd(a.ctr + a.base * x, 1u);
            pend = v;
            return;
        }
        if ((threadIdx.x & 63u) == 0) v = atomicAdd(a.ctr, 1u);
        pend = v;                                  /* raw: decoded (and waited for) in take() */
    }
    __device__ __forceinline__ unsigned take(const Args &a)
    {
        if (QM == 0 || QM == 4 || QM == 6 || QM == 8 || QM == 9 || QM == 10) return pend;
        if (QM == 7) {
            const unsigned t = __builtin_amdgcn_readfirstlane(pend);
            if (!(t & 0x80000000u)) return t;
            const unsigned x = (unsigned)__builtin_amdgcn_s_getreg((2 << 11) | 20) & 7u;
            return a.nstatic + 8u * (t & 0x7fffffffu) + x;
        }
        const unsigned t = __builtin_amdgcn_readfirstlane(pend);
        if (QM == 5) {
            const unsigned x = (unsigned)__builtin_amdgcn_s_getreg((2 << 11) | 20) & 7u, G = a.nstatic;
            return t == 0xffffffffu ? t : (t / G) * 8u * G + x * G + (t % G);
        }
        return t - a.base + (QM == 3 ? a.nstatic : 0u);
    }
};

template <int NV, int NM, int NL, int CH, int DIST, int NT, int QM, int WPG = 4, int OP = 0>
__global__ __launch_bounds__(WPG * 64) void k_skel(Args a)
{
    static_assert(CH > DIST, "the issue cursor is at most one chunk ahead");
    extern __shared__ __attribute__((aligned(16))) uint8_t dyn[];
    __shared__ unsigned s_q;
    if (QM == 4 || QM == 10) {
        if (threadIdx.x == 0) s_q = 0;
        __syncthreads();
    }
    const unsigned lane = threadIdx.x & 63u;
    uint8_t *ring = dyn + (threadIdx.x >> 6) * ((DIST + 1) * kSlot + kStage + 256);
    uint8_t *stage = ring + (DIST + 1) * kSlot;
    uint8_t *dummy = stage + kStage;
    const unsigned nw = gridDim.x * WPG;
    const unsigned wv = __builtin_amdgcn_readfirstlane(blockIdx.x * WPG + (threadIdx.x >> 6));
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    const unsigned long long c0 = __builtin_amdgcn_s_memtime();
    const unsigned nchunks = a.nsteps / CH;
    Q<QM> q{nw, wv, 0, 0, &s_q};
    q.fetch(a);
    unsigned cc = q.take(a);                        /* compute chunk */
    if (cc >= nchunks) {
        if (a.ts && lane == 0) { a.ts[6 * wv] = 0; a.ts[6 * wv + 1] = 0; }
        if (QM == 5 || QM == 7) {
            unsigned last = 0;
            if (lane == 0) last = atomicAdd(a.ctr + 256, 1u) == nw - 1;
            if (__builtin_amdgcn_readfirstlane(last) && lane < 9) atomicExch(a.ctr + (lane == 8 ? 256 : a.base * lane), 0u);
        }
        return;
    }
    q.fetch(a);                                    /* the chunk after: taken when the issue cursor gets there */
    unsigned ic = cc, ik = 0;                      /* issue cursor: chunk, step in it */
    unsigned ck = 0;                               /* compute step in cc */
    const uint32_t off0 = (lane / 12u) * kPitch + 16u * (lane % 12u);
    const uint32_t off1 = ((64u + lane) / 12u) * kPitch + 16u * ((64u + lane) % 12u);
    auto issue = [&](uint8_t *slot) {
        if (ic < nchunks) {
            const unsigned s = ic * CH + ik;
            const uint8_t *b = a.in + (size_t)(s / kStepsPerRow) * 8 * kPitch + (s % kStepsPerRow) * 192u;
            __builtin_amdgcn_global_load_lds((gp)(b + off0), (lp)slot, 16, 0, 0);
            if (lane < 32) __builtin_amdgcn_global_load_lds((gp)(b + off1), (lp)(slot + 1024), 16, 0, 0);
        } else {
            __builtin_amdgcn_global_load_lds((gp)a.in, (lp)dummy, 4, 0, 0);
            __builtin_amdgcn_global_load_lds((gp)a.in, (lp)dummy, 4, 0, 0);
        }
        if (ic < nchunks && ++ik == CH) {
            ik = 0;
            ic = q.take(a);
            if (ic < nchunks) q.fetch(a);
        }
    };
#pragma unroll
    for (int k = 0; k < DIST; k++) {
        issue(ring + k * kSlot);
        for (int i = 0; i < 3; i++) __builtin_amdgcn_global_load_lds((gp)a.in, (lp)dummy, 4, 0, 0);
    }
    f2 acc[8];
#pragma unroll
    for (int i = 0; i < 8; i++) acc[i] = f2{(float)lane, (float)i};
    const f2 k1 = NT == 2 ? f2{0.0f, 0.0f} : f2{1.0001f, 0.9999f}, k2 = NT == 2 ? f2{0.0f, 0.0f} : f2{0.5f, 0.25f};
    if (NT == 2) {
#pragma unroll
        for (int i = 0; i < 8; i++) acc[i] = f2{0.0f, 0.0f};
    }
    f4 macc[4] = {};
    unsigned slot = 0;
    for (;;) {
        const unsigned sc = cc * CH + ck;
        __builtin_amdgcn_s_waitcnt(wait_imm<DIST>());
        __builtin_amdgcn_wave_barrier();
        asm volatile("" ::: "memory");
        uint8_t *sp = ring + slot * kSlot;
        issue(ring + (slot == 0 ? DIST : slot - 1) * kSlot);
        const u4 d = *(const u4 *)(sp + (lane % 96) * 16);
        if (NT != 2) {
            acc[0].x += __uint_as_float(d.x & 0x3fffffffu);
            acc[1].x += __uint_as_float(d.y & 0x3fffffffu);
        }
        h8 av = __builtin_bit_cast(h8, NT == 2 ? u4{0, 0, 0, 0} : d);
#pragma unroll
        for (int i = 0; i < NM; i++)
            macc[i & 3] = __builtin_amdgcn_mfma_f32_16x16x32_f16(av, av, macc[i & 3], 0, 0, 0);
#pragma unroll
        for (int i = 0; i < NV; i++) {
            if (OP == 0) asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(acc[i & 7]) : "v"(k1), "v"(k2));
            if (OP == 1) asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(acc[i & 7]) : "v"(k2));
            if (OP == 2) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(acc[i & 7].x) : "v"(k1.x), "v"(k2.x));
            if (OP == 3) asm volatile("v_perm_b32 %0, %0, %1, %2" : "+v"(acc[i & 7].x) : "v"(d.w), "v"(0x05040702u));
            if (OP == 4) asm volatile("v_pk_mul_f32 %0, %0, %1" : "+v"(acc[i & 7]) : "v"(k1));
        }
        if (NM) acc[2].x += macc[0].x + macc[1].y + macc[2].z + macc[3].w;
#pragma unroll
        for (int i = 0; i < NL; i++)
            *(uint16_t *)(stage + (i % 3) * 1152 + ((lane * 37u + (unsigned)i * 131u) & 511u) * 2u) =
                (uint16_t)(__float_as_uint(acc[i & 7].x) ^ (d.z >> (i & 15)));
        __builtin_amdgcn_wave_barrier();
        asm volatile("" ::: "memory");
        const unsigned f = sc / kStepsPerFrame, bi = (sc - f * kStepsPerFrame) * 8u;
        int16_t *ob = a.out + (size_t)f * 3 * kNb * 64 + (size_t)bi * 64 + lane * 8;
#pragma unroll
        for (int c = 0; c < 3; c++) {
            u4 v = *(const u4 *)(stage + c * 1152 + lane * 16);
            if (NL == 0) v.x ^= __float_as_uint(acc[c].x + acc[c + 3].y);
            if (NT) __builtin_nontemporal_store(v, (u4 *)(ob + (size_t)c * kNb * 64));
            else *(u4 *)(ob + (size_t)c * kNb * 64) = v;
        }
        __builtin_amdgcn_wave_barrier();
        asm volatile("" ::: "memory");
        if (QM == 6) asm volatile("s_barrier" ::: "memory");   /* lock-step within the workgroup */
        if (QM == 8 || QM == 9) {
            /* rotating priority: each wave of a CU gets the top priority a quarter of the time */
            const unsigned ph = (QM == 8 ? (cc * CH + ck) : cc) + (wv >> 2) + (wv & 3);
            switch (ph & 3) {
            case 0: __builtin_amdgcn_s_setprio(0); break;
            case 1: __builtin_amdgcn_s_setprio(1); break;
            case 2: __builtin_amdgcn_s_setprio(2); break;
            default: __builtin_amdgcn_s_setprio(3); break;
            }
        }
        slot = slot == DIST ? 0 : slot + 1;
        if (++ck == CH) {
            ck = 0;
            cc = ic;                                /* the issue cursor is already in the next chunk */
            if (cc >= nchunks) break;
        }
    }
    if (acc[5].y == 3.0f) a.out[0] = 1;
    if (QM == 5 || QM == 7) {
        /* the last wave to finish resets the counters for the next launch (stream order) */
        __builtin_amdgcn_s_waitcnt(0);
        unsigned last = 0;
        if (lane == 0) last = atomicAdd(a.ctr + 256, 1u) == nw - 1;
        if (__builtin_amdgcn_readfirstlane(last) && lane < 9) atomicExch(a.ctr + (lane == 8 ? 256 : a.base * lane), 0u);
    }
    if (a.ts && lane == 0) {
        a.ts[6 * wv] = t0;
        a.ts[6 * wv + 1] = __builtin_amdgcn_s_memrealtime();
        a.ts[6 * wv + 2] = (unsigned)__builtin_amdgcn_s_getreg((31 << 11) | 20);
        a.ts[6 * wv + 3] = (unsigned)__builtin_amdgcn_s_getreg((31 << 11) | 4);
        a.ts[6 * wv + 4] = c0;
        a.ts[6 * wv + 5] = __builtin_amdgcn_s_memtime();
    }
}

template <int NT>
__global__ __launch_bounds__(256) void k_ideal(const u4 *__restrict__ in, u4 *__restrict__ out, size_t n)
{
    for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
        const u4 v = in[i];
        const u4 x = v * 3u, y = v ^ 0x5a5a5a5au;
        if (NT) {
            __builtin_nontemporal_store(x, out + i);
            __builtin_nontemporal_store(y, out + n + i);
        } else {
            out[i] = x;
            out[n + i] = y;
        }
    }
}

static uint8_t *g_in[2];
static int16_t *g_out;
static unsigned *g_ctr;
static unsigned long long *g_ts;
static int g_cus;
static hipEvent_t e0, e1;

template <class L>
static void timeit(const char *name, L launch)
{
    int which = 0;
    for (int i = 0; i < 300; i++) launch(g_in[(which++) & 1], false);
    CK(hipDeviceSynchronize());
    std::vector<float> v;
    for (int r = 0; r < 5; r++) {
        CK(hipEventRecord(e0));
        for (int i = 0; i < 20; i++) launch(g_in[(which++) & 1], false);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        v.push_back(ms * 1e3f / 20);
    }
    std::sort(v.begin(), v.end());
    const double bytes = 8.0 * kW * kH * 9;
    printf("%-44s min %7.1f us  med %7.1f us  frac(min) %.3f", name, v[0], v[2], bytes / (v[0] * 1e-6) / 8e12);
    /* one more launch with per-wave timestamps: spread of wave end times */
    launch(g_in[(which++) & 1], true);
    CK(hipDeviceSynchronize());
    printf("\n");
    fflush(stdout);
}

static unsigned g_ctr_val = 0, g_stride = 32;

template <int NV, int NM, int NL, int CH, int DIST, int NT, int QM, int WPG = 4, int OP = 0>
static void skel(int wpe, int grid_mult = 1, double static_frac = 0.0, int superchunk = 0)
{
    char name[160];
    snprintf(name, sizeof name, "skel v%d m%d l%d c%d d%d nt%d q%d w%d g%d sf%.2f wg%d sc%d op%d", NV, NM, NL, CH, DIST,
             NT, QM, wpe, grid_mult, static_frac, WPG, superchunk, OP);
    const size_t per_wg = WPG * ((DIST + 1) * kSlot + kStage + 256);
    /* wpe waves per SIMD: wpe * 4 / WPG workgroups per CU */
    const size_t lds = std::max(per_wg, (size_t)(160 * 1024 * WPG / (4 * wpe) - 64) & ~(size_t)15);
    auto kern = k_skel<NV, NM, NL, CH, DIST, NT, QM, WPG, OP>;
    CK(hipFuncSetAttribute((const void *)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    const unsigned nsteps = 8 * kStepsPerFrame, nchunks = nsteps / CH;
    unsigned grid = g_cus * wpe * 4 / WPG * grid_mult;
    if (grid_mult == 0) grid = (nchunks + WPG - 1) / WPG;  /* non-persistent: one chunk per wave */
    const unsigned nw = grid * WPG;
    unsigned nstatic = (unsigned)(static_frac * nchunks) / nw * nw;
    if (QM == 4 || QM == 5) {
        nstatic = superchunk;                       /* chunks per super-chunk / XCD interleave */
    }
    std::vector<unsigned long long> ts(6 * nw);
    timeit(name, [&](uint8_t *in, bool stamp) {
        if (stamp) CK(hipMemset(g_ts, 0, 6 * nw * sizeof(unsigned long long)));
        Args a{in, g_out, nsteps, g_ctr, QM == 5 ? g_stride : (QM == 7 ? 32u : g_ctr_val), stamp ? g_ts : nullptr, nstatic};
        hipLaunchKernelGGL(kern, dim3(grid), dim3(WPG * 64), lds, 0, a);
        /* every wave ends with one failing dequeue: the counter moves by the dynamic chunks + nw */
        if (QM == 1 || QM == 3) g_ctr_val += (nchunks - nstatic) + nw;
        if (stamp) {
            CK(hipMemcpy(ts.data(), g_ts, ts.size() * 8, hipMemcpyDeviceToHost));
            unsigned long long mn = ~0ull;
            std::vector<double> ends;
            std::vector<double> clk;
            for (unsigned w = 0; w < nw; w++)
                if (ts[6 * w]) {
                    mn = std::min(mn, ts[6 * w]);
                    const double dr = (double)(ts[6 * w + 1] - ts[6 * w]);
                    if (dr > 500) clk.push_back((double)(ts[6 * w + 5] - ts[6 * w + 4]) / dr * 100.0);
                }
            std::sort(clk.begin(), clk.end());
            double xsum[8] = {}, xn[8] = {};
            /* per CU (xcc, se, cu): spread of its waves' ends */
            std::vector<std::pair<unsigned, double>> cu;
            for (unsigned w = 0; w < nw; w++) {
                if (!ts[6 * w]) continue;
                const double e = (ts[6 * w + 1] - mn) * 0.01;
                ends.push_back(e);
                const unsigned x = (unsigned)ts[6 * w + 2] & 7u, hw = (unsigned)ts[6 * w + 3];
                xsum[x] += e;
                xn[x] += 1;
                cu.push_back({x << 16 | ((hw >> 13) & 7u) << 8 | ((hw >> 8) & 15u), e});
            }
            std::sort(ends.begin(), ends.end());
            const size_t m = ends.size();
            printf("  | ends p1 %.1f p10 %.1f p50 %.1f p90 %.1f max %.1f", ends[m / 100], ends[m / 10],
                   ends[m / 2], ends[m * 9 / 10], ends[m - 1]);
            if (!clk.empty()) printf(" | clk MHz p50 %.0f", clk[clk.size() / 2]);
            printf(" | xcd means");
            for (int x = 0; x < 8; x++) printf(" %.0f", xn[x] ? xsum[x] / xn[x] : -1.0);
            std::sort(cu.begin(), cu.end());
            double spread = 0, cmax_lo = 1e30, cmax_hi = 0;
            int ncu = 0;
            for (size_t i = 0; i < cu.size();) {
                size_t j = i;
                double lo = 1e30, hi = 0;
                while (j < cu.size() && cu[j].first == cu[i].first) {
                    lo = std::min(lo, cu[j].second);
                    hi = std::max(hi, cu[j].second);
                    j++;
                }
                spread += hi - lo;
                cmax_lo = std::min(cmax_lo, hi);
                cmax_hi = std::max(cmax_hi, hi);
                ncu++;
                i = j;
            }
            printf(" | %d CUs: mean in-CU spread %.1f, CU last-end %.1f..%.1f", ncu, spread / ncu, cmax_lo, cmax_hi);
            /* by SIMD id, and by the wave's rank (by block index) among the CU's workgroups */
            double ss[4] = {}, sn[4] = {};
            std::vector<std::pair<unsigned long long, std::pair<unsigned, double>>> byc;   /* (cu key, (block, end)) */
            for (unsigned w = 0; w < nw; w++) {
                if (!ts[6 * w]) continue;
                const unsigned hw = (unsigned)ts[6 * w + 3], x = (unsigned)ts[6 * w + 2] & 7u;
                const double e = (ts[6 * w + 1] - mn) * 0.01;
                ss[(hw >> 4) & 3] += e;
                sn[(hw >> 4) & 3] += 1;
                const unsigned long long key = (unsigned long long)x << 16 | ((hw >> 13) & 7u) << 8 | ((hw >> 8) & 15u);
                byc.push_back({key, {w / WPG, e}});
            }
            printf(" | simd means");
            for (int i = 0; i < 4; i++) printf(" %.0f", sn[i] ? ss[i] / sn[i] : -1.0);
            std::sort(byc.begin(), byc.end());
            double rs[8] = {}, rn[8] = {};
            for (size_t i = 0; i < byc.size();) {
                size_t j = i;
                while (j < byc.size() && byc[j].first == byc[i].first) j++;
                /* rank workgroups of this CU by block index */
                std::vector<unsigned> blks;
                for (size_t k = i; k < j; k++) blks.push_back(byc[k].second.first);
                std::sort(blks.begin(), blks.end());
                blks.erase(std::unique(blks.begin(), blks.end()), blks.end());
                for (size_t k = i; k < j; k++) {
                    const int rk = (int)(std::lower_bound(blks.begin(), blks.end(), byc[k].second.first) - blks.begin());
                    if (rk < 8) { rs[rk] += byc[k].second.second; rn[rk] += 1; }
                }
                i = j;
            }
            printf(" | wg-rank means");
            for (int i = 0; i < 8 && rn[i]; i++) printf(" %.0f", rs[i] / rn[i]);
        }
    });
}

int main(int argc, char **argv)
{
    const char *which = argc > 1 ? argv[1] : "all";
    const size_t in_bytes = 8ull * kW * kH * 3;
    CK(hipMalloc(&g_in[0], in_bytes + 4096));
    CK(hipMalloc(&g_in[1], in_bytes + 4096));
    CK(hipMalloc(&g_out, 2 * in_bytes));
    CK(hipMalloc(&g_ctr, 8 << 20));          /* counters up to 1 MiB apart (8 XCDs) */
    CK(hipMalloc(&g_ts, 6 * 1024 * 1024 * sizeof(unsigned long long)));
    CK(hipMemset(g_ctr, 0, 8 << 20));
    {
        std::vector<uint8_t> h(in_bytes);
        uint64_t z = 12345;
        for (size_t i = 0; i < in_bytes; i += 8) {
            z += 0x9E3779B97F4A7C15ULL;
            uint64_t t = z;
            t = (t ^ (t >> 30)) * 0xBF58476D1CE4E5B9ULL;
            t = (t ^ (t >> 27)) * 0x94D049BB133111EBULL;
            t ^= t >> 31;
            memcpy(&h[i], &t, std::min<size_t>(8, in_bytes - i));
        }
        CK(hipMemcpy(g_in[0], h.data(), in_bytes, hipMemcpyHostToDevice));
        CK(hipMemcpy(g_in[1], h.data(), in_bytes, hipMemcpyHostToDevice));
    }
    CK(hipMemset(g_out, 0, 2 * in_bytes));
    CK(hipDeviceGetAttribute(&g_cus, hipDeviceAttributeMultiprocessorCount, 0));
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const size_t n = in_bytes / 16;
    timeit("ideal_np_nt", [&](uint8_t *in, bool) {
        hipLaunchKernelGGL(k_ideal<1>, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, 0, (const u4 *)in, (u4 *)g_out, n);
    });
    if (!strcmp(which, "all") || !strcmp(which, "a")) {
        skel<0, 0, 0, 4, 2, 1, 0>(3);
        skel<0, 0, 0, 4, 2, 1, 0>(3, 0);
        skel<0, 0, 0, 4, 2, 1, 10, 12>(3);
        skel<0, 0, 0, 4, 2, 1, 10, 8>(2);
        skel<0, 0, 0, 4, 2, 1, 10, 16>(4);
        skel<192, 16, 24, 4, 2, 1, 0>(3);
        skel<192, 16, 24, 4, 2, 1, 10, 12>(3);
        skel<192, 16, 24, 4, 2, 1, 10, 16>(4);
    }
    if (!strcmp(which, "r4b")) {
        /* the VALU cliff: persistent vs non-persistent at 64..192 packed FMAs, and op kinds */
        skel<0, 0, 0, 3, 2, 1, 0>(4);
        skel<64, 16, 24, 3, 2, 1, 0>(4);
        skel<128, 16, 24, 3, 2, 1, 0>(4);
        skel<160, 16, 24, 3, 2, 1, 0>(4);
        skel<0, 0, 0, 4, 2, 1, 0>(4, 0);
        skel<64, 16, 24, 4, 2, 1, 0>(4, 0);
        skel<128, 16, 24, 4, 2, 1, 0>(4, 0);
        skel<144, 16, 24, 4, 2, 1, 0>(4, 0);
        skel<160, 16, 24, 4, 2, 1, 0>(4, 0);
        skel<176, 16, 24, 4, 2, 1, 0>(4, 0);
        skel<192, 16, 24, 4, 2, 1, 0>(4, 0);
        skel<128, 16, 24, 2, 1, 1, 0>(4, 0);
        skel<128, 16, 24, 6, 2, 1, 0>(4, 0);
        skel<192, 16, 24, 4, 2, 1, 0, 4, 1>(4, 0);   /* pk_add */
        skel<192, 16, 24, 4, 2, 1, 0, 4, 4>(4, 0);   /* pk_mul */
        skel<192, 16, 24, 4, 2, 1, 0, 4, 2>(4, 0);   /* scalar fma */
        skel<192, 16, 24, 4, 2, 1, 0, 4, 3>(4, 0);   /* perm */
        skel<128, 16, 48, 4, 2, 1, 0>(4, 0);         /* 48 LDS writes */
        skel<128, 16, 24, 4, 2, 1, 0>(3, 0);
        skel<128, 16, 24, 4, 2, 1, 0>(2, 0);
    }
    if (!strcmp(which, "r4c")) {
        /* occupancy (waves per SIMD, pinned by LDS) and MFMA count at k_mxs-like compute, non-persistent */
        skel<0, 0, 0, 3, 2, 1, 0>(4, 0);
        skel<128, 16, 24, 3, 2, 1, 0>(3, 0);
        skel<128, 16, 24, 3, 2, 1, 0>(4, 0);
        skel<128, 16, 24, 3, 2, 1, 0>(5, 0);
        skel<128, 16, 24, 3, 2, 1, 0>(6, 0);
        skel<128, 16, 24, 2, 1, 1, 0>(5, 0);
        skel<128, 16, 24, 2, 1, 1, 0>(6, 0);
        skel<128, 0, 24, 3, 2, 1, 0>(4, 0);
        skel<128, 8, 24, 3, 2, 1, 0>(4, 0);
        skel<96, 16, 24, 3, 2, 1, 0>(4, 0);
        skel<96, 16, 24, 3, 2, 1, 0>(5, 0);
        skel<128, 16, 24, 3, 1, 1, 0>(4, 0);       /* 3 steps through 2 slots */
        skel<128, 16, 24, 3, 1, 1, 0>(5, 0);
    }
    if (!strcmp(which, "r4")) {
        /* round 4: non-persistent grids (one chunk per wave) with random-operand compute, and the
         * VALU -> MFMA trade (same memory pattern, 4 waves per SIMD) */
        skel<0, 0, 0, 3, 2, 1, 0>(4);              /* persistent, memory only */
        skel<192, 16, 24, 3, 2, 1, 0>(4);          /* persistent, k_mx-sized compute */
        skel<0, 0, 0, 3, 2, 1, 0>(4, 0);           /* non-persistent, memory only */
        skel<0, 0, 0, 8, 2, 1, 0>(4, 0);
        skel<192, 16, 24, 3, 2, 1, 0>(4, 0);       /* non-persistent, k_mx-sized compute */
        skel<192, 16, 24, 4, 2, 1, 0>(4, 0);
        skel<192, 16, 24, 8, 2, 1, 0>(4, 0);
        skel<192, 16, 24, 16, 2, 1, 0>(4, 0);
        skel<128, 16, 24, 4, 2, 1, 0>(4, 0);
        skel<96, 16, 24, 4, 2, 1, 0>(4, 0);
        skel<64, 16, 24, 4, 2, 1, 0>(4, 0);
        skel<96, 40, 24, 4, 2, 1, 0>(4, 0);        /* column pass on the matrix cores: fewer VALU, more MFMA */
        skel<64, 64, 24, 4, 2, 1, 0>(4, 0);
        skel<64, 88, 24, 4, 2, 1, 0>(4, 0);
        skel<96, 40, 24, 3, 2, 1, 0>(4);
        skel<64, 64, 24, 3, 2, 1, 0>(4);
        skel<192, 16, 24, 4, 2, 2, 0>(4, 0);       /* zero operands */
    }
    return 0;
}
