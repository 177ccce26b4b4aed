/*
 * jpgx_plan.cpp -- host side of the C-ABI shim: argument validation, quantisation tables,
 * the underflow bytes, and the rigorous fp32 guard band.  No device code here.
 *
 * Guard band.  The kernel computes each quotient t = F(u,v)/Q[u][v] in fp32 (xform_math.h,
 * FOps).  BoundOps below pushes an interval [lo,hi] of the exact value and a bound E on the
 * fp32 error through the very same template code, starting from pixel bytes in [0,255]:
 *     add/sub:  E = Ea + Eb + 2^-24 (|c| + Ea + Eb)
 *     a*k:      E = Ea|k_f| + |a| |k_f - k| + 2^-24 (...)
 *     fma:      E = Ea|k_f| + |a| |k_f - k| + Eb + 2^-24 (...)
 * and adds the error of the fp32 scale.  If the fp32 quotient sits farther than E_t from a
 * half-integer, the reference's double quotient rounds (src/quantise.c:58, C round()) to the
 * same integer; otherwise the kernel flags the coefficient for the exact-order fp64 path.
 */
#include <math.h>
#include <string.h>

#include <algorithm>
#include <memory>

#include "jpgx_internal.h"
#include "jx_consts.h"
#include "xform_math.h"

/* pristine base tables, src/quantise.c:8-25 (row index = first subscript) */
static const int kLum[8][8] = JX_Q_LUM_INIT;
static const int kChr[8][8] = JX_Q_CHR_INIT;

namespace {

struct Bnd {
    double lo, hi, E;
};

struct BoundOps {
    typedef Bnd T;
    static double mag(const Bnd &a) { return std::max(fabs(a.lo), fabs(a.hi)); }
    static Bnd round_(double lo, double hi, double err)
    {
        const double u = 0x1p-24;
        Bnd c{lo, hi, 0};
        c.E = err + u * (mag(c) + err);
        return c;
    }
    static void span(double a, double b, double &lo, double &hi)
    {
        lo = std::min(a, b);
        hi = std::max(a, b);
    }
    static Bnd add(Bnd a, Bnd b) { return round_(a.lo + b.lo, a.hi + b.hi, a.E + b.E); }
    static Bnd sub(Bnd a, Bnd b) { return round_(a.lo - b.hi, a.hi - b.lo, a.E + b.E); }
    static Bnd mulc(Bnd a, jx_const k)
    {
        double lo, hi;
        span(a.lo * k.x, a.hi * k.x, lo, hi);
        return round_(lo, hi, a.E * fabs((double)k.f) + mag(a) * fabs((double)k.f - k.x));
    }
    static Bnd fmac(Bnd a, jx_const k, Bnd b)
    {
        double lo, hi;
        span(a.lo * k.x, a.hi * k.x, lo, hi);
        return round_(lo + b.lo, hi + b.hi,
                      a.E * fabs((double)k.f) + mag(a) * fabs((double)k.f - k.x) + b.E);
    }
    static Bnd lit(jx_const k) { return Bnd{k.x, k.x, fabs((double)k.f - k.x)}; }
};

/* sub: 0 = one pixel per sample (4:4:4 and the reference's parity modes); 1 = true 4:2:2,
 * 2 = true 4:2:0, in the kernels' (k_chroma, k_sub422) operation order: the colour transform
 * of the pair's / quad's byte sums (exact integers <= 510 / 1020 in fp32), times 0.5 / 0.25.
 * The exact value is the average of the pixels' samples (the oracle's definition); the colour
 * transform being linear, it equals the transform of the sums scaled, in real arithmetic. */
template <int CH>
void coef_bounds(Bnd F[8][8], int sub = 0)
{
    const Bnd byte{0.0, sub == 1 ? 510.0 : (sub == 2 ? 1020.0 : 255.0), 0.0};
    Bnd px[8], row[8];
    Bnd p = jx_pixel<BoundOps, CH>(byte, byte, byte);
    if (sub == 1) p = BoundOps::mulc(p, JX_K(0.5));
    if (sub == 2) p = BoundOps::mulc(p, JX_K(0.25));
    for (int x = 0; x < 8; x++) px[x] = p;
    jx_fdct8<BoundOps>(px, row);   /* every pixel row has the same bound */
    for (int u = 0; u < 8; u++) {
        Bnd col[8], out[8];
        for (int y = 0; y < 8; y++) col[y] = row[u];
        jx_fdct8<BoundOps>(col, out);
        for (int v = 0; v < 8; v++) F[v][u] = out[v];
    }
}

}  // namespace

extern "C" {

int jpgx_validate(int width, int height, const jpgx_params *p)
{
    if (!p) return JPGX_EARG;
    if (p->sample_ratio < 0 || p->sample_ratio > 2) return JPGX_ESAMPLE;
    if (p->quality < 1 || p->quality > 97) return JPGX_EQUALITY;
    /* src/preprocess.c:82-98 pads by w%8 / w%16 / h%16 (not up to a multiple), after which
     * its copy loop is wrong: only exact multiples have defined reference behaviour. */
    const int wm = p->sample_ratio == 0 ? 8 : 16, hm = p->sample_ratio == 2 ? 16 : 8;
    if (width <= 0 || height <= 0 || width % wm || height % hm) return JPGX_EGEOMETRY;
    return JPGX_OK;
}

static unsigned long long req2size(unsigned long long n)
{
    unsigned long long s = (n + 8 + 15) & ~15ULL;
    return s < 32 ? 32 : s;
}

void jpgx_glibc_underflow(long long n_pixels, long long bmp_file_size, uint8_t out[8])
{
    /* glibc malloc (64-bit): the chunk-size word sits 8 bytes before the user pointer.
     * r_new is an sbrk chunk (size | PREV_INUSE) unless it is at or above the mmap
     * threshold (size rounded to pages | IS_MMAPPED).  The threshold starts at 128 KiB and
     * rises to the size of the mmapped file buffer freed at src/bitmap.c:151 when that
     * chunk is at most 32 MiB (DEFAULT_MMAP_THRESHOLD_MAX). */
    const unsigned long long page = 4096, thr0 = 128 * 1024, thr_max = 32ULL << 20;
    unsigned long long thr = thr0;
    const unsigned long long fchunk = req2size((unsigned long long)bmp_file_size);
    if (fchunk >= thr0) {
        const unsigned long long mm = (fchunk + 8 + page - 1) & ~(page - 1);
        if (mm > thr && mm <= thr_max) thr = mm;
    }
    const unsigned long long nb = req2size((unsigned long long)n_pixels);
    const unsigned long long size =
        nb >= thr ? (((nb + 8 + page - 1) & ~(page - 1)) | 2ULL) : (nb | 1ULL);
    for (int k = 0; k < 8; k++) out[k] = (uint8_t)(size >> (8 * k));
}

void jpgx_default_params(jpgx_params *p, int width, int height, int quality, int sample_ratio)
{
    memset(p, 0, sizeof *p);
    p->quality = quality;
    p->sample_ratio = sample_ratio;
    const long long n = (long long)width * height;
    jpgx_glibc_underflow(n, 54 + 3 * n, p->underflow[0]);
    memcpy(p->underflow[1], p->underflow[0], 8);
    memcpy(p->underflow[2], p->underflow[0], 8);
}

int jpgx_scale_table(int which, int quality, int out[8][8])
{
    if (quality < 1 || quality > 97) return JPGX_EQUALITY;
    const int(*base)[8] = which == 0 ? kLum : kChr;
    const int s = quality < 50 ? 5000 / quality : 200 - 2 * quality;  /* quantise.c:81 */
    for (int i = 0; i < 8; i++)
        for (int j = 0; j < 8; j++) out[i][j] = (s * base[i][j] + 50) / 100;  /* :82 */
    return JPGX_OK;
}

void jx_under_dwords(const uint8_t under[3][8], uint32_t out[6])
{
    /* the missing pixel row, interleaved like the input: pixel x = (r_x, g_x, b_x) */
    uint8_t row[24];
    for (int x = 0; x < 8; x++)
        for (int k = 0; k < 3; k++) row[3 * x + k] = under[k][x];
    memcpy(out, row, sizeof row);
}

/* long-double evaluation of the same 1-D transform code (near-exact constants) */
struct LDOps {
    typedef long double T;
    static T add(T a, T b) { return a + b; }
    static T sub(T a, T b) { return a - b; }
    static T mulc(T a, jx_const k) { return a * (long double)k.x; }
    static T fmac(T a, jx_const k, T b) { return a * (long double)k.x + b; }
    static T lit(jx_const k) { return (long double)k.x; }
};

/* Factor that turns output k of jx_fdct8 into sum_x in[x] cos((2x+1)k pi/16): evaluated on
 * in[x] = cos((2x+1)k pi/16) (where that sum is 8 for k = 0, else 4). */
static long double dct_kfactor(int k)
{
    const long double pi = 3.141592653589793238462643383279502884L;
    long double in[8], out[8];
    for (int x = 0; x < 8; x++) in[x] = cosl((2 * x + 1) * k * pi / 16);
    jx_fdct8<LDOps>(in, out);
    return (k == 0 ? 8.0L : 4.0L) / out[k];
}

int jx_plan_tables_mode(int quality, int sub, float w[3][64], float lim[3][64], int16_t q[2][64])
{
    int qs[2][8][8];
    int rc = jpgx_scale_table(0, quality, qs[0]);
    if (rc) return rc;
    jpgx_scale_table(1, quality, qs[1]);
    for (int t = 0; t < 2; t++)
        for (int u = 0; u < 8; u++)
            for (int v = 0; v < 8; v++) q[t][u * 8 + v] = (int16_t)qs[t][u][v];

    Bnd F[3][8][8];
    coef_bounds<0>(F[0]);                  /* luma is never averaged */
    coef_bounds<1>(F[1], sub);
    coef_bounds<2>(F[2], sub);
    const long double a0 = 1.0L / sqrtl(2.0L);
    for (int ch = 0; ch < 3; ch++) {
        const int t = ch == 0 ? 0 : 1;
        for (int v = 0; v < 8; v++)
            for (int u = 0; u < 8; u++) {
                /* exact scale: 1/4 a(u) a(v) k(u) k(v) / Q[u][v] (dct.c:54, quantise.c:58) */
                const long double au = u == 0 ? a0 : 1.0L, av = v == 0 ? a0 : 1.0L;
                const long double ku = dct_kfactor(u), kv = dct_kfactor(v);
                const long double ws = 0.25L * au * av * ku * kv / (long double)qs[t][u][v];
                const float wf = (float)ws;
                const Bnd &b = F[ch][v][u];
                const double mF = BoundOps::mag(b) + b.E;
                /* error of t_fp vs the reference's real-arithmetic quotient, plus the final
                 * fma rounding of d (< 2^-25), plus slack for the reference's own double
                 * rounding (< 1e-10) and for this bound's own double arithmetic */
                double et = b.E * fabs((double)wf) + mF * (double)fabsl((long double)wf - ws) + 0x1p-25;
                et = et * 1.01 + 1e-7;
                w[ch][v * 8 + u] = wf;
                lim[ch][v * 8 + u] = (float)(0.5 - et);
            }
    }
    return JPGX_OK;
}

int jx_plan_tables(int quality, float w[3][64], float lim[3][64], int16_t q[2][64])
{
    return jx_plan_tables_mode(quality, 0, w, lim, q);
}

int jpgx_guard_band(int quality, float scale[3][64], float lim[3][64])
{
    int16_t q[2][64];
    return jx_plan_tables(quality, scale, lim, q);
}

void jpgx_stripe(int block_rows, int nshards, int k, int *row_begin, int *row_end)
{
    /* contiguous, sizes differ by at most one block row: the first block_rows % n get +1 */
    const int base = block_rows / nshards, extra = block_rows % nshards;
    *row_begin = k * base + std::min(k, extra);
    *row_end = *row_begin + base + (k < extra ? 1 : 0);
}

const char *jpgx_version(void) { return "jpgx 0.1 (gfx950)"; }

size_t jpgx_chroma_blocks(int width, int row_begin, int row_end, int sample_ratio, unsigned flags)
{
    if (width <= 0 || row_end < row_begin) return 0;
    const size_t rows = (size_t)(row_end - row_begin);
    if (!(flags & JPGX_FLAG_SUBSAMPLE) || sample_ratio == 0) return rows * (size_t)(width / 8);
    return (sample_ratio == 2 ? rows / 2 : rows) * (size_t)(width / 16);
}

size_t jpgx_workspace_size(const jpgx_frames *fr)
{
    /* every kernel keeps its exact-pass queues in LDS */
    (void)fr;
    return 0;
}

}  /* extern "C" */

/* ---- packed-pair equivalence (host) --------------------------------------------------------
 * The kernel's packed path (xform_math.h: PairOps, jx_fdct8_pk) must produce, lane by lane, the
 * very fp32 values of the scalar FOps code the guard band was derived for.  HostPair evaluates
 * the packed code with one correctly rounded scalar operation per lane, as v_pk_* does. */
namespace {
struct HF2 {
    float x, y;
};
struct HostPair {
    typedef HF2 V;
    static V mk(float a, float b) { return V{a, b}; }
    static float lo(V a) { return a.x; }
    static float hi(V a) { return a.y; }
    static V add(V a, V b) { return V{a.x + b.x, a.y + b.y}; }
    static V sub(V a, V b) { return V{a.x - b.x, a.y - b.y}; }
    static V mul(V a, V b) { return V{a.x * b.x, a.y * b.y}; }
    static V fma(V a, V b, V c) { return V{fmaf(a.x, b.x, c.x), fmaf(a.y, b.y, c.y)}; }
};

inline uint32_t bits(float f)
{
    uint32_t u;
    memcpy(&u, &f, 4);
    return u;
}

uint64_t sm64(uint64_t &s)
{
    uint64_t z = (s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

/* one block-channel both ways: scalar rows/cols (the bound's code) vs the kernel's packed
 * order (rows: jx_fdct8_pk on pixel pairs; columns: jx_fdct8 over PairOps on column pairs) */
template <int CH>
long long block_mismatch(const uint8_t px[8][8][3], const float w[64])
{
    typedef PairOps<HostPair> PO;
    float T[8][8], Fs[8][8];
    for (int y = 0; y < 8; y++) {
        float in[8];
        for (int x = 0; x < 8; x++)
            in[x] = jx_pixel<FOps, CH>((float)px[y][x][0], (float)px[y][x][1], (float)px[y][x][2]);
        jx_fdct8<FOps>(in, T[y]);
    }
    for (int u = 0; u < 8; u++) {
        float col[8], out[8];
        for (int y = 0; y < 8; y++) col[y] = T[y][u];
        jx_fdct8<FOps>(col, out);
        for (int v = 0; v < 8; v++) Fs[v][u] = out[v];
    }
    HF2 Tp[8][4];
    for (int y = 0; y < 8; y++) {
        HF2 in[4];
        for (int k = 0; k < 4; k++) {
            const HF2 r{(float)px[y][2 * k][0], (float)px[y][2 * k + 1][0]};
            const HF2 g{(float)px[y][2 * k][1], (float)px[y][2 * k + 1][1]};
            const HF2 b{(float)px[y][2 * k][2], (float)px[y][2 * k + 1][2]};
            in[k] = jx_pixel<PO, CH>(r, g, b);
        }
        jx_fdct8_pk<HostPair>(in, Tp[y]);
    }
    long long bad = 0;
    const float magic = 12582912.0f;
    for (int j = 0; j < 4; j++) {
        HF2 col[8], out[8];
        for (int y = 0; y < 8; y++) col[y] = Tp[y][j];
        jx_fdct8<PO>(col, out);
        for (int v = 0; v < 8; v++)
            for (int l = 0; l < 2; l++) {
                const int u = jx_pk_k(j, l);
                const float Fp = l ? out[v].y : out[v].x;
                if (bits(Fp) != bits(Fs[v][u])) bad++;
                /* quantiser: tm = fma(F,w,M), d = fma(F,w,-(tm-M)) in both forms */
                const float ww = w[v * 8 + u];
                const HF2 Fw = HostPair::mk(Fp, Fp), W = HostPair::mk(ww, ww);
                const HF2 tm = HostPair::fma(Fw, W, HostPair::mk(magic, magic));
                const HF2 rr = HostPair::sub(tm, HostPair::mk(magic, magic));
                const HF2 d = HostPair::fma(Fw, W, HostPair::mk(-rr.x, -rr.y));
                const float tms = fmaf(Fs[v][u], ww, magic), ds = fmaf(Fs[v][u], ww, -(tms - magic));
                if (bits(tm.x) != bits(tms) || bits(d.x) != bits(ds)) bad++;
            }
    }
    return bad;
}
}  // namespace

extern "C" long long jx_selftest_pk(long long nblocks, unsigned long long seed)
{
    float w[3][64], lim[3][64];
    int16_t q[2][64];
    jx_plan_tables(90, w, lim, q);
    uint64_t s = seed;
    long long bad = 0;
    uint8_t px[8][8][3];
    for (long long n = 0; n < nblocks; n++) {
        const int kind = (int)(n % 4);  /* random, flat, two-level, ramps */
        const uint64_t r0 = sm64(s);
        for (int y = 0; y < 8; y++)
            for (int x = 0; x < 8; x++)
                for (int c = 0; c < 3; c++) {
                    uint8_t v;
                    if (kind == 0) v = (uint8_t)(sm64(s) >> 56);
                    else if (kind == 1) v = (uint8_t)(r0 >> (8 * c));
                    else if (kind == 2) v = ((r0 >> (x + 8 * y)) & 1) ? 255 : (uint8_t)(r0 >> 40);
                    else v = (uint8_t)((x * (int)(r0 & 31) + y * (int)((r0 >> 5) & 31) + c * 7) & 255);
                    px[y][x][c] = v;
                }
        bad += block_mismatch<0>(px, w[0]) + block_mismatch<1>(px, w[1]) + block_mismatch<2>(px, w[2]);
    }
    return bad;
}

extern "C" {

}  /* extern "C" */

/* ---- k_mx: colour conversion + row DCT as one f16 MFMA product --------------------------
 *
 * k_mx multiplies each pixel row, 24 bytes b_k (k = 3x + p, plane p of pixel x), by B[k][n] =
 * a[c][p] cos((2x+1)u pi/16), n = 8c + u, with a bias row (input 1.0) carrying the level shift,
 * -8 * 128 for Y at u = 0 (preprocess.c:160-162,186-188: Y - 128; the level-shifted chroma has
 * no constant; the true cosines of u > 0 sum to 0).  B is split into JX_MX_PARTS f16 parts:
 *   Bh  B rounded to a multiple of 2^-11 (|B| < 1: 11 bits; bias: its f16),
 *   Bl  2^12 (B - Bh),  [Bm  2^12 (B - Bh) - Bl]   (each rounded to f16).
 * Encoding (the kernel's A is one v_perm per two bytes): A holds the byte zero-extended to 16
 * bits, i.e. the f16 subnormal b 2^-24 (exact), the bias lanes 1.0; B's byte rows are stored
 * x 2^15 and the bias row x 2^-9, so every product is b B 2^-9 (exact in fp32) and the MFMA's
 * results are R 2^-9.  Scaling by a power of two changes no rounding, so the kernel's fp32
 * values are those of the true-scale arithmetic below times 2^-9 bit for bit; the column pass
 * scales with them, and the quantiser's w x 2^9 (JX_MX_RSCALE) gives the very fp32 F w.
 * acc_h = sum_k b_k Bh_k is EXACT whatever the order of the MFMA's additions: every product
 * and every partial sum is a multiple of 2^-11 below 2^13 in magnitude (24 bits).  acc_l =
 * sum_k b_k (Bl_k [+ Bm_k]) 2^-12 is below 1 in magnitude; each of its additions is charged
 * one ulp.  R = fl(acc_h + 2^-12 acc_l) (one fma) then enters the column pass (jx_fdct8,
 * FOps, two blocks per v_pk_* pair) as usual.
 *
 * Operand layout (v_mfma_f32_16x16x32_f16: lane l holds A[row l & 15][k = 8 (l >> 4) + e] and
 * B[k = 8 (l >> 4) + e][column l & 15], e = 0..7): k < 24 is byte k of the pixel row, k = 24
 * the bias (A = 1.0), k > 24 weight 0.  Three B matrices ("which"): 0 = columns j = 8c + u for
 * c = Y, Cb; 1 = Cr at u = j for j < 8, zero columns j >= 8; 2 = zero columns j < 8, Cr at
 * u = j - 8 for j >= 8 (k_mx sums A_set0 B1 + A_set1 B2: the two sets concatenated along K).
 */
static const double kMxA[3][3] = {{0.299, 0.587, 0.114},
                                  {-0.168736, 0.331264, -0.5},
                                  {0.5, -0.418688, -0.081312}};

/* round to the nearest f16 (ties to even); bit pattern in *bits */
static long double f16_round(long double x, uint16_t *bits)
{
    if (x == 0) {
        *bits = 0;
        return 0;
    }
    const int e = ilogbl(x);
    const int qe = std::max(e - 10, -24);
    const long double v = rintl(ldexpl(x, -qe)) * ldexpl(1.0L, qe);
    const long double av = fabsl(v);
    uint16_t s = v < 0 ? 0x8000 : 0;
    const int ev = ilogbl(av);
    if (ev < -14) {
        s |= (uint16_t)llrintl(ldexpl(av, 24));
    } else {
        const long long mant = llrintl(ldexpl(av, 10 - ev)) - 1024;
        s |= (uint16_t)(((ev + 15) << 10) | mant);
    }
    *bits = s;
    return v;
}

/* exact B[k][n] (k < 24: matrix, k = 24: bias row; n < 24) */
static long double mx_exact(int k, int n)
{
    if (n >= 24) return 0;
    const int c = n / 8, u = n % 8;
    const long double pi = 3.141592653589793238462643383279502884L;
    if (k < 24) {
        const int x = k / 3, p = k % 3;
        return (long double)kMxA[c][p] * cosl((2 * x + 1) * u * pi / 16);
    }
    if (k == 24 && u == 0 && c == 0) return -1024.0L;
    return 0;
}

/* f16 encodings of the split parts (see above): a byte row's value x 2^15, the bias row's
 * x 2^-9; returns the true-scale value the encoding represents */
constexpr int kMxBExp = 15, kMxBiasExp = -9;
static long double mx_enc(long double v, bool bias, uint16_t *bits)
{
    const int e = bias ? kMxBiasExp : kMxBExp;
    return ldexpl(f16_round(ldexpl(v, e), bits), -e);
}

struct MxSplit {
    long double h[25][32], l[25][32], m[25][32];      /* m = 0 unless JX_MX_PARTS == 3 */
    uint16_t bh[25][32], bl[25][32], bm[25][32];
};

static int mx_split(MxSplit &S)
{
    memset(&S, 0, sizeof S);
    for (int k = 0; k < 25; k++)
        for (int n = 0; n < 24; n++) {
            const long double B = mx_exact(k, n);
            const bool bias = k == 24;
            const long double hv = mx_enc(bias ? B : rintl(ldexpl(B, 11)) / 2048.0L, bias, &S.bh[k][n]);
            if (ldexpl(hv, 11) != rintl(ldexpl(hv, 11))) return JPGX_EARG;
            S.h[k][n] = hv;
            /* the lo parts are stored scaled by 2^JX_MX_LOEXP (round 4: 2^0); k_mx takes R =
             * acc_h + 2^-LOEXP acc_l, exact scaling.  S.l / S.m hold the unscaled values. */
            const long double ls = mx_enc(ldexpl(B - hv, JX_MX_LOEXP), bias, &S.bl[k][n]);
            S.l[k][n] = ldexpl(ls, -JX_MX_LOEXP);
            if (JX_MX_PARTS == 3) {
                const long double ms = mx_enc(ldexpl(B - hv, JX_MX_LOEXP) - ls, bias, &S.bm[k][n]);
                S.m[k][n] = ldexpl(ms, -JX_MX_LOEXP);
            }
        }
    for (int n = 0; n < 24; n++) {              /* acc_h exactness: partial sums < 2^13 */
        long double sh = fabsl(S.h[24][n]);
        for (int k = 0; k < 24; k++) sh += 255.0L * fabsl(S.h[k][n]);
        if (sh >= 8192.0L) return JPGX_EARG;
    }
    return JPGX_OK;
}

extern "C" int jx_mx_parts(void) { return JX_MX_PARTS; }
extern "C" int jx_mx_loexp(void) { return JX_MX_LOEXP; }

extern "C" int jx_mx_operands(uint16_t ops[3 * JX_MX_PARTS][64][8])
{
    std::unique_ptr<MxSplit> S_(new MxSplit);   /* heap, per call: reentrant across threads */
    MxSplit &S = *S_;
    const int rc = mx_split(S);
    if (rc) return rc;
    /* operand 3 * part + which; lane l holds B[k = 8 (l >> 4) + e][plan column of l & 15] */
    for (int part = 0; part < JX_MX_PARTS; part++)
        for (int which = 0; which < 3; which++)
            for (int l = 0; l < 64; l++)
                for (int e = 0; e < 8; e++) {
                    const int k = 8 * (l >> 4) + e, j = l & 15;
                    int n = -1;
                    if (which == 0) n = j;
                    else if (which == 1 && j < 8) n = 16 + j;
                    else if (which == 2 && j >= 8) n = 16 + j - 8;
                    uint16_t v = 0;
                    if (n >= 0 && k <= 24)
                        v = part == 0 ? S.bh[k][n] : (part == 1 ? S.bl[k][n] : S.bm[k][n]);
                    ops[3 * part + which][l][e] = v;
                }
    return JPGX_OK;
}

/* Interval + error bound of R (the column pass input) for column n = 8c + u. */
static Bnd mx_row_bound(const MxSplit &S, int n)
{
    long double loh = S.h[24][n], hih = S.h[24][n];
    long double lol = S.l[24][n] + S.m[24][n], hil = lol;
    long double sl = fabsl(S.l[24][n]) + fabsl(S.m[24][n]);
    long double rep = fabsl(mx_exact(24, n) - S.h[24][n] - S.l[24][n] - S.m[24][n]);
    for (int k = 0; k < 24; k++) {             /* bytes 0..255 */
        const long double bh = S.h[k][n], bo = S.l[k][n] + S.m[k][n];
        loh += std::min(0.0L, 255.0L * bh);
        hih += std::max(0.0L, 255.0L * bh);
        lol += std::min(0.0L, 255.0L * bo);
        hil += std::max(0.0L, 255.0L * bo);
        sl += 255.0L * (fabsl(S.l[k][n]) + fabsl(S.m[k][n]));
        rep += 255.0L * fabsl(mx_exact(k, n) - S.h[k][n] - S.l[k][n] - S.m[k][n]);
    }
    /* acc_l: per lo part one MFMA of 32 products (K = 32: 25 weights, 7 zeros; the Cr tile's
     * second, K-concatenated MFMA adds exact zeros in every column) plus the accumulator input;
     * every addition charged one ulp of the magnitude bound, twice over for an unknown
     * summation tree and rounding mode */
    const double nadd = 2.0 * (33.0 * (JX_MX_PARTS - 1));
    const double el = (double)(nadd * sl * 0x1p-23L + rep);
    return BoundOps::add(Bnd{(double)loh, (double)hih, 0.0},
                         Bnd{(double)lol - el, (double)hil + el, el});
}

extern "C" int jx_plan_tables_mx(int quality, float w[24][8], float lim[24][8], int16_t q[2][64])
{
    int qs[2][8][8];
    int rc = jpgx_scale_table(0, quality, qs[0]);
    if (rc) return rc;
    jpgx_scale_table(1, quality, qs[1]);
    for (int t = 0; t < 2; t++)
        for (int u = 0; u < 8; u++)
            for (int v = 0; v < 8; v++) q[t][u * 8 + v] = (int16_t)qs[t][u][v];
    std::unique_ptr<MxSplit> S_(new MxSplit);   /* heap, per call: reentrant across threads */
    MxSplit &S = *S_;
    rc = mx_split(S);
    if (rc) return rc;
    const long double a0 = 1.0L / sqrtl(2.0L);
    for (int n = 0; n < 24; n++) {
        const int c = n / 8, u = n % 8, t = c == 0 ? 0 : 1;
        const Bnd R = mx_row_bound(S, n);
        Bnd col[8], out[8];
        for (int y = 0; y < 8; y++) col[y] = R;
        jx_fdct8<BoundOps>(col, out);
        for (int v = 0; v < 8; v++) {
            const long double au = u == 0 ? a0 : 1.0L, av = v == 0 ? a0 : 1.0L;
            const long double ws = 0.25L * au * av * dct_kfactor(v) / (long double)qs[t][u][v];
            const float wf = (float)ws;
            const Bnd &b = out[v];
            const double mF = BoundOps::mag(b) + b.E;
            double et = b.E * fabs((double)wf) + mF * (double)fabsl((long double)wf - ws) + 0x1p-25;
            et = et * 1.01 + 1e-7;
            w[n][v] = wf;
            lim[n][v] = (float)(0.5 - et);
        }
    }
    return JPGX_OK;
}

/* ---- k_mx422 / k_mx420: true 4:2:2 / 4:2:0 on the matrix cores --------------------------
 *
 * Y is k_mx's Y (plan columns n = u, the 4:4:4 split S), its B laid out K-concatenated: the
 * product A_set0 B_Y0 + A_set1 B_Y1 puts set 0's blocks in C columns 0..7 and set 1's in
 * 8..15 (B_Y0 zero in columns 8..15, B_Y1 zero in 0..7), exactly as k_mx's Cr tile.
 * Chroma (the EXTENSION's definition, oracle/cpu_ref.c cpuref_chroma_sample): a chroma row of a
 * chroma block is, for 4:2:2 (sub 1), the 16 pixels (48 bytes) of one pixel row of its MCU, the
 * sample X the average of pixels 2X, 2X+1 of the level-shifted chroma; for 4:2:0 (sub 2) the 16
 * pixels of two pixel rows (96 bytes, k = 48 r + 3x + p), the sample the average of the 2 x 2
 * quad.  The row transform is linear in the bytes:
 *   R(u) = sum_{r, x < 16, p} b_{48r+3x+p} w a[c][p] cos((2 floor(x/2) + 1) u pi/16),
 * w = 1/2 (4:2:2) or 1/4 (4:2:0), a = kMxA[c], c = Cb, Cr, b = the byte (the level-shifted
 * chroma has no constant: no bias row), n = 8 c' + u (c' = 0 Cb, 1 Cr).  K = 32 MFMAs over
 * k = 0..31, 32..63 [, 64..95].  Same encoding and split as k_mx: Bh a multiple of 2^-11 (acc_h
 * exact in any order: every partial sum a multiple of 2^-11 below 2^13), the lo part(s) scaled
 * by 2^12, each of acc_l's additions charged one ulp (65 per 4:2:2 chroma row, 97 per 4:2:0 one:
 * 32 products per MFMA plus the accumulator).
 */
static int mxc_nk(int sub) { return 48 * sub; }
static int mxc_ksteps(int sub) { return sub == 1 ? 2 : 3; }

static long double mxc_exact(int sub, int k, int n)
{
    if (n >= 16 || k >= mxc_nk(sub)) return 0;
    const int c = 1 + n / 8, u = n % 8, kk = k % 48, x = kk / 3, p = kk % 3;
    const long double pi = 3.141592653589793238462643383279502884L;
    return (sub == 1 ? 0.5L : 0.25L) * (long double)kMxA[c][p] * cosl((2 * (x / 2) + 1) * u * pi / 16);
}

struct MxcSplit {
    long double h[96][16], l[96][16], m[96][16];
    uint16_t bh[96][16], bl[96][16], bm[96][16];
};

static int mxc_split(int sub, MxcSplit &S)
{
    memset(&S, 0, sizeof S);
    const int nk = mxc_nk(sub);
    for (int k = 0; k < nk; k++)
        for (int n = 0; n < 16; n++) {
            const long double B = mxc_exact(sub, k, n);
            const long double hv = mx_enc(rintl(ldexpl(B, 11)) / 2048.0L, false, &S.bh[k][n]);
            if (ldexpl(hv, 11) != rintl(ldexpl(hv, 11))) return JPGX_EARG;
            S.h[k][n] = hv;
            const long double ls = mx_enc(ldexpl(B - hv, JX_MX_LOEXP), false, &S.bl[k][n]);
            S.l[k][n] = ldexpl(ls, -JX_MX_LOEXP);
            if (JX_MX_PARTS == 3) {
                const long double ms = mx_enc(ldexpl(B - hv, JX_MX_LOEXP) - ls, false, &S.bm[k][n]);
                S.m[k][n] = ldexpl(ms, -JX_MX_LOEXP);
            }
        }
    for (int n = 0; n < 16; n++) {              /* acc_h exactness: partial sums < 2^13 */
        long double sh = 0;
        for (int k = 0; k < nk; k++) sh += 255.0L * fabsl(S.h[k][n]);
        if (sh >= 8192.0L) return JPGX_EARG;
    }
    return JPGX_OK;
}

/* operand [part][which][lane][e]: which 0 / 1 = Y of set 0 / set 1 (K = 32: 24 bytes + bias),
 * 2.. = chroma k-steps (k = 32 (which - 2) + 8 (l >> 4) + e); lane l holds B[k][column l & 15] */
static int mxc_operands(int sub, uint16_t (*ops)[5][64][8])
{
    std::unique_ptr<MxSplit> S_(new MxSplit);   /* heap, per call: reentrant across threads */
    MxSplit &S = *S_;
    std::unique_ptr<MxcSplit> C_(new MxcSplit);
    MxcSplit &C = *C_;
    int rc = mx_split(S);
    if (!rc) rc = mxc_split(sub, C);
    if (rc) return rc;
    for (int part = 0; part < JX_MX_PARTS; part++)
        for (int which = 0; which < 5; which++)
            for (int l = 0; l < 64; l++)
                for (int e = 0; e < 8; e++) {
                    const int j = l & 15;
                    uint16_t v = 0;
                    if (which < 2) {
                        const int k = 8 * (l >> 4) + e;
                        const bool on = which == 0 ? j < 8 : j >= 8;
                        if (on && k <= 24) {
                            const int n = j & 7;
                            v = part == 0 ? S.bh[k][n] : (part == 1 ? S.bl[k][n] : S.bm[k][n]);
                        }
                    } else {
                        const int k = 32 * (which - 2) + 8 * (l >> 4) + e;
                        if (k < mxc_nk(sub)) v = part == 0 ? C.bh[k][j] : (part == 1 ? C.bl[k][j] : C.bm[k][j]);
                    }
                    ops[part][which][l][e] = v;
                }
    return JPGX_OK;
}

extern "C" int jx_mx422_operands(uint16_t ops[JX_MX_PARTS][4][64][8])
{
    std::unique_ptr<uint16_t[][5][64][8]> o5(new uint16_t[JX_MX_PARTS][5][64][8]);
    const int rc = mxc_operands(1, o5.get());
    if (rc) return rc;
    for (int part = 0; part < JX_MX_PARTS; part++) memcpy(ops[part], o5[part], sizeof ops[part]);
    return JPGX_OK;
}

extern "C" int jx_mx420_operands(uint16_t ops[JX_MX_PARTS][5][64][8])
{
    return mxc_operands(2, ops);
}

/* Interval + error bound of a chroma row transform R (column n = 8 c' + u) */
static Bnd mxc_row_bound(int sub, const MxcSplit &S, int n)
{
    long double loh = 0, hih = 0, lol = 0, hil = 0, sl = 0, rep = 0;
    for (int k = 0; k < mxc_nk(sub); k++) {    /* bytes 0..255 */
        const long double bh = S.h[k][n], bo = S.l[k][n] + S.m[k][n];
        loh += std::min(0.0L, 255.0L * bh);
        hih += std::max(0.0L, 255.0L * bh);
        lol += std::min(0.0L, 255.0L * bo);
        hil += std::max(0.0L, 255.0L * bo);
        sl += 255.0L * (fabsl(S.l[k][n]) + fabsl(S.m[k][n]));
        rep += 255.0L * fabsl(mxc_exact(sub, k, n) - S.h[k][n] - S.l[k][n] - S.m[k][n]);
    }
    /* acc_l: per lo part mxc_ksteps MFMAs of 32 products plus the accumulator input, every
     * addition charged one ulp of the magnitude bound, twice over (unknown summation tree and
     * rounding mode) */
    const double nadd = 2.0 * ((32.0 * mxc_ksteps(sub) + 1.0) * (JX_MX_PARTS - 1));
    const double el = (double)(nadd * sl * 0x1p-23L + rep);
    return BoundOps::add(Bnd{(double)loh, (double)hih, 0.0},
                         Bnd{(double)lol - el, (double)hil + el, el});
}

/* plan columns n = 8 c + u as jx_mxtab: c = 0 Y (k_mx's bound), 1 Cb, 2 Cr (subsampled rows) */
static int mxc_plan_tables(int sub, int quality, float w[24][8], float lim[24][8], int16_t q[2][64])
{
    int qs[2][8][8];
    int rc = jpgx_scale_table(0, quality, qs[0]);
    if (rc) return rc;
    jpgx_scale_table(1, quality, qs[1]);
    for (int t = 0; t < 2; t++)
        for (int u = 0; u < 8; u++)
            for (int v = 0; v < 8; v++) q[t][u * 8 + v] = (int16_t)qs[t][u][v];
    std::unique_ptr<MxSplit> S_(new MxSplit);   /* heap, per call: reentrant across threads */
    MxSplit &S = *S_;
    std::unique_ptr<MxcSplit> C_(new MxcSplit);
    MxcSplit &C = *C_;
    rc = mx_split(S);
    if (!rc) rc = mxc_split(sub, C);
    if (rc) return rc;
    const long double a0 = 1.0L / sqrtl(2.0L);
    for (int n = 0; n < 24; n++) {
        const int c = n / 8, u = n % 8, t = c == 0 ? 0 : 1;
        const Bnd R = c == 0 ? mx_row_bound(S, n) : mxc_row_bound(sub, C, n - 8);
        Bnd col[8], out[8];
        for (int y = 0; y < 8; y++) col[y] = R;
        jx_fdct8<BoundOps>(col, out);
        for (int v = 0; v < 8; v++) {
            const long double au = u == 0 ? a0 : 1.0L, av = v == 0 ? a0 : 1.0L;
            const long double ws = 0.25L * au * av * dct_kfactor(v) / (long double)qs[t][u][v];
            const float wf = (float)ws;
            const Bnd &b = out[v];
            const double mF = BoundOps::mag(b) + b.E;
            double et = b.E * fabs((double)wf) + mF * (double)fabsl((long double)wf - ws) + 0x1p-25;
            et = et * 1.01 + 1e-7;
            w[n][v] = wf;
            lim[n][v] = (float)(0.5 - et);
        }
    }
    return JPGX_OK;
}

extern "C" int jx_plan_tables_mx422(int quality, float w[24][8], float lim[24][8], int16_t q[2][64])
{
    return mxc_plan_tables(1, quality, w, lim, q);
}

extern "C" int jx_plan_tables_mx420(int quality, float w[24][8], float lim[24][8], int16_t q[2][64])
{
    return mxc_plan_tables(2, quality, w, lim, q);
}

/* Host emulation of the subsampled chroma fast path (acc_h exact, acc_l in fp32, R = fl(acc_h +
 * 2^-12 acc_l), FOps column pass, quantiser) against the definition's exact quotient on random
 * MCUs: unflagged mismatches (must be 0), flagged count, worst error / band. */
static long long mxc_selftest(int sub, long long nblocks, unsigned long long seed, int quality,
                              long long *flagged, double *ratio)
{
    std::unique_ptr<MxcSplit> C_(new MxcSplit);
    MxcSplit &C = *C_;
    if (mxc_split(sub, C)) return -1;
    float w[24][8], lim[24][8];
    int16_t q[2][64];
    if (mxc_plan_tables(sub, quality, w, lim, q)) return -1;
    const long double pi = 3.141592653589793238462643383279502884L;
    const long double a0 = 1.0L / sqrtl(2.0L);
    const int nk = mxc_nk(sub);
    uint64_t s = seed;
    long long bad = 0, nfl = 0;
    double worst = 0;
    for (long long bk = 0; bk < nblocks; bk++) {
        int px[8][96];                          /* chroma row y: [r][16 pixels][3] */
        for (int y = 0; y < 8; y++)
            for (int k = 0; k < nk; k++) {
                s = s * 6364136223846793005ULL + 1442695040888963407ULL;
                px[y][k] = (int)(s >> 56);
                if ((bk & 3) == 1) px[y][k] = px[0][k % 3];      /* flat blocks too */
                if ((bk & 3) == 2) px[y][k] = (k % 3 == 0) ? 255 : 0;
            }
        for (int n = 0; n < 16; n++) {
            const int c = 1 + n / 8, u = n % 8, pn = 8 + n;
            float R[8];
            for (int y = 0; y < 8; y++) {
                long double ah = 0;
                float al = 0.0f;
                for (int k = 0; k < nk; k++) {
                    const int sv = px[y][k];
                    ah += sv * C.h[k][n];
                    al = al + (float)(sv * C.l[k][n]);
                    if (JX_MX_PARTS == 3) al = al + (float)(sv * C.m[k][n]);
                }
                R[y] = (float)ah + al;
            }
            float F[8];
            jx_fdct8<FOps>(R, F);
            for (int v = 0; v < 8; v++) {
                long double sum = 0;
                for (int y = 0; y < 8; y++)
                    for (int X = 0; X < 8; X++) {
                        long double cs = 0;
                        for (int r = 0; r < sub; r++)
                            for (int h = 0; h < 2; h++) {
                                const int x = 2 * X + h, o = 48 * r + 3 * x;
                                cs += (long double)kMxA[c][0] * px[y][o] + (long double)kMxA[c][1] * px[y][o + 1] +
                                      (long double)kMxA[c][2] * px[y][o + 2];
                            }
                        sum += (sub == 1 ? 0.5L : 0.25L) * cs * cosl((2 * X + 1) * u * pi / 16) *
                               cosl((2 * y + 1) * v * pi / 16);
                    }
                const long double au = u == 0 ? a0 : 1.0L, av = v == 0 ? a0 : 1.0L;
                const long double qx = 0.25L * au * av * sum / q[1][u * 8 + v];
                const float tm = fmaf(F[v], w[pn][v], 12582912.0f);
                const float rr = tm - 12582912.0f;
                const float d = fmaf(F[v], w[pn][v], -rr);
                const double qf = (double)F[v] * (double)w[pn][v];
                const double band = 0.5 - (double)lim[pn][v];
                worst = std::max(worst, (double)fabsl((long double)qf - qx) / band);
                if (fabsf(d) >= lim[pn][v]) {
                    nfl++;
                    continue;
                }
                if ((long double)rr != roundl(qx)) bad++;
            }
        }
    }
    if (flagged) *flagged = nfl;
    if (ratio) *ratio = worst;
    return bad;
}

extern "C" long long jx_selftest_mx422(long long nblocks, unsigned long long seed, int quality,
                                       long long *flagged, double *ratio)
{
    return mxc_selftest(1, nblocks, seed, quality, flagged, ratio);
}

extern "C" long long jx_selftest_mx420(long long nblocks, unsigned long long seed, int quality,
                                       long long *flagged, double *ratio)
{
    return mxc_selftest(2, nblocks, seed, quality, flagged, ratio);
}

/* Host emulation of k_mx's fast path on random blocks (acc_h exact, acc_l summed in fp32,
 * R = fl(acc_h + acc_l), then the kernel's FOps column pass and quantiser): counts the
 * coefficients whose unflagged fp32 result differs from round(exact quotient) (must be 0)
 * and the flagged ones.  ratio[0] = max |fp32 quotient - exact| / (0.5 - lim). */
extern "C" long long jx_selftest_mx(long long nblocks, unsigned long long seed, int quality,
                                    long long *flagged, double *ratio)
{
    std::unique_ptr<MxSplit> S_(new MxSplit);   /* heap, per call: reentrant across threads */
    MxSplit &S = *S_;
    if (mx_split(S)) return -1;
    float w[24][8], lim[24][8];
    int16_t q[2][64];
    if (jx_plan_tables_mx(quality, w, lim, q)) return -1;
    const long double pi = 3.141592653589793238462643383279502884L;
    const long double a0 = 1.0L / sqrtl(2.0L);
    uint64_t s = seed;
    long long bad = 0, nfl = 0;
    double worst = 0;
    for (long long bk = 0; bk < nblocks; bk++) {
        int px[8][24];
        for (int y = 0; y < 8; y++)
            for (int k = 0; k < 24; k++) {
                s = s * 6364136223846793005ULL + 1442695040888963407ULL;
                px[y][k] = (int)(s >> 56);
                if ((bk & 3) == 1) px[y][k] = px[0][k % 3];      /* flat blocks too */
            }
        for (int n = 0; n < 24; n++) {
            const int c = n / 8, u = n % 8;
            float R[8];
            for (int y = 0; y < 8; y++) {
                long double ah = S.h[24][n];
                float al = (float)(S.l[24][n] + S.m[24][n]);
                for (int k = 0; k < 24; k++) {
                    const int sv = px[y][k];
                    ah += sv * S.h[k][n];
                    al = al + (float)(sv * S.l[k][n]);
                    if (JX_MX_PARTS == 3) al = al + (float)(sv * S.m[k][n]);
                }
                R[y] = (float)ah + al;
            }
            float F[8];
            jx_fdct8<FOps>(R, F);
            for (int v = 0; v < 8; v++) {
                /* exact: 1/4 a(u) a(v) sum_x sum_y X c_u(x) c_v(y) / Q, X from double colours */
                long double sum = 0;
                for (int y = 0; y < 8; y++)
                    for (int x = 0; x < 8; x++) {
                        long double X = (long double)kMxA[c][0] * px[y][3 * x] +
                                        (long double)kMxA[c][1] * px[y][3 * x + 1] +
                                        (long double)kMxA[c][2] * px[y][3 * x + 2];
                        X += c == 0 ? -128.0L : 0.0L;
                        sum += X * cosl((2 * x + 1) * u * pi / 16) * cosl((2 * y + 1) * v * pi / 16);
                    }
                const long double au = u == 0 ? a0 : 1.0L, av = v == 0 ? a0 : 1.0L;
                const long double qx = 0.25L * au * av * sum / q[c == 0 ? 0 : 1][u * 8 + v];
                const float tm = fmaf(F[v], w[n][v], 12582912.0f);
                const float rr = tm - 12582912.0f;
                const float d = fmaf(F[v], w[n][v], -rr);
                const double qf = (double)F[v] * (double)w[n][v];
                const double band = 0.5 - (double)lim[n][v];
                worst = std::max(worst, (double)fabsl((long double)qf - qx) / band);
                if (fabsf(d) >= lim[n][v]) {
                    nfl++;
                    continue;
                }
                if ((long double)rr != roundl(qx)) bad++;
            }
        }
    }
    if (flagged) *flagged = nfl;
    if (ratio) *ratio = worst;
    return bad;
}
