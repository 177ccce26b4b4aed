/*
 * xform_math.h -- the fast-path arithmetic of the block transform, written ONCE as templates
 * over an "ops" policy so that the same source text is
 *   (a) instantiated with FOps (fp32, explicit FMAs) inside the gfx950 kernel, and
 *   (b) instantiated with BoundOps on the host, which propagates a rigorous interval + error
 *       bound through exactly the same operation sequence.  (b) yields, per quality and per
 *       coefficient, the guard band that decides when the fp32 quotient is too close to a
 *       rounding boundary and must be recomputed by the exact-order fp64 path.
 *
 * Reference semantics being approximated (exact values in real arithmetic):
 *   pixel:  preprocess.c:160-162 then level_shift preprocess.c:186-188
 *   DCT:    dct.c:43-56   F(u,v) = 1/4 a(u) a(v) sum_x sum_y X[y][x] cos((2x+1)u pi/16) cos((2y+1)v pi/16)
 * The 1-D transform below is the unnormalised 8-point DCT-II computed by an even/odd
 * decomposition with each output scaled by a constant (jx_fdct8); nothing is normalised: the
 * scale factors and the quantiser divisor are folded into one per-coefficient w(u,v) on the host.
 */
#ifndef JPGX_XFORM_MATH_H
#define JPGX_XFORM_MATH_H

#if defined(__HIPCC__) || defined(__HIP__)
#define JX_HD __host__ __device__ __forceinline__
#else
#define JX_HD inline
#endif

/* A constant as the kernel uses it (f) and its exact real value (x, to double precision). */
struct jx_const {
    float f;
    double x;
};

#define JX_K(v) jx_const{(float)(v), (double)(v)}

/* cos(k*pi/16), 40 digits */
#define JX_C1 0.9807852804032304491261822361342390369739
#define JX_C2 0.9238795325112867561281831893967882868224
#define JX_C3 0.8314696123025452370787883776179057567386
#define JX_C4 0.7071067811865475244008443621048490392848
#define JX_C5 0.5555702330196022247428308139485328743749
#define JX_C6 0.3826834323650897717284599840303988667613
#define JX_C7 0.1950903220161282678482848684770222409277

/* ---- fp32 policy (device) ------------------------------------------------------------- */
struct FOps {
    typedef float T;
    static JX_HD T add(T a, T b) { return a + b; }
    static JX_HD T sub(T a, T b) { return a - b; }
    static JX_HD T mulc(T a, jx_const k) { return a * k.f; }
    static JX_HD T fmac(T a, jx_const k, T b) { return __builtin_fmaf(a, k.f, b); }
    static JX_HD T lit(jx_const k) { return k.f; }
};

/*
 * Pixel value of channel CH from the three input bytes (reference planes 0,1,2 = "r,g,b"),
 * level shift included:  Y-128,  Cb-128 = -(0.168736r - 0.331264g + 0.5b),
 * Cr-128 = 0.5r - 0.418688g - 0.081312b.
 */
template <class O, int CH>
JX_HD typename O::T jx_pixel(typename O::T r, typename O::T g, typename O::T b)
{
    if (CH == 0)
        return O::fmac(r, JX_K(0.299), O::fmac(g, JX_K(0.587), O::fmac(b, JX_K(0.114), O::lit(JX_K(-128.0)))));
    if (CH == 1)
        return O::fmac(r, JX_K(-0.168736), O::fmac(g, JX_K(0.331264), O::mulc(b, JX_K(-0.5))));
    return O::fmac(r, JX_K(0.5), O::fmac(g, JX_K(-0.418688), O::mulc(b, JX_K(-0.081312))));
}

/*
 * Unnormalised, SCALED 8-point DCT-II, even/odd split, 28 ops: out[k] = sum_x in[x]
 * cos((2x+1)k pi/16) / f(k), with f(0) = 1, f(4) = C4, f(2) = C2, f(6) = -C2, f(k odd) = Ck.
 * Each output's factor is the one that makes its first term a plain addend (no product): the
 * odd outputs are d0 + (Ck'/Ck) d1 + ..., the (2, 6) rotation e2 + (C6/C2) e3 and
 * e3 - (C6/C2) e2.  The factors go into the per-coefficient scale w(u,v) on the host
 * (jpgx_plan.cpp dct_kfactor evaluates them from this very code).  Round 4: 34 -> 28 ops.
 */
#define JX_KR(a, b) jx_const{(float)((a) / (b)), (double)((a) / (b))}
template <class O>
JX_HD void jx_fdct8(const typename O::T *in, typename O::T *out)
{
    typedef typename O::T T;
    const T s0 = O::add(in[0], in[7]), d0 = O::sub(in[0], in[7]);
    const T s1 = O::add(in[1], in[6]), d1 = O::sub(in[1], in[6]);
    const T s2 = O::add(in[2], in[5]), d2 = O::sub(in[2], in[5]);
    const T s3 = O::add(in[3], in[4]), d3 = O::sub(in[3], in[4]);
    const T e0 = O::add(s0, s3), e1 = O::add(s1, s2);
    const T e2 = O::sub(s0, s3), e3 = O::sub(s1, s2);
    out[0] = O::add(e0, e1);
    out[4] = O::sub(e0, e1);
    out[2] = O::fmac(e3, JX_KR(JX_C6, JX_C2), e2);
    out[6] = O::fmac(e2, JX_KR(-JX_C6, JX_C2), e3);
    out[1] = O::fmac(d3, JX_KR(JX_C7, JX_C1), O::fmac(d2, JX_KR(JX_C5, JX_C1), O::fmac(d1, JX_KR(JX_C3, JX_C1), d0)));
    out[3] = O::fmac(d3, JX_KR(-JX_C5, JX_C3), O::fmac(d2, JX_KR(-JX_C1, JX_C3), O::fmac(d1, JX_KR(-JX_C7, JX_C3), d0)));
    out[5] = O::fmac(d3, JX_KR(JX_C3, JX_C5), O::fmac(d2, JX_KR(JX_C7, JX_C5), O::fmac(d1, JX_KR(-JX_C1, JX_C5), d0)));
    out[7] = O::fmac(d3, JX_KR(-JX_C1, JX_C7), O::fmac(d2, JX_KR(JX_C3, JX_C7), O::fmac(d1, JX_KR(-JX_C5, JX_C7), d0)));
}

/* ---- packed pairs ------------------------------------------------------------------------
 * The same fp32 operations, two per instruction (v_pk_fma_f32 / v_pk_add_f32 / v_pk_mul_f32 on
 * gfx950, whose lane-wise results are those of the scalar instructions).  P is a pair policy:
 *   V           the pair type,  mk(a,b) / lo(v) / hi(v)
 *   add sub mul fma             lane-wise fp32 operations, one rounding each
 * Every function below performs, lane by lane, exactly the scalar operation sequence of the
 * FOps code above, so the guard band bounds (BoundOps over that scalar code) hold unchanged;
 * jx_selftest_pk (jpgx_plan.cpp) checks the equivalence bit for bit on the host.
 */

/* O-policy over pairs: two independent instances of the scalar code, one per lane */
template <class P>
struct PairOps {
    typedef typename P::V T;
    static JX_HD T add(T a, T b) { return P::add(a, b); }
    static JX_HD T sub(T a, T b) { return P::sub(a, b); }
    static JX_HD T mulc(T a, jx_const k) { return P::mul(a, P::mk(k.f, k.f)); }
    static JX_HD T fmac(T a, jx_const k, T b) { return P::fma(a, P::mk(k.f, k.f), b); }
    static JX_HD T lit(jx_const k) { return P::mk(k.f, k.f); }
};

/*
 * One 8-point jx_fdct8 with its work split over the two lanes of every pair: 14 packed
 * operations instead of 28 scalar ones.  in = (x0,x1),(x2,x3),(x4,x5),(x6,x7); out = the
 * pairs (out0,out4),(out2,out6),(out1,out3),(out5,out7).  Swapped and broadcast operands
 * become op_sel modifiers, negated ones neg modifiers (a + (-b) == a - b exactly).
 */
template <class P>
JX_HD void jx_fdct8_pk(const typename P::V *in, typename P::V *out)
{
    typedef typename P::V V;
#define JX_F(a, b) (JX_KR(a, b)).f
    const V x76 = P::mk(P::hi(in[3]), P::lo(in[3])), x54 = P::mk(P::hi(in[2]), P::lo(in[2]));
    const V s01 = P::add(in[0], x76), d01 = P::sub(in[0], x76);   /* (s0,s1), (d0,d1) */
    const V s23 = P::add(in[1], x54), d23 = P::sub(in[1], x54);   /* (s2,s3), (d2,d3) */
    const V s32 = P::mk(P::hi(s23), P::lo(s23));
    const V e01 = P::add(s01, s32), e23 = P::sub(s01, s32);       /* (e0,e1), (e2,e3) */
    /* (e0+e1, e0-e1) as fma(e1, (1,-1), e0): fma(x, +-1, y) rounds y +- x once, exactly as
     * the scalar add/sub (a lane-dependent sign has no neg modifier) */
    out[0] = P::fma(P::mk(P::hi(e01), P::hi(e01)), P::mk(1.0f, -1.0f), P::mk(P::lo(e01), P::lo(e01)));
    /* (e2 + k e3, e3 - k e2) */
    out[1] = P::fma(P::mk(P::hi(e23), P::lo(e23)), P::mk(JX_F(JX_C6, JX_C2), JX_F(-JX_C6, JX_C2)), e23);
    const V d0 = P::mk(P::lo(d01), P::lo(d01)), d1 = P::mk(P::hi(d01), P::hi(d01));
    const V d2 = P::mk(P::lo(d23), P::lo(d23)), d3 = P::mk(P::hi(d23), P::hi(d23));
    out[2] = P::fma(d3, P::mk(JX_F(JX_C7, JX_C1), JX_F(-JX_C5, JX_C3)),
             P::fma(d2, P::mk(JX_F(JX_C5, JX_C1), JX_F(-JX_C1, JX_C3)),
             P::fma(d1, P::mk(JX_F(JX_C3, JX_C1), JX_F(-JX_C7, JX_C3)), d0)));
    out[3] = P::fma(d3, P::mk(JX_F(JX_C3, JX_C5), JX_F(-JX_C1, JX_C7)),
             P::fma(d2, P::mk(JX_F(JX_C7, JX_C5), JX_F(JX_C3, JX_C7)),
             P::fma(d1, P::mk(JX_F(-JX_C1, JX_C5), JX_F(-JX_C5, JX_C7)), d0)));
#undef JX_F
}

/* coefficient index k of lane 0 / lane 1 of output pair j of jx_fdct8_pk */
JX_HD constexpr int jx_pk_k(int j, int lane)
{
    return lane == 0 ? (j == 0 ? 0 : j == 1 ? 2 : j == 2 ? 1 : 5)
                     : (j == 0 ? 4 : j == 1 ? 6 : j == 2 ? 3 : 7);
}

#endif
