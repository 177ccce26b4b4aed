"""CPU check of the exact pass's fast decision (csrc/jpgx_mx.hip mx_exact_sum / mx_exact_one): the
device forms t' = fl(s_par R) with R = fl(K / Q) (jx_mxtab.r, MxExLds::recip) from a tree-ordered
fp64 sum s_par; when |frac(|t'|) - 1/2| > 2^-33, rint(t') must equal round() of the reference's
t = fl(fl(K s_seq) / Q) from its sequential sum (dct.c:46-54, quantise.c:58).  Both device trees are
modelled: the 8-lane groups' (8 in-lane additions + 3 butterfly levels) and the whole wave's of a
single flagged coefficient (6 levels: x ^ 1, x ^ 2, 7 - x, row_mirror, permlane16 / permlane32
swaps).  Random, extreme and tie-heavy blocks, in numpy fp64 (IEEE double, one rounding per op)."""
import numpy as np

M = 2.0 ** -33
ALPHA0 = 1.0 / np.sqrt(2.0)


def _cos():
    c = np.empty((8, 8))
    for k in range(8):
        for x in range(8):
            c[k, x] = np.cos(((2 * x + 1) * k * np.pi) / 16)
    return c


def _round_away(t):
    a = np.abs(t)
    r = np.floor(a)
    r = r + (a - r >= 0.5)
    return np.sign(t) * r


def _decide(X, u, v, q, wave=False):
    """X: (N, 8, 8) [x][y] level-shifted values; returns (reference, fast, decided)"""
    C = _cos()
    cu, cv = C[u][:, :, None], C[v][:, None, :]          # (N, 8, 1), (N, 1, 8)
    t = (X * cu) * cv                                      # (N, x, y): fl(fl(X cu) cv)
    seq = np.zeros(X.shape[0])
    for x in range(8):
        for y in range(8):
            seq = seq + t[:, x, y]
    if wave:
        # mx_exact_one: lane 8 y + x holds t[x, y]; 3 levels over x, then y pairs, quads, halves
        w = t.copy()                                      # (N, x, y)
        w = w + w[:, [1, 0, 3, 2, 5, 4, 7, 6], :]
        w = w + w[:, [2, 3, 0, 1, 6, 7, 4, 5], :]
        w = w + w[:, [7, 6, 5, 4, 3, 2, 1, 0], :]
        assert np.all(w == w[:, :1, :])
        r = w[:, 0, :]                                    # (N, y): the row sums
        r = r + r[:, [1, 0, 3, 2, 5, 4, 7, 6]]            # row_mirror: y pairs
        r = r + r[:, [2, 3, 0, 1, 6, 7, 4, 5]]            # permlane16 swap: y quads
        r = r + r[:, [4, 5, 6, 7, 0, 1, 2, 3]]            # permlane32 swap: halves
        assert np.all(r == r[:, :1])
        par = r[:, 0]
    else:
        lane = t[:, :, 0].copy()
        for y in range(1, 8):
            lane = lane + t[:, :, y]
        l1 = lane + lane[:, [1, 0, 3, 2, 5, 4, 7, 6]]
        l2 = l1 + l1[:, [2, 3, 0, 1, 6, 7, 4, 5]]
        par = l2 + l2[:, [7, 6, 5, 4, 3, 2, 1, 0]]
        assert np.all(par == par[:, :1])                  # every lane holds the same total
        par = par[:, 0]
    qa = np.where(u == 0, 0.25 * ALPHA0, 0.25)
    al = np.where(v == 0, ALPHA0, 1.0)
    K = qa * al
    ref = _round_away((K * seq) / q)
    tp = par * (K / q)                                    # the device: t' = fl(s_par fl(K / Q))
    a = np.abs(tp)
    decided = np.abs((a - np.floor(a)) - 0.5) > M
    return ref, np.rint(tp), decided


def test_fast_decision_matches_the_sequential_sum():
    rng = np.random.default_rng(5)
    n = 200000
    X = rng.uniform(-171.0, 171.0, (n, 8, 8))
    X[: n // 4] = np.where(rng.random((n // 4, 8, 8)) < 0.5, -170.6, 127.0)   # extremes
    X[n // 4: n // 2] = np.round(X[n // 4: n // 2])                            # integer-valued
    u = rng.integers(0, 8, n)
    v = rng.integers(0, 8, n)
    q = rng.integers(1, 256, n).astype(np.float64)
    for wave in (False, True):
        ref, fast, decided = _decide(X, u, v, q, wave)
        assert decided.mean() > 0.99
        assert np.array_equal(ref[decided], fast[decided])


def test_flat_blocks_fall_back():
    """flat blocks: s = 64 X exactly, DC halves are exact ties that only the sequential sum's
    own rounding of K decides -- the fast path must leave them undecided"""
    X = np.repeat(np.arange(-128.0, 128.0)[:, None, None], 64, axis=1).reshape(-1, 8, 8)
    n = X.shape[0]
    u = np.zeros(n, np.int64)
    v = np.zeros(n, np.int64)
    for qv in (1, 2, 4, 8, 16, 32):
        q = np.full(n, float(qv))
        for wave in (False, True):
            ref, fast, decided = _decide(X, u, v, q, wave)
            assert np.array_equal(ref[decided], fast[decided])
            if qv == 16:
                assert not decided.all()                      # X odd: 8 X / 16 is a half
