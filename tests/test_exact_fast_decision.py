"""CPU check of the exact pass's fast decision (csrc/jpgx_mx.hip mx_exact_sum, JX_MX_FASTEXACT):
when the tree-ordered fp64 sum gives t = fl(fl(K s) / Q) with |frac(|t|) - 1/2| > 2^-33, rint(t)
must equal round() of the reference's sequential sum (dct.c:46-54, quantise.c:58) -- here on
random, extreme and tie-heavy blocks, in numpy fp64 (IEEE double, one rounding per operation)."""
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


def _decide(X, u, v, q):
    """X: (N, 8, 8) [x][y] level-shifted values; returns (reference, fast, decided)"""
    C = _cos()
    cu, cv = C[u][:, :, None], C[v][:, None, :]          # (N, 8, 1), (N, 1, 8)
    t = (X * cu) * cv                                      # (N, x, y): fl(fl(X cu) cv)
    seq = np.zeros(X.shape[0])
    for x in range(8):
        for y in range(8):
            seq = seq + t[:, x, y]
    lane = t[:, :, 0].copy()
    for y in range(1, 8):
        lane = lane + t[:, :, y]
    l1 = lane + lane[:, [1, 0, 3, 2, 5, 4, 7, 6]]
    l2 = l1 + l1[:, [2, 3, 0, 1, 6, 7, 4, 5]]
    par = l2 + l2[:, [7, 6, 5, 4, 3, 2, 1, 0]]
    assert np.all(par == par[:, :1])                      # every lane holds the same total
    par = par[:, 0]
    qa = np.where(u == 0, 0.25 * ALPHA0, 0.25)
    al = np.where(v == 0, ALPHA0, 1.0)
    K = qa * al
    ref = _round_away((K * seq) / q)
    tp = (K * par) / q
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
    ref, fast, decided = _decide(X, u, v, q)
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
        ref, fast, decided = _decide(X, u, v, q)
        assert np.array_equal(ref[decided], fast[decided])
        if qv == 16:
            assert not decided.all()                          # X odd: 8 X / 16 is a half
