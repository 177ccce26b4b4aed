"""The LDS stage layouts of the MFMA kernels (csrc/jpgx_mx.hip, round 6), restated and checked
against the LDS bank rules of MI355X_MICROARCH.md (LDS section): ds_write_b16 banks are (a / 4) % 32
per 32-lane half; ds_read_b128 banks are (a / 4) % 64 per 16-lane group {0-3, 12-15, 20-27}, ...
 * every block's 64 zig-zag coefficients occupy distinct bytes of its 128-byte slot;
 * each of the 24 (4:4:4) / 16 (4:2:x) column writes of a step is at most 2-way per 32-lane half
   (the minimum: zig-zag rows v = 1..6 put 3-4 of a block's dwords on one dword position mod 4);
 * the 16-byte stage reads of the stores are conflict-free.
PMC (profiles/r06_bank_conflicts.txt): k_mxs 89.3 -> 53.3 SQ_LDS_BANK_CONFLICT cycles per step,
k_mxs422 65.0 -> 41.0, k_mxs420 42.9 -> 24.9."""
from collections import Counter, defaultdict

ZZ = [[0, 1, 5, 6, 14, 15, 27, 28], [2, 4, 7, 13, 16, 26, 29, 42], [3, 8, 12, 17, 25, 30, 41, 43],
      [9, 11, 18, 24, 31, 40, 44, 53], [10, 19, 23, 32, 39, 45, 52, 54], [20, 22, 33, 38, 46, 51, 55, 60],
      [21, 34, 37, 47, 50, 56, 59, 61], [35, 36, 48, 49, 57, 58, 62, 63]]      # zig_zag.c:6-15
G32 = [range(32), range(32, 64)]
G128 = [[0, 1, 2, 3, 12, 13, 14, 15] + list(range(20, 28)), list(range(4, 12)) + [16, 17, 18, 19] + list(range(28, 32))]
G128 += [[x + 32 for x in g] for g in G128]


def mxs_h(s):
    return (5 if s & 1 else 0) ^ (2 if s >= 12 else 0)


def mx2_h(s):
    return (5 if s & 1 else 0) ^ (2 if s & 4 else 0)


def coef(h, s, z):
    return 128 * s + 16 * ((z >> 3) ^ h(s)) + 2 * (z & 7)


def mx_pos(c, jb):
    return jb if c == 0 else (12 + jb if c == 1 else (8 + jb if jb < 4 else 16 + jb))


def ways(addrs, groups, nbank, width):
    """max distinct dwords on one bank per group, per group"""
    out = []
    for g in groups:
        banks = defaultdict(set)
        for lane in g:
            for d in range(width // 4 or 1):
                dw = addrs[lane] // 4 + d
                banks[dw % nbank].add(dw)
        out.append(max(len(v) for v in banks.values()))
    return out


def test_slots_hold_distinct_bytes():
    for h, n in ((mxs_h, 24), (mx2_h, 16)):
        seen = {coef(h, s, z) for s in range(n) for z in range(64)}
        assert len(seen) == 64 * n and max(seen) < 128 * n


def test_k_mxs_stage():
    slot = lambda k, lane: mx_pos((lane & 15) >> 3, lane >> 4) + 4 * k          # noqa: E731
    extra = 0
    for k in range(3):
        for v in range(8):
            w = ways([coef(mxs_h, slot(k, l), ZZ[v][l & 7]) for l in range(64)], G32, 32, 2)
            assert max(w) <= 2, (k, v, w)
            extra += sum(x - 1 for x in w)
    assert extra == 36                                   # 60 for the padded 144-B slots of round 5
    ro = [128 * (l >> 3) + 16 * ((l & 7) ^ mxs_h(l >> 3)) for l in range(64)]
    rcb = [128 * (12 + (l >> 3)) + 16 * ((l & 7) ^ mxs_h(12 + (l >> 3))) for l in range(64)]
    s_cr = lambda l: (l >> 3) + (8 if (l >> 3) < 4 else 16)                      # noqa: E731
    rr = [128 * s_cr(l) + 16 * ((l & 7) ^ mxs_h(s_cr(l))) for l in range(64)]
    for a in (ro, rcb, rr):
        assert ways(a, G128, 64, 16) == [1, 1, 1, 1]
    # the closed forms the kernel uses (mx_ro), also static_assert'ed in the source
    for l in range(64):
        r = (l << 4) ^ ((l & 8) * 10)
        assert r == ro[l] and (r ^ 32) + 1536 == rcb[l] and (r ^ (l & 32)) + 1024 + ((l & 32) << 5) == rr[l]


def test_k_mxs42x_stage():
    extra = 0
    for k in range(2):                                   # Y column, chroma column (8 slots on)
        for v in range(8):
            addrs = [coef(mx2_h, ((l & 15) >> 3) * 4 + (l >> 4) + 8 * k, ZZ[v][l & 7]) for l in range(64)]
            w = ways(addrs, G32, 32, 2)
            assert max(w) <= 2, (k, v, w)
            extra += sum(x - 1 for x in w)
    assert extra == 24
    pm = lambda g: (g & 1) * 2 + (g >> 1)                # noqa: E731  (k_mxs420's chroma order)
    reads = [[coef(mx2_h, l >> 3, 8 * (l & 7)) for l in range(64)],
             [coef(mx2_h, 8 + (l >> 3), 8 * (l & 7)) for l in range(64)],
             [coef(mx2_h, 8 + 4 * (l >> 5) + pm((l >> 3) & 3), 8 * (l & 7)) for l in range(64)]]
    for a in reads:
        assert ways(a, G128, 64, 16) == [1, 1, 1, 1]
    for l in range(64):
        assert ((l << 4) ^ ((l & 8) * 10) ^ (l & 32)) == reads[0][l]
