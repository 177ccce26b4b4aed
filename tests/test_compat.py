"""The reference-compatible host API (include/jpgx_compat.h): Block API, JpgData adapter, DC
recurrence, BMP reader -- checked against the oracle and the reference's own known answers.
CPU only except the encode_bmp tests, which run the GPU path."""
import os

import numpy as np
import pytest

import oracle as O
from conftest import GOLDEN, coef_sha, sha
from jpgx import compat as C
from test_oracle import CHR, KAT_IN, LUM


def test_kat_through_block_api(golden, capfd):
    """test_dct() (src/jpg_driver.c:54-150): set 64 values, show, dct_block, quantise_lum with
    the UNSCALED global table, zig_zag_block."""
    b = C.Block()
    for y in range(8):
        for x in range(8):
            b.set(x, y, KAT_IN[y, x])
    assert b.get(3, 1) == KAT_IN[1, 3]
    b.show()
    shown = capfd.readouterr().out
    assert shown.startswith("\n  -76.00   -73.00 ") and shown.count("\n") == 9
    b.dct()
    assert [f"{v:.2f}" for v in b.values()[:5]] == ["-415.37", "-30.19", "-61.20", "27.24",
                                                   "56.12"]
    assert np.array_equal(C.legacy_table(0), LUM)
    b.quantise_lum()
    assert b.zig_zag().tolist() == golden["kat_zigzag"]


def test_copy_is_deep():
    b = C.Block(np.arange(64.0))
    c = b.copy()
    b.set(0, 0, 99.0)
    assert c.get(0, 0) == 0.0 and c.values()[63] == 63.0


def test_dct_quantise_zigzag_match_oracle():
    rng = np.random.default_rng(7)
    for trial in range(50):
        v = rng.integers(-128, 128, 64).astype(np.float64) + rng.random(64) * (trial % 2)
        b = C.Block(v)
        b.dct()
        F = O.dct_block(v)
        assert np.array_equal(b.values(), F)           # bit-exact doubles
        q = rng.integers(1, 98)
        table = O.scale_table(LUM if trial % 3 else CHR, int(q))
        b.quantise(table)
        qv = O.quantise_block(F, table)
        assert np.array_equal(b.values(), qv)
        assert np.array_equal(b.zig_zag(), O.zigzag_block(qv))


def test_legacy_tables_rescale_in_place():
    """quantise() rescales the global tables each call (src/quantise.c:34-35)."""
    t = C.legacy_table(1)
    saved = t.copy()
    try:
        C.scale_table_inplace(t, 75)
        assert np.array_equal(t, O.scale_table(CHR, 75))
        C.scale_table_inplace(t, 75)                   # the reference's double scaling
        assert np.array_equal(t, O.scale_table(O.scale_table(CHR, 75), 75))
        v = np.linspace(-500, 500, 64)
        b = C.Block(v)
        b.quantise_chr()
        assert np.array_equal(b.values(), O.quantise_block(v, t))
    finally:
        t[:] = saved


def test_scale_table_inplace_all_qualities():
    for q in range(1, 98):
        t = LUM.astype(np.int32).copy()
        C.scale_table_inplace(t, q)
        assert np.array_equal(t, O.scale_table(LUM, q))


def _coef(seed, W=64, H=48, q=75):
    return O.blocks(O.gen_splitmix(seed, W, H), q)


def test_jpgdata_adapter_and_dpcm():
    W, H = 64, 48
    coef = _coef(3, W, H)
    j = C.jpgdata_from_coef(W, H, coef)
    try:
        assert j.num_blocks_Y == j.num_blocks_Cb == j.num_blocks_Cr == (W // 8) * (H // 8)
        assert np.array_equal(C.jpgdata_zigzag(j), coef.astype(np.int32))
        C.dpcm(j)
        ref = O.dpcm(coef)
        assert np.array_equal(C.jpgdata_zigzag(j), ref)
        assert np.array_equal(C.dpcm_dc(coef), ref[:, :, 0])
    finally:
        C.free_jpgdata(j)


def test_dpcm_stripe_carry_stitches():
    """The DC recurrence of block-row stripes computed separately, stitched by carry, equals
    the whole-frame recurrence."""
    coef = _coef(5, 128, 96, 90)
    whole = C.dpcm_dc(coef)
    nb = coef.shape[1]
    carry = np.zeros(3, np.int32)
    parts = []
    for s in np.array_split(np.arange(nb), 5):
        d = C.dpcm_dc(coef[:, s[0]:s[-1] + 1], carry)
        parts.append(d)
        carry = d[:, -1].copy()
    assert np.array_equal(np.concatenate(parts, axis=1), whole)


def test_dpcm_leaves_int16_range():
    coef = np.zeros((3, 4, 64), np.int16)
    coef[:, :, 0] = [[30000, -30000, 30000, -30000]] * 3
    dc = C.dpcm_dc(coef)
    assert dc[0].tolist() == [30000, -60000, 90000, -120000]


@pytest.mark.parametrize("name", ["cam", "tiger"])
def test_bmp_read_matches_oracle(name):
    path = os.path.join(GOLDEN, "images", f"{name}.bmp")
    rgb, fs = C.bmp_read(path)
    data = open(path, "rb").read()
    assert fs == len(data)
    assert np.array_equal(rgb, O.bmp_decode(data))


def test_bmp_read_errors(tmp_path):
    with pytest.raises(Exception):
        C.bmp_read(str(tmp_path / "missing.bmp"))
    p = tmp_path / "short.bmp"
    p.write_bytes(b"BM" + b"\0" * 20)
    with pytest.raises(Exception):
        C.bmp_read(str(p))


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["cam", "tiger"])
def test_encode_bmp_matches_reference(golden, name):
    """encode_bmp_to_jpeg up to dpcm (src/jpg_encode.c:19-47) on the bundled images, against
    the hashes of the real reference's zig_zag_* and post-dpcm arrays."""
    path = os.path.join(GOLDEN, "images", f"{name}.bmp")
    ent = golden["images"][name]
    for q, h in ent["coef_sha256"].items():
        j = C.encode_bmp(path, int(q))
        try:
            assert coef_sha(C.jpgdata_zigzag(j).astype(np.int16)) == h, (name, q)
        finally:
            C.free_jpgdata(j)
        j = C.encode_bmp(path, int(q), do_dpcm=True)
        try:
            assert sha(C.jpgdata_zigzag(j).astype("<i4")) == ent["dpcm_sha256"][q], (name, q)
        finally:
            C.free_jpgdata(j)
