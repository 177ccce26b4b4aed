"""The reference-compatible host API (include/jpgx_compat.h): Block API, JpgData adapter, DC
recurrence, BMP reader -- checked against the oracle and the reference's own known answers.
CPU only except the encode_bmp tests, which run the GPU path."""
import os

import numpy as np
import pytest

import oracle as O
from conftest import GOLDEN, coef_sha, sha
import jpgx
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


# ---- JFIF writer (the build's own entropy stage; parity unpinned: the reference's Huffman
# stage never terminates) -- checked by decoding the file back to the coefficients -----------
def _roundtrip(coef, W, H, q):
    from jfif_decode import decode
    data = C.write_jfif(coef, W, H, q)
    d = decode(data)
    assert (d["width"], d["height"]) == (W, H)
    want = np.clip(coef.astype(np.int32), -1023, 1023)
    want[:, :, 0] = coef[:, :, 0]                      # DC is not clamped
    assert np.array_equal(d["coef"], want)
    return data, d


@pytest.mark.parametrize("q", [1, 25, 50, 75, 90, 97])
def test_jfif_roundtrip_random(q):
    W, H = 48, 40
    coef = O.blocks(O.gen_splitmix(q, W, H), q)
    data, d = _roundtrip(coef, W, H, q)
    # DQT = the divisors the reference applied: its scaled tables, transposed (quantise.c:58)
    scan = np.array([[0, 1, 5, 6, 14, 15, 27, 28], [2, 4, 7, 13, 16, 26, 29, 42],
                     [3, 8, 12, 17, 25, 30, 41, 43], [9, 11, 18, 24, 31, 40, 44, 53],
                     [10, 19, 23, 32, 39, 45, 52, 54], [20, 22, 33, 38, 46, 51, 55, 60],
                     [21, 34, 37, 47, 50, 56, 59, 61], [35, 36, 48, 49, 57, 58, 62, 63]])
    wide = max(O.scale_table(LUM, q).max(), O.scale_table(CHR, q).max()) > 255
    assert d["sof"] == (0xC1 if wide else 0xC0)        # 16-bit tables: extended sequential
    assert wide == (q <= 23)
    for t, base in ((0, LUM), (1, CHR)):
        qs = np.maximum(O.scale_table(base, q), 1)     # the true divisors, never clamped
        zz = np.zeros(64, np.int32)
        for v in range(8):
            for u in range(8):
                zz[scan[v, u]] = qs[u, v]
        assert d["dqt"][t] == zz.tolist()
    assert d["qsel"] == [0, 1, 1]


def test_jfif_roundtrip_edge_values():
    """runs of zeros longer than 16 (ZRL), all-zero blocks (EOB only), extreme magnitudes
    (categories 10/11), clamping above the baseline AC range, DC differences near +-2047"""
    W, H = 24, 16
    nb = 6
    coef = np.zeros((3, nb, 64), np.int16)
    coef[0, 0, 0], coef[0, 1, 0], coef[0, 2, 0] = -1024, 1016, -1024
    coef[1, 0, 0], coef[1, 1, 0] = -1364, 672
    coef[0, 0, 63] = 5                                # one AC after a 62-zero run
    coef[0, 1, 1], coef[0, 1, 2] = 1023, -1023
    coef[2, 3, 17] = 1200                             # clamped to 1023
    coef[2, 4, 1:64] = np.arange(1, 64) * (-1) ** np.arange(63)
    _roundtrip(coef, W, H, 97)


@pytest.mark.parametrize("q", [75, 1])
def test_jfif_decodes_with_pil(q):
    """a standard decoder (PIL/libjpeg) accepts the file: baseline at q = 75, extended
    sequential with 16-bit quantisation tables at q = 1 (divisors up to 6050)"""
    import io
    Image = pytest.importorskip("PIL.Image")
    W, H = 64, 48
    coef = O.blocks(O.gen_splitmix(11, W, H), q)
    img = Image.open(io.BytesIO(C.write_jfif(coef, W, H, q)))
    img.load()
    assert img.size == (W, H)
    if q == 1:
        assert max(max(t) for t in img.quantization.values()) > 255
    assert img.size == (W, H) and img.mode == "RGB"


def test_jfif_small_buffer_and_bad_args():
    import ctypes
    from jpgx import lib
    coef = np.zeros((3, 4, 64), np.int16)
    buf = (ctypes.c_uint8 * 64)()
    n = ctypes.c_size_t()
    rc = lib.jpgx_write_jfif(coef.ctypes.data, 16, 16, 50, ctypes.cast(buf, ctypes.c_void_p), 64,
                             ctypes.byref(n))
    assert rc == -4 and n.value > 64                  # EARG, with the size needed
    rc = lib.jpgx_write_jfif(coef.ctypes.data, 12, 16, 50, ctypes.cast(buf, ctypes.c_void_p), 64,
                             ctypes.byref(n))
    assert rc == -4
    rc = lib.jpgx_write_jfif(coef.ctypes.data, 16, 16, 98, ctypes.cast(buf, ctypes.c_void_p), 64,
                             ctypes.byref(n))
    assert rc == -2


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["cam", "tiger"])
def test_encode_bmp_to_jpeg_file(golden, name, tmp_path):
    """The reference's entry point end to end: BMP -> GPU block transform -> JPEG file, whose
    coefficients are the reference's (golden hashes of its zig_zag_* arrays)."""
    from jfif_decode import decode
    src = os.path.join(GOLDEN, "images", f"{name}.bmp")
    for q, h in golden["images"][name]["coef_sha256"].items():
        dst = str(tmp_path / f"{name}_{q}.jpg")
        C.encode_bmp_to_jpeg(src, dst, int(q))
        d = decode(open(dst, "rb").read())
        assert coef_sha(d["coef"].astype(np.int16)) == h, (name, q)


def test_fill_jpgdata_refuses_to_leak():
    """a JpgData that already holds zig_zag arrays is refused (JPGX_EARG, nothing changed);
    after jpgx_free_jpgdata it can be filled again."""
    import ctypes
    W, H = 16, 8
    coef = O.blocks(O.gen_splitmix(3, W, H), 50)
    j = C.jpgdata_from_coef(W, H, coef)
    nb = j.num_blocks_Y
    rc = C.lib.jpgx_fill_jpgdata(ctypes.byref(j), np.ascontiguousarray(coef, np.int16).ctypes.data)
    assert rc == jpgx.EARG and j.num_blocks_Y == nb
    assert np.array_equal(C.jpgdata_zigzag(j), coef)
    C.lib.jpgx_free_jpgdata(ctypes.byref(j))
    assert not j.zig_zag_Y
    rc = C.lib.jpgx_fill_jpgdata(ctypes.byref(j), np.ascontiguousarray(coef, np.int16).ctypes.data)
    assert rc == jpgx.OK and np.array_equal(C.jpgdata_zigzag(j), coef)
    C.lib.jpgx_free_jpgdata(ctypes.byref(j))


@pytest.mark.gpu
@pytest.mark.parametrize("sr,flags", [(0, 0), (1, 0), (1, jpgx.FLAG_SUBSAMPLE), (2, jpgx.FLAG_SUBSAMPLE)])
def test_encode_rgb_to_jpeg_in_memory(tmp_path, sr, flags):
    """jpgx_encode_rgb_to_jpeg (the reference's declared encode_rgb_to_jpeg,
    src/headers/jpg_encode.h:99): an in-memory image, row-padded, to a JFIF file whose decoded
    coefficients are the oracle's (4:4:4 parity output, or the true-subsampling extension)."""
    from jfif_decode import decode
    W, H, q = 96, 64, 80
    big = O.gen_splitmix(61 + sr, W + 16, H)
    rgb = big[:, :W]                                  # pitch (W + 16) * 3
    dst = str(tmp_path / "m.jpg")
    C.encode_rgb_to_jpeg(rgb, dst, q, sr, flags)
    d = decode(open(dst, "rb").read())
    img = np.ascontiguousarray(rgb)
    if flags & jpgx.FLAG_SUBSAMPLE:
        assert np.array_equal(d["coef"][0], O.blocks(img, q, sr)[0])
        c = O.chroma_sub(img, q, sr)
        assert np.array_equal(d["coef"][1], c[0]) and np.array_equal(d["coef"][2], c[1])
    else:
        assert np.array_equal(d["coef"].astype(np.int16), O.blocks(img, q))
    with pytest.raises(jpgx.JpgxError) as e:
        C.encode_rgb_to_jpeg(np.ascontiguousarray(rgb[:, :90]), dst, q)
    assert e.value.rc == jpgx.EGEOMETRY


@pytest.mark.gpu
def test_config0_512_bmp_to_jpeg(golden, tmp_path):
    """BASELINE configs[0] through the drop-in: a 512x512 BMP (the golden G frame, seed 1) ->
    jpgx_encode_bmp_to_jpeg at q=90 (4:4:4) -> a JPEG whose decoded coefficients hash to the
    real reference's zig_zag_* output for that BMP (tests/golden/golden.json)."""
    from jfif_decode import decode
    ent = next(e for e in golden["synthetic"] if (e["kind"], e["W"], e["H"]) == ("G", 512, 512))
    src, dst = str(tmp_path / "in.bmp"), str(tmp_path / "out.jpg")
    O.write_bmp(src, O.gen_splitmix(ent["seed"], 512, 512))
    C.encode_bmp_to_jpeg(src, dst, 90)
    d = decode(open(dst, "rb").read())
    assert coef_sha(d["coef"].astype(np.int16)) == ent["coef_sha256"]["90"]
