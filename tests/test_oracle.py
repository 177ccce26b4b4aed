"""Pin the oracle (oracle/cpu_ref.c) to the reference's own known answers and to outputs of
the real reference (tests/golden/golden.json, made by tests/golden/make_golden.py)."""
import os

import numpy as np
import pytest

import oracle as O
from conftest import GOLDEN, coef_sha, sha

# The reference's KAT input (src/jpg_driver.c:60-130): values[y*8+x], already level shifted.
KAT_IN = np.array([
    [-76, -73, -67, -62, -58, -67, -64, -55], [-65, -69, -73, -38, -19, -43, -59, -56],
    [-66, -69, -60, -15, 16, -24, -62, -55], [-65, -70, -57, -6, 26, -22, -58, -59],
    [-61, -67, -60, -24, -2, -40, -60, -58], [-49, -63, -68, -58, -51, -60, -70, -53],
    [-43, -57, -64, -69, -73, -67, -63, -45], [-41, -49, -59, -60, -63, -52, -50, -34]],
    np.float64)
# src/quantise.c:8-15 (unscaled luminance table, which test_dct() uses as is)
LUM = np.array([[16, 11, 10, 16, 24, 40, 51, 61], [12, 12, 14, 19, 26, 58, 60, 55],
                [14, 13, 16, 24, 40, 57, 69, 56], [14, 17, 22, 29, 51, 87, 80, 62],
                [18, 22, 37, 56, 68, 109, 103, 77], [24, 35, 55, 64, 81, 104, 113, 92],
                [49, 64, 78, 87, 103, 121, 120, 101], [72, 92, 95, 98, 112, 100, 103, 99]],
               np.int32)
CHR = np.full((8, 8), 99, np.int32)
CHR[:4, :4] = [[17, 18, 24, 47], [18, 21, 26, 66], [24, 26, 56, 99], [47, 66, 99, 99]]


def test_scale_table_against_formula():
    for q in (1, 10, 25, 49, 50, 51, 75, 90, 95, 97):
        s = 5000 // q if q < 50 else 200 - 2 * q
        for base in (LUM, CHR):
            assert np.array_equal(O.scale_table(base, q), (s * base + 50) // 100)
    assert np.array_equal(O.scale_table(LUM, 50), LUM)


def test_kat_block_api(golden):
    """dct_block -> quantise_lum (UNSCALED table) -> zig_zag_block, as test_dct() does."""
    F = O.dct_block(KAT_IN)
    # jpg_driver.c prints the DCT row v=0 with %8.2f: -415.37 -30.19 -61.20 27.24 56.12 ...
    assert [f"{x:.2f}" for x in F[:5]] == ["-415.37", "-30.19", "-61.20", "27.24", "56.12"]
    qv = O.quantise_block(F, LUM)
    zz = O.zigzag_block(qv)
    assert zz.tolist() == golden["kat_zigzag"]


def test_kat_refcost_mode_identical():
    assert np.array_equal(O.dct_block(KAT_IN, O.MODE_REFCOST), O.dct_block(KAT_IN, O.MODE_TABLE))


@pytest.mark.parametrize("name", ["cam", "tiger"])
def test_bundled_images(golden, name):
    path = os.path.join(GOLDEN, "images", f"{name}.bmp")
    data = open(path, "rb").read()
    rgb = O.bmp_decode(data)
    uf = O.glibc_underflow(rgb.shape[0] * rgb.shape[1], len(data))
    ent = golden["images"][name]
    assert np.array_equal(np.tile(uf, (3, 1)), np.array(ent["underflow"]))  # model == glibc
    for q, h in ent["coef_sha256"].items():
        out = O.blocks(rgb, int(q), underflow=uf)
        assert coef_sha(out) == h, (name, q)
        assert sha(O.dpcm(out).astype("<i4")) == ent["dpcm_sha256"][q], (name, q, "dpcm")
    if name == "cam":
        assert np.array_equal(O.blocks(rgb, 75, underflow=uf), np.load(
            os.path.join(GOLDEN, "cam_q75_ref.npy")))


def _frame(ent):
    if ent["kind"] == "G":
        return O.gen_splitmix(ent["seed"], ent["W"], ent["H"])
    return O.gen_tie(ent["W"], ent["H"])


def test_synthetic_frames(golden):
    for ent in golden["synthetic"]:
        if ent["W"] * ent["H"] > 512 * 512:
            continue
        rgb = _frame(ent)
        assert sha(rgb) == ent["input_sha256"]
        for q, h in ent["coef_sha256"].items():
            out = O.blocks(rgb, int(q), underflow=ent["underflow"])
            assert coef_sha(out) == h, (ent["kind"], ent["W"], ent["H"], q)
            if "coef" in ent:
                assert np.array_equal(out, np.array(ent["coef"][q]))
        if "coef_sha256_sr1" in ent:
            q0 = next(iter(ent["coef_sha256"]))
            assert coef_sha(O.blocks(rgb, int(q0), sample_ratio=1,
                                     underflow=ent["underflow"])) == ent["coef_sha256_sr1"]


def test_underflow_model_vs_glibc(golden):
    """The top-chunk formula equals what glibc really left in front of the planes for every
    fixture except tiny images, where a freed chunk can be reused (24x16: r_new got a
    416-byte chunk) -- the reason the ABI takes per-plane bytes."""
    for ent in golden["synthetic"]:
        model = np.tile(O.glibc_underflow(ent["W"] * ent["H"]), (3, 1))
        if ent["W"] * ent["H"] >= 64 * 48:
            assert np.array_equal(model, np.array(ent["underflow"])), (ent["W"], ent["H"])
    odd = next(e for e in golden["synthetic"] if (e["W"], e["H"]) == (24, 16))
    assert odd["underflow"][0] != odd["underflow"][1]


@pytest.mark.parametrize("W,H,q", [(1920, 1080, "90"), (3840, 2160, "90"), (3840, 2160, "75")])
def test_large_frames(golden, W, H, q):
    ent = next(e for e in golden["synthetic"] if e["W"] == W and e["H"] == H)
    rgb = _frame(ent)
    assert sha(rgb) == ent["input_sha256"]
    out = O.blocks(rgb, int(q), nthreads=0, underflow=ent["underflow"])
    assert coef_sha(out) == ent["coef_sha256"][q]


def test_row_ranges_stitch():
    rgb = O.gen_splitmix(5, 64, 64)
    whole = O.blocks(rgb, 80)
    parts = [O.blocks(rgb, 80, rows=(a, b)) for a, b in [(0, 3), (3, 4), (4, 8)]]
    assert np.array_equal(np.concatenate(parts, axis=1), whole)


def test_invalid_arguments():
    rgb = O.gen_splitmix(1, 16, 16)
    for q in (0, 98, 100, -3):
        with pytest.raises(ValueError):
            O.blocks(rgb, q)
    with pytest.raises(ValueError):
        O.blocks(O.gen_splitmix(1, 12, 16), 50)
    with pytest.raises(ValueError):
        O.blocks(O.gen_splitmix(1, 24, 16), 50, sample_ratio=1)   # 4:2:2 needs W % 16
    with pytest.raises(ValueError):
        O.blocks(O.gen_splitmix(1, 16, 8), 50, sample_ratio=2)    # 4:2:0 needs H % 16


@pytest.mark.skipif(not O.ref_available(), reason="reference build (oracle/_ref) absent")
@pytest.mark.parametrize("W,H,seed,q,sr", [(32, 16, 21, 33, 0), (48, 40, 22, 66, 0),
                                           (64, 32, 23, 5, 1), (96, 64, 24, 95, 2)])
def test_against_reference_binary(tmp_path, W, H, seed, q, sr):
    """Fresh cases straight against the reference compiled from its own sources."""
    rgb = O.gen_splitmix(seed, W, H)
    bmp = str(tmp_path / "f.bmp")
    O.write_bmp(bmp, rgb)
    ref = O.ref_dump(bmp, q, sample_ratio=sr)
    assert np.array_equal(O.blocks(rgb, q, sample_ratio=sr), ref)
