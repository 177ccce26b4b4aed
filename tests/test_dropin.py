"""The drop-in proven at the C level.

* Block API: tests/c/dropin_block.c is written against the reference's unprefixed names
  (new_block, set_value_block, dct_block, quantise_lum, zig_zag_block: src/headers/block.h:15-40,
  dct.h:10, quantise.h:9-10, zig_zag.h:11), compiled with include/jpgx_refnames.h and linked
  only against libjpgx.so; it reproduces the reference's own KAT (src/jpg_driver.c:54-150).
* Entropy front end: tests/c/dropin_entropy.c is compiled against the reference's headers
  (src/headers/jpg_encode.h) and linked with the reference's OWN dpcm.o and huffman.o
  (src/dpcm.c:6-21, src/huffman.c:23-44, built in place by oracle/Makefile) plus libjpgx.so.
  A JpgData filled by jpgx_fill_jpgdata (here) or jpgx_encode_bmp on the GPU (test_gpu_...)
  goes through the reference's unchanged dpcm() and the frequency half of huffman_encode();
  the post-dpcm DCs and the four freq tables must equal what the real reference produced on
  its own (tests/golden/entropy_stats.json)."""
import hashlib
import json
import os
import subprocess
import tempfile

import numpy as np
import pytest

import oracle as O
from conftest import GOLDEN, REPO
from test_oracle import KAT_IN, LUM

CDIR = os.path.join(REPO, "tests", "c")
BUILD = os.path.join(CDIR, "_build")


def _make(target):
    subprocess.run(["make", "-s", "-C", CDIR, target], check=True, stdout=subprocess.DEVNULL)
    return os.path.join(BUILD, "dropin_" + target)


def _entropy_binary():
    exe = os.path.join(BUILD, "dropin_entropy")
    if os.path.exists("/root/reference/src") and os.path.exists(os.path.join(O.REF_DIR, "dpcm.o")):
        return _make("entropy")
    if not os.path.exists(exe):
        pytest.skip("the reference's dpcm.o / huffman.o are not built here")
    return exe


def _entropy_cases():
    with open(os.path.join(GOLDEN, "entropy_stats.json")) as f:
        return json.load(f)["cases"]


def _check(exe_args, case):
    with tempfile.TemporaryDirectory() as td:
        dc, hist = os.path.join(td, "dc.bin"), os.path.join(td, "hist.bin")
        subprocess.run(exe_args + [dc, hist], check=True)
        d = np.fromfile(dc, np.int32)
        h = np.fromfile(hist, np.int32).reshape(4, 257)
    assert hashlib.sha256(d.astype("<i4").tobytes()).hexdigest() == case["dc_sha256"]
    assert h.tolist() == case["hist"]


def test_block_api_through_refnames(golden):
    exe = _make("block")
    inp = " ".join(str(int(v)) for v in KAT_IN.reshape(-1)) + " 0\n"
    out = subprocess.run([exe], input=inp, capture_output=True, text=True, check=True).stdout
    toks = out.split()
    dct = np.array([float(t) for t in toks[:64]])
    zz = [int(t) for t in toks[64:128]]
    assert [f"{v:.2f}" for v in dct[:5]] == ["-415.37", "-30.19", "-61.20", "27.24", "56.12"]
    assert zz == golden["kat_zigzag"]


@pytest.mark.parametrize("q", [10, 50, 90])
def test_block_api_scaled_table_matches_oracle(q):
    """quality > 0: scale_table (src/quantise.c:74-86) rescales the global table in place first;
    the zig-zag output equals the oracle's transform of the same block."""
    exe = _make("block")
    rng = np.random.default_rng(q)
    v = rng.integers(-128, 128, 64).astype(np.float64)
    inp = " ".join(str(int(x)) for x in v) + f" {q}\n"
    out = subprocess.run([exe], input=inp, capture_output=True, text=True, check=True).stdout
    zz = [int(t) for t in out.split()[64:128]]
    F = O.dct_block(v)
    want = O.zigzag_block(O.quantise_block(F, O.scale_table(LUM, q)))
    assert zz == [int(x) for x in want]


@pytest.mark.parametrize("idx", range(4))
def test_reference_dpcm_and_huffman_consume_jpgx_jpgdata(idx):
    """jpgx_fill_jpgdata's JpgData (from coefficients equal to the reference's: the oracle,
    pinned in test_oracle.py) fed to the reference's own dpcm() and huffman freq pass."""
    exe = _entropy_binary()
    case = [c for c in _entropy_cases() if "image" in c][idx]
    data = open(os.path.join(GOLDEN, "images", f"{case['image']}.bmp"), "rb").read()
    rgb = O.bmp_decode(data)
    H, W = rgb.shape[:2]
    with open(os.path.join(GOLDEN, "golden.json")) as f:
        ent = json.load(f)["images"][case["image"]]
    coef = O.blocks(rgb, case["q"], underflow=ent["underflow"])
    with tempfile.TemporaryDirectory() as td:
        cb = os.path.join(td, "coef.bin")
        coef.astype("<i2").tofile(cb)
        _check([exe, "coef", cb, str(W), str(H)], case)


@pytest.mark.gpu
@pytest.mark.parametrize("idx", range(4))
def test_gpu_encode_bmp_into_reference_entropy_stage(idx, cuda):
    """The whole drop-in: jpgx_encode_bmp on the GPU fills the reference's JpgData in place of
    src/jpg_encode.c:32-44; the reference's own dpcm() and huffman frequency pass follow."""
    exe = _entropy_binary()
    case = [c for c in _entropy_cases() if "image" in c][idx]
    bmp = os.path.join(GOLDEN, "images", f"{case['image']}.bmp")
    _check([exe, "bmp", bmp, str(case["q"])], case)
