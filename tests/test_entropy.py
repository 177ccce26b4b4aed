"""Entropy-stage statistics: the reference's DC recurrence (src/dpcm.c:6-21)
and huffman_encode's frequency pass (src/huffman.c:23-44, 182-235).  The oracle restatement is
pinned against the REAL reference's frequency tables (tests/golden/entropy_stats.json, made by
tests/golden/make_entropy_golden.py from the compiled reference); the GPU kernels
(jpgx_entropy_stats_gpu) must match the oracle exactly (integer work)."""
import hashlib
import json
import os

import numpy as np
import pytest

import jpgx
import oracle as O
from conftest import GOLDEN


def _cases():
    return json.load(open(os.path.join(GOLDEN, "entropy_stats.json")))["cases"]


def _rgb(case):
    if "image" in case:
        return O.bmp_decode(open(os.path.join(GOLDEN, "images", f"{case['image']}.bmp"), "rb").read())
    return O.gen_splitmix(case["seed"], case["W"], case["H"]) if case["kind"] == "G" else O.gen_tie(case["W"], case["H"])


def _underflow(case, golden):
    if "image" in case:
        return golden["images"][case["image"]]["underflow"]
    for ent in golden["synthetic"]:
        if (ent["kind"], ent["W"], ent["H"], ent["seed"]) == (case.get("kind"), case.get("W"),
                                                               case.get("H"), case.get("seed")):
            return ent["underflow"]
    return None


def test_oracle_matches_reference_frequency_tables(golden):
    for case in _cases():
        if case.get("W", 0) * case.get("H", 0) > 512 * 512:
            continue                                  # the 1080p case runs on the GPU test
        coef = O.blocks(_rgb(case), case["q"], underflow=_underflow(case, golden))
        dc, hist = O.entropy_stats(coef)
        assert np.array_equal(hist, np.array(case["hist"], np.int32)), case.get("image", case.get("kind"))
        assert hashlib.sha256(dc.astype("<i4").tobytes()).hexdigest() == case["dc_sha256"]


def test_histogram_quirks_by_construction():
    """Hand-made blocks: EOB only when the last AC is zero, ZRL per 16 zeros, run|size."""
    coef = np.zeros((3, 3, 64), np.int16)
    coef[0, 0, 0] = 5                                 # DC class 3
    coef[0, 0, 1] = 1                                 # (0 | 1), then EOB
    coef[0, 1, 0] = 5                                 # dpcm: 5 - 5 = 0 -> class 0
    coef[0, 1, 20] = -3                               # 19 zeros: ZRL, then (3 | 2) = 3, EOB
    coef[0, 2, 63] = 7                                # last AC non-zero: no EOB; 62 zeros:
    dc, hist = O.entropy_stats(coef)                  # 3 ZRL, then (14 | 3) = 15
    assert list(dc[:3]) == [5, 0, 0]
    assert hist[0, 3] == 1 and hist[0, 0] == 2 and hist[0, 256] == 1
    assert hist[1, 0x00] == 2 + 0 and hist[1, 0xF0] == 1 + 3
    assert hist[1, 1] == 1 and hist[1, 3] == 1 and hist[1, 15] == 1


def test_host_dpcm_matches_oracle():
    rgb = O.gen_splitmix(9, 128, 64)
    coef = O.blocks(rgb, 75)
    dc, _ = O.entropy_stats(coef)
    nb = coef.shape[1]
    got = np.empty(3 * nb, np.int32)
    import ctypes
    f = jpgx.lib.jpgx_dpcm_dc
    f.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_void_p]
    carry = (ctypes.c_int32 * 3)(0, 0, 0)
    assert f(coef.ctypes.data, nb, ctypes.cast(carry, ctypes.c_void_p), got.ctypes.data) == 0
    assert np.array_equal(got, dc)


def _gpu_stats(coef, nb_y, nb_c, cuda, carry=None):
    import torch
    d = torch.from_numpy(np.ascontiguousarray(coef.reshape(-1, 64))).to(cuda)
    dc, hist = jpgx.entropy_stats_gpu(d, nb_y, nb_c, carry)
    return dc.cpu().numpy(), hist.cpu().numpy()


@pytest.mark.gpu
def test_gpu_stats_golden(golden, cuda):
    for case in _cases():
        coef = jpgx.encode_blocks(__import__("torch").from_numpy(_rgb(case)).to(cuda), case["q"],
                                  underflow=_underflow(case, golden)).cpu().numpy()
        nb = coef.shape[1]
        dc, hist = _gpu_stats(coef, nb, nb, cuda)
        assert np.array_equal(hist, np.array(case["hist"], np.int32)), case.get("image", case.get("kind"))
        assert hashlib.sha256(dc.astype("<i4").tobytes()).hexdigest() == case["dc_sha256"]


@pytest.mark.gpu
@pytest.mark.parametrize("W,H,q", [(8, 8, 50), (40, 16, 90), (1920, 1080, 75), (3840, 2160, 90)])
def test_gpu_stats_vs_oracle(cuda, W, H, q):
    rgb = O.gen_splitmix(W + q, W, H)
    coef = jpgx.encode_blocks(__import__("torch").from_numpy(rgb).to(cuda), q).cpu().numpy()
    nb = coef.shape[1]
    dc, hist = _gpu_stats(coef, nb, nb, cuda)
    rdc, rhist = O.entropy_stats(coef)
    assert np.array_equal(dc, rdc)
    assert np.array_equal(hist, rhist)


@pytest.mark.gpu
def test_gpu_stats_stripes_with_carry(cuda):
    """Two stripes with the first one's last DCs carried in: the second stripe's dc equals the
    whole image's; its histogram plus the first's (minus one reserved count) equals the whole."""
    rgb = O.gen_splitmix(77, 640, 480)
    coef = O.blocks(rgb, 90)
    nb = coef.shape[1]
    dc_all, hist_all = O.entropy_stats(coef)
    s = (480 // 8 // 2) * (640 // 8)
    a, b = coef[:, :s], coef[:, s:]
    dca, ha = _gpu_stats(a, s, s, cuda)
    carry = [int(dca[c * s + s - 1]) for c in range(3)]
    dcb, hb = _gpu_stats(b, nb - s, nb - s, cuda, carry)
    want_b = np.concatenate([dc_all[c * nb + s:(c + 1) * nb] for c in range(3)])
    assert np.array_equal(dcb, want_b)
    tot = ha.astype(np.int64) + hb
    tot[:, 256] -= 1
    assert np.array_equal(tot, hist_all)


@pytest.mark.gpu
@pytest.mark.parametrize("sr", [1, 2])
def test_gpu_stats_subsampled_layout(cuda, sr):
    import torch
    W, H = 256, 128
    rgb = O.gen_splitmix(5, W, H)
    out = jpgx.encode_blocks(torch.from_numpy(rgb).to(cuda), 75, sr, flags=jpgx.FLAG_SUBSAMPLE)
    nb = (H // 8) * (W // 8)
    nbc = jpgx.chroma_blocks(W, 0, H // 8, sr, jpgx.FLAG_SUBSAMPLE)
    dc, hist = jpgx.entropy_stats_gpu(out, nb, nbc)
    rdc, rhist = O.entropy_stats(out.cpu().numpy(), nb, nbc)
    assert np.array_equal(dc.cpu().numpy(), rdc)
    assert np.array_equal(hist.cpu().numpy(), rhist)


def _gap_rule_hist(coef):
    """k_ent_ac's rule restated (csrc/jpgx_entropy.hip, round 6): a lane walks its block's 63 AC
    coefficients with the previous nonzero position p (0 = the DC position); coefficient i has run
    r = i - p - 1 and adds one count to bin ((r & 15) | class) when nonzero (class = the frexp
    exponent of the coefficient as a float) or to bin 32 + (r & 15) when zero; a zero with r & 15 == 15
    completes a group of 16 zeros, so ZRL = bin 47 minus the groups in the trailing zeros,
    sum over blocks of (63 - L) >> 4 (L = the last nonzero position); EOB iff coefficient 63 is zero.
    Returns the AC histogram [257]."""
    z = np.asarray(coef, np.int64).reshape(-1, 64)
    nb = z.shape[0]
    bins = np.zeros(48, np.int64)
    prev = np.zeros(nb, np.int64)
    for i in range(1, 64):
        v = z[:, i]
        cls = np.frexp(v.astype(np.float32))[1].astype(np.int64)      # 0 for 0
        r = i - 1 - prev
        nz = cls != 0
        b = np.where(nz, (r & 15) | cls, 32 | (r & 15))
        np.add.at(bins, b, 1)
        prev = np.where(nz, i, prev)
    h = np.zeros(257, np.int64)
    h[1:32] = bins[1:32]
    h[0xF0] = bins[47] - int(((63 - prev) >> 4).sum())
    h[0] = int((z[:, 63] == 0).sum())
    return h


@pytest.mark.parametrize("kind", ["dense", "sparse", "long_runs", "extremes"])
def test_device_gap_rule_matches_oracle(kind):
    """The histogram rule the GPU kernel uses, against the oracle's sequential huffman.c loop."""
    rng = np.random.default_rng({"dense": 1, "sparse": 2, "long_runs": 3, "extremes": 4}[kind])
    nb = 3000
    if kind == "dense":
        c = rng.integers(-300, 301, (3, nb, 64))
    elif kind == "sparse":
        c = rng.integers(-40, 41, (3, nb, 64)) * (rng.random((3, nb, 64)) < 0.08)
    elif kind == "long_runs":                     # runs of 16+, 32+ zeros, all-zero AC blocks
        c = np.zeros((3, nb, 64), np.int64)
        for b in range(nb):
            for i in rng.choice(64, rng.integers(0, 4), replace=False):
                c[0, b, i] = c[1, b, (i * 7) % 64] = c[2, b, 63 - i] = rng.integers(1, 9) * rng.choice([-1, 1])
    else:                                         # int16 extremes: classes up to 16
        c = rng.choice(np.array([0, 1, -1, 32767, -32768, 2048, -2047]), (3, nb, 64))
    c = c.astype(np.int16)
    _, hist = O.entropy_stats(c)
    for ch, row in ((0, 1), (1, 3)):
        blocks = c[0] if ch == 0 else c[1:].reshape(-1, 64)
        want = hist[row].astype(np.int64)
        got = _gap_rule_hist(blocks)
        got[256] = want[256]                      # the reserved count
        assert np.array_equal(got, want), (kind, ch)


@pytest.mark.gpu
def test_gpu_stats_batch_equals_per_frame(cuda):
    """The batch call (one set of launches over frames with a padded frame stride) equals one
    call per frame, and the oracle on frame 1."""
    import torch
    W, H, F = 640, 480, 3
    nb = (H // 8) * (W // 8)
    out = torch.zeros((F, 3 * nb + 5, 64), dtype=torch.int16, device=cuda)    # padded frames
    for f in range(F):
        out[f, :3 * nb] = jpgx.encode_blocks(torch.from_numpy(O.gen_splitmix(40 + f, W, H)).to(cuda),
                                             50 + 20 * f).reshape(3 * nb, 64)
    dcb, hb = jpgx.entropy_stats_gpu_batch(out, nb, nb)
    for f in range(F):
        dc, h = jpgx.entropy_stats_gpu(out[f, :3 * nb].contiguous(), nb, nb)
        assert torch.equal(dcb[f], dc) and torch.equal(hb[f], h), f
    rdc, rh = O.entropy_stats(out[1, :3 * nb].cpu().numpy(), nb, nb)
    assert np.array_equal(dcb[1].cpu().numpy(), rdc) and np.array_equal(hb[1].cpu().numpy(), rh)


def test_batch_entry_point_rejects_bad_arguments():
    """Argument checks of jpgx_entropy_stats_gpu_batch that need no device."""
    import ctypes
    L = jpgx.lib
    nb = 100
    ws = ctypes.create_string_buffer(int(L.jpgx_entropy_workspace_size_batch(nb, nb, 2)) + 16)
    p16 = ctypes.addressof(ws) + (-ctypes.addressof(ws)) % 16
    args = lambda stride, nf, carry: L.jpgx_entropy_stats_gpu_batch(      # noqa: E731
        p16, stride, nf, nb, nb, carry, p16, p16, p16, len(ws.raw) - 16, None)
    carry = (ctypes.c_int32 * 3)(1, 2, 3)
    assert args(3 * nb * 64 - 64, 2, None) == jpgx.EARG                # stride below a frame
    assert args(3 * nb * 64 + 8, 2, None) == jpgx.EARG                 # not whole blocks
    assert args(3 * nb * 64, 0, None) == jpgx.EARG                     # no frames
    assert args(3 * nb * 64, 2, ctypes.cast(carry, ctypes.c_void_p)) == jpgx.EARG   # carry with a batch


@pytest.mark.gpu
@pytest.mark.parametrize("sr", [0, 1, 2])
def test_gpu_stats_batch_sliced_and_subsampled(cuda, sr):
    """A sliced view of a padded batch (frames nb_y + 2 nb_c + 5 blocks apart, the first
    nb_y + 2 nb_c of each used: the frame stride is the tensor's, not the slice's size) and
    subsampled layouts (nb_c = nb_y / 2, nb_y / 4: different DC workgroup counts per channel)
    equal one call per frame and the oracle."""
    import torch
    W, H, F = 256, 192, 3
    fl = jpgx.FLAG_SUBSAMPLE if sr else 0
    nb = (H // 8) * (W // 8)
    nbc = jpgx.chroma_blocks(W, 0, H // 8, sr, fl)
    per = nb + 2 * nbc
    pad = torch.zeros((F, per + 5, 64), dtype=torch.int16, device=cuda)
    for f in range(F):
        pad[f, :per] = jpgx.encode_blocks(torch.from_numpy(O.gen_splitmix(60 + f, W, H)).to(cuda),
                                          60 + 10 * f, sr, flags=fl).reshape(per, 64)
    view = pad[:, :per]
    assert not view.is_contiguous() and view.stride(0) == (per + 5) * 64
    dcb, hb = jpgx.entropy_stats_gpu_batch(view, nb, nbc)
    for f in range(F):
        dc, h = jpgx.entropy_stats_gpu(pad[f, :per].contiguous(), nb, nbc)
        assert torch.equal(dcb[f], dc) and torch.equal(hb[f], h), f
        rdc, rh = O.entropy_stats(pad[f, :per].cpu().numpy(), nb, nbc)
        assert np.array_equal(dcb[f].cpu().numpy(), rdc) and np.array_equal(hb[f].cpu().numpy(), rh)


def test_batch_binding_rejects_bad_layouts():
    """The Python binding refuses what the C entry point cannot see (no device needed: CPU
    tensors stand in, the checks run before any call)."""
    import torch
    nb = 16
    with pytest.raises(ValueError):
        jpgx.entropy_stats_gpu_batch(torch.zeros((2, 3 * nb, 64), dtype=torch.int32), nb, nb)
    with pytest.raises(ValueError):                       # frames not contiguous
        jpgx.entropy_stats_gpu_batch(torch.zeros((2, 64, 3 * nb), dtype=torch.int16).transpose(1, 2), nb, nb)
    with pytest.raises(ValueError):                       # frame shorter than nb_y + 2 nb_c blocks
        jpgx.entropy_stats_gpu_batch(torch.zeros((2, 3 * nb - 1, 64), dtype=torch.int16), nb, nb)


def test_batch_entry_point_rejects_too_many_frames():
    """nframes > 65535 (the histogram launch's grid.y) is refused up front, before any launch."""
    import ctypes
    L = jpgx.lib
    nb = 1
    need = int(L.jpgx_entropy_workspace_size_batch(nb, nb, 65536))
    ws = ctypes.create_string_buffer(need + 16)
    p16 = ctypes.addressof(ws) + (-ctypes.addressof(ws)) % 16
    assert L.jpgx_entropy_stats_gpu_batch(p16, 3 * 64, 65536, nb, nb, None, p16, p16, p16, need,
                                          None) == jpgx.EARG
