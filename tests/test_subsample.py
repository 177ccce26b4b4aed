"""True 4:2:2 / 4:2:0 chroma subsampling (JPGX_FLAG_SUBSAMPLE): an EXTENSION.  The reference's
subsample_422/420 (src/downsample.c:24-32) only print, so its semantics are defined by the
oracle restatement (oracle/cpu_ref.h: level shift, then the pair/quad average, standard tiling
of the subsampled planes) and parity with the reference is unpinned for the chroma planes; the
luma plane is the reference's own (pinned).  CPU tests pin the oracle's definition by exact
properties; GPU tests require the HIP path to match the oracle bit for bit."""
import numpy as np
import pytest

import jpgx
import oracle as O


def _last_col_mask(nb, bpr):
    m = np.ones(nb, bool)
    m[bpr - 1::bpr] = False          # the reference's 4:4:4 tiling has the x0 = -8 quirk there
    return m


@pytest.mark.parametrize("q", [50, 90])
def test_oracle_pair_duplicates_match_444(q):
    """A frame whose horizontal pixel pairs are equal: every 4:2:2 chroma sample is
    (p + p) * 0.5 = p exactly, so the chroma blocks equal the 4:4:4 chroma blocks of the
    half-width frame (outside the quirk column)."""
    rgb = O.gen_splitmix(11, 96, 48)
    sub = O.chroma_sub(np.repeat(rgb, 2, axis=1), q, 1)
    full = O.blocks(rgb, q)
    m = _last_col_mask(full.shape[1], 96 // 8)
    assert np.array_equal(sub[:, m], full[1:, m])


@pytest.mark.parametrize("q", [50, 90])
def test_oracle_quad_duplicates_match_444(q):
    rgb = O.gen_splitmix(12, 64, 64)
    sub = O.chroma_sub(np.repeat(np.repeat(rgb, 2, axis=1), 2, axis=0), q, 2)
    full = O.blocks(rgb, q)
    m = _last_col_mask(full.shape[1], 64 // 8)
    assert np.array_equal(sub[:, m], full[1:, m])


def test_oracle_sample_definition():
    """cpuref_chroma_sample against a direct numpy evaluation of the definition."""
    rgb = O.gen_splitmix(3, 32, 16)
    r, g, b = (rgb[..., k].astype(np.float64) for k in range(3))
    cb = (128 - (0.168736 * r - 0.331264 * g + 0.5 * b)) - 128
    cr = (128 + (0.5 * r - 0.418688 * g - 0.081312 * b)) - 128
    L = O.lib()
    p = O._u8(np.ascontiguousarray(rgb))
    for ch, c in ((1, cb), (2, cr)):
        for (X, Y) in ((0, 0), (5, 3), (15, 15)):
            assert L.cpuref_chroma_sample(p, 96, 1, ch, X, Y) == (c[Y, 2 * X] + c[Y, 2 * X + 1]) * 0.5
        for (X, Y) in ((0, 0), (7, 7), (15, 2)):
            want = ((c[2 * Y, 2 * X] + c[2 * Y, 2 * X + 1]) + (c[2 * Y + 1, 2 * X] + c[2 * Y + 1, 2 * X + 1])) * 0.25
            assert L.cpuref_chroma_sample(p, 96, 2, ch, X, Y) == want


def test_chroma_blocks_and_validation():
    S = jpgx.FLAG_SUBSAMPLE
    assert jpgx.chroma_blocks(64, 0, 4, 0, S) == 4 * 8
    assert jpgx.chroma_blocks(64, 0, 4, 1, 0) == 4 * 8
    assert jpgx.chroma_blocks(64, 0, 4, 1, S) == 4 * 4
    assert jpgx.chroma_blocks(64, 0, 4, 2, S) == 2 * 4
    assert jpgx.chroma_blocks(64, 2, 6, 2, S) == 2 * 4


def test_guard_band_for_averages_is_no_looser_than_needed():
    """The averaged sample's interval is the single pixel's, its fp32 error bound no larger
    than a pixel's plus the add: the chroma bands stay of the 4:4:4 order of magnitude."""
    sc, lim = jpgx.guard_band(75)
    assert (0.5 - lim).max() < 1e-3


def _dev(a, cuda):
    import torch
    return torch.from_numpy(np.ascontiguousarray(a)).to(cuda)


@pytest.fixture(params=["fused", "two-pass"])
def impl(request, monkeypatch):
    """True 4:2:2 / 4:2:0 run as k_mx422 / k_mx420 (one pass: the product library) or as
    k_xform's Y + k_chroma<1> / <2> (the test-only cross-check library libjpgx_alt.so)."""
    if request.param == "two-pass":
        monkeypatch.setattr(jpgx, "lib", jpgx.alt_library())
    return request.param


def _check(rgb, q, sr, cuda, flags=0):
    H, W = rgb.shape[:2]
    out = jpgx.encode_blocks(_dev(rgb, cuda), q, sr, flags=jpgx.FLAG_SUBSAMPLE | flags)
    out = out.cpu().numpy()
    nb = (H // 8) * (W // 8)
    nbc = jpgx.chroma_blocks(W, 0, H // 8, sr, jpgx.FLAG_SUBSAMPLE)
    y, c = jpgx.split_sub(out, nb, nbc)
    ref_y = O.blocks(rgb, q, sr)[0]
    ref_c = O.chroma_sub(rgb, q, sr)
    assert np.array_equal(y, ref_y), f"luma {np.argwhere(y != ref_y)[:5].tolist()}"
    bad = np.argwhere(c != ref_c)
    assert len(bad) == 0, f"chroma sr{sr} q{q}: {len(bad)} mismatches, first {bad[:5].tolist()}"


@pytest.mark.gpu
@pytest.mark.parametrize("sr", [1, 2])
@pytest.mark.parametrize("q", [25, 50, 75, 90, 97])
def test_gpu_subsample_random(cuda, impl, sr, q):
    _check(O.gen_splitmix(100 + q, 256, 128), q, sr, cuda)


@pytest.mark.gpu
@pytest.mark.parametrize("sr", [1, 2])
def test_gpu_subsample_force_exact(cuda, impl, sr):
    _check(O.gen_splitmix(7, 128, 64), 75, sr, cuda, flags=jpgx.FLAG_FORCE_EXACT)


@pytest.mark.gpu
@pytest.mark.parametrize("sr", [1, 2])
def test_gpu_subsample_tie_and_flat(cuda, impl, sr):
    _check(O.gen_tie(256, 128), 50, sr, cuda)
    rgb = np.zeros((64, 128, 3), np.uint8)
    rgb[..., 0], rgb[..., 1], rgb[..., 2] = 255, 0, 128
    _check(rgb, 90, sr, cuda)


@pytest.mark.gpu
@pytest.mark.parametrize("sr", [1, 2])
@pytest.mark.parametrize("every", [5, 29])
def test_gpu_subsample_sparse_ties(cuda, impl, sr, every):
    """sparse flat tie blocks in a random frame: one or a few flagged coefficients per step (the
    inline exact pass's whole-wave path and its 8-lane batches), Y and chroma"""
    rgb = O.gen_splitmix(500 + every, 1024, 256)
    tie = O.gen_tie(1024, 256)
    for bi in range(3, 128 * 32, every):
        r, c = divmod(bi, 128)
        rgb[8 * r:8 * r + 8, 8 * c:8 * c + 8] = tie[8 * r:8 * r + 8, 8 * c:8 * c + 8]
    for q in (50, 97):
        _check(rgb, q, sr, cuda)


@pytest.mark.gpu
@pytest.mark.parametrize("sr", [1, 2])
def test_gpu_subsample_multi_v(cuda, impl, sr):
    """Y blocks whose column u = 0 holds two flagged coefficients (test_gpu_parity.MULTI_V at q50):
    Y columns with several flag bits (8-lane batches) beside the chroma of the same MCUs"""
    from test_gpu_parity import MULTI_V
    rgb = O.gen_splitmix(940 + sr, 1024, 128)
    pats = MULTI_V[50]
    for i, bi in enumerate(range(5, 128 * 16, 11)):
        r, c = divmod(bi, 128)
        rgb[8 * r:8 * r + 8, 8 * c:8 * c + 8] = np.array(pats[i % len(pats)], np.uint8)[:, None, None]
    _check(rgb, 50, sr, cuda)


@pytest.mark.gpu
@pytest.mark.parametrize("sr", [1, 2])
def test_gpu_subsample_1080p_class(cuda, impl, sr):
    _check(O.gen_splitmix(2, 1920, 1072), 90, sr, cuda)


@pytest.mark.gpu
@pytest.mark.parametrize("sr", [1, 2])
def test_gpu_subsample_stripes_and_batch(cuda, impl, sr):
    """Stripes of a batch of frames through the device entry point equal the whole frames."""
    import torch
    W, H, F = 256, 128, 3
    frames = [O.gen_splitmix(40 + f, W, H) for f in range(F)]
    d_in = _dev(np.stack(frames), cuda)
    S = jpgx.FLAG_SUBSAMPLE
    nb = (H // 8) * (W // 8)
    nbc = jpgx.chroma_blocks(W, 0, H // 8, sr, S)
    per = nb + 2 * nbc
    want = [np.concatenate([O.blocks(fr, 75, sr)[0], O.chroma_sub(fr, 75, sr).reshape(-1, 64)])
            for fr in frames]
    out = torch.zeros((F, per, 64), dtype=torch.int16, device=cuda)
    p = jpgx.default_params(W, H, 75, sr, flags=S)
    for (r0, r1) in ((0, 6), (6, 16)):
        nbs = (r1 - r0) * (W // 8)
        nbcs = jpgx.chroma_blocks(W, r0, r1, sr, S)
        o = torch.zeros((F, nbs + 2 * nbcs, 64), dtype=torch.int16, device=cuda)
        fr = jpgx.frames(W, H, nframes=F, rows=(r0, r1), in_frame_stride=W * H * 3,
                         out_frame_stride=(nbs + 2 * nbcs) * 64)
        ws = torch.empty(max(jpgx.workspace_size(fr), 1), dtype=torch.uint8, device=cuda)
        jpgx.blocks_gpu(fr, p, d_in.data_ptr() + r0 * 8 * W * 3, o, ws)
        c0 = jpgx.chroma_blocks(W, 0, r0, sr, S)
        out[:, r0 * (W // 8):r1 * (W // 8)] = o[:, :nbs]
        for ch in range(2):
            out[:, nb + ch * nbc + c0:nb + ch * nbc + c0 + nbcs] = o[:, nbs + ch * nbcs:nbs + (ch + 1) * nbcs]
    got = out.cpu().numpy()
    for f in range(F):
        assert np.array_equal(got[f], want[f]), f"frame {f}"


@pytest.mark.gpu
@pytest.mark.parametrize("sr", [1, 2])
def test_gpu_subsample_4k_batch_golden(cuda, impl, sr):
    """4 x 3840x2160 q75 true 4:2:2 / 4:2:0 frames in one launch, generated on the GPU, every
    frame hashed against the oracle hashes in tests/golden/big_golden.json (sub_4k_q75)."""
    import hashlib
    import json
    import os

    import torch
    from conftest import GOLDEN
    with open(os.path.join(GOLDEN, "big_golden.json")) as f:
        ent = json.load(f)["sub_4k_q75"]
    W, H, q = ent["W"], ent["H"], ent["quality"]
    S = jpgx.FLAG_SUBSAMPLE
    F = len(ent["seeds"])
    d_in = torch.empty(F * W * H * 3, dtype=torch.uint8, device=cuda)
    for i, seed in enumerate(ent["seeds"]):
        jpgx.gen_splitmix_gpu(d_in[i * W * H * 3:(i + 1) * W * H * 3], seed)
    nb = (H // 8) * (W // 8)
    per = nb + 2 * jpgx.chroma_blocks(W, 0, H // 8, sr, S)
    out = torch.empty((F, per, 64), dtype=torch.int16, device=cuda)
    fr = jpgx.frames(W, H, nframes=F, out_frame_stride=per * 64)
    jpgx.blocks_gpu(fr, jpgx.default_params(W, H, q, sr, flags=S), d_in, out, 0)
    got = out.cpu().numpy()
    bad = [seed for i, seed in enumerate(ent["seeds"])
           if hashlib.sha256(got[i].astype("<i2").tobytes()).hexdigest()
           != ent[f"sr{sr}_coef_sha256"][i]]
    assert not bad, f"frames with wrong coefficients (seeds): {bad}"


@pytest.mark.gpu
@pytest.mark.parametrize("W,H", [(272, 48), (48, 32), (528, 16)])
def test_gpu_sub420_partial_tiles_and_frames(cuda, impl, W, H):
    """MCU rows of 17, 3 and 33 MCUs (partial 16-MCU tiles, a row's last block in the quirk
    column), 3 frames in one launch, and a 2-block-row stripe pair through the device entry."""
    import torch
    F, q = 3, 70
    frames = [O.gen_splitmix(300 + W + f, W, H) for f in range(F)]
    S = jpgx.FLAG_SUBSAMPLE
    nb = (H // 8) * (W // 8)
    per = nb + 2 * jpgx.chroma_blocks(W, 0, H // 8, 2, S)
    out = torch.zeros((F, per, 64), dtype=torch.int16, device=cuda)
    fr = jpgx.frames(W, H, nframes=F, out_frame_stride=per * 64)
    jpgx.blocks_gpu(fr, jpgx.default_params(W, H, q, 2, flags=S), _dev(np.stack(frames), cuda),
                    out, 0)
    got = out.cpu().numpy()
    for f in range(F):
        want = np.concatenate([O.blocks(frames[f], q, 2)[0],
                               O.chroma_sub(frames[f], q, 2).reshape(-1, 64)])
        bad = np.argwhere(got[f] != want)
        assert len(bad) == 0, f"frame {f}: {len(bad)} mismatches, first {bad[:4].tolist()}"


@pytest.mark.gpu
@pytest.mark.parametrize("W,H,F", [(16, 8, 3), (48, 24, 3), (80, 16, 5), (144, 8, 7)])
@pytest.mark.parametrize("kind", ["random", "tie", "exact"])
def test_gpu_sub422_small_rows(cuda, impl, W, H, F, kind):
    """Block-rows of 2, 6, 10 and 18 blocks: several row-last (x0 = -8 quirk) Y blocks in one
    8-block step, MCUs whose right block is the quirk block, steps across rows and frames and a
    partial last step; tie frames flag chroma coefficients there (the inline exact pass reads a
    quirk MCU's right half from its true rows), FORCE_EXACT sends every coefficient through it."""
    import torch
    q = 50 if kind == "tie" else 85
    frames = [O.gen_tie(W, H) if kind == "tie" else O.gen_splitmix(500 + W + f, W, H)
              for f in range(F)]
    S = jpgx.FLAG_SUBSAMPLE
    flags = S | (jpgx.FLAG_FORCE_EXACT if kind == "exact" else 0)
    nb = (H // 8) * (W // 8)
    per = nb + 2 * jpgx.chroma_blocks(W, 0, H // 8, 1, S)
    guard = 2048
    buf = torch.full((F * per * 64 + guard,), 0x7A7A, dtype=torch.int16, device=cuda)
    fr = jpgx.frames(W, H, nframes=F, out_frame_stride=per * 64)
    jpgx.blocks_gpu(fr, jpgx.default_params(W, H, q, 1, flags=flags), _dev(np.stack(frames), cuda),
                    buf, 0)
    got = buf.cpu().numpy()
    assert (got[F * per * 64:] == 0x7A7A).all(), "write past the end of the output"
    for f in range(F):
        want = np.concatenate([O.blocks(frames[f], q, 1)[0],
                               O.chroma_sub(frames[f], q, 1).reshape(-1, 64)])
        bad = np.argwhere(got[f * per * 64:(f + 1) * per * 64].reshape(per, 64) != want)
        assert len(bad) == 0, f"frame {f}: {len(bad)} mismatches, first {bad[:4].tolist()}"


@pytest.mark.gpu
@pytest.mark.parametrize("W,H,F", [(16, 16, 3), (48, 32, 3), (80, 16, 5), (144, 48, 1), (400, 32, 2)])
@pytest.mark.parametrize("kind", ["random", "tie", "exact"])
def test_gpu_sub420_small_rows(cuda, impl, W, H, F, kind):
    """MCU rows of 1, 3, 5, 9 and 25 MCUs: every MCU or many of them the row's last (x0 = -8
    quirk in both block rows of its right column), steps and step pairs across MCU rows and
    frames, an odd MCU count (a pair whose second step lies past the end); tie frames flag
    chroma coefficients (the inline exact pass: a general pair's MCUs from global memory, a simple
    pair's from its LDS slots), FORCE_EXACT sends every coefficient through it; a sentinel region
    after the output must stay intact."""
    import torch
    q = 50 if kind == "tie" else 85
    frames = [O.gen_tie(W, H) if kind == "tie" else O.gen_splitmix(700 + W + f, W, H)
              for f in range(F)]
    S = jpgx.FLAG_SUBSAMPLE
    flags = S | (jpgx.FLAG_FORCE_EXACT if kind == "exact" else 0)
    nb = (H // 8) * (W // 8)
    per = nb + 2 * jpgx.chroma_blocks(W, 0, H // 8, 2, S)
    guard = 2048
    buf = torch.full((F * per * 64 + guard,), 0x7A7A, dtype=torch.int16, device=cuda)
    fr = jpgx.frames(W, H, nframes=F, out_frame_stride=per * 64)
    jpgx.blocks_gpu(fr, jpgx.default_params(W, H, q, 2, flags=flags), _dev(np.stack(frames), cuda),
                    buf, 0)
    got = buf.cpu().numpy()
    assert (got[F * per * 64:] == 0x7A7A).all(), "write past the end of the output"
    for f in range(F):
        want = np.concatenate([O.blocks(frames[f], q, 2)[0],
                               O.chroma_sub(frames[f], q, 2).reshape(-1, 64)])
        bad = np.argwhere(got[f * per * 64:(f + 1) * per * 64].reshape(per, 64) != want)
        assert len(bad) == 0, f"frame {f}: {len(bad)} mismatches, first {bad[:4].tolist()}"


@pytest.mark.gpu
def test_gpu_sub422_tiles_cross_frames(cuda, impl):
    """nb = 170 blocks per frame (not a multiple of 64): tiles straddle frame ends, the last tile
    is partial, every block row ends in the x0 = -8 quirk column (34 blocks per row)."""
    import torch
    W, H, F, q = 272, 40, 3, 80
    frames = [O.gen_splitmix(90 + f, W, H) for f in range(F)]
    S = jpgx.FLAG_SUBSAMPLE
    nb = (H // 8) * (W // 8)
    per = nb + 2 * jpgx.chroma_blocks(W, 0, H // 8, 1, S)
    out = torch.zeros((F, per, 64), dtype=torch.int16, device=cuda)
    fr = jpgx.frames(W, H, nframes=F, out_frame_stride=per * 64)
    jpgx.blocks_gpu(fr, jpgx.default_params(W, H, q, 1, flags=S), _dev(np.stack(frames), cuda),
                    out, 0)
    got = out.cpu().numpy()
    for f in range(F):
        want = np.concatenate([O.blocks(frames[f], q, 1)[0],
                               O.chroma_sub(frames[f], q, 1).reshape(-1, 64)])
        assert np.array_equal(got[f], want), f"frame {f}"


@pytest.mark.parametrize("sr", [1, 2])
@pytest.mark.parametrize("q", [50, 90])
def test_jfif_subsampled_roundtrip(sr, q):
    """jpgx_write_jfif_sub on the oracle's Y + subsampled chroma: the independent decoder
    (tests/jfif_decode.py, MCU interleave of T.81 A.2.3) returns the same coefficients."""
    from jpgx import compat as C
    from jfif_decode import decode
    W, H = 96, 64
    rgb = O.gen_splitmix(21 + sr, W, H)
    y, c = O.blocks(rgb, q, sr)[0], O.chroma_sub(rgb, q, sr)
    data = C.write_jfif_sub(np.concatenate([y, c.reshape(-1, 64)]), W, H, q, sr)
    d = decode(data)
    assert d["sampling"] == ((2, 1) if sr == 1 else (2, 2))
    assert np.array_equal(d["coef"][0], y)
    assert np.array_equal(d["coef"][1], c[0]) and np.array_equal(d["coef"][2], c[1])


@pytest.mark.parametrize("sr", [1, 2])
def test_jfif_subsampled_decodes_with_pil(sr):
    """libjpeg (PIL) decodes the subsampled file; on a smooth frame its image is close to the
    decode of the 4:4:4 file of the same pipeline (same Cb sign quirk in both)."""
    import io
    Image = pytest.importorskip("PIL.Image")
    from jpgx import compat as C
    W, H = 128, 64
    yy, xx = np.mgrid[0:H, 0:W]
    rgb = np.stack([(xx * 2) % 256, (yy * 4) % 256, ((xx + yy) * 1.5) % 256], -1).astype(np.uint8)
    full = O.blocks(rgb, 90)
    y, c = O.blocks(rgb, 90, sr)[0], O.chroma_sub(rgb, 90, sr)
    a = np.asarray(Image.open(io.BytesIO(C.write_jfif(full, W, H, 90))).convert("RGB"), float)
    img = Image.open(io.BytesIO(C.write_jfif_sub(np.concatenate([y, c.reshape(-1, 64)]), W, H, 90, sr)))
    assert img.size == (W, H)
    b = np.asarray(img.convert("RGB"), float)
    psnr = 10 * np.log10(255 ** 2 / np.mean((a - b) ** 2))
    assert psnr > 30, psnr


@pytest.mark.gpu
@pytest.mark.parametrize("sr", [1, 2])
def test_gpu_encode_bmp_to_jpeg_subsampled(tmp_path, cuda, sr):
    """BMP in, truly subsampled JPEG out (jpgx_encode_bmp_to_jpeg_ex on the GPU)."""
    from jpgx import compat as C
    from jfif_decode import decode
    W, H = 256, 128
    rgb = O.gen_splitmix(31, W, H)
    src, dst = str(tmp_path / "in.bmp"), str(tmp_path / "out.jpg")
    O.write_bmp(src, rgb)
    C.encode_bmp_to_jpeg_ex(src, dst, 75, sr, jpgx.FLAG_SUBSAMPLE)
    d = decode(open(dst, "rb").read())
    assert np.array_equal(d["coef"][0], O.blocks(rgb, 75, sr)[0])
    c = O.chroma_sub(rgb, 75, sr)
    assert np.array_equal(d["coef"][1], c[0]) and np.array_equal(d["coef"][2], c[1])


def test_subsample_argument_errors():
    """Validation happens before any device work: no GPU needed."""
    S = jpgx.FLAG_SUBSAMPLE
    W, H = 64, 64
    fake = 1 << 20                                   # never dereferenced
    p = jpgx.default_params(W, H, 75, 0, flags=S)
    fr = jpgx.frames(W, H)
    rc = jpgx.lib.jpgx_blocks_gpu(__import__("ctypes").byref(fr), __import__("ctypes").byref(p),
                                  fake, fake, fake, 0, None)
    assert rc == jpgx.ESAMPLE                       # the flag needs sample_ratio 1 or 2
    p = jpgx.default_params(W, H, 75, 2, flags=S)
    fr = jpgx.frames(W, H, rows=(1, 4))
    rc = jpgx.lib.jpgx_blocks_gpu(__import__("ctypes").byref(fr), __import__("ctypes").byref(p),
                                  fake, fake, fake, 0, None)
    assert rc == jpgx.EARG                          # 4:2:0 stripes start on even block rows
