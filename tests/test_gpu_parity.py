"""GPU parity: libjpgx.so (HIP, gfx950) against the oracle and the reference's golden vectors.
Bit-exact int16 coefficients are required everywhere (integer output: no tolerance)."""
import os

import numpy as np
import pytest

import jpgx
import oracle as O
from conftest import GOLDEN, coef_sha

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True, params=["xform", "mx"])
def kernel(request, monkeypatch):
    """Every parity test runs on both 4:4:4 kernels: k_mxs (colour + row DCT on the matrix
    cores, csrc/jpgx_mx.hip: the product library's kernel) and k_xform (all-VALU), which only
    the test-only cross-check library libjpgx_alt.so dispatches."""
    if request.param == "xform":
        monkeypatch.setattr(jpgx, "lib", jpgx.alt_library())
    return request.param


def _dev(a, cuda):
    import torch
    return torch.from_numpy(np.ascontiguousarray(a)).to(cuda)


def _gpu(rgb, q, cuda, sr=0, underflow=None, flags=0):
    out = jpgx.encode_blocks(_dev(rgb, cuda), q, sr, underflow=underflow, flags=flags)
    return out.cpu().numpy()


def _frame(ent):
    if ent["kind"] == "G":
        return O.gen_splitmix(ent["seed"], ent["W"], ent["H"])
    return O.gen_tie(ent["W"], ent["H"])


def test_golden_synthetic(golden, cuda):
    for ent in golden["synthetic"]:
        rgb = _frame(ent)
        for q, h in ent["coef_sha256"].items():
            out = _gpu(rgb, int(q), cuda, underflow=ent["underflow"])
            if coef_sha(out) != h:
                ref = O.blocks(rgb, int(q), underflow=ent["underflow"])
                bad = np.argwhere(out != ref)
                pytest.fail(f"{ent['kind']} {ent['W']}x{ent['H']} q{q}: {len(bad)} mismatches, "
                            f"first {bad[:5].tolist()}")
        if "coef_sha256_sr1" in ent:
            q0 = int(next(iter(ent["coef_sha256"])))
            out = _gpu(rgb, q0, cuda, sr=1, underflow=ent["underflow"])
            assert coef_sha(out) == ent["coef_sha256_sr1"]


@pytest.mark.parametrize("name", ["cam", "tiger"])
def test_golden_images(golden, cuda, name):
    data = open(os.path.join(GOLDEN, "images", f"{name}.bmp"), "rb").read()
    rgb = O.bmp_decode(data)
    ent = golden["images"][name]
    for q, h in ent["coef_sha256"].items():
        assert coef_sha(_gpu(rgb, int(q), cuda, underflow=ent["underflow"])) == h, (name, q)


def test_force_exact_path(golden, cuda):
    """Every coefficient through the exact fp64 path must still be bit-exact."""
    for ent in golden["synthetic"]:
        if ent["W"] * ent["H"] > 512 * 512:
            continue
        rgb = _frame(ent)
        q = next(iter(ent["coef_sha256"]))
        out = _gpu(rgb, int(q), cuda, underflow=ent["underflow"], flags=jpgx.FLAG_FORCE_EXACT)
        assert coef_sha(out) == ent["coef_sha256"][q], (ent["W"], ent["H"], q)


@pytest.mark.parametrize("q", list(range(1, 98, 4)) + [97])
def test_quality_sweep(cuda, q):
    rgb = O.gen_splitmix(1000 + q, 136, 64)
    assert np.array_equal(_gpu(rgb, q, cuda), O.blocks(rgb, q))


@pytest.mark.parametrize("W,H", [(8, 8), (8, 64), (64, 8), (16, 16), (24, 40), (520, 8)])
def test_edge_geometries(cuda, W, H):
    rgb = O.gen_splitmix(W * 1000 + H, W, H)
    uf = np.arange(24, dtype=np.uint8).reshape(3, 8) * 7 + 3   # distinct per plane
    for q in (30, 90):
        assert np.array_equal(_gpu(rgb, q, cuda, underflow=uf), O.blocks(rgb, q, underflow=uf))


def test_tie_frame_every_dc_is_a_tie(cuda):
    """T frame at q50: every Y DC is an exact .5 tie (fp32 and fp64-separable fail here)."""
    rgb = O.gen_tie(512, 512)
    assert np.array_equal(_gpu(rgb, 50, cuda), O.blocks(rgb, 50))


def _sparse_tie(W, H, seed, every):
    """Random frame with every `every`-th block replaced by a flat tie block (gen_tie): at q50 its
    Y DC is an exact .5 tie, so steps carry one flagged coefficient (the inline exact pass's
    whole-wave path, whose tree sum then sees a near-tie and falls back) or several (its 8-lane
    batches)."""
    rgb = O.gen_splitmix(seed, W, H)
    tie = O.gen_tie(W, H)
    bpr = W // 8
    for bi in range(3, (W // 8) * (H // 8), every):
        r, c = divmod(bi, bpr)
        rgb[8 * r:8 * r + 8, 8 * c:8 * c + 8] = tie[8 * r:8 * r + 8, 8 * c:8 * c + 8]
    return rgb


# Gray blocks whose rows are constant across x (only column u = 0 non-zero) with two coefficients
# of that column at (or within 1e-5 of) a .5 boundary: at q50 v = 0 and v = 4 are both exact ties
# (found by a search over the reference's double arithmetic), at q90 v = 1 and v = 2 -- one
# column with two flagged coefficients per such block (a lane with several flag bits: the exact
# pass's 8-lane batches, never the single-coefficient path).
MULTI_V = {50: [[182, 101, 34, 200, 52, 82, 221, 160], [143, 34, 169, 120, 73, 231, 148, 66], [80, 198, 94, 81, 204, 128, 10, 29], [165, 172, 249, 77, 160, 231, 2, 120], [115, 230, 107, 220, 81, 126, 15, 122], [93, 65, 27, 115, 251, 160, 158, 227]],
           90: [[53, 16, 72, 210, 179, 226, 163, 184]]}


@pytest.mark.parametrize("q", [50, 90])
def test_multi_v_flagged_columns(cuda, q):
    rgb = O.gen_splitmix(900 + q, 1024, 128)
    pats = MULTI_V[q]
    bpr = 1024 // 8
    for i, bi in enumerate(range(5, bpr * 16, 11)):
        r, c = divmod(bi, bpr)
        col = np.array(pats[i % len(pats)], np.uint8)[:, None, None]
        rgb[8 * r:8 * r + 8, 8 * c:8 * c + 8] = col
    assert np.array_equal(_gpu(rgb, q, cuda), O.blocks(rgb, q))


@pytest.mark.parametrize("every", [5, 13, 61])
def test_sparse_tie_exact_pass(cuda, every):
    rgb = _sparse_tie(1024, 256, 77 + every, every)
    for q in (50, 90, 97):
        assert np.array_equal(_gpu(rgb, q, cuda), O.blocks(rgb, q)), f"q{q}"


@pytest.mark.parametrize("W,F", [(8, 1), (24, 1), (520, 1), (24, 3), (40, 5)])
def test_tail_step_guard_region(cuda, W, F):
    """Launches whose block count is not a multiple of 8 (the last step's missing blocks are
    clamped copies of the last one) on tie frames (flagged DCs, so the exact pass runs on the
    last step): the output equals the oracle and a sentinel region after it stays untouched."""
    import torch
    H, q = 8, 50
    frames = [O.gen_tie(W, H) for _ in range(F)]
    nb = (H // 8) * (W // 8)
    guard = 4096
    buf = torch.full((F * 3 * nb * 64 + guard,), 0x7A7A, dtype=torch.int16, device=cuda)
    fr = jpgx.frames(W, H, nframes=F)
    ws = torch.empty(max(jpgx.workspace_size(fr), 1), dtype=torch.uint8, device=cuda)
    jpgx.blocks_gpu(fr, jpgx.default_params(W, H, q), _dev(np.stack(frames), cuda), buf, ws)
    got = buf.cpu().numpy()
    assert (got[F * 3 * nb * 64:] == 0x7A7A).all(), "write past the end of the output"
    for f in range(F):
        assert np.array_equal(got[f * 3 * nb * 64:(f + 1) * 3 * nb * 64].reshape(3, nb, 64),
                              O.blocks(frames[f], q)), f


def test_batch_and_stripes(cuda):
    """A batch of frames in one launch, and block-row stripes with the one-row halo, give the
    same output as frame-by-frame whole images."""
    import torch
    W, H, F, q = 96, 64, 3, 85
    frames = [O.gen_splitmix(70 + f, W, H) for f in range(F)]
    host = np.stack(frames)
    d_in = _dev(host, cuda)
    p = jpgx.default_params(W, H, q)
    nb = (H // 8) * (W // 8)
    fr = jpgx.frames(W, H, nframes=F)
    out = torch.zeros((F, 3, nb, 64), dtype=torch.int16, device=cuda)
    ws = torch.empty(jpgx.workspace_size(fr), dtype=torch.uint8, device=cuda)
    jpgx.blocks_gpu(fr, p, d_in, out, ws)
    got = out.cpu().numpy()
    for f in range(F):
        assert np.array_equal(got[f], O.blocks(frames[f], q)), f
    # stripes: rows [r0, r1) of every frame, input pointer at pixel row 8*r0
    bpr = W // 8
    for r0, r1 in [(0, 3), (3, 5), (5, 8)]:
        frs = jpgx.frames(W, H, nframes=F, rows=(r0, r1))
        nbs = (r1 - r0) * bpr
        o = torch.zeros((F, 3, nbs, 64), dtype=torch.int16, device=cuda)
        ws = torch.empty(jpgx.workspace_size(frs), dtype=torch.uint8, device=cuda)
        base = d_in.data_ptr() + r0 * 8 * W * 3
        jpgx.blocks_gpu(frs, p, base, o, ws)
        o = o.cpu().numpy()
        for f in range(F):
            assert np.array_equal(o[f], O.blocks(frames[f], q, rows=(r0, r1))), (f, r0, r1)


def test_host_buffer_entry_points(cuda):
    rgb = O.gen_splitmix(9, 200, 120)
    ref = O.blocks(rgb, 77)
    assert np.array_equal(jpgx.encode_blocks(rgb, 77), ref)
    n = jpgx.device_count()
    assert np.array_equal(jpgx.encode_blocks_multi(rgb, 77, n), ref)
    with pytest.raises(jpgx.JpgxError):
        jpgx.encode_blocks_multi(rgb, 77, n + 1)


def test_invalid_arguments_gpu(cuda):
    import torch
    rgb = torch.zeros((16, 16, 3), dtype=torch.uint8, device=cuda)
    with pytest.raises(jpgx.JpgxError) as e:
        jpgx.encode_blocks(rgb, 98)
    assert e.value.rc == jpgx.EQUALITY
    with pytest.raises(jpgx.JpgxError) as e:
        jpgx.encode_blocks(torch.zeros((16, 12, 3), dtype=torch.uint8, device=cuda), 50)
    assert e.value.rc == jpgx.EGEOMETRY
    fr = jpgx.frames(16, 16)
    out = torch.zeros((3, 4, 64), dtype=torch.int16, device=cuda)
    with pytest.raises(jpgx.JpgxError) as e:        # misaligned input pointer
        jpgx.blocks_gpu(fr, jpgx.default_params(16, 16, 50), rgb.data_ptr() + 3, out, 0)
    assert e.value.rc == jpgx.EARG
    with pytest.raises(jpgx.JpgxError) as e:        # stripe beyond the frame
        jpgx.blocks_gpu(jpgx.frames(16, 16, rows=(1, 3)), jpgx.default_params(16, 16, 50), rgb,
                        out, 0)
    assert e.value.rc == jpgx.EARG
    assert jpgx.workspace_size(fr) == 0             # no workspace: NULL / 0 bytes accepted
    jpgx.blocks_gpu(fr, jpgx.default_params(16, 16, 50), rgb, out, 0)
    torch.cuda.synchronize()
    assert np.array_equal(out.cpu().numpy(), O.blocks(np.zeros((16, 16, 3), np.uint8), 50))
    ws = torch.empty(64, dtype=torch.uint8, device=cuda)
    with pytest.raises(jpgx.JpgxError) as e:        # misaligned workspace pointer
        jpgx.blocks_gpu(fr, jpgx.default_params(16, 16, 50), rgb, out, ws.data_ptr() + 4)
    assert e.value.rc == jpgx.EWORKSPACE


def test_gpu_generators_match_oracle(cuda):
    import torch
    for W, H, seed in [(64, 40, 3), (3840, 16, 77)]:
        d = torch.empty((H, W, 3), dtype=torch.uint8, device=cuda)
        jpgx.gen_splitmix_gpu(d, seed)
        assert np.array_equal(d.cpu().numpy(), O.gen_splitmix(seed, W, H))
    d = torch.empty((64, 48, 3), dtype=torch.uint8, device=cuda)
    jpgx.gen_tie_gpu(d, 48, 64)
    assert np.array_equal(d.cpu().numpy(), O.gen_tie(48, 64))


def test_large_frames_hash(golden, cuda):
    """1080p q90 and 4K q90/q75 generated on the GPU, hashed against the reference."""
    import torch
    for ent in golden["synthetic"]:
        if ent["W"] * ent["H"] < 1920 * 1080:
            continue
        W, H = ent["W"], ent["H"]
        d = torch.empty((H, W, 3), dtype=torch.uint8, device=cuda)
        jpgx.gen_splitmix_gpu(d, ent["seed"])
        for q, h in ent["coef_sha256"].items():
            out = jpgx.encode_blocks(d, int(q), underflow=ent["underflow"]).cpu().numpy()
            assert coef_sha(out) == h, (W, H, q)
        if (W, H) == (3840, 2160):
            # BASELINE configs[2] literally: 4K, sample_ratio 1 ("4:2:2"), q=75 -- the
            # reference's chroma_subsample is a no-op (src/downsample.c:24-32), so its output is
            # the 4:4:4 one (every sr1 golden above equals its sr0 hash)
            out = jpgx.encode_blocks(d, 75, sample_ratio=1, underflow=ent["underflow"]).cpu().numpy()
            assert coef_sha(out) == ent["coef_sha256"]["75"]


@pytest.mark.parametrize("q", [10, 50, 75, 90])
def test_force_exact_with_ties(cuda, q):
    """FORCE_EXACT on a frame with flat tie blocks: batches of the exact pass mix coefficients the
    fast decision settles with exact .5 ties that must take the sequential sum (mx_exact_sum)"""
    rgb = _sparse_tie(256, 128, 11, 3)
    assert np.array_equal(_gpu(rgb, q, cuda, flags=jpgx.FLAG_FORCE_EXACT), O.blocks(rgb, q))
