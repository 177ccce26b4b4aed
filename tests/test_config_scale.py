"""BASELINE.json configs[4] at its full size: a 16384x16384 frame, sample_ratio 1 (the
reference's "4:2:2", whose output is 4:4:4), q=50, split into the 8 block-row stripes of an
8-GPU node and stitched.  Pinned to the REAL reference, run once on this very frame in the
build container (tests/golden/make_big_golden.py -> big_golden.json, about 24 min): the
whole-frame output hash, per-channel and per-stripe hashes, and the glibc chunk word the
reference really read in front of each plane (the x0 = -8 underflow of block-row 0 in the mmap
case, src/preprocess.c:127-129,159-160 after src/bitmap.c:113,151).  The stripe launches are
also checked against the whole-frame launch, and the entropy stage's DC recurrence / Huffman
frequency tables stitch across stripes with the carried DCs (the host-side dpcm + huffman
stitch of that config)."""
import hashlib
import json
import os

import numpy as np
import pytest

import jpgx
import oracle as O
from conftest import GOLDEN

pytestmark = pytest.mark.gpu

W = H = 16384
Q, SR, SEED, NGPU = 50, 1, 5, 8


@pytest.fixture(scope="module")
def ref():
    with open(os.path.join(GOLDEN, "big_golden.json")) as f:
        g = json.load(f)["frame16k_q50_sr1"]
    assert (g["W"], g["H"], g["quality"], g["sample_ratio"], g["seed"]) == (W, H, Q, SR, SEED)
    return g


def _sha(t) -> str:
    return hashlib.sha256(t.contiguous().cpu().numpy().astype("<i2").tobytes()).hexdigest()


@pytest.fixture(scope="module")
def frame(cuda):
    import torch
    d_in = torch.empty(W * H * 3, dtype=torch.uint8, device=cuda)
    jpgx.gen_splitmix_gpu(d_in, SEED)
    p = jpgx.default_params(W, H, Q, SR)
    nb = (W // 8) * (H // 8)
    out = torch.empty((3, nb, 64), dtype=torch.int16, device=cuda)
    fr = jpgx.frames(W, H)
    ws = torch.empty(jpgx.workspace_size(fr), dtype=torch.uint8, device=cuda)
    jpgx.blocks_gpu(fr, p, d_in, out, ws)
    torch.cuda.synchronize()
    yield d_in, out, p
    del d_in, out, ws
    torch.cuda.empty_cache()


def test_underflow_is_the_real_mmap_chunk_word(ref):
    # the bytes the reference really read (a 16384^2 plane is mmapped: size
    # rounded to pages | IS_MMAPPED), equal to jpgx_glibc_underflow's model
    assert [bytes(u).hex() for u in ref["underflow"]] == ["0210001000000000"] * 3
    assert jpgx.glibc_underflow(W * H).hex() == "0210001000000000"


def test_input_is_the_reference_frame(frame, ref):
    d_in, _, _ = frame
    h = hashlib.sha256()
    step = 1 << 28
    for o in range(0, d_in.numel(), step):
        h.update(d_in[o:o + step].cpu().numpy().tobytes())
    assert h.hexdigest() == ref["input_sha256"]


def test_whole_frame_equals_reference(frame, ref):
    """Every coefficient of the 16384^2 frame equals the real reference's output."""
    _, out, _ = frame
    assert _sha(out[:, :W // 8]) == ref["block_row0_sha256"]      # the mmap-underflow row
    assert [_sha(out[c]) for c in range(3)] == ref["channel_sha256"]
    assert _sha(out) == ref["coef_sha256"]


def test_stripes_equal_whole_frame(frame, cuda, ref):
    import torch
    d_in, out, p = frame
    bpr = W // 8
    for k in range(NGPU):
        r0, r1 = jpgx.stripe(H // 8, NGPU, k)
        fr = jpgx.frames(W, H, rows=(r0, r1))
        o = torch.empty((3, (r1 - r0) * bpr, 64), dtype=torch.int16, device=cuda)
        ws = torch.empty(jpgx.workspace_size(fr), dtype=torch.uint8, device=cuda)
        jpgx.blocks_gpu(fr, p, d_in.data_ptr() + r0 * 8 * W * 3, o, ws)
        assert [r0, r1] == ref["stripes8"][k]["rows"]
        assert torch.equal(o, out[:, r0 * bpr:r1 * bpr]), (k, r0, r1)
        assert _sha(o) == ref["stripes8"][k]["coef_sha256"], (k, r0, r1)
        del o, ws


def test_entropy_stats_stitch_across_stripes(frame):
    d_in, out, p = frame
    nb = out.shape[1]
    dc_all, hist_all = jpgx.entropy_stats_gpu(out, nb, nb)
    s = jpgx.stripe(H // 8, 2, 0)[1] * (W // 8)
    a = out[:, :s].contiguous()
    b = out[:, s:].contiguous()
    dca, ha = jpgx.entropy_stats_gpu(a, s, s)
    carry = [int(dca[c * s + s - 1]) for c in range(3)]
    dcb, hb = jpgx.entropy_stats_gpu(b, nb - s, nb - s, carry)
    dc_all = dc_all.cpu().numpy()
    # the whole frame against the oracle: 4.19 M blocks per channel, so k_ent_dc's loop over more
    # than 1,024 earlier chunk sums (reached above ~524 K blocks per channel) runs here
    rdc, rhist = O.entropy_stats(out.cpu().numpy())
    assert np.array_equal(dc_all, rdc)
    assert np.array_equal(hist_all.cpu().numpy(), rhist)
    want_b = np.concatenate([dc_all[c * nb + s:(c + 1) * nb] for c in range(3)])
    assert np.array_equal(dcb.cpu().numpy(), want_b)
    tot = ha.cpu().numpy().astype(np.int64) + hb.cpu().numpy()
    tot[:, 256] -= 1                        # freq[256] = 1 once per huffman_encode call
    assert np.array_equal(tot, hist_all.cpu().numpy())


def test_jfif_stitch_of_the_stripes(frame, ref):
    """The host entropy stage of configs[4]: the 16384^2 frame's coefficients
    -> one JFIF with restart intervals of 16 MCU rows (DRI = 32768 MCUs; every GPU stripe
    boundary, 256 rows, is an interval boundary), coded on 8 host threads -- one per stripe -- and
    concatenated; the independent T.81 decoder (tests/c/jfif_dec.c, 8 threads over the RSTm
    markers) returns every coefficient: the whole-frame hash of the real reference.  Parity of
    the bitstream itself is unpinned (the reference's Huffman stage never terminates)."""
    import time

    import jpgx.compat as C
    from test_jfif_restart import jfd_decode
    import ctypes
    import subprocess
    from conftest import REPO
    subprocess.run(["make", "-s", "-C", os.path.join(REPO, "tests", "c"), "jfd"], check=True)
    lib = ctypes.CDLL(os.path.join(REPO, "tests", "c", "_build", "libjfd.so"))
    lib.jfd_decode.restype = ctypes.c_int
    lib.jfd_decode.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_size_t,
                               ctypes.c_int, ctypes.c_void_p]
    _, out, _ = frame
    coef = out.cpu().numpy()
    t0 = time.perf_counter()
    data = C.write_jfif_ex(coef, W, H, Q, 0, restart_rows=16, nthreads=NGPU, cap=coef.nbytes // 2)
    dt = time.perf_counter() - t0
    print(f"\n16384^2 q{Q}: JFIF {len(data) / 1e6:.1f} MB in {dt:.2f} s on {NGPU} threads "
          f"({W * H / dt / 1e6:.0f} Mpx/s)")
    got, info = jfd_decode(lib, data, coef.size, NGPU)
    assert info[4] == 16 * (W // 8) and info[5] == (H // 8) // 16 - 1
    assert hashlib.sha256(got.astype("<i2").tobytes()).hexdigest() == ref["coef_sha256"]
