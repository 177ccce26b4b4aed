"""BASELINE.json configs[4] at its full size: a 16384x16384 frame, sample_ratio 1 (the
reference's "4:2:2", whose output is 4:4:4), q=50, split into the 8 block-row stripes of an
8-GPU node and stitched.  The oracle cannot run the whole frame in test time, so the checks are
size-independent: every stripe launch equals the same block-rows of the whole-frame launch
(the halo row and the x0 = -8 quirk across stripe seams), sampled block-rows (the first, whose
last block reads the glibc chunk word of a 16384^2 plane -- the mmap case of
jpgx_glibc_underflow -- the rows on both sides of a seam, the last) equal the oracle bit for
bit, and the entropy stage's DC recurrence / Huffman frequency tables stitch across stripes
with the carried DCs (the host-side dpcm + huffman stitch of that config)."""
import numpy as np
import pytest

import jpgx
import oracle as O

pytestmark = pytest.mark.gpu

W = H = 16384
Q, SR, SEED, NGPU = 50, 1, 5, 8


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


def test_underflow_is_the_mmap_chunk_word():
    # a 16384^2 plane is mmapped: size rounded to pages | IS_MMAPPED
    assert jpgx.glibc_underflow(W * H).hex() == "0210001000000000"


def test_stripes_equal_whole_frame(frame, cuda):
    import torch
    d_in, out, p = frame
    bpr = W // 8
    for k in range(NGPU):
        r0, r1 = jpgx.stripe(H // 8, NGPU, k)
        fr = jpgx.frames(W, H, rows=(r0, r1))
        o = torch.empty((3, (r1 - r0) * bpr, 64), dtype=torch.int16, device=cuda)
        ws = torch.empty(jpgx.workspace_size(fr), dtype=torch.uint8, device=cuda)
        jpgx.blocks_gpu(fr, p, d_in.data_ptr() + r0 * 8 * W * 3, o, ws)
        assert torch.equal(o, out[:, r0 * bpr:r1 * bpr]), (k, r0, r1)
        del o, ws


def test_sampled_block_rows_match_oracle(frame):
    d_in, out, p = frame
    bpr = W // 8
    under = np.frombuffer(bytes(p.underflow[0]) + bytes(p.underflow[1]) + bytes(p.underflow[2]),
                          np.uint8).reshape(3, 8)
    seam = jpgx.stripe(H // 8, NGPU, 1)[0]
    for r in (0, 1, seam - 1, seam, H // 8 - 1):
        top = max(0, 8 * r - 8)
        rows = d_in[top * W * 3:(8 * r + 8) * W * 3].cpu().numpy().reshape(-1, W, 3)
        want = O.blocks(rows, Q, SR, underflow=under, rows=(0, 1) if r == 0 else (1, 2))
        got = out[:, r * bpr:(r + 1) * bpr].cpu().numpy()
        assert np.array_equal(got, want), r


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
    want_b = np.concatenate([dc_all[c * nb + s:(c + 1) * nb] for c in range(3)])
    assert np.array_equal(dcb.cpu().numpy(), want_b)
    tot = ha.cpu().numpy().astype(np.int64) + hb.cpu().numpy()
    tot[:, 256] -= 1                        # freq[256] = 1 once per huffman_encode call
    assert np.array_equal(tot, hist_all.cpu().numpy())
