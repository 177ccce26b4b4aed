"""BASELINE.json configs[3] at its full size: a batch of 64 synthetic 3840x2160 frames, 4:4:4,
q=90, row-stripe sharded across 8 GPUs -- run here on ONE GPU as the 8 rank plans bench.py
uses at N=8 (bench.rank_plan: each rank's block-row stripe of every frame, the one-pixel-row
halo above a stripe that does not start at row 0, the per-rank splitmix seeds that make its
bytes equal the same rows of the global frame).  The 8 stripe outputs of every frame are
stitched and hashed against tests/golden/big_golden.json (the oracle restatement, pinned to
the real reference on frame 1000 and at 4K in test_oracle.py).

Every stripe seam crosses the x0 = -8 quirk (src/preprocess.c:199-211: the last block of a
block-row reads the previous pixel row, i.e. the halo row for a stripe's first block-row), so
general steps (register-loaded, with the quirk block) fall at every stripe's block-row ends and
frame ends inside one launch of k_mxs's short-lived waves (three 8-block steps per wave), with
the inline exact pass on the flagged steps of every frame."""
import hashlib
import json
import os

import numpy as np
import pytest

import bench
import jpgx
from conftest import GOLDEN

pytestmark = pytest.mark.gpu

NGPU, FPG = 8, 8


@pytest.fixture(scope="module")
def batch():
    with open(os.path.join(GOLDEN, "big_golden.json")) as f:
        return json.load(f)["batch64_4k_q90"]


@pytest.fixture(params=["xform", "mx"])
def kernel(request, monkeypatch):
    """k_mxs (the product library's 4:4:4 kernel) and k_xform (the test-only libjpgx_alt.so)"""
    if request.param == "xform":
        monkeypatch.setattr(jpgx, "lib", jpgx.alt_library())
    return request.param


def _frame_sha(parts):
    """sha256 of one frame's [3][nb][64] int16 output given its stripes' [3][nb_r][64] parts."""
    import torch
    whole = torch.cat(parts, dim=1).contiguous().cpu().numpy()
    return hashlib.sha256(whole.astype("<i2").tobytes()).hexdigest()


def _run_rank(plan, W, H, q, cuda, flags=0, frames=None):
    """One rank's launch over its stripe of the frames `frames` (default: the whole batch),
    inputs generated on the device exactly as bench.py does."""
    import torch
    fl = list(range(plan["B"])) if frames is None else list(frames)
    B, fstride = len(fl), plan["fstride"]
    d_in = torch.empty(B * fstride, dtype=torch.uint8, device=cuda)
    for i, f in enumerate(fl):
        jpgx.gen_splitmix_gpu(d_in[i * fstride:(i + 1) * fstride], plan["seeds"][f])
    nb = plan["nb"]
    out = torch.empty((B, 3, nb, 64), dtype=torch.int16, device=cuda)
    fr = jpgx.frames(W, H, nframes=B, rows=(plan["r0"], plan["r1"]), in_pitch=plan["row_bytes"],
                     in_frame_stride=fstride, out_frame_stride=3 * nb * 64)
    ws = torch.empty(jpgx.workspace_size(fr), dtype=torch.uint8, device=cuda)
    p = jpgx.default_params(W, H, q, flags=flags)
    jpgx.blocks_gpu(fr, p, d_in.data_ptr() + plan["halo"] * plan["row_bytes"], out, ws)
    torch.cuda.synchronize()
    del d_in, ws
    return out


def test_plan_covers_the_batch(batch):
    W, H = batch["W"], batch["H"]
    plans = [bench.rank_plan(W, H, FPG, NGPU, r, jpgx) for r in range(NGPU)]
    assert all(p["B"] == len(batch["frames"]) for p in plans)
    assert plans[0]["r0"] == 0 and plans[-1]["r1"] == H // 8
    for a, b in zip(plans, plans[1:]):
        assert a["r1"] == b["r0"] and b["halo"] == 1
    assert [f["seed"] for f in batch["frames"]] == [1000 + f for f in range(64)]


def test_batch64_as_eight_rank_stripes(batch, cuda, kernel):
    """The whole of configs[3]: 8 rank launches of 64 frame-stripes each, every frame's
    stitched output bit-exact against its golden hash."""
    import torch
    W, H, q = batch["W"], batch["H"], batch["quality"]
    outs = [_run_rank(bench.rank_plan(W, H, FPG, NGPU, r, jpgx), W, H, q, cuda)
            for r in range(NGPU)]
    bad = []
    for f, ent in enumerate(batch["frames"]):
        if _frame_sha([o[f] for o in outs]) != ent["coef_sha256"]:
            bad.append(ent["seed"])
    del outs
    torch.cuda.empty_cache()
    assert not bad, f"frames with wrong coefficients (seeds): {bad}"


def test_batch64_single_launch(batch, cuda, kernel):
    """The same 64 frames as ONE launch on one GPU (no stripes): 1,036,800 steps of 8 blocks,
    three steps per short-lived k_mxs wave (345,600 waves, steps crossing frame ends)."""
    import torch
    W, H, q = batch["W"], batch["H"], batch["quality"]
    out = _run_rank(bench.rank_plan(W, H, FPG * NGPU, 1, 0, jpgx), W, H, q, cuda)
    bad = [ent["seed"] for f, ent in enumerate(batch["frames"])
           if _frame_sha([out[f]]) != ent["coef_sha256"]]
    del out
    torch.cuda.empty_cache()
    assert not bad, f"frames with wrong coefficients (seeds): {bad}"


def test_batch_force_exact_multi_tile(batch, cuda, kernel):
    """FLAG_FORCE_EXACT over 8 frames in one launch: every coefficient through the in-kernel
    exact fp64 pass (k_mxs: every step's 192 coefficients in 8-lane batches, inline before the
    step's stores; k_xform: its per-tile queues overflowing and draining on every tile)."""
    import torch
    W, H, q = batch["W"], batch["H"], batch["quality"]
    plan = bench.rank_plan(W, H, FPG, 1, 0, jpgx)
    out = _run_rank(plan, W, H, q, cuda, flags=jpgx.FLAG_FORCE_EXACT, frames=range(8))
    bad = [batch["frames"][f]["seed"] for f in range(8)
           if _frame_sha([out[f]]) != batch["frames"][f]["coef_sha256"]]
    del out
    torch.cuda.empty_cache()
    assert not bad, f"frames with wrong coefficients (seeds): {bad}"


def test_rank_inputs_equal_global_frame_rows(batch, cuda):
    """The per-rank seeds of bench.rank_plan regenerate exactly the rows of the global frame
    (checked on frame 1000 against the golden input hash, stitched from the 8 ranks' stripes
    without their halo rows)."""
    import torch
    W, H = batch["W"], batch["H"]
    rows = []
    for r in range(NGPU):
        p = bench.rank_plan(W, H, FPG, NGPU, r, jpgx)
        d = torch.empty(p["fstride"], dtype=torch.uint8, device=cuda)
        jpgx.gen_splitmix_gpu(d, p["seeds"][0])
        rows.append(d[p["halo"] * p["row_bytes"]:].cpu().numpy())
    whole = np.concatenate(rows)
    assert whole.size == W * H * 3
    assert hashlib.sha256(whole.tobytes()).hexdigest() == batch["frames"][0]["input_sha256"]
