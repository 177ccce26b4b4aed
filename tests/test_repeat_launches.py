"""Repeated launches against the oracle (GPU): the round-4 chained-MFMA operand hazard
(profiles/r04_mfma_valu_war.txt) showed as a few wrong 8x8 blocks in 1-3 % of
launches -- rare enough to pass every single-launch parity test.  Here each launch mode runs many
times on the same two 4K frames and every block of every launch is compared, on the GPU, with the
oracle's output (bit-exact).  The ISA-level rule that prevents it is checked on every build by
tests/test_isa.py; this is the behavioural check."""
import numpy as np
import pytest

import jpgx
import oracle as O

pytestmark = pytest.mark.gpu

W, H, Q, SEEDS = 3840, 2160, 75, (1000, 1001)
LAUNCHES = 40


@pytest.fixture(scope="module")
def frames():
    return [O.gen_splitmix(s, W, H) for s in SEEDS]


@pytest.mark.parametrize("sr", [0, 1, 2])
def test_repeated_launches_match_the_oracle(cuda, frames, sr):
    import torch
    S = jpgx.FLAG_SUBSAMPLE if sr else 0
    nb = (H // 8) * (W // 8)
    nbc = jpgx.chroma_blocks(W, 0, H // 8, sr, S) if sr else nb
    per = nb + 2 * nbc
    if sr:
        want = np.stack([np.concatenate([O.blocks(f, Q, sr)[0], O.chroma_sub(f, Q, sr).reshape(-1, 64)])
                         for f in frames])
    else:
        want = np.stack([O.blocks(f, Q).reshape(-1, 64) for f in frames])
    d_in = torch.from_numpy(np.ascontiguousarray(np.stack(frames))).to(cuda)
    d_want = torch.from_numpy(want).to(cuda)
    fr = jpgx.frames(W, H, nframes=len(frames), out_frame_stride=per * 64)
    p = jpgx.default_params(W, H, Q, sr, flags=S)
    out = torch.empty((len(frames), per, 64), dtype=torch.int16, device=cuda)
    wrong = []
    for r in range(LAUNCHES):
        out.fill_(0x5a5a)
        jpgx.blocks_gpu(fr, p, d_in, out, 0)
        bad = torch.nonzero((out != d_want).any(dim=2))
        if len(bad):
            wrong.append((r, len(bad), bad[:4].cpu().tolist()))
    assert not wrong, f"launches with wrong blocks (launch, count, first [frame, block]): {wrong}"
