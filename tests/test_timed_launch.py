"""jpgx_blocks_gpu_timed (include/jpgx.h): the same output as jpgx_blocks_gpu, and its event pair
brackets the transform kernel itself (bench.py's roofline.kernel_ms)."""
import numpy as np
import pytest

import jpgx
import oracle as O

@pytest.mark.gpu
@pytest.mark.parametrize("sr,flags", [(0, 0), (1, jpgx.FLAG_SUBSAMPLE), (2, jpgx.FLAG_SUBSAMPLE)])
def test_timed_launch_matches_and_times(cuda, sr, flags):
    import torch
    W, H = 640, 480
    rgb = torch.from_numpy(O.gen_splitmix(31, W, H)).to(cuda)
    ref = jpgx.encode_blocks(rgb, 90, sr, flags=flags)
    nb = (H // 8) * (W // 8)
    nbc = jpgx.chroma_blocks(W, 0, H // 8, sr, flags)
    out = torch.full((nb + 2 * nbc, 64), 0x5a5a, dtype=torch.int16, device=cuda)
    fr = jpgx.frames(W, H)
    fr.out_frame_stride = (nb + 2 * nbc) * 64
    p = jpgx.default_params(W, H, 90, sr, flags=flags)
    ws = torch.empty(max(jpgx.workspace_size(fr), 1), dtype=torch.uint8, device=cuda)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    e1.record()                                   # the handles exist
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    jpgx.blocks_gpu(fr, p, rgb, out, ws, kernel_events=(e0, e1))
    b.record()
    torch.cuda.synchronize()
    assert np.array_equal(out.cpu().numpy().reshape(-1), ref.cpu().numpy().reshape(-1))
    k, around = e0.elapsed_time(e1), a.elapsed_time(b)
    assert 0.0 < k <= around * 1.001 + 1e-3, (k, around)


def test_timed_entry_requires_both_events():
    import ctypes
    fr = jpgx.frames(64, 64)
    p = jpgx.default_params(64, 64, 90)
    assert jpgx.lib.jpgx_blocks_gpu_timed(ctypes.byref(fr), ctypes.byref(p), 16, 16, 16, 0, None, None,
                                          None) == jpgx.EARG
