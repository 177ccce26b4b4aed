"""Host-buffer path (csrc/jpgx_host.cpp): images in host memory, block-row shards (several per
GPU here: the box has one), chunked through the device with two chunks in flight, staged through
pinned buffers or DMA'd directly from page-locked caller memory.  Every result is compared
bit-exactly with the oracle (or the golden hash of the reference's output), whatever the shard
count, chunk size, pitch or buffer kind."""
import hashlib
import json
import os

import numpy as np
import pytest

import jpgx
import oracle as O
from conftest import GOLDEN

pytestmark = pytest.mark.gpu


def _want(rgb, q, sr=0, flags=0):
    if flags & jpgx.FLAG_SUBSAMPLE:
        return np.concatenate([O.blocks(rgb, q, sr)[0], O.chroma_sub(rgb, q, sr).reshape(-1, 64)])
    return O.blocks(rgb, q)


@pytest.mark.parametrize("nshards,chunk_rows", [(1, 0), (1, 1), (3, 0), (4, 3), (7, 2)])
def test_shards_on_one_device(cuda, nshards, chunk_rows):
    """17 block rows: shards of 2-5 rows, chunks of 1-3 rows (every chunk seam and shard seam
    crosses the x0 = -8 halo read), slot reuse after two chunks."""
    rgb = O.gen_splitmix(500 + nshards, 200, 136)
    want = O.blocks(rgb, 83)
    with jpgx.HostContext(nshards, [0] * nshards, chunk_rows) as ctx:
        assert np.array_equal(ctx.blocks(rgb, 83), want)
        assert np.array_equal(ctx.blocks(rgb, 83), want)      # buffers reused


@pytest.mark.parametrize("sr", [1, 2])
@pytest.mark.parametrize("nshards,chunk_rows", [(1, 0), (3, 2), (2, 1)])
def test_true_subsampling_shards_and_chunks(cuda, sr, nshards, chunk_rows):
    """True 4:2:2 / 4:2:0 through shards and chunks (4:2:0 in MCU-row pairs)."""
    rgb = O.gen_splitmix(600 + sr, 160, 144)
    fl = jpgx.FLAG_SUBSAMPLE
    with jpgx.HostContext(nshards, [0] * nshards, chunk_rows) as ctx:
        assert np.array_equal(ctx.blocks(rgb, 75, sr, flags=fl), _want(rgb, 75, sr, fl))


def test_growth_pitch_and_quality_changes(cuda):
    """One context over images of growing size, a row-padded input view and new qualities."""
    with jpgx.HostContext(2, [0, 0], 2) as ctx:
        for (W, H, q) in [(64, 32, 40), (520, 96, 90), (1024, 256, 12)]:
            big = O.gen_splitmix(W + H, W + 24, H)
            view = big[:, :W]                                 # pitch (W + 24) * 3
            assert view.strides[0] == (W + 24) * 3
            assert np.array_equal(ctx.blocks(view, q), O.blocks(np.ascontiguousarray(view), q))


def test_page_locked_buffers_are_dmad_directly(cuda):
    rgb = O.gen_splitmix(77, 640, 360)
    out = np.empty((3, 80 * 45, 64), np.int16)
    jpgx.host_register(rgb)
    jpgx.host_register(out)
    try:
        with jpgx.HostContext(3, [0, 0, 0], 4) as ctx:
            ctx.blocks(rgb, 90, out=out)
    finally:
        jpgx.host_unregister(rgb)
        jpgx.host_unregister(out)
    assert np.array_equal(out, O.blocks(rgb, 90))


def test_4k_pooled_entry_points_match_reference_hash(cuda):
    """jpgx_blocks and jpgx_blocks_multi (pooled contexts) on the 4K q90 frame whose output the
    real reference hashed (tests/golden/big_golden.json, batch frame 1000)."""
    with open(os.path.join(GOLDEN, "big_golden.json")) as f:
        ent = json.load(f)["batch64_4k_q90"]["frames"][0]
    rgb = O.gen_splitmix(ent["seed"], 3840, 2160)
    for _ in range(2):
        out = jpgx.encode_blocks(rgb, 90)
        assert hashlib.sha256(out.astype("<i2").tobytes()).hexdigest() == ent["coef_sha256"]
    out = jpgx.encode_blocks_multi(rgb, 90, jpgx.device_count())
    assert hashlib.sha256(out.astype("<i2").tobytes()).hexdigest() == ent["coef_sha256"]
    with jpgx.HostContext(4, [0] * 4) as ctx:
        out = ctx.blocks(rgb, 90)
    assert hashlib.sha256(out.astype("<i2").tobytes()).hexdigest() == ent["coef_sha256"]
    jpgx.lib.jpgx_host_release()


def test_host_context_errors(cuda):
    n = jpgx.device_count()
    with pytest.raises(jpgx.JpgxError) as e:
        jpgx.HostContext(2, [0, n])
    assert e.value.rc == jpgx.ENODEV
    with pytest.raises(jpgx.JpgxError) as e:
        jpgx.HostContext(0)
    assert e.value.rc == jpgx.EARG
    with jpgx.HostContext(1) as ctx:
        with pytest.raises(jpgx.JpgxError) as e:
            ctx.blocks(O.gen_splitmix(1, 16, 12), 50)
        assert e.value.rc == jpgx.EGEOMETRY
        with pytest.raises(jpgx.JpgxError) as e:
            ctx.blocks(O.gen_splitmix(1, 16, 16), 98)
        assert e.value.rc == jpgx.EQUALITY
