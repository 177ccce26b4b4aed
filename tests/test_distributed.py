"""The N>1 path on CPU: two gloo ranks run bench.py's sharding (rank_plan: block-row stripes,
halo row, per-rank splitmix seeds) and its max-over-ranks timing reduction; each rank computes
its stripe with the oracle (the CPU checker -- the GPU kernel's stripe path is covered by
test_gpu_parity), and the stitched stripes must equal the whole frame.  No data-path
collective exists: all_gather here only brings the results to the checker."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

W, H, FRAMES = 96, 80, 2


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank(rank, world, port, q):
    import torch
    import torch.distributed as dist

    import bench
    import jpgx
    import oracle as O

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        plan = bench.rank_plan(W, H, FRAMES, world, rank, jpgx)
        assert plan["B"] == FRAMES * world
        outs = []
        for f in range(plan["B"]):
            # the rank's bytes, generated from its own seed, placed at their frame rows
            stripe = O.gen_splitmix(plan["seeds"][f], W, plan["rows_px"])
            frame = np.zeros((H, W, 3), np.uint8)
            top = 8 * plan["r0"] - plan["halo"]
            frame[top:top + plan["rows_px"]] = stripe
            outs.append(O.blocks(frame, q, rows=(plan["r0"], plan["r1"])))
        t = bench.max_over_ranks(float(rank + 1), world)
        assert t == float(world)
        gathered = [None] * world
        dist.all_gather_object(gathered, (plan["r0"], plan["r1"], outs))
        if rank == 0:
            spans = sorted((g[0], g[1]) for g in gathered)
            assert spans[0][0] == 0 and spans[-1][1] == H // 8
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))   # disjoint, complete
            for f in range(FRAMES * world):
                full = O.blocks(O.gen_splitmix(1000 + f, W, H), q)
                stitched = np.concatenate([g[2][f] for g in sorted(gathered)], axis=1)
                assert np.array_equal(stitched, full), f
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("q", [50, 90])
def test_two_rank_stripes_stitch(q):
    mp.spawn(_rank, args=(2, _free_port(), q), nprocs=2, join=True)


def _check_rank(rank, world, port, corrupt):
    """bench.check_output's N>1 leg: frame 0's stripes gathered and hashed against the golden
    64 x 4K q90 batch (each rank's stripe computed here by the oracle, as the GPU would)."""
    import torch
    import torch.distributed as dist

    import bench
    import jpgx
    import oracle as O

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        Wk, Hk, q = 3840, 2160, 90
        plan = bench.rank_plan(Wk, Hk, 1, world, rank, jpgx)
        stripe = O.gen_splitmix(plan["seeds"][0], Wk, plan["rows_px"])
        frame = np.zeros((Hk, Wk, 3), np.uint8)
        top = 8 * plan["r0"] - plan["halo"]
        frame[top:top + plan["rows_px"]] = stripe
        out = O.blocks(frame, q, rows=(plan["r0"], plan["r1"]))
        if corrupt and rank == world - 1:
            out[2, -1, 63] ^= 1
        d_out = torch.from_numpy(out.reshape(1, -1, 64))
        res = bench.check_output(d_out, plan, Wk, Hk, q, False, world, torch.device("cpu"), jpgx)
        assert res["frames_checked"] == 1 and res["ok"] is (not corrupt), res
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,corrupt", [(2, False), (3, False), (2, True)])
def test_bench_output_check_gathers_stripes(world, corrupt):
    mp.spawn(_check_rank, args=(world, _free_port(), corrupt), nprocs=world, join=True)


def test_bench_output_check_single_rank():
    """The N=1 leg hashes every frame of the step's output."""
    import torch

    import bench
    import jpgx
    import oracle as O
    plan = bench.rank_plan(3840, 2160, 2, 1, 0, jpgx)
    outs = np.stack([O.blocks(O.gen_splitmix(s, 3840, 2160), 90) for s in plan["seeds"]])
    d_out = torch.from_numpy(outs.reshape(2, -1, 64))
    res = bench.check_output(d_out, plan, 3840, 2160, 90, False, 1, None, jpgx)
    assert res["ok"] and res["frames_checked"] == 2
    d_out[1, 5, 7] += 1
    res = bench.check_output(d_out, plan, 3840, 2160, 90, False, 1, None, jpgx)
    assert not res["ok"] and res["frames_wrong"] == [1001]
    assert bench.check_output(d_out, plan, 1920, 1080, 90, False, 1, None, jpgx) is None


def test_bench_repeat_check_counts_differing_launches():
    """bench.py's repeated-launch check: every launch after the checked one is compared with it."""
    import torch

    import bench
    d_out = torch.arange(64, dtype=torch.int16).view(1, 1, 64).clone()
    calls = [0]

    def step():
        calls[0] += 1
        d_out[0, 0, 5] = 5 if calls[0] not in (3, 7) else -1      # launches 3 and 7 differ

    res = bench.repeat_check(step, d_out, 10, 1, torch.device("cpu"))
    assert res == {"repeat_launches": 10, "repeat_launches_differing": 2} and calls[0] == 10
