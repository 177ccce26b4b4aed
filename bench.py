"""Benchmark: RGB -> quantised zig-zag int16 coefficients (the reference's per-block hot path,
preprocess.c -> dct.c -> quantise.c -> zig_zag.c) on MI355X through libjpgx.so.

Workload (BASELINE.json metric "Mpixels/sec RGB->quantised-coeff, 4K 4:4:4 q=90"):
  every GPU processes, per step, its block-row stripe of a global batch of
  frames_per_gpu * N synthetic 3840x2160 RGB frames (4:4:4, q=90) -- configs[3]'s
  "batch of 64 x 4K frames, row-stripe sharded across 8 GPUs" at N=8, weak scaling.
  Frames are generated on the device (splitmix64) before timing; a step is one
  jpgx_blocks_gpu() call over all frames of the stripe (one k_mxs launch, whose in-kernel
  exact path recomputes the guard-band coefficients).
  8 frames per GPU = 597 MB moved per step, more than the 256 MiB Infinity Cache.

Launch: python bench.py [--gpus N --steps K --warmup W]; for N > 1 one process per GPU, either
under the driver's torch.distributed.run or started by bench.py itself (a child
torch.distributed.run) when WORLD_SIZE is unset; RCCL carries only the barrier and the max-time
reduction (the stripes need no data exchange).  Rank 0 prints ONE JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "jpeg-encoder-and-decoder_amd"))

METRIC = "Mpixels/sec RGB→quantised-coeff, 4K 4:4:4 q=90; % HBM roofline"
HBM_PEAK_GBS = 8000.0          # MI355X HBM3E spec (MI355X_MICROARCH.md)
BYTES_PER_PX = 9               # 3 B RGB in + 3 channels x 2 B int16 out
SPLITMIX_C = 0x9E3779B97F4A7C15


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def _port_rate(width, height, quality, seconds, threads):
    """The oracle (exact-order fp64 naive DCT with two cos() calls per term: the reference's
    own algorithmic cost, src/dct.c:43-56) on the first block-rows of one frame."""
    import oracle
    frame = oracle.gen_splitmix(1, width, height)
    t = time.perf_counter()
    oracle.blocks(frame, quality, mode=oracle.MODE_REFCOST, nthreads=threads, rows=(0, 1))
    per_row = time.perf_counter() - t
    rows = max(1, min(height // 8, int(seconds / max(per_row, 1e-6))))
    t = time.perf_counter()
    oracle.blocks(frame, quality, mode=oracle.MODE_REFCOST, nthreads=threads, rows=(0, rows))
    dt = time.perf_counter() - t
    return rows * 8 * width / dt / 1e6, rows, dt


def _reference_rate(width, quality, seconds, jpgx):
    """The real reference (oracle/_ref/ref_dump: the reference's own preprocess -> zig_zag
    stage sources compiled by oracle/Makefile, 1 thread) on a width x (8*rows) synthetic BMP,
    wall time of the process; its output is compared with the GPU path's on the same image."""
    import subprocess
    import tempfile

    import numpy as np
    import oracle
    exe = os.path.join(REPO, "oracle", "_ref", "ref_dump")

    def run(rows, td):
        img = oracle.gen_splitmix(1, width, 8 * rows)
        bmp, out = os.path.join(td, "s.bmp"), os.path.join(td, "s.bin")
        oracle.write_bmp(bmp, img)
        t = time.perf_counter()
        subprocess.run([exe, bmp, out, str(quality), "0"], check=True,
                       stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
        dt = time.perf_counter() - t
        ref = np.fromfile(out, np.int32).reshape(3, -1, 64)
        return img, ref, dt

    with tempfile.TemporaryDirectory() as td:
        _, _, dt = run(2, td)
        rows = max(2, int(seconds / max(dt / 2, 1e-4)))
        img, ref, dt = run(rows, td)
    gpu = jpgx.encode_blocks(img, quality)
    return width * 8 * rows / dt / 1e6, rows, dt, bool(np.array_equal(gpu, ref))


def host_cpus():
    """(usable cores, how that was determined, CPU model): the process's affinity set, capped
    by a cgroup v2 CPU quota when one is set (a GPU box may show the whole machine's CPUs)."""
    n, how = len(os.sched_getaffinity(0)), "sched_getaffinity"
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            quota, period = f.read().split()[:2]
        if quota != "max":
            q = max(1, -(-int(quota) // int(period)))
            if q < n:
                n, how = q, f"cgroup cpu.max quota ({quota}/{period})"
    except (OSError, ValueError):
        pass
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return n, how, model


def cpu_baseline(width, height, quality, seconds, jpgx):
    """CPU rates on bounded samples of the bench workload (rates are per pixel, so a sample of
    the frame's first block-rows gives the same Mpixels/s as a whole frame at this per-block
    cost; the sample is named in each entry)."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    allc, how, model = host_cpus()
    p_all, rows_all, dt_all = _port_rate(width, height, quality, seconds / 3, allc)
    extra = {"cpu_model": model, "host_cores": allc, "host_cores_from": how,
             "port_all_cores": {"value": round(p_all, 4), "cores": allc,
                                "sample": f"block-rows 0..{rows_all} of a {width}x{height} "
                                          f"frame ({rows_all * 8 * width} px, rate per pixel), "
                                          f"OpenMP over blocks with {allc} threads, "
                                          f"{dt_all:.1f} s"}}
    if os.path.exists(os.path.join(REPO, "oracle", "_ref", "ref_dump")):
        v, rows, dt, same = _reference_rate(width, quality, seconds, jpgx)
        return {"value": round(v, 4), "unit": "Mpixels/s", "cores": 1, "kind": "reference",
                "sample": f"{width}x{8 * rows} synthetic BMP (splitmix seed 1), q={quality}: a "
                          f"sub-frame of {8 * rows} of the {height} rows, its per-pixel rate "
                          f"reported; the reference's preprocess->zig_zag compiled -O2 "
                          f"(oracle/_ref), process wall {dt:.1f} s incl. BMP read",
                "gpu_output_identical": same, **extra}
    v, rows, dt = _port_rate(width, height, quality, seconds, 1)
    return {"value": round(v, 4), "unit": "Mpixels/s", "cores": 1, "kind": "port",
            "sample": f"block-rows 0..{rows} of one {width}x{height} frame ({rows * 8 * width} "
                      f"px), q={quality}, oracle/cpu_ref.c exact-order fp64 with cos() per term, "
                      f"{dt:.1f} s", **extra}


def measured_traffic(kname):
    """HBM bytes per launch from the committed PMC profile (tools/pmc_summary.py, FETCH_SIZE x2
    + WRITE_SIZE per MI355X_MICROARCH.md), as a ratio to the algorithmic bytes -- only if it
    was measured on this exact kernel source.  rocprofv3 --pmc cannot run inside bench.py."""
    import glob
    sys.path.insert(0, os.path.join(REPO, "tools"))
    from pmc_summary import kernel_source_sha
    sha = kernel_source_sha(kname)
    for path in sorted(glob.glob(os.path.join(REPO, "profiles", f"r*_{kname}_pmc.json")),
                       reverse=True):
        with open(path) as f:
            prof = json.load(f)
        if prof.get("kernel_source_sha256") == sha and "traffic_over_algorithmic" in prof:
            return prof["traffic_over_algorithmic"], os.path.relpath(path, REPO)
    return None, None


def rank_plan(W, H, frames_per_gpu, world, rank, jpgx, unit=1):
    """What rank `rank` of `world` holds: its block-row stripe [r0, r1) of every frame of the
    global batch (weak scaling: frames_per_gpu * world frames), the one-pixel-row halo above a
    stripe that does not start at row 0 (the x0 = -8 quirk reads it), and the splitmix seed
    that makes the rank's bytes equal to the same rows of the global frame (byte k of a frame
    is mix(seed + (k+1)*C), so starting at byte k0 is seed + k0*C)."""
    B = frames_per_gpu * world
    r0, r1 = jpgx.stripe(H // 8 // unit, world, rank)     # unit 2: true 4:2:0 MCU rows
    r0, r1 = r0 * unit, r1 * unit
    halo = 1 if r0 > 0 else 0
    row_bytes = W * 3
    rows_px = (r1 - r0) * 8 + halo
    k0 = (8 * r0 - halo) * row_bytes
    seeds = [(1000 + f + k0 * SPLITMIX_C) % (1 << 64) for f in range(B)]
    return {"B": B, "r0": r0, "r1": r1, "halo": halo, "row_bytes": row_bytes,
            "rows_px": rows_px, "fstride": rows_px * row_bytes,
            "nb": (r1 - r0) * (W // 8), "seeds": seeds}


def max_over_ranks(x, world, device=None):
    """The job's time is the slowest rank's (the only collective on the path)."""
    if world == 1:
        return x
    import torch
    import torch.distributed as dist
    t = torch.tensor([x], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def check_output(d_out, plan, W, H, q, subsample, world, device, jpgx):
    """After the timed region: hash the last step's output against tests/golden/big_golden.json
    (the 64-frame 4K q90 batch, seeds 1000+f, pinned to the reference): every frame at N=1; at
    N>1 frame 0, its stripes gathered to every rank (outside the timed region, the only data a
    collective ever carries here).  None when the workload has no committed golden."""
    import hashlib

    import torch
    path = os.path.join(REPO, "tests", "golden", "big_golden.json")
    if subsample or not os.path.exists(path):
        return None
    with open(path) as f:
        gold = json.load(f)["batch64_4k_q90"]
    if (W, H, q) != (gold["W"], gold["H"], gold["quality"]):
        return None
    frames = gold["frames"]
    nb = plan["nb"]

    def sha(t):
        return hashlib.sha256(t.contiguous().cpu().numpy().astype("<i2").tobytes()).hexdigest()

    if world == 1:
        n = min(plan["B"], len(frames))
        bad = [frames[f]["seed"] for f in range(n)
               if sha(d_out[f].view(3, nb, 64)) != frames[f]["coef_sha256"]]
        return {"frames_checked": n, "frames_wrong": bad, "ok": not bad,
                "against": "tests/golden/big_golden.json batch64_4k_q90"}
    import torch.distributed as dist
    sizes = [rank_plan(W, H, 1, world, r, jpgx)["nb"] for r in range(world)]
    nbmax = max(sizes)
    mine = torch.zeros((3, nbmax, 64), dtype=torch.int16, device=device)
    mine[:, :nb] = d_out[0].view(3, nb, 64).to(device)
    parts = [torch.empty_like(mine) for _ in range(world)]
    dist.all_gather([p.view(torch.uint8) for p in parts], mine.view(torch.uint8))  # no int16
    whole = torch.cat([p[:, :n] for p, n in zip(parts, sizes)], dim=1)
    ok = sha(whole) == frames[0]["coef_sha256"]
    return {"frames_checked": 1, "frames_wrong": [] if ok else [frames[0]["seed"]], "ok": ok,
            "against": "tests/golden/big_golden.json batch64_4k_q90 (frame 0, all stripes)"}


def repeat_check(step, d_out, launches, world, device):
    """After the golden check: `launches` more launches (alternating input sets, identical
    content), each compared on the GPU with the checked output -- a wrong-output fault that
    comes and goes from launch to launch would show here on every bench run.
    Counts are summed over ranks."""
    import torch
    import torch.distributed as dist
    ref = d_out.clone()
    wrong = torch.zeros((), dtype=torch.int64, device=d_out.device)
    for _ in range(launches):
        step()
        wrong += torch.ne(d_out, ref).any().to(torch.int64)
    n = torch.tensor([launches, int(wrong.item())], dtype=torch.int64, device=device)
    if world > 1:
        dist.all_reduce(n)
    del ref
    return {"repeat_launches": int(n[0]), "repeat_launches_differing": int(n[1])}


ALT_LIB = os.path.join(REPO, "jpeg-encoder-and-decoder_amd", "lib", "libjpgx_alt.so")


def alt_selected():
    """--kernel xform: the test-only cross-check library (k_xform / two-pass 4:2:x)"""
    return os.path.abspath(os.environ.get("JPGX_LIB", "")) == ALT_LIB


def sub_kernel_name(sr):
    """The kernels a true-subsampling launch runs (jpgx_blocks_gpu's dispatch)."""
    if alt_selected():
        return f"k_xform(Y)+k_chroma<{sr}>"
    return mx_kernel_name(sr)


def mx_kernel_name(sr):
    """The MFMA kernel this library's launch runs for sample ratio sr (0 = 4:4:4): k_mxs /
    k_mxs422 / k_mxs420 (short-lived waves)."""
    import ctypes

    import jpgx
    f = jpgx.lib.jx_mx_kernel_name
    f.restype = ctypes.c_char_p
    f.argtypes = [ctypes.c_int]
    return f(sr).decode()


def launch_ranks(n):
    """`bench.py --gpus N` (N > 1) started without torch.distributed.run: start the N ranks
    here, one process per GPU, as a child torch.distributed.run (never an exec), before this
    process makes any GPU call; its exit code is ours.  Refused when the node has fewer GPUs than
    N, unless JPGX_BENCH_BACKEND=gloo asks for the rehearsal with ranks sharing the GPUs."""
    import subprocess

    import torch
    ndev = torch.cuda.device_count()          # counts devices without initialising the GPU
    rehearsal = os.environ.get("JPGX_BENCH_BACKEND") == "gloo"
    if n > ndev and not rehearsal:
        log(f"bench: --gpus {n} but this node has {ndev} GPU(s)")
        return 2
    # --standalone: the launcher binds its own free port on 127.0.0.1 and keeps it (no window
    # between picking a port here and binding it there for another process to take it)
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--standalone", "--local-addr", "127.0.0.1",
           "--nnodes=1", f"--nproc-per-node={n}", os.path.abspath(__file__)] + sys.argv[1:]
    log(f"bench: starting {n} ranks: {' '.join(cmd[2:])}")
    return subprocess.run(cmd, env=env).returncode


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--input-sets", type=int, default=2,
                    help="copies of the input batch read by consecutive steps in turn (1 = the "
                         "same input every step, which the Infinity Cache partly holds)")
    ap.add_argument("--settle-ms", type=float, default=1000.0,
                    help="after the W warmup steps, keep stepping (untimed) until this much time "
                         "has passed, so the timed steps see the GPU's loaded steady state and not "
                         "its ramp out of idle (about 20 ms of load; profiles/r02_ramp.json) -- and "
                         "a rocprofv3 summary of the same command averages mostly steady-state "
                         "launches (with 200 ms the ramp's ~150 slow launches raised the mean by "
                         "~3 %%); 0 = off")
    ap.add_argument("--kernel-timing", choices=["events", "span"], default="span",
                    help="roofline.kernel_ms from the span of the K launches / K (queue gaps "
                         "included; default) or from per-launch kernel begin/end events "
                         "(jpgx_blocks_gpu_timed, the interval rocprofv3 reports; slows the loop)")
    ap.add_argument("--launch", choices=["eager", "graph"], default="eager",
                    help="the K timed launches as K eager launches (default) or as one HIP graph "
                         "(captured after the warmup, untimed; the settle and the timed region replay "
                         "it): within the box's noise of eager (0.677-0.685 vs 0.670-0.682 of 8 TB/s "
                         "on one box, profiles/r06_launch_gaps.txt), the queue gap being ~1 us of "
                         "~110; --kernel-timing events implies eager")
    ap.add_argument("--frames-per-gpu", type=int, default=8)
    ap.add_argument("--width", type=int, default=3840)
    ap.add_argument("--height", type=int, default=2160)
    ap.add_argument("--quality", type=int, default=90)
    ap.add_argument("--sample-ratio", type=int, default=0)
    ap.add_argument("--verify-launches", type=int, default=256,
                    help="after the timed region and the golden check, this many more launches "
                         "compared with the checked output on the GPU (0 = off)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--kernel", choices=["xform", "mx"], default=None,
                    help="4:4:4 transform kernel: k_mxs (the product: colour and row DCT on the "
                         "matrix cores) or k_xform (all-VALU, from the test-only cross-check "
                         "library lib/libjpgx_alt.so), DESIGN.md 4")
    ap.add_argument("--subsample", action="store_true",
                    help="true 4:2:2 / 4:2:0 chroma (JPGX_FLAG_SUBSAMPLE, an extension; needs "
                         "--sample-ratio 1 or 2): not the headline metric")
    args = ap.parse_args()
    if args.gpus < 1:
        raise SystemExit("--gpus must be >= 1")
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus))
    if args.kernel == "xform":
        os.environ["JPGX_LIB"] = ALT_LIB
    elif args.kernel == "mx" and alt_selected():
        os.environ.pop("JPGX_LIB")                # --kernel mx: the product library, whatever the env said
    kname = "k_xform" if alt_selected() else mx_kernel_name(0)

    import torch
    import torch.distributed as dist

    import jpgx

    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        raise SystemExit(f"bench: --gpus {args.gpus} but WORLD_SIZE={world}: one rank per GPU")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # one process per GPU over RCCL ("nccl").  JPGX_BENCH_BACKEND=gloo (with ranks placed on
    # local_rank % device_count) rehearses the N>1 path on a box with fewer GPUs than ranks;
    # it is never how numbers are taken.
    backend = os.environ.get("JPGX_BENCH_BACKEND", "nccl")
    dev = torch.device("cuda", local % max(1, torch.cuda.device_count()))
    torch.cuda.set_device(dev)
    if world > 1:
        dist.init_process_group(backend)
    cdev = dev if backend == "nccl" else torch.device("cpu")     # collectives' tensors
    N = world

    W, H, q = args.width, args.height, args.quality
    flags = jpgx.FLAG_SUBSAMPLE if args.subsample else 0
    if args.subsample and args.sample_ratio not in (1, 2):
        raise SystemExit("--subsample needs --sample-ratio 1 or 2")
    unit = 2 if args.subsample and args.sample_ratio == 2 else 1
    plan = rank_plan(W, H, args.frames_per_gpu, N, rank, jpgx, unit)
    B, r0, r1, halo = plan["B"], plan["r0"], plan["r1"], plan["halo"]
    row_bytes, fstride, nb = plan["row_bytes"], plan["fstride"], plan["nb"]

    # device-resident inputs: frame f's stripe (+ one halo pixel row) generated in place
    d_in = torch.empty(B * fstride, dtype=torch.uint8, device=dev)
    for f in range(B):
        jpgx.gen_splitmix_gpu(d_in[f * fstride:(f + 1) * fstride], plan["seeds"][f])
    nbc = jpgx.chroma_blocks(W, r0, r1, args.sample_ratio, flags)
    per = nb + 2 * nbc                                   # blocks per frame stripe output
    bytes_per_px = 3 + 2 * per / max(nb, 1)              # 9 for 4:4:4; 7 / 6 true 4:2:2 / 4:2:0
    d_out = torch.empty((B, per, 64), dtype=torch.int16, device=dev)
    fr = jpgx.frames(W, H, nframes=B, rows=(r0, r1), in_pitch=row_bytes, in_frame_stride=fstride,
                     out_frame_stride=per * 64)
    d_ws = torch.empty(jpgx.workspace_size(fr), dtype=torch.uint8, device=dev)
    params = jpgx.default_params(W, H, q, args.sample_ratio, flags=flags)
    # Consecutive steps read alternate copies of the batch (--input-sets): like a stream of new
    # frames, a step's input is then not still resident in the 256 MiB Infinity Cache from the
    # step before (2 x 199 MB per GPU at 8 frames; the frames sweep in DESIGN.md 4.3 measures
    # what residency would be worth).  The copies are identical, so the output is checkable.
    inputs = [d_in] + [d_in.clone() for _ in range(args.input_sets - 1)]
    rgb_ptrs = [t.data_ptr() + halo * row_bytes for t in inputs]
    torch.cuda.synchronize()
    nstep = [0]

    def step(ev_mid=None, kev=None):
        jpgx.blocks_gpu(fr, params, rgb_ptrs[nstep[0] % len(rgb_ptrs)], d_out, d_ws,
                        event_between=ev_mid, kernel_events=kev)
        nstep[0] += 1

    # per-launch kernel events (jpgx_blocks_gpu_timed: hipExtLaunchKernel sets them to the kernel's
    # own begin / end, the interval rocprofv3's kernel trace reports); recorded once so that their
    # handles exist
    kevs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
            for _ in range(args.steps if args.kernel_timing == "events" else 0)]
    for a, b in kevs:
        a.record()
        b.record()

    # W warmup steps, each timed on its own (reported as the cold start), then untimed steps
    # until --settle-ms have passed: after idle the GPU's power management takes ~20 ms of load
    # to reach its steady state (the first launches run 15-35% slower; profiles/r02_ramp.json)
    cold = []
    t_w = time.perf_counter()
    for _ in range(args.warmup):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        step()
        e1.record()
        cold.append((e0, e1))
    settle_steps = 0
    # --launch graph: the K steps' launches captured once into a HIP graph after the
    # warmup (untimed; the capture executes nothing), the settle loop then replays it, and the timed
    # region is one more replay -- the same K launches, input sets alternating as before.  (Capture
    # and instantiation idle the GPU for a while: without the settle after them the timed replay
    # ran ~30 % slow, the ramp out of idle.)
    graph, launch_mode = None, "eager"
    if args.launch == "graph" and args.kernel_timing != "events":
        try:
            torch.cuda.synchronize()
            graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(graph, stream=torch.cuda.Stream(), capture_error_mode="thread_local"):
                for _ in range(args.steps):
                    step()
            launch_mode = "hip-graph"
        except Exception as e:            # noqa: BLE001 -- fall back to eager launches, say so
            graph, launch_mode = None, f"eager (graph capture failed: {type(e).__name__})"
            torch.cuda.synchronize()
    torch.cuda.synchronize()
    t_s = time.perf_counter()
    while True:
        if graph is not None:
            graph.replay()
            settle_steps += args.steps
        else:
            for _ in range(10):
                step()
            settle_steps += 10
        torch.cuda.synchronize()
        if (time.perf_counter() - t_s) * 1e3 >= args.settle_ms:
            break
    cold_ms = [a.elapsed_time(b) for a, b in cold]
    # Kernel timing inside the timed region (one launch per step: the exact pass runs inside the
    # kernel).  --kernel-timing span (default): HIP events on the launch stream around the K
    # back-to-back launches; span / K is `kernel_ms` (the queue gaps between launches included).
    # --kernel-timing events: every launch goes through jpgx_blocks_gpu_timed, whose
    # hipExtLaunchKernel sets a pair of HIP events to that kernel's own begin and end (the interval
    # a rocprofv3 kernel trace reports) and `kernel_ms` is their mean -- but those launches cost the
    # wall clock ~5 us each (round 6: 118.5 vs 112.3-113.8 us per step, kernel 110.2 vs span 110.6-
    # 112.2 us), so it is not the default.  The wall clock around the loop, bracketed by barrier +
    # synchronize, gives the step time and `value` either way.
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ev0.record()
    if graph is not None:
        graph.replay()
    else:
        for i in range(args.steps):
            step(kev=kevs[i] if args.kernel_timing == "events" else None)
    ev1.record()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = max_over_ranks(time.perf_counter() - t0, world, cdev)

    span_ms = ev0.elapsed_time(ev1) / args.steps
    launch_ms = [a.elapsed_time(b) for a, b in kevs] if args.kernel_timing == "events" else None
    xform_ms = sum(launch_ms) / len(launch_ms) if launch_ms else span_ms
    px_rank_step = B * (r1 - r0) * 8 * W
    px_total = B * W * H * args.steps                 # all ranks
    value = px_total / elapsed / 1e6
    ms_per_step = elapsed / args.steps * 1e3
    achieved = bytes_per_px * px_rank_step / (xform_ms * 1e-3) / 1e9

    check = check_output(d_out, plan, W, H, q, args.subsample, world, cdev, jpgx)
    if args.verify_launches > 0:
        rep = repeat_check(step, d_out, args.verify_launches, world, cdev)
        if check is None:          # no committed golden at this config: self-consistency only
            check = {"frames_checked": 0, "ok": True,
                     "against": "the last timed launch's output (no committed golden at this config)"}
        check.update(rep)
        check["ok"] = check["ok"] and rep["repeat_launches_differing"] == 0
    if rank == 0:
        t_ratio, t_src = measured_traffic(kname) if not args.subsample else (None, None)
        cpu = None
        if N == 1 and not args.no_cpu_baseline:
            cpu = cpu_baseline(W, H, q, args.cpu_seconds, jpgx)
        line = {
            "metric": METRIC if not args.subsample else
                      f"Mpixels/sec RGB->quantised-coeff, true {'4:2:2' if args.sample_ratio == 1 else '4:2:0'} "
                      f"q={q} (extension, not the headline)",
            "value": round(value, 1), "unit": "Mpixels/s", "n_gpus": N,
            "steps": args.steps, "warmup": args.warmup,
            "settle": {"ms": args.settle_ms, "extra_untimed_steps": settle_steps,
                       "warmup_step_ms": [round(x, 4) for x in cold_ms]},
            "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f32",
            "data": "synthetic (splitmix64 RGB frames generated in HBM)",
            "config": {"workload": f"{args.frames_per_gpu} x {W}x{H} RGB frames per GPU, "
                                   f"{['4:4:4', 'true 4:2:2', 'true 4:2:0'][args.sample_ratio] if args.subsample else '4:4:4'}"
                                   f", q={q}, block-row stripes",
                       "global_batch_frames": B, "width": W, "height": H, "quality": q,
                       "sample_ratio": args.sample_ratio, "parallelism": f"stripes{N}",
                       "collectives": ("none" if N == 1 else
                                       f"{backend}: barrier, max-time, output check"),
                       "kernel_timing": ("per-launch kernel begin/end HIP events (hipExtLaunchKernel)"
                                         if launch_ms else "HIP events around the K launches on their stream"),
                       "launch": launch_mode,
                       "input_sets": args.input_sets},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                         "traffic": (round(t_ratio * bytes_per_px * px_rank_step)
                                     if t_ratio else None),
                         "traffic_source": t_src,
                         "kernel": kname if not args.subsample else sub_kernel_name(args.sample_ratio),
                         "kernel_ms": round(xform_ms, 4),
                         "kernel_ms_min_max": ([round(min(launch_ms), 4), round(max(launch_ms), 4)]
                                               if launch_ms else None),
                         "span_ms_per_launch": round(span_ms, 4),
                         "bytes_per_launch": bytes_per_px * px_rank_step},
            "cpu_baseline": cpu,
            "output_check": check,
        }
        print(json.dumps(line), flush=True)
    bad = check is not None and not check["ok"]
    if bad and rank == 0:
        log(f"bench: output differs from the golden hashes: {check}")
    if world > 1:
        dist.destroy_process_group()
    if bad:
        sys.exit(3)


if __name__ == "__main__":
    main()
