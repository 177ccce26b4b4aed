"""bench.py itself on the GPU: the N=1 line (contract keys, roofline, its own output check
against the golden hashes) and the N>1 path rehearsed with two ranks on the box's one GPU
(`bench.py --gpus 2` starts them itself; gloo collectives: the stripes, per-rank seeds, barrier, max-over-ranks
timing and the cross-rank output check all run; RCCL needs one GPU per rank)."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KEYS = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
        "scaling", "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"}


def _line(out):
    lines = [ln for ln in out.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out
    return json.loads(lines[0])


@pytest.mark.parametrize("launch", ["graph", "eager"])
def test_bench_single_gpu_line(launch):
    """The timed K launches as one HIP-graph replay (default) or K eager launches: either way the
    last timed launch's output is checked against the golden hashes."""
    r = subprocess.run([sys.executable, "bench.py", "--steps", "3", "--warmup", "1", "--launch", launch,
                        "--no-cpu-baseline"], cwd=REPO, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    d = _line(r.stdout)
    assert d["config"]["launch"] == {"graph": "hip-graph", "eager": "eager"}[launch]
    assert KEYS <= d.keys() and d["n_gpus"] == 1
    assert d["output_check"]["ok"] and d["output_check"]["frames_checked"] == 8
    assert d["output_check"]["repeat_launches"] == 256
    assert d["output_check"]["repeat_launches_differing"] == 0
    rf = d["roofline"]
    assert rf["bound"] == "hbm" and 0 < rf["frac"] < 1 and rf["kernel"] == "k_mxs"


def test_bench_two_ranks_rehearsal():
    """`bench.py --gpus 2` started directly: it launches its two ranks itself."""
    env = dict(os.environ, JPGX_BENCH_BACKEND="gloo")
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--steps", "3", "--warmup", "1",
                        "--frames-per-gpu", "2"], cwd=REPO, env=env, capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    d = _line(r.stdout)
    assert d["n_gpus"] == 2 and d["config"]["global_batch_frames"] == 4
    assert d["cpu_baseline"] is None
    assert d["output_check"]["ok"] and "all stripes" in d["output_check"]["against"]
    assert d["output_check"]["repeat_launches"] == 2 * 256        # summed over the ranks


def test_bench_refuses_more_gpus_than_the_node_has():
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    env.pop("JPGX_BENCH_BACKEND", None)
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "64", "--steps", "1"], cwd=REPO,
                       env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode != 0 and not [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
