"""bench.py's multi-rank path on CPU (gloo): `bench.py --gpus 2` with no
torch.distributed environment re-launches itself with 2 ranks; every rank runs
the same barrier / timing / counter all-reduce steps as the GPU bench, here
with --cpu-stub's stub decode.  The reduced counters must equal the closed form
over the GLOBAL frame range (frames are keyed by global index), and rank 0
prints one JSON line with n_gpus = 2."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(gpus, batch, steps):
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    env.pop("RANK", None)
    env.pop("LOCAL_RANK", None)
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(gpus), "--cpu-stub",
                        "--steps", str(steps), "--warmup", "1", "--batch", str(batch)],
                       capture_output=True, text=True, timeout=240, env=env, cwd=ROOT)
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, p.stdout
    return json.loads(lines[0])


def _expected(world, batch, steps):
    frames = world * batch
    flipped = sum(1 for f in range(frames) if f % 7 == 0)  # one bit flipped per such frame
    return [flipped * steps, flipped * steps, frames * steps]


def test_bench_self_launch_two_ranks():
    r = _run(2, 64, 3)
    assert r["n_gpus"] == 2 and r["stub"] is True and r["steps"] == 3
    assert len(r["rank_ms_per_step"]) == 2
    assert r["ms_per_step"] == max(r["rank_ms_per_step"])  # max over ranks
    assert r["counts"] == _expected(2, 64, 3)
    assert r["value"] > 0


def test_bench_single_rank_counts():
    r = _run(1, 96, 2)
    assert r["n_gpus"] == 1 and r["counts"] == _expected(1, 96, 2)


def test_bench_self_launch_eight_ranks():
    """The driver's N=8 shape end to end on CPU: self-launch -> torch.distributed.run
    -> 8 gloo ranks, each timing its own shard; counters all-reduced over the
    global frame range, one max-over-ranks step time, one time per rank."""
    r = _run(8, 32, 2)
    assert r["n_gpus"] == 8 and r["stub"] is True and r["steps"] == 2
    assert len(r["rank_ms_per_step"]) == 8
    assert r["ms_per_step"] == max(r["rank_ms_per_step"])
    assert r["counts"] == _expected(8, 32, 2)
    assert r["value"] > 0
