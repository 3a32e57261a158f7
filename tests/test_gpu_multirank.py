"""The multi-rank GPU bench path on one GPU: `bench.py --gpus 2` self-launches
two ranks (torch.distributed.run); with --dist-backend gloo both may share the
box's single GPU (RCCL refuses duplicate devices, so the real 8-GPU run uses
nccl).  Each rank decodes its own shard of global frame indices; the reduced
counters must cover both shards, and the aggregate value is reported with
per-rank step times, max over ranks."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_two_ranks_on_one_gpu(gpu):
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dist-backend", "gloo",
                        "--skip-cpu", "--sections", "polar,ldpc", "--batch", "8192", "--steps", "3", "--warmup", "1",
                        "--snr", "0.0"],
                       capture_output=True, text=True, timeout=240, env=env, cwd=ROOT)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, p.stdout[-2000:]
    r = json.loads(lines[0])
    assert r["n_gpus"] == 2 and len(r["rank_ms_per_step"]) == 2
    assert r["ms_per_step"] == max(r["rank_ms_per_step"])
    assert r["config"]["global_batch"] == 16384
    assert 0.0 < r["fer"] < 1.0  # counters of both shards, at 0 dB some frames fail
    assert r["value"] > 0 and r["ldpc"]["value"] > 0
