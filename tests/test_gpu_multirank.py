"""The multi-rank GPU bench path on one GPU: `bench.py --gpus 2` self-launches
two ranks (torch.distributed.run); with --dist-backend gloo both may share the
box's single GPU (RCCL refuses duplicate devices, so the real 8-GPU run uses
nccl).  Each rank decodes its own shard of global frame indices; the reduced
counters must cover both shards, and every key reports per-rank step times,
its value taken at the max over ranks.  VERDICT r02 missing 3: every section
the driver's 8-GPU run executes (headline, end-to-end, default frozen set,
published SC configuration, configs[0], LDPC BP-20 + valid codewords, CA-SCL
L=32 with its harness.ber sweep, both configs[4] keys) runs here with 2 ranks
at small batches (benchmarks/ber_simulation.py:167-192 for the sweep)."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(args, tmp_path, timeout=300):
    """Run bench.py with 2 ranks; returns the full result (the --detail-out file:
    per-rank times of every key) after checking the one compact stdout line."""
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    detail = str(tmp_path / "detail.json")
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dist-backend", "gloo",
                        "--skip-cpu", "--detail-out", detail] + args, capture_output=True, text=True,
                       timeout=timeout, env=env, cwd=ROOT)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, p.stdout[-2000:]
    line = json.loads(lines[0])
    with open(detail) as f:
        full = json.load(f)
    assert line["value"] == pytest.approx(full["value"], rel=1e-5) and line["n_gpus"] == full["n_gpus"] == 2
    return full


def _ranks(d, steps, frames_per_gpu):
    assert len(d["rank_ms_per_step"]) == 2 and all(t > 0 for t in d["rank_ms_per_step"])
    assert abs(d["ms_per_step"] - max(d["rank_ms_per_step"])) < 1e-9
    if "frames_counted" in d:
        assert d["frames_counted"] == 2 * frames_per_gpu * steps
    assert d["value"] > 0


def test_bench_two_ranks_on_one_gpu(gpu, tmp_path):
    r = _bench(["--sections", "polar,ldpc", "--batch", "8192", "--steps", "3", "--warmup", "1", "--snr", "0.0"],
               tmp_path)
    assert r["n_gpus"] == 2 and len(r["rank_ms_per_step"]) == 2
    assert r["ms_per_step"] == max(r["rank_ms_per_step"])
    assert r["config"]["global_batch"] == 16384
    assert 0.0 < r["fer"] < 1.0  # counters of both shards, at 0 dB some frames fail
    assert r["value"] > 0 and r["ldpc"]["value"] > 0


def test_bench_every_section_two_ranks(gpu, tmp_path):
    B, LB, steps = 4096, 2048, 2
    r = _bench(["--batch", str(B), "--long-batch", str(LB), "--steps", str(steps), "--warmup", "1",
                "--extra-steps", str(steps), "--sweep-frames", "8192", "--sweep-max-errors", "40", "--snr", "1.0"],
               tmp_path, timeout=420)
    assert r["n_gpus"] == 2
    _ranks(r, steps, B)
    assert r["end_to_end"]["value"] > 0
    _ranks(r["default_frozen_set"], steps, B)
    _ranks(r["polar_sc_default"], steps, B)
    _ranks(r["config0_sc_256"], steps, 0)
    _ranks(r["ldpc"], steps, B)
    _ranks(r["ldpc"]["valid_codewords"], steps, 0)
    c = r["cascl_l32"]
    _ranks(c, steps, B)
    pts = c["sweep"]["points"]
    assert [p["snr_db"] for p in pts] == [-2.0, -1.0, 0.0, 1.0, 2.0, 3.0, 4.0, 5.0]
    for p in pts:
        # frames sharded over both ranks, one all-reduce per round: a point ends at
        # the frame budget or at the first round past max_errors
        assert p["frames"] == 8192 or (p["frame_errors"] >= 40 and p["frames"] % 2 == 0)
    assert pts[0]["frame_errors"] >= 40 and pts[-1]["frames"] == 8192
    lb = r["long_block"]
    _ranks(lb["polar_4096_l8"], steps, LB)
    _ranks(lb["ldpc_8192_ms20"], steps, LB)
    _ranks(lb["ldpc_8192_ms20_no_early_stop"], steps, LB)
