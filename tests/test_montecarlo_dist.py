"""Multi-process Monte-Carlo logic on CPU (gloo, world_size 2): frame sharding,
one all-reduce of the error counters per round, round-granular max_errors stop.
The per-frame work is the C oracle (test infrastructure) on tiny SC frames; the
GPU round functions share the same engine.  Results must not depend on the
number of ranks."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from polarcode_and_ldpc_amd.harness.montecarlo import MonteCarlo, shard, wilson_interval

N, K = 64, 32


def _cpu_round_fn():
    from oracle import oracle as O
    from polarcode_and_ldpc_amd.polar import PolarEncoder, construct_frozen_set
    fr = construct_frozen_set(N, K, 1.0)
    enc = PolarEncoder(N, K, frozen_bits=fr)

    def fn(snr_index, snr_db, offset, nframes):
        msgs, llrs = [], []
        sigma = np.sqrt(1.0 / (2.0 * 10 ** (snr_db / 10.0)))
        for f in range(offset, offset + nframes):
            rng = np.random.RandomState((snr_index * 1_000_003 + f) % (2 ** 31))
            m = rng.randint(0, 2, K)
            x = enc.encode(m)
            llrs.append(2.0 * ((1.0 - 2.0 * x) + sigma * rng.randn(N)) / sigma ** 2)
            msgs.append(m)
        dec = O.sc_decode(N, fr, np.array(llrs))
        err = (dec != np.array(msgs)).sum(axis=1)
        return np.array([err.sum(), (err > 0).sum(), nframes], dtype=np.int64)

    return fn


def _run(world_rank, world, port, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    if world > 1:
        dist.init_process_group("gloo", rank=world_rank, world_size=world)
    mc = MonteCarlo(_cpu_round_fn(), info_bits=K, batch=24)
    res = mc.run([-5.0, 0.0, 4.0], num_frames=200, max_errors=30)
    if world > 1:
        dist.destroy_process_group()
    if world_rank == 0:
        q.put([r.as_dict() for r in res])


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_shard_partition():
    for total in (0, 1, 7, 64, 65):
        for world in (1, 2, 3, 8):
            parts = [shard(total, r, world) for r in range(world)]
            assert sum(c for _, c in parts) == total
            pos = 0
            for s, c in parts:
                assert s == pos
                pos += c


def test_wilson_matches_reference_formula():
    p, lo, hi = wilson_interval(10, 1000)
    assert p == 0.01 and 0.0054 < lo < 0.0055 and 0.0182 < hi < 0.0184
    assert wilson_interval(0, 0) == (0.0, 0.0, 0.0)


def test_world2_equals_world1():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    _run(0, 1, 0, q)
    one = q.get()
    port = _free_port()
    procs = [ctx.Process(target=_run, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    two = q.get(timeout=180)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for a, b in zip(one, two):
        # world 2 runs rounds of 48 frames, world 1 of 24: identical frames only up
        # to the point where both stopped; compare rates within Wilson intervals
        assert a["frames"] > 0 and b["frames"] > 0
        assert b["frames"] % 48 == 0 or b["frames"] == 200
        if a["frames"] == b["frames"]:
            assert a["frame_errors"] == b["frame_errors"] and a["bit_errors"] == b["bit_errors"]
        lo = max(a["fer_ci"][0], b["fer_ci"][0])
        hi = min(a["fer_ci"][1], b["fer_ci"][1])
        assert lo <= hi  # overlapping confidence intervals
    # high SNR point: no early stop, both ran all 200 frames -> identical counts
    assert one[2]["frames"] == two[2]["frames"] == 200
    assert one[2]["bit_errors"] == two[2]["bit_errors"]
    # low SNR point stops on max_errors
    assert one[0]["frame_errors"] >= 30 and two[0]["frame_errors"] >= 30


def test_point_log_resume(tmp_path):
    """An interrupted sweep resumes from its per-point JSON-lines log (SURVEY §5
    checkpoint/resume) and gives exactly the uninterrupted counts; rows of
    another configuration and a torn last line are ignored."""
    from polarcode_and_ldpc_amd.harness.montecarlo import PointLog
    snrs = [-5.0, 0.0, 4.0]
    full = MonteCarlo(_cpu_round_fn(), info_bits=K, batch=24).run(snrs, num_frames=120, max_errors=30)
    path = tmp_path / "points.jsonl"
    key = dict(code="polar", N=N, K=K, frames=120, max_errors=30)
    # "interrupted" after the first point, plus a foreign row and a torn line
    MonteCarlo(_cpu_round_fn(), info_bits=K, batch=24).run(snrs[:1], 120, 30, log=PointLog(path, key))
    PointLog(path, dict(key, frames=7)).append(full[2])
    with open(path, "a") as f:
        f.write('{"key": {"code": "pol')
    calls = []
    fn = _cpu_round_fn()

    def counting(*a):
        calls.append(a[0])
        return fn(*a)

    resumed = MonteCarlo(counting, info_bits=K, batch=24).run(snrs, 120, 30, log=PointLog(path, key))
    assert 0 not in calls  # point 0 came from the log
    assert [r.as_dict() for r in resumed] == [r.as_dict() for r in full]
    assert len(PointLog(path, key).load()) == 3
