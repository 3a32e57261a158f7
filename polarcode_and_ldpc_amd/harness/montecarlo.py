"""Monte-Carlo BER/FER engine: frames sharded over GPUs, one all-reduce per round.

Semantics follow benchmarks/ber_simulation.py:132-293 of the reference:
per SNR point, frames of random messages are encoded, sent through BPSK/AWGN
and decoded; BER = bit errors / (frames * K), FER = frame errors / frames, and a
point stops once `max_errors` frame errors are seen (:191-192) or `num_frames`
frames are done (:167).  Differences, by design:
  * frames run in rounds of `batch` frames per rank; the stop test is applied
    after each round (the reference stops at the exact frame), so a point may
    overshoot max_errors by less than one round -- BER/FER stay unbiased;
  * frame f of SNR point s uses the noise/message stream (seed, s, f) (Philox on
    the device), so results are identical for any number of GPUs;
  * the only collective is one all-reduce (SUM) of int64[3] = {bit errors,
    frame errors, frames} per round (RCCL over xGMI on GPUs, gloo on CPU).
"""
from __future__ import annotations

import math
from dataclasses import asdict, dataclass, field
from typing import Callable, List, Optional, Sequence

import numpy as np


def wilson_interval(errors: int, total: int, confidence: float = 0.95):
    """(rate, lower, upper): the Wilson score interval of
    src/utils/metrics.py:138-167 (calculate_ber_with_confidence)."""
    if total == 0:
        return 0.0, 0.0, 0.0
    from statistics import NormalDist
    z = NormalDist().inv_cdf(1 - (1 - confidence) / 2)
    p = errors / total
    den = 1 + z ** 2 / total
    center = (p + z ** 2 / (2 * total)) / den
    margin = z * math.sqrt(p * (1 - p) / total + z ** 2 / (4 * total ** 2)) / den
    return p, max(0.0, center - margin), min(1.0, center + margin)


def shard(total: int, rank: int, world: int):
    """Contiguous shard [start, start+count) of `total` frames for `rank`."""
    base, extra = divmod(total, world)
    start = rank * base + min(rank, extra)
    return start, base + (1 if rank < extra else 0)


@dataclass
class PointResult:
    snr_db: float
    frames: int
    frame_errors: int
    bit_errors: int
    info_bits: int
    ber: float = 0.0
    fer: float = 0.0
    ber_ci: tuple = field(default_factory=tuple)
    fer_ci: tuple = field(default_factory=tuple)
    rounds: int = 0

    def finalize(self):
        tb = self.frames * self.info_bits
        self.ber, lo, hi = wilson_interval(self.bit_errors, tb)
        self.ber_ci = (lo, hi)
        self.fer, lo, hi = wilson_interval(self.frame_errors, self.frames)
        self.fer_ci = (lo, hi)
        return self

    def as_dict(self):
        return asdict(self)


RoundFn = Callable[[int, float, int, int], np.ndarray]
"""round_fn(snr_index, snr_db, global_frame_offset, nframes) -> int64[3] local
counts {bit errors, frame errors, frames} for frames [offset, offset+nframes)."""


class MonteCarlo:
    def __init__(self, round_fn: RoundFn, info_bits: int, batch: int, group=None, device=None):
        self.round_fn = round_fn
        self.info_bits = info_bits
        self.batch = int(batch)
        self.group = group
        self.device = device
        import torch.distributed as dist
        self._dist = dist if (dist.is_available() and dist.is_initialized()) else None
        self.rank = self._dist.get_rank(group) if self._dist else 0
        self.world = self._dist.get_world_size(group) if self._dist else 1

    def _allreduce(self, counts: np.ndarray) -> np.ndarray:
        if self.world == 1:
            return counts
        import torch
        # RCCL reduces device tensors; gloo (CPU tests, one-GPU rehearsals) host ones
        dev = "cpu" if self._dist.get_backend(self.group) == "gloo" else self.device
        t = torch.as_tensor(counts, dtype=torch.int64, device=dev)
        self._dist.all_reduce(t, group=self.group)
        return t.cpu().numpy()

    def _finished(self, log: "Optional[PointLog]") -> dict:
        """Finished points of `log`, read on rank 0 and broadcast, so that every
        rank skips the same SNR points even when the ranks do not share a file
        system (or the file changes between their reads): a disagreement would
        pair different points' all-reduces."""
        done = log.load() if (log is not None and self.rank == 0) else {}
        if self.world > 1:
            box = [sorted((k, v.as_dict()) for k, v in done.items())]
            self._dist.broadcast_object_list(box, src=self._dist.get_global_rank(self.group, 0)
                                             if self.group is not None else 0, group=self.group)
            done = {}
            for k, d in box[0]:
                done[k] = PointResult(snr_db=d["snr_db"], frames=d["frames"], frame_errors=d["frame_errors"],
                                      bit_errors=d["bit_errors"], info_bits=d["info_bits"],
                                      rounds=d.get("rounds", 0)).finalize()
        return done

    def run_point(self, snr_index: int, snr_db: float, num_frames: int, max_errors: int) -> PointResult:
        res = PointResult(snr_db=float(snr_db), frames=0, frame_errors=0, bit_errors=0, info_bits=self.info_bits)
        done = 0
        while done < num_frames and res.frame_errors < max_errors:
            round_total = min(self.batch * self.world, num_frames - done)
            start, count = shard(round_total, self.rank, self.world)
            local = np.zeros(3, dtype=np.int64)
            if count > 0:
                local = np.asarray(self.round_fn(snr_index, snr_db, done + start, count), dtype=np.int64)
            tot = self._allreduce(local)
            res.bit_errors += int(tot[0])
            res.frame_errors += int(tot[1])
            res.frames += int(tot[2])
            res.rounds += 1
            done += round_total
        return res.finalize()

    def run(self, snr_db_range: Sequence[float], num_frames: int, max_errors: int,
            log: "Optional[PointLog]" = None) -> List[PointResult]:
        """One PointResult per SNR point.  With a PointLog, points already in the
        log (same run key) are taken from it, and each new point is appended as
        soon as it finishes (rank 0), so an interrupted sweep resumes where it
        stopped.  Point i always draws the stream (seed, i, frame): a resumed
        sweep gives the same counts as an uninterrupted one."""
        done = self._finished(log)
        out = []
        for i, s in enumerate(snr_db_range):
            key = round(float(s), 9)
            if key in done:
                out.append(done[key])
                continue
            p = self.run_point(i, s, num_frames, max_errors)
            if log is not None and self.rank == 0:
                log.append(p)
            out.append(p)
        return out


class PointLog:
    """Append-only JSON-lines record of finished SNR points (SURVEY §5
    checkpoint / resume; the reference writes its results once at the end,
    src/utils/visualization.py:84-112).  Each row carries the run key (code,
    decoder, code construction digest, frames, max_errors, frames per round,
    seed, decoder library build id): rows of another configuration -- or of
    another build of the decoder library -- in the same file are ignored."""

    def __init__(self, path, key: dict):
        import json
        import os
        self.path = str(path)
        self.key = json.loads(json.dumps(key, sort_keys=True))
        d = os.path.dirname(self.path)
        if d:
            os.makedirs(d, exist_ok=True)

    def load(self):
        import json
        import os
        done = {}
        if not os.path.exists(self.path):
            return done
        with open(self.path) as f:
            for line in f:
                line = line.strip()
                if not line:
                    continue
                try:
                    row = json.loads(line)
                except ValueError:
                    continue  # a row cut short by an interruption
                if row.get("key") != self.key:
                    continue
                p = row["point"]
                r = PointResult(snr_db=p["snr_db"], frames=p["frames"], frame_errors=p["frame_errors"],
                                bit_errors=p["bit_errors"], info_bits=p["info_bits"], rounds=p.get("rounds", 0))
                done[round(float(r.snr_db), 9)] = r.finalize()
        return done

    def append(self, p: PointResult):
        import json
        import os
        with open(self.path, "ab+") as f:
            f.seek(0, os.SEEK_END)
            if f.tell() > 0:  # a torn last row (interrupted write) keeps its own line
                f.seek(-1, os.SEEK_END)
                if f.read(1) != b"\n":
                    f.write(b"\n")
            f.write((json.dumps({"key": self.key, "point": p.as_dict()}) + "\n").encode())
            f.flush()
            os.fsync(f.fileno())


# ---------------------------------------------------------------------------
# GPU round functions (device-resident frame source + decode + count)

def _stream_seed(seed: int, snr_index: int) -> int:
    return (int(seed) * 0x9E3779B97F4A7C15 + (snr_index + 1) * 0xBF58476D1CE4E5B9) & (2 ** 64 - 1)


def polar_round_fn(decoder, seed: int = 0, crc_polynomial: Optional[str] = None):
    """Round function for a drop-in SC/SCL decoder (polar.SCDecoder/SCLDecoder).
    Random K-bit messages (CRC appended when crc_polynomial is given, as
    src/polar/encoder.py:74-78 does), device polar encoder, device AWGN,
    decode, device error count over the K decoded bits."""
    import torch
    from .. import _native
    from ..channel.awgn import AWGNChannel
    N, K = decoder.N, decoder._n_info
    bufs = {}

    def fn(snr_index, snr_db, offset, nframes):
        if bufs.get("B", 0) < nframes:
            bufs.update(B=nframes, msg=torch.empty((nframes, K), dtype=torch.uint8, device="cuda"),
                        cw=torch.empty((nframes, N), dtype=torch.uint8, device="cuda"),
                        llr=torch.empty((nframes, N), dtype=torch.float64, device="cuda"),
                        out=torch.empty((nframes, K), dtype=torch.uint8, device="cuda"))
        msg, cw, llr, out = (bufs[k][:nframes] for k in ("msg", "cw", "llr", "out"))
        s = _stream_seed(seed, snr_index)
        if crc_polynomial is None:
            _native.random_bits(s, offset, msg)
        else:  # data bits + their CRC, on the device (pl_crc_append)
            from ..polar.utils import CRC_POLYNOMIALS
            name = crc_polynomial if crc_polynomial in CRC_POLYNOMIALS else "CRC-8"
            L = int(name.split("-")[1])
            _native.random_bits(s, offset, msg)
            _native.crc_append(msg, K - L, L, CRC_POLYNOMIALS[name])
        _native.polar_encode(decoder.plan, msg, cw)
        AWGNChannel(snr_db).llr_batch_device(cw, N, nframes, seed=s ^ 0xA5A5A5A5, frame_offset=offset, out=llr)
        decoder.plan.decode(llr, out)
        counts = torch.zeros(3, dtype=torch.int64, device="cuda")
        _native.count_errors(msg, out, K, counts)
        return counts.cpu().numpy()

    return fn


def ldpc_round_fn(decoder, seed: int = 0, info_bits: Optional[int] = None, encoder=None):
    """Round function for BPDecoder/MSDecoder.

    encoder None: the all-zero codeword (BP and min-sum are codeword-symmetric);
    errors over the first `info_bits` positions, like ber_simulation.py:265-269
    (decoded[:k]).  encoder = an LDPCEncoder: random k-bit messages (device
    Philox), valid codewords on the device (LDPCEncoder.encode_batch_device,
    pl_gf2_encode), errors over the encoder's info positions -- the whole Monte
    Carlo chain device-resident."""
    import torch
    from .. import _native
    from ..channel.awgn import AWGNChannel
    n = decoder.n
    if encoder is not None:
        k = encoder.k
        info = torch.from_numpy(np.asarray(encoder.info_positions, dtype=np.int64)).cuda()
    else:
        k = info_bits if info_bits is not None else n - decoder.m
    bufs = {}

    def fn(snr_index, snr_db, offset, nframes):
        if bufs.get("B", 0) < nframes:
            bufs.update(B=nframes, llr=torch.empty((nframes, n), dtype=torch.float64, device="cuda"),
                        out=torch.empty((nframes, n), dtype=torch.uint8, device="cuda"),
                        its=torch.empty((nframes,), dtype=torch.int32, device="cuda"),
                        zero=torch.zeros((nframes, n), dtype=torch.uint8, device="cuda"),
                        msg=torch.empty((nframes, k), dtype=torch.uint8, device="cuda"),
                        cw=torch.empty((nframes, n), dtype=torch.uint8, device="cuda"))
        llr, out, its, zero, msg, cw = (bufs[x][:nframes] for x in ("llr", "out", "its", "zero", "msg", "cw"))
        s = _stream_seed(seed, snr_index)
        counts = torch.zeros(3, dtype=torch.int64, device="cuda")
        if encoder is None:
            AWGNChannel(snr_db).llr_batch_device(None, n, nframes, seed=s, frame_offset=offset, out=llr)
            decoder.plan.decode(llr, out, its)
            _native.count_errors(zero, out, k, counts)
        else:
            _native.random_bits(s, offset, msg)
            encoder.encode_batch_device(msg, out=cw)
            AWGNChannel(snr_db).llr_batch_device(cw, n, nframes, seed=s ^ 0xA5A5A5A5, frame_offset=offset, out=llr)
            decoder.plan.decode(llr, out, its)
            _native.count_errors(msg, out.index_select(1, info).contiguous(), k, counts)
        return counts.cpu().numpy()

    return fn


def stub_round_fn(seed: int = 0, info_bits: int = 16):
    """Deterministic CPU round function (tests and plumbing rehearsals only): the
    counts of frame f at SNR point i depend only on (seed, i, f), like the
    device round functions' Philox streams, so any sharding gives the same
    points.  Frame error iff hash(seed, i, f) % 1000 < 400 >> i; bit errors
    1 + f % 5 per erroneous frame."""
    def fn(snr_index, snr_db, offset, nframes):
        f = np.arange(offset, offset + nframes, dtype=np.uint64)
        h = (f * np.uint64(2654435761) + np.uint64((seed * 1000003 + snr_index * 97) & 0xFFFFFFFF)) % np.uint64(1000)
        err = h < np.uint64(400 >> min(snr_index, 16))
        bits = np.where(err, 1 + (f % np.uint64(5)), 0).astype(np.int64)
        return np.array([int(bits.sum()), int(err.sum()), int(nframes)], dtype=np.int64)
    return fn
