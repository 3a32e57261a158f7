"""Batched GPU counterpart of benchmarks/throughput_test.py (:22-353).

Same entry points, arguments and JSON fields as the reference
(`run_throughput_test`, `measure_polar_throughput`, `measure_ldpc_throughput`;
info-Mbps = frames * K / seconds / 1e6, :217, :237), but every phase processes
all `num_iterations` frames in one device batch instead of a Python loop:
encoding (device polar encoder; host LDPC encoder, as the reference), decoding
(one kernel launch over resident LLRs), end to end (device message source +
encode + AWGN + decode).  Times are wall-clock around synchronised device work.
"""
from __future__ import annotations

import time
from pathlib import Path
from typing import Dict, Optional

import numpy as np
import torch

from .. import _native
from ..channel.awgn import AWGNChannel
from ..ldpc.decoder import BPDecoder
from ..ldpc.encoder import LDPCEncoder
from ..polar.decoder import SCDecoder, SCLDecoder
from ..polar.encoder import PolarEncoder
from ..utils.visualization import save_results


def _timed(fn):
    torch.cuda.synchronize()
    t0 = time.time()
    out = fn()
    torch.cuda.synchronize()
    return time.time() - t0, out


def measure_polar_throughput(config: Dict, num_iterations: int, snr_db: float, list_size: int = 0,
                             seed: int = 42) -> Dict:
    """throughput_test.py:185-269.  list_size 0 = SCDecoder (the reference's
    choice), >= 1 = SCLDecoder(list_size)."""
    N, K = config["encoding"]["N"], config["encoding"]["K"]
    enc = PolarEncoder(N, K)
    fr = enc.get_frozen_bits_positions()
    dec = SCDecoder(N, K, frozen_bits=fr) if list_size <= 0 else SCLDecoder(N, K, list_size, frozen_bits=fr)
    B = int(num_iterations)
    ch = AWGNChannel(snr_db)
    msg = torch.empty((B, K), dtype=torch.uint8, device="cuda")
    cw = torch.empty((B, N), dtype=torch.uint8, device="cuda")
    llr = torch.empty((B, N), dtype=torch.float64, device="cuda")
    out = torch.empty((B, K), dtype=torch.uint8, device="cuda")

    def source():
        _native.random_bits(seed, 0, msg)

    def encode():
        _native.polar_encode(dec.plan, msg, cw)

    def channel():
        ch.llr_batch_device(cw, N, B, seed=seed, out=llr)

    def decode():
        dec.plan.decode(llr, out)

    for f in (source, encode, channel, decode):  # warm-up (throughput_test.py:204-209)
        f()
    source()
    t_enc, _ = _timed(encode)
    channel()
    t_dec, _ = _timed(decode)
    t_e2e, _ = _timed(lambda: [f() for f in (source, encode, channel, decode)])
    bits = B * K
    return {"N": N, "K": K, "rate": K / N, "num_iterations": B, "encoding_time": t_enc, "decoding_time": t_dec,
            "end_to_end_time": t_e2e, "encoding_throughput": bits / t_enc / 1e6,
            "decoding_throughput": bits / t_dec / 1e6, "end_to_end_throughput": bits / t_e2e / 1e6,
            "decoder": "SC" if list_size <= 0 else "SCL", "list_size": int(list_size)}


def measure_ldpc_throughput(config: Dict, num_iterations: int, snr_db: float, seed: int = 42) -> Dict:
    """throughput_test.py:272-353: LDPCEncoder(n, k, dv, dc, seed=42) (so the
    same H and, for its rank-deficient H, the same invalid codewords as the
    reference's timing), BPDecoder(H, max_iter)."""
    n, k = config["encoding"]["n"], config["encoding"]["k"]
    dv, dc = config["encoding"].get("dv", 3), config["encoding"].get("dc", 6)
    max_iter = config["decoding"].get("max_iterations", 50)
    enc = LDPCEncoder(n, k, dv=dv, dc=dc, seed=42)
    dec = BPDecoder(enc.H, max_iter=max_iter)
    B = int(num_iterations)
    rs = np.random.RandomState(seed)
    msgs = rs.randint(0, 2, (B, k))
    ch = AWGNChannel(snr_db)
    llr = torch.empty((B, n), dtype=torch.float64, device="cuda")
    out = torch.empty((B, n), dtype=torch.uint8, device="cuda")
    its = torch.empty((B,), dtype=torch.int32, device="cuda")

    def encode():
        return torch.from_numpy(enc.encode_batch(msgs).astype(np.uint8)).cuda()

    cw = encode()
    ch.llr_batch_device(cw, n, B, seed=seed, out=llr)
    dec.plan.decode(llr, out, its)  # warm-up
    t_enc, cw = _timed(encode)
    ch.llr_batch_device(cw, n, B, seed=seed, out=llr)
    t_dec, _ = _timed(lambda: dec.plan.decode(llr, out, its))

    def e2e():
        c = encode()
        ch.llr_batch_device(c, n, B, seed=seed, out=llr)
        dec.plan.decode(llr, out, its)

    t_e2e, _ = _timed(e2e)
    bits = B * k
    return {"n": n, "k": k, "rate": k / n, "num_iterations": B, "encoding_time": t_enc, "decoding_time": t_dec,
            "end_to_end_time": t_e2e, "encoding_throughput": bits / t_enc / 1e6,
            "decoding_throughput": bits / t_dec / 1e6, "end_to_end_throughput": bits / t_e2e / 1e6,
            "max_iter": max_iter, "mean_iterations": float(its.double().mean())}


def run_throughput_test(polar_config: Dict, ldpc_config: Dict, output_dir: Path, num_iterations: int = 100,
                        snr_db: float = 3.0, list_size: int = 0) -> Dict:
    """throughput_test.py:22-109: results {num_iterations, snr_db, polar, ldpc}
    saved to output_dir/data/throughput_results.json."""
    results = {"num_iterations": num_iterations, "snr_db": snr_db,
               "polar": measure_polar_throughput(polar_config, num_iterations, snr_db, list_size),
               "ldpc": measure_ldpc_throughput(ldpc_config, num_iterations, snr_db)}
    save_results(results, Path(output_dir) / "data" / "throughput_results.json")
    return results


if __name__ == "__main__":
    import argparse
    import json
    ap = argparse.ArgumentParser(description="batched GPU throughput test (throughput_test.py fields)")
    ap.add_argument("--frames", type=int, default=65536)
    ap.add_argument("--snr", type=float, default=3.0)
    ap.add_argument("--N", type=int, default=1024)
    ap.add_argument("--K", type=int, default=512)
    ap.add_argument("--list-size", type=int, default=0)
    ap.add_argument("--n", type=int, default=504)
    ap.add_argument("--k", type=int, default=252)
    ap.add_argument("--max-iter", type=int, default=20)
    ap.add_argument("--out", default="results")
    a = ap.parse_args()
    r = run_throughput_test({"encoding": {"N": a.N, "K": a.K}},
                            {"encoding": {"n": a.n, "k": a.k}, "decoding": {"max_iterations": a.max_iter}},
                            Path(a.out), a.frames, a.snr, a.list_size)
    print(json.dumps(r, indent=1))
