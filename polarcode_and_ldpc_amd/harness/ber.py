"""Batched, multi-GPU counterpart of benchmarks/ber_simulation.py (:24-293).

`run_ber_simulation` keeps the reference's arguments and result layout
({'snr_db', 'polar': {'self': {'ber', 'fer'}}, 'ldpc': {'self': ...}} saved to
output_dir/data/ber_simulation_results.json) and adds per-point frame / error
counts with Wilson intervals.  Frames are generated, decoded and counted on the
device in rounds (harness/montecarlo.py): the max_errors stop is applied per
round, frames are sharded over the ranks of an initialised torch.distributed
group with one all-reduce of the counters per round.

Code choices follow the reference's simulate_* (:132-293): polar frozen set from
PolarLibWrapper(N, K, 2.0) (offline substitute: bit-reversed Bhattacharyya),
LDPC H from LDPCLibWrapper(n, k, dv, dc, seed=42) (offline substitute), BP with
max_iterations, errors over the k message positions.  LDPC frames use the
all-zero codeword (BP is codeword-symmetric); polar frames use random messages
through the device encoder.
"""
from __future__ import annotations

from pathlib import Path
from typing import Dict, Optional, Sequence

import numpy as np

from ..utils.visualization import save_results
from .montecarlo import MonteCarlo, PointLog, ldpc_round_fn, polar_round_fn


def _digest(*arrays) -> str:
    import hashlib
    h = hashlib.sha1()
    for a in arrays:
        a = np.ascontiguousarray(a)
        h.update(str(a.shape).encode())
        h.update(a.astype(np.int64).tobytes())
    return h.hexdigest()[:16]


def _log(log_path, mc, **key):
    """PointLog whose run key names everything a point's counts depend on: the
    code construction (digest of the frozen set / H), the decoder, the frame
    budget, the frames per round and the decoder library build."""
    if not log_path:
        return None
    from .. import _native
    return PointLog(log_path, dict(key, round_frames=mc.batch * mc.world, lib=_native.build_id()))


def simulate_polar(snr_db_range: Sequence[float], num_frames: int, max_errors: int, config: Dict,
                   list_size: int = 0, crc_polynomial: Optional[str] = None, batch: int = 65536, seed: int = 0,
                   group=None, log_path=None):
    """ber_simulation.py:132-198 -> (ber, fer, points).  list_size 0 = SC (the
    reference), >= 1 = SCL, with crc_polynomial = CA-SCL (CRC inside the K bits).
    log_path: JSON-lines file of finished points; a rerun resumes from it."""
    import torch
    from ..lib_wrappers import PolarLibWrapper
    from ..polar.decoder import CASCLDecoder, SCDecoder, SCLDecoder
    N, K = config["encoding"]["N"], config["encoding"]["K"]
    fr = PolarLibWrapper(N, K, 2.0).get_frozen_bits_positions()
    if list_size <= 0:
        dec = SCDecoder(N, K, frozen_bits=fr)
    elif crc_polynomial:
        dec = CASCLDecoder(N, K, list_size, frozen_bits=fr, crc_polynomial=crc_polynomial)
    else:
        dec = SCLDecoder(N, K, list_size, frozen_bits=fr)
    mc = MonteCarlo(polar_round_fn(dec, seed=seed, crc_polynomial=crc_polynomial), info_bits=K, batch=batch,
                    group=group, device=torch.device("cuda", torch.cuda.current_device()))
    log = _log(log_path, mc, code="polar", N=N, K=K, list_size=list_size, crc=crc_polynomial, frames=num_frames,
               max_errors=max_errors, seed=seed, frozen=_digest(np.sort(np.asarray(fr))))
    pts = mc.run(snr_db_range, num_frames, max_errors, log=log)
    return np.array([p.ber for p in pts]), np.array([p.fer for p in pts]), pts


def simulate_ldpc(snr_db_range: Sequence[float], num_frames: int, max_errors: int, config: Dict,
                  batch: int = 65536, seed: int = 0, group=None, random_codewords: bool = False, log_path=None):
    """ber_simulation.py:201-293 -> (ber, fer, points).  random_codewords: random
    messages encoded into valid codewords on the device (LDPCEncoder.
    encode_batch_device) instead of the all-zero codeword."""
    import torch
    from ..ldpc.decoder import BPDecoder
    from ..ldpc.encoder import LDPCEncoder
    from ..lib_wrappers import LDPCLibWrapper
    n, k = config["encoding"]["n"], config["encoding"]["k"]
    cons = config.get("construction", config["encoding"])
    lib = LDPCLibWrapper(n, k, dv=cons.get("dv", 3), dc=cons.get("dc", 6), seed=42)
    H = lib.get_parity_check_matrix()
    dec = BPDecoder(H, max_iter=config["decoding"].get("max_iterations", 50))
    enc = LDPCEncoder(n, lib.k, H=H) if random_codewords else None
    mc = MonteCarlo(ldpc_round_fn(dec, seed=seed, info_bits=lib.k, encoder=enc), info_bits=lib.k, batch=batch,
                    group=group, device=torch.device("cuda", torch.cuda.current_device()))
    log = _log(log_path, mc, code="ldpc", n=n, k=lib.k, max_iter=dec.max_iter, random=random_codewords,
               frames=num_frames, max_errors=max_errors, seed=seed, dv=cons.get("dv", 3), dc=cons.get("dc", 6),
               H=_digest(np.asarray(H) & 1))
    pts = mc.run(snr_db_range, num_frames, max_errors, log=log)
    return np.array([p.ber for p in pts]), np.array([p.fer for p in pts]), pts


def run_ber_simulation(snr_db_range: np.ndarray, num_frames: int, max_errors: int, polar_config: Dict,
                       ldpc_config: Dict, output_dir: Path, use_third_party: bool = False, batch: int = 65536,
                       list_size: int = 0, crc_polynomial: Optional[str] = None, resume: bool = False) -> Dict:
    """ber_simulation.py:296-... -> results dict (also saved as JSON).  resume:
    keep per-point rows in output_dir/data/ber_points.jsonl and take finished
    points from it (opt-in: a fresh call always simulates)."""
    snr = np.asarray(snr_db_range, dtype=float)
    results = {"snr_db": snr.tolist(), "polar": {}, "ldpc": {}}
    points = Path(output_dir) / "data" / "ber_points.jsonl" if resume else None
    pb, pf, pp = simulate_polar(snr, num_frames, max_errors, polar_config, list_size, crc_polynomial, batch,
                                log_path=points)
    results["polar"]["self"] = {"ber": pb.tolist(), "fer": pf.tolist(), "points": [p.as_dict() for p in pp]}
    lb, lf, lp = simulate_ldpc(snr, num_frames, max_errors, ldpc_config, batch, log_path=points)
    results["ldpc"]["self"] = {"ber": lb.tolist(), "fer": lf.tolist(), "points": [p.as_dict() for p in lp]}
    if use_third_party:
        print("Warning: third-party libraries (polarcodes, pyldpc) are not available offline")
    save_results(results, Path(output_dir) / "data" / "ber_simulation_results.json")
    return results


def _parse_range(s: str):
    a, b, c = (float(x) for x in s.split(":"))
    return np.arange(a, b + c / 2, c)


def main(argv=None):
    """CLI (one process per GPU under torchrun; RCCL all-reduce of the counters):
    python -m polarcode_and_ldpc_amd.harness.ber --code polar --N 1024 --K 512 \\
        --list-size 32 --crc CRC-8 --snr=-2:5:1 --frames 1000000 --max-errors 100"""
    import argparse
    import json
    import os
    import torch
    import torch.distributed as dist
    ap = argparse.ArgumentParser()
    ap.add_argument("--code", choices=["polar", "ldpc"], default="polar")
    ap.add_argument("--N", type=int, default=1024)
    ap.add_argument("--K", type=int, default=512)
    ap.add_argument("--list-size", type=int, default=0)
    ap.add_argument("--crc", default=None)
    ap.add_argument("--n", type=int, default=504)
    ap.add_argument("--k", type=int, default=252)
    ap.add_argument("--max-iter", type=int, default=20)
    ap.add_argument("--snr", default="-2:5:1")
    ap.add_argument("--frames", type=int, default=1 << 20)
    ap.add_argument("--max-errors", type=int, default=100)
    ap.add_argument("--batch", type=int, default=65536)
    ap.add_argument("--out", default=None)
    ap.add_argument("--log", "--resume-log", dest="log", default=None,
                    help="JSON-lines file of finished SNR points; a rerun resumes from it (under torchrun spell it "
                         "--resume-log: torchrun's own parser takes --log for an abbreviation of --log-dir)")
    ap.add_argument("--ldpc-codewords", choices=["zero", "random"], default="zero",
                    help="LDPC frames: all-zero codeword, or random messages encoded on the device")
    ap.add_argument("--cpu-stub", action="store_true",
                    help="plumbing check on CPU: gloo ranks and a deterministic stub round function "
                         "(montecarlo.stub_round_fn) instead of the device decoders; not a simulation")
    a = ap.parse_args(argv)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if not a.cpu_stub:
        torch.cuda.set_device(local)
    if world > 1:
        if a.cpu_stub:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    snr = _parse_range(a.snr)
    if a.cpu_stub:
        from .montecarlo import stub_round_fn
        mc = MonteCarlo(stub_round_fn(seed=7, info_bits=a.K), info_bits=a.K, batch=a.batch)
        log = _log(a.log, mc, code="stub", K=a.K, frames=a.frames, max_errors=a.max_errors)
        pts = mc.run(snr, a.frames, a.max_errors, log=log)
        ber, fer = np.array([p.ber for p in pts]), np.array([p.fer for p in pts])
    elif a.code == "polar":
        ber, fer, pts = simulate_polar(snr, a.frames, a.max_errors, {"encoding": {"N": a.N, "K": a.K}},
                                       a.list_size, a.crc, a.batch, log_path=a.log)
    else:
        ber, fer, pts = simulate_ldpc(snr, a.frames, a.max_errors,
                                      {"encoding": {"n": a.n, "k": a.k}, "decoding": {"max_iterations": a.max_iter}},
                                      a.batch, random_codewords=a.ldpc_codewords == "random", log_path=a.log)
    if int(os.environ.get("RANK", "0")) == 0:
        res = {"code": a.code, "snr_db": snr.tolist(), "ber": ber.tolist(), "fer": fer.tolist(), "gpus": world,
               "points": [p.as_dict() for p in pts]}
        print(json.dumps(res))
        if a.out:
            save_results(res, a.out)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
