#!/usr/bin/env python3
"""Reference-side BER/FER samples for tests/test_gpu_ber_parity.py.

The frame loop is the reference's own (benchmarks/ber_simulation.py:167-192 for
polar, :245-269 for LDPC): per frame ``np.random.randint(0, 2, K)`` message, the
reference encoder's ``encode``, ``AWGNChannel(snr, seed=None).transmit`` (global
NumPy RNG, src/channel/awgn.py:75-112), decode, ``np.sum(message != decoded)``.
Encoder and channel are the reference's classes, imported read-only from
/root/reference/src (this script runs in the build container only; the output is
data).  Decoders:

  * SC N=256 and BP-20 (504,252): the reference's own SCDecoder / BPDecoder;
  * SCL L=8 / L=32 N=1024 and MS-20 n=8192: the pinned C oracle
    (oracle/refcpu.c, bit-exact with the reference decoders on every golden
    vector, tests/test_oracle_golden.py) -- the reference's Python SCL at L=32
    and MSDecoder at n=8192 take seconds per frame.

LDPC points transmit the all-zero codeword (BP and min-sum are
codeword-symmetric; the reference's BER loop encodes with pyldpc's G, which is
absent here) and count errors over the first k positions.

Every point draws CHUNKS chunks of FRAMES_PER_CHUNK frames; chunk c seeds the
global RNG with ``seed + c`` before its frame loop.  The seeds below were fixed
before any GPU run of the test that reads them (round 4), so the device
Monte-Carlo is compared against a sample nobody chose after the fact.

Output: tests/golden/ber_points.npz -- for each point ``<name>_err`` (uint16 bit
errors per frame, in frame order), ``<name>_meta`` (JSON: code, SNR, seed,
decoder, frames).

Usage:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_ber_golden.py [-j 8] [--only name,...]
"""
import argparse
import json
import os
import sys
import time
from multiprocessing import Pool

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
FRAMES_PER_CHUNK = 512
CHUNKS = 32  # 16 384 frames per point

# name: (kind, params, snr_db, seed).  Seeds fixed in round 4 before any GPU run.
POINTS = {
    "sc256_m20": ("sc", dict(N=256, K=128), -2.0, 410000),
    "sc256_m10": ("sc", dict(N=256, K=128), -1.0, 420000),
    "sc256_p00": ("sc", dict(N=256, K=128), 0.0, 430000),
    "scl8_m20": ("scl", dict(N=1024, K=512, L=8), -2.0, 440000),
    "scl8_m15": ("scl", dict(N=1024, K=512, L=8), -1.5, 450000),
    "scl8_m10": ("scl", dict(N=1024, K=512, L=8), -1.0, 460000),
    "scl32_m20": ("scl", dict(N=1024, K=512, L=32), -2.0, 470000),
    "scl32_m15": ("scl", dict(N=1024, K=512, L=32), -1.5, 480000),
    "ms20_m12": ("ms", dict(n=8192, dv=3, dc=6, hseed=11, max_iter=20), -1.2, 490000),
    "ms20_m10": ("ms", dict(n=8192, dv=3, dc=6, hseed=11, max_iter=20), -1.0, 500000),
    "bp20_m10": ("bp", dict(n=504, k=252, hseed=42, max_iter=20), -1.0, 510000),
    "bp20_p05": ("bp", dict(n=504, k=252, hseed=42, max_iter=20), 0.5, 520000),
    # round 5: CA-SCL L=32 + CRC-8 at the low end of the
    # configs[3] sweep; seeds fixed before any GPU run of the test that reads them
    "cascl32_m20": ("cascl", dict(N=1024, K=512, L=32, crc="CRC-8"), -2.0, 530000),
    "cascl32_m15": ("cascl", dict(N=1024, K=512, L=32, crc="CRC-8"), -1.5, 540000),
}


def _imp():
    sys.dont_write_bytecode = True
    for p in (os.path.join(REF, "src"), ROOT):
        if p not in sys.path:
            sys.path.insert(0, p)
    import polar, ldpc, channel  # noqa: F401  (the reference packages)
    return polar, ldpc, channel


def _H(kind, p):
    sys.path.insert(0, ROOT)
    if kind == "ms":
        from polarcode_and_ldpc_amd.ldpc.matrix import regular_construction
        return np.asarray(regular_construction(p["n"], p["dv"], p["dc"], seed=p["hseed"]))
    _, ldpc, _ = _imp()
    return np.asarray(ldpc.LDPCEncoder(p["n"], p["k"], dv=3, dc=6, seed=p["hseed"]).H)


def _chunk(task):
    name, c = task
    kind, p, snr, seed = POINTS[name]
    polar, ldpc, channel = _imp()
    from oracle import oracle
    # H first: the reference's LDPCEncoder(seed=42) reseeds NumPy's global RNG
    # (mackay_construction, src/ldpc/matrix.py:34-35); built after the chunk's
    # seed it made every BP chunk draw the same 512 frames (round 4, caught by
    # the GPU parity test's first run and fixed here; seeds unchanged)
    H = _H(kind, p) if kind in ("bp", "ms") else None
    np.random.seed(seed + c)
    ch = channel.AWGNChannel(snr_db=snr, seed=None)
    nf = FRAMES_PER_CHUNK
    if kind == "cascl":
        # the reference's encoder with use_crc (src/polar/encoder.py:63-87: K - crc
        # data bits, crc_encode appends the CRC); no reference CA-SCL decoder exists
        # (decoder.py:202-203,259 store use_crc and never read it), so the frames
        # are decoded by the oracle's restatement of the build-defined CA-SCL
        # (oracle.cascl_decode, pinned frame by frame against the GPU kernel)
        from polarcode_and_ldpc_amd.polar import construct_frozen_set
        from polar.utils import crc_encode
        N, K, crc = p["N"], p["K"], p["crc"]
        fr = construct_frozen_set(N, K, 2.0)
        enc = polar.PolarEncoder(N, K, frozen_bits=fr, use_crc=True, crc_polynomial=crc)
        msgs, llrs = [], []
        for _ in range(nf):
            m = np.random.randint(0, 2, enc.K_data)
            msgs.append(crc_encode(m, crc))
            llrs.append(ch.transmit(enc.encode(m), return_llr=True))
        msgs, llrs = np.array(msgs), np.array(llrs)
        dec = oracle.cascl_decode(N, p["L"], fr, llrs, crc_polynomial=crc, threads=1)
        err = (dec != msgs).sum(axis=1)
    elif kind in ("sc", "scl"):
        from polarcode_and_ldpc_amd.polar import construct_frozen_set
        N, K = p["N"], p["K"]
        fr = construct_frozen_set(N, K, 2.0)  # ber_simulation.py:146-148 (PolarLibWrapper substitute)
        enc = polar.PolarEncoder(N, K, frozen_bits=fr)
        msgs, llrs = [], []
        for _ in range(nf):
            m = np.random.randint(0, 2, K)
            msgs.append(m)
            llrs.append(ch.transmit(enc.encode(m), return_llr=True))
        msgs, llrs = np.array(msgs), np.array(llrs)
        if kind == "sc":
            d = polar.SCDecoder(N, K, frozen_bits=fr)
            dec = np.array([d.decode(l) for l in llrs])
        else:
            dec = oracle.scl_decode(N, p["L"], fr, llrs, threads=1)
        err = (dec != msgs).sum(axis=1)
    else:
        n = H.shape[1]
        k = n - H.shape[0] if kind == "ms" else p["k"]
        llrs = np.array([ch.transmit(np.zeros(n, dtype=int), return_llr=True) for _ in range(nf)])
        if kind == "bp":
            d = ldpc.BPDecoder(H, max_iter=p["max_iter"])
            err = np.array([d.decode(l)[:k].sum() for l in llrs])
        else:
            from polarcode_and_ldpc_amd.ldpc import dense_to_csr
            rp, ci = dense_to_csr(H)
            bits, _ = oracle.ldpc_decode(rp, ci, n, llrs, "ms", p["max_iter"], True, 1.0, threads=1)
            err = bits[:, :k].sum(axis=1)
    return name, c, np.asarray(err, dtype=np.uint16)


def main():
    global REF
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default=REF)
    ap.add_argument("--only", default=None)
    ap.add_argument("-j", type=int, default=8)
    a = ap.parse_args()
    REF = a.ref
    names = [n for n in POINTS if a.only is None or n in a.only.split(",")]
    out_path = os.path.join(HERE, "ber_points.npz")
    out = dict(np.load(out_path)) if os.path.exists(out_path) else {}
    # the slow points first so the pool drains evenly
    order = {"bp": 0, "cascl": 1, "scl": 1, "sc": 2, "ms": 3}
    tasks = sorted([(n, c) for n in names for c in range(CHUNKS)], key=lambda t: (order[POINTS[t[0]][0]], t))
    got = {n: [None] * CHUNKS for n in names}
    t0 = time.time()
    with Pool(a.j) as pool:
        for i, (name, c, err) in enumerate(pool.imap_unordered(_chunk, tasks)):
            got[name][c] = err
            if all(x is not None for x in got[name]):
                kind, p, snr, seed = POINTS[name]
                e = np.concatenate(got[name])
                out[name + "_err"] = e
                dec = "reference" if kind in ("sc", "bp") else "oracle/refcpu.c"
                out[name + "_meta"] = np.array(json.dumps(dict(
                    kind=kind, params=p, snr_db=snr, seed=seed, chunks=CHUNKS,
                    frames_per_chunk=FRAMES_PER_CHUNK, frames=int(e.size), decoder=dec)))
                np.savez_compressed(out_path, **out)
                print("%s: %d frames, FER %.4f, BER/frame %.3f  (%.0f s)" % (
                    name, e.size, (e > 0).mean(), e.mean(), time.time() - t0), flush=True)
            elif i % 16 == 0:
                print("  %d/%d chunks (%.0f s)" % (i + 1, len(tasks), time.time() - t0), flush=True)


if __name__ == "__main__":
    main()
