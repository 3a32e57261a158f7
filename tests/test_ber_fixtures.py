"""The reference-side BER/FER samples (tests/golden/ber_points.npz, written by
tests/golden/make_ber_golden.py) that tests/test_gpu_ber_parity.py compares the
device Monte-Carlo with: every point present with >= 16 384 frames and the
seeds the generator fixes, and the first frames of each point's first chunk
regenerated here -- the reference frame loop (benchmarks/ber_simulation.py:
167-192) restated with this build's host encoder and channel (equal to the
reference's, tests/test_host.py), decoded by the C oracle (equal to the
reference decoders, tests/test_oracle_golden.py) -- give the stored per-frame
bit errors.  CPU only."""
import importlib.util
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN, golden


def _generator():
    spec = importlib.util.spec_from_file_location("make_ber_golden", os.path.join(GOLDEN, "make_ber_golden.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_every_point_present_with_fixed_seeds():
    g = _generator()
    d = golden("ber_points.npz")
    for name, (kind, params, snr, seed) in g.POINTS.items():
        meta = json.loads(str(d[name + "_meta"]))
        err = d[name + "_err"]
        # distinct chunks (a generator that reseeded the RNG inside a chunk once
        # made all 32 BP chunks the same 512 frames)
        chunks = err.reshape(g.CHUNKS, g.FRAMES_PER_CHUNK)
        assert len({c.tobytes() for c in chunks}) > g.CHUNKS // 2, name
        assert meta["kind"] == kind and meta["snr_db"] == snr and meta["seed"] == seed, name
        assert meta["params"] == json.loads(json.dumps(params)), name
        assert meta["frames"] == err.size == g.CHUNKS * g.FRAMES_PER_CHUNK >= 16384, name


@pytest.mark.parametrize("name", ["sc256_m10", "scl8_m15", "scl32_m20", "ms20_m12", "bp20_m10", "cascl32_m15"])
def test_first_frames_regenerate(oracle, name):
    from polarcode_and_ldpc_amd.channel import AWGNChannel
    g = _generator()
    kind, p, snr, seed = g.POINTS[name]
    d = golden("ber_points.npz")
    want = d[name + "_err"][:6].astype(np.int64)
    if kind in ("bp", "ms"):  # H before the seed: LDPCEncoder(seed=42) reseeds the global RNG
        from polarcode_and_ldpc_amd.ldpc import LDPCEncoder
        from polarcode_and_ldpc_amd.ldpc.matrix import regular_construction
        if kind == "ms":
            H = np.asarray(regular_construction(p["n"], p["dv"], p["dc"], seed=p["hseed"]))
            k = H.shape[1] - H.shape[0]
        else:
            H = np.asarray(LDPCEncoder(p["n"], p["k"], dv=3, dc=6, seed=p["hseed"]).H)
            k = p["k"]
    np.random.seed(seed)  # chunk 0
    ch = AWGNChannel(snr)
    if kind == "cascl":  # PolarEncoder(use_crc=True): K - crc data bits, crc_encode appends the CRC
        from polarcode_and_ldpc_amd.polar import PolarEncoder, construct_frozen_set
        from polarcode_and_ldpc_amd.polar.utils import crc_encode
        N, K = p["N"], p["K"]
        fr = construct_frozen_set(N, K, 2.0)
        enc = PolarEncoder(N, K, frozen_bits=fr, use_crc=True, crc_polynomial=p["crc"])
        msgs, llrs = [], []
        for _ in range(6):
            m = np.random.randint(0, 2, enc.K_data)
            msgs.append(crc_encode(m, p["crc"]))
            llrs.append(ch.transmit(enc.encode(m), return_llr=True))
        msgs, llrs = np.array(msgs), np.array(llrs)
        got = (oracle.cascl_decode(N, p["L"], fr, llrs, crc_polynomial=p["crc"], threads=6) != msgs).sum(axis=1)
    elif kind in ("sc", "scl"):
        from polarcode_and_ldpc_amd.polar import PolarEncoder, construct_frozen_set
        N, K = p["N"], p["K"]
        fr = construct_frozen_set(N, K, 2.0)
        enc = PolarEncoder(N, K, frozen_bits=fr)
        msgs, llrs = [], []
        for _ in range(6):
            m = np.random.randint(0, 2, K)
            msgs.append(m)
            llrs.append(ch.transmit(enc.encode(m), return_llr=True))
        msgs, llrs = np.array(msgs), np.array(llrs)
        dec = oracle.sc_decode(N, fr, llrs) if kind == "sc" else oracle.scl_decode(N, p["L"], fr, llrs, threads=6)
        got = (dec != msgs).sum(axis=1)
    else:
        from polarcode_and_ldpc_amd.ldpc import dense_to_csr
        n = H.shape[1]
        llrs = np.array([ch.transmit(np.zeros(n, dtype=int), return_llr=True) for _ in range(6)])
        rp, ci = dense_to_csr(H)
        bits, _ = oracle.ldpc_decode(rp, ci, n, llrs, kind, p["max_iter"], True, 1.0, threads=6)
        got = bits[:, :k].sum(axis=1)
    assert np.array_equal(got, want), (name, got, want)
