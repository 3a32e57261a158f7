"""Host-side (CPU) checks of the harness parity layer: the reference-layout
import shim, lib_wrappers substitutes, LDPC/metrics helpers, channels' host
paths.  No GPU calls."""
import json
import sys

import numpy as np
import pytest

ROOT = __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__)))


def test_compat_shim_resolves_reference_imports():
    """The imports of benchmarks/*.py and tests/*.py of the reference resolve
    through polarcode_and_ldpc_amd/compat/src to this package's objects."""
    import polarcode_and_ldpc_amd.polar as P
    shim = ROOT + "/polarcode_and_ldpc_amd/compat/src"
    sys.path.insert(0, shim)
    sys.path.insert(0, ROOT + "/polarcode_and_ldpc_amd/compat")
    try:
        from channel import AWGNChannel, BSCChannel, RayleighFadingChannel  # noqa: F401
        from ldpc import BPDecoder, LDPCEncoder, check_syndrome, create_tanner_graph, peg_construction  # noqa: F401
        from lib_wrappers import LDPCLibWrapper, PolarLibWrapper  # noqa: F401
        from polar import PolarEncoder, SCDecoder, SCLDecoder, construct_polar_code  # noqa: F401
        from src.polar.decoder import SCDecoder as S2
        from utils import plot_ber_curves, save_results  # noqa: F401
        from utils.metrics import calculate_ber, calculate_fer  # noqa: F401
        assert SCDecoder is P.SCDecoder and S2 is P.SCDecoder
    finally:
        sys.path.remove(shim)
        sys.path.remove(ROOT + "/polarcode_and_ldpc_amd/compat")


def test_ldpc_lib_wrapper_substitute_is_a_valid_systematic_code():
    from polarcode_and_ldpc_amd.lib_wrappers import LDPCLibWrapper
    w = LDPCLibWrapper(504, 252, dv=3, dc=6, seed=42)
    H, G = w.get_parity_check_matrix(), w.get_generator_matrix()
    assert H.shape == (w.m, 504) and G.shape == (504, w.k)
    assert not ((H @ G) % 2).any()
    m = np.random.RandomState(0).randint(0, 2, w.k)
    c = w.encode(m)
    assert np.array_equal(c[:w.k], m) and not ((H @ c) % 2).any()


def test_polar_lib_wrapper_substitute():
    from polarcode_and_ldpc_amd.lib_wrappers import PolarLibWrapper
    from polarcode_and_ldpc_amd.polar import construct_frozen_set
    w = PolarLibWrapper(1024, 512, 2.0)
    assert np.array_equal(w.get_frozen_bits_positions(), construct_frozen_set(1024, 512, 2.0))
    assert len(w.get_info_bits_positions()) == 512 and w.get_code_rate() == 0.5


def test_ldpc_helpers():
    from polarcode_and_ldpc_amd.ldpc import (calculate_girth, check_syndrome, create_tanner_graph,
                                             peg_construction)
    H = peg_construction(12, 6, 2)
    assert (H.sum(axis=0) == 2).all() and H.sum(axis=1).max() - H.sum(axis=1).min() <= 1
    vn, cn = create_tanner_graph(H)
    assert all(H[c, v] == 1 for c in range(6) for v in cn[c]) and sum(map(len, vn)) == H.sum()
    assert check_syndrome(H, np.zeros(12, int))
    assert calculate_girth(H) in (4, 6)


def test_metrics_match_reference_formulas():
    from polarcode_and_ldpc_amd.utils import (calculate_ber, calculate_ber_with_confidence, calculate_fer,
                                              calculate_throughput)
    from scipy import stats
    assert calculate_ber(np.array([0, 1, 1, 0]), np.array([0, 0, 1, 1])) == 0.5
    assert calculate_fer([np.zeros(3), np.ones(3)], [np.zeros(3), np.zeros(3)]) == 0.5
    assert calculate_throughput(10 ** 6, 0.5) == 2.0 and calculate_throughput(1, 0) == 0.0
    ber, lo, hi = calculate_ber_with_confidence(37, 10000)
    z = stats.norm.ppf(0.975)
    p, n = 37 / 10000, 10000
    c = (p + z * z / (2 * n)) / (1 + z * z / n)
    h = z * np.sqrt(p * (1 - p) / n + z * z / (4 * n * n)) / (1 + z * z / n)
    assert ber == p and abs(lo - (c - h)) < 1e-12 and abs(hi - (c + h)) < 1e-12


def test_save_results_json(tmp_path):
    from polarcode_and_ldpc_amd.utils import save_results
    save_results({"a": np.arange(3), "b": {"c": np.float64(1.5), "d": np.int32(2)}}, tmp_path / "x" / "r.json")
    assert json.load(open(tmp_path / "x" / "r.json")) == {"a": [0, 1, 2], "b": {"c": 1.5, "d": 2}}


def test_host_channels_follow_reference_rng_use():
    """BSC / Rayleigh host methods draw from NumPy's global RNG exactly as the
    reference (src/channel/bsc.py:33-49, fading.py:31-63)."""
    from polarcode_and_ldpc_amd.channel import BSCChannel, RayleighFadingChannel
    bits = np.random.RandomState(1).randint(0, 2, 64)
    out = BSCChannel(0.2, seed=7).transmit(bits)
    np.random.seed(7)
    flip = np.random.random(64) < 0.2
    assert np.array_equal(out, np.where(flip, 1 - bits, bits))
    llr = RayleighFadingChannel(1.0, seed=9).transmit(bits)
    np.random.seed(9)
    s = 1.0 - 2.0 * bits
    hr, hi = np.random.normal(0, 1 / np.sqrt(2), 64), np.random.normal(0, 1 / np.sqrt(2), 64)
    h = np.abs(hr + 1j * hi)
    sd = np.sqrt(1.0 / (2.0 * 10 ** 0.1))
    y = h * s + np.random.normal(0, sd, 64)
    assert np.allclose(llr, 2.0 * y * h / sd ** 2, rtol=0, atol=0)


def test_valid_generator_spans_the_code():
    """§8 f row 3: the seed-42 (504, 252) H is rank-deficient (rank 251, rank of
    H2 236), so the reference's encoders emit non-codewords; valid_generator's
    rows are codewords, independent, with the message at `info`."""
    from polarcode_and_ldpc_amd.ldpc import LDPCEncoder, regular_construction, valid_generator
    from polarcode_and_ldpc_amd._native import pack_gf2_columns
    enc = LDPCEncoder(504, 252, dv=3, dc=6, seed=42)
    H = np.asarray(enc.H).astype(np.int64)
    G, info = enc.valid_generator()
    assert G.shape == (252, 504) and len(np.unique(info)) == 252
    assert not ((H @ G.T.astype(np.int64)) % 2).any()
    assert np.array_equal(G[:, info], np.eye(252, dtype=np.uint8))
    assert not ((H @ np.asarray(enc.encode(np.ones(252, int))).astype(np.int64)) % 2 == 0).all()  # reference quirk
    H2 = np.asarray(regular_construction(504, 3, 6, seed=3)).astype(np.int64)
    G2, info2 = valid_generator(H2)
    assert not ((H2 @ G2.T.astype(np.int64)) % 2).any() and G2.shape[0] == len(info2)
    P = pack_gf2_columns(G).view(np.uint32)
    i, j = 37, 411
    assert ((P[i // 32, j] >> (i % 32)) & 1) == G[i, j]
    assert P.shape == (8, 504)
