"""BER/FER parity of the device Monte-Carlo chain with the reference's CPU path
(BASELINE.json north_star: "BER/FER curves agree within Monte-Carlo error at
every SNR point"), and the distribution of the device AWGN source.

Device side (the product path): harness.montecarlo -- device random messages
(Philox), device polar encoder or the all-zero LDPC codeword, pl_awgn_llr
(Philox4x32-10 + Box-Muller), the HIP decoder, device error count; 65 536 -
131 072 frames per point.

Reference side (round 4): tests/golden/ber_points.npz,
16 384 frames per point made in the build container by
tests/golden/make_ber_golden.py with seeds fixed before any GPU run: the
reference's own frame loop (benchmarks/ber_simulation.py:167-192:
np.random.randint messages, the reference encoder, AWGNChannel.transmit with
np.random.normal), decoded by the reference's SCDecoder / BPDecoder (SC N=256,
BP-20) or by the pinned C oracle (SCL L=8 / L=32, MS-20; the reference's
Python SCL at L=32 and MSDecoder at n=8192 take seconds per frame).  The GPU
box only runs the device Monte-Carlo.

Criteria:
  * FER: the 95 % Wilson intervals of src/utils/metrics.py:138-167 overlap;
  * BER: bit errors within a frame are correlated (a wrong frame carries many),
    so a Wilson interval over bits is far too narrow; the BER check is a
    two-sample z-test on bit errors per frame (frames are the independent
    units), |z| < 3.5.
"""
import json
import math

import numpy as np
import pytest
import torch

from conftest import golden

pytestmark = pytest.mark.gpu


def _ref_point(name, kind, snr):
    """Per-frame bit errors of a reference-side point, with its metadata checked."""
    d = golden("ber_points.npz")
    meta = json.loads(str(d[name + "_meta"]))
    assert meta["kind"] == kind and meta["snr_db"] == snr and meta["frames"] >= 16384, meta
    return d[name + "_err"].astype(np.int64)


def _compare(dev, host_err, K, label):
    from polarcode_and_ldpc_amd.harness.montecarlo import wilson_interval
    nh = len(host_err)
    fh, bh = int((host_err > 0).sum()), int(host_err.sum())
    _, lo_d, hi_d = wilson_interval(dev.frame_errors, dev.frames)
    _, lo_h, hi_h = wilson_interval(fh, nh)
    assert lo_d <= hi_h and lo_h <= hi_d, "%s FER: device %.4g [%.4g, %.4g] vs reference %.4g [%.4g, %.4g]" % (
        label, dev.fer, lo_d, hi_d, fh / nh, lo_h, hi_h)
    # BER: per-frame bit-error counts are the independent units
    var = float(np.var(host_err, ddof=1)) if nh > 1 else 0.0
    md, mh = dev.bit_errors / dev.frames, bh / nh
    se = math.sqrt(var / dev.frames + var / nh)
    z = 0.0 if se == 0 else (md - mh) / se
    assert abs(z) < 3.5, "%s BER: device %.4g vs reference %.4g (z = %.2f)" % (label, md / K, mh / K, z)
    return dict(fer_dev=dev.fer, fer_ref=fh / nh, ber_dev=md / K, ber_ref=mh / K, z=z)


@pytest.mark.parametrize("snr,name", [(-2.0, "sc256_m20"), (-1.0, "sc256_m10"), (0.0, "sc256_p00")])
def test_sc_n256_ber_fer_parity(gpu, snr, name):
    """SC N=256 K=128 (the reference's own SCDecoder on the reference side)."""
    from polarcode_and_ldpc_amd.harness.montecarlo import MonteCarlo, polar_round_fn
    from polarcode_and_ldpc_amd.polar import SCDecoder, construct_frozen_set
    N, K = 256, 128
    fr = construct_frozen_set(N, K, 2.0)  # ber_simulation.py:146-148 (PolarLibWrapper substitute)
    dev = MonteCarlo(polar_round_fn(SCDecoder(N, K, frozen_bits=fr), seed=101), info_bits=K,
                     batch=65536).run([snr], 131072, 10 ** 12)[0]
    r = _compare(dev, _ref_point(name, "sc", snr), K, "SC N=256 @ %g dB" % snr)
    assert r["fer_ref"] > 0.005  # a point with errors to compare


@pytest.mark.parametrize("snr,name", [(-2.0, "scl8_m20"), (-1.5, "scl8_m15"), (-1.0, "scl8_m10")])
def test_scl_l8_n1024_ber_fer_parity(gpu, snr, name):
    """SCL L=8 N=1024 in its waterfall (Es/N0, the reference's SNR)."""
    from polarcode_and_ldpc_amd.harness.montecarlo import MonteCarlo, polar_round_fn
    from polarcode_and_ldpc_amd.polar import SCLDecoder, construct_frozen_set
    N, K, L = 1024, 512, 8
    fr = construct_frozen_set(N, K, 2.0)
    dev = MonteCarlo(polar_round_fn(SCLDecoder(N, K, L, frozen_bits=fr), seed=102), info_bits=K,
                     batch=65536).run([snr], 131072, 10 ** 12)[0]
    r = _compare(dev, _ref_point(name, "scl", snr), K, "SCL L=8 N=1024 @ %g dB" % snr)
    assert r["fer_ref"] > 0.001


@pytest.mark.parametrize("snr,name", [(-2.0, "scl32_m20"), (-1.5, "scl32_m15")])
def test_scl_l32_n1024_ber_fer_parity(gpu, snr, name):
    """Plain SCL L=32 N=1024 (the reference's SCLDecoder at the configs[3] list
    size; its use_crc is inert) at the low end of the configs[3] sweep.  Round 3
    compared 2 048 host frames drawn from a seed chosen after the first seed's
    sample failed (a 3.2-sigma outlier); this version compares
    16 384 reference-side frames whose seeds were fixed before any GPU run."""
    from polarcode_and_ldpc_amd.harness.montecarlo import MonteCarlo, polar_round_fn
    from polarcode_and_ldpc_amd.polar import SCLDecoder, construct_frozen_set
    N, K, L = 1024, 512, 32
    fr = construct_frozen_set(N, K, 2.0)
    dev = MonteCarlo(polar_round_fn(SCLDecoder(N, K, L, frozen_bits=fr), seed=104), info_bits=K,
                     batch=32768).run([snr], 65536, 10 ** 12)[0]
    r = _compare(dev, _ref_point(name, "scl", snr), K, "SCL L=32 N=1024 @ %g dB" % snr)
    assert r["fer_ref"] > 0.005


@pytest.mark.parametrize("snr,name", [(-1.2, "ms20_m12"), (-1.0, "ms20_m10")])
def test_ms20_8192_ber_fer_parity(gpu, snr, name):
    """Min-Sum (normalization 1.0) max_iter=20 with early stop on the n=8192
    (3,6)-regular code of the configs[4] bench (every check degree 6: the
    reference's MSDecoder raises on degree-1 checks), all-zero codeword, errors
    over the first k positions; the waterfall of this code."""
    from polarcode_and_ldpc_amd.harness.montecarlo import MonteCarlo, ldpc_round_fn
    from polarcode_and_ldpc_amd.ldpc import MSDecoder
    from polarcode_and_ldpc_amd.ldpc.matrix import regular_construction
    H = regular_construction(8192, 3, 6, seed=11)
    k = 8192 - H.shape[0]
    dec = MSDecoder(H, max_iter=20, normalization=1.0, early_stop=True)
    dev = MonteCarlo(ldpc_round_fn(dec, seed=105, info_bits=k), info_bits=k, batch=16384).run([snr], 65536,
                                                                                           10 ** 12)[0]
    r = _compare(dev, _ref_point(name, "ms", snr), k, "MS-20 n=8192 @ %g dB" % snr)
    assert r["fer_ref"] > 0.01


@pytest.mark.parametrize("snr,name", [(-1.0, "bp20_m10"), (0.5, "bp20_p05")])
def test_bp20_504_ber_fer_parity(gpu, snr, name):
    """BP-20 on the seed-42 (504, 252) code, all-zero codeword (BP is
    codeword-symmetric; the device side is harness.montecarlo.ldpc_round_fn),
    errors over the first k positions as ber_simulation.py:265-269; the
    reference side is the reference's own BPDecoder."""
    from polarcode_and_ldpc_amd.harness.montecarlo import MonteCarlo, ldpc_round_fn
    from polarcode_and_ldpc_amd.ldpc import BPDecoder, LDPCEncoder
    enc = LDPCEncoder(504, 252, dv=3, dc=6, seed=42)
    dec = BPDecoder(enc.H, max_iter=20)
    dev = MonteCarlo(ldpc_round_fn(dec, seed=103, info_bits=252), info_bits=252,
                     batch=65536).run([snr], 131072, 10 ** 12)[0]
    r = _compare(dev, _ref_point(name, "bp", snr), 252, "BP-20 (504,252) @ %g dB" % snr)
    assert r["fer_ref"] > 0.001


def test_awgn_llr_moments_and_tails(gpu):
    """pl_awgn_llr against the reference channel's distribution: for the all-zero
    codeword LLR = 2 (1 + sigma z) / sigma^2 (awgn.py:47, :75, :88), so mean
    2 / sigma^2 and variance 4 / sigma^2; z standard normal including both tails;
    the two Box-Muller outputs of a pair uncorrelated; and a two-sample KS test
    against np.random.normal (the reference's noise source)."""
    from scipy import stats
    from polarcode_and_ldpc_amd.channel import AWGNChannel
    snr = 1.0
    ch = AWGNChannel(snr)
    s2 = ch.noise_std ** 2
    B, n = 4096, 1024
    llr = ch.llr_batch_device(None, n, B, seed=77).double()
    M = B * n
    mean = llr.mean().item()
    var = llr.var().item()
    assert abs(mean / (2.0 / s2) - 1.0) < 5 * (math.sqrt(4.0 / s2 / M) / (2.0 / s2))
    assert abs(var / (4.0 / s2) - 1.0) < 5 * math.sqrt(2.0 / M)
    z = ((llr * s2 / 2.0 - 1.0) / ch.noise_std).flatten()
    for t in (1.0, 2.0, 3.0, 4.0):
        p = 2 * stats.norm.sf(t)
        for side in (z > t, z < -t):
            got = side.double().mean().item()
            assert abs(got - p / 2) < 5 * math.sqrt(p / 2 / M) + 1e-7, (t, got, p / 2)
    zz = z.view(B, n // 2, 2)
    corr = torch.corrcoef(torch.stack([zz[..., 0].flatten(), zz[..., 1].flatten()]))[0, 1].item()
    assert abs(corr) < 5 / math.sqrt(M / 2)
    zs = z[:: 16].cpu().numpy()
    rng = np.random.RandomState(5)
    ks = stats.ks_2samp(zs, rng.normal(0.0, 1.0, size=zs.size))
    assert ks.pvalue > 1e-3, ks
    assert stats.kstest(zs, "norm").pvalue > 1e-3
    # codeword signs: BPSK 0 -> +1, 1 -> -1 (awgn.py:47) on the same noise
    cw = torch.ones((B, n), dtype=torch.uint8, device="cuda")
    neg = ch.llr_batch_device(cw, n, B, seed=77)
    assert torch.allclose(neg - (llr - 4.0 / s2), torch.zeros_like(neg), atol=1e-9 * (4.0 / s2))


@pytest.mark.parametrize("snr,name", [(-2.0, "cascl32_m20"), (-1.5, "cascl32_m15")])
def test_cascl_l32_crc8_ber_fer_parity(gpu, snr, name):
    """CA-SCL L=32 + CRC-8 N=1024 K=512 (configs[3] itself) at the low end of its
    sweep.  Device: harness.montecarlo.polar_round_fn with crc_polynomial
    (Philox data bits + pl_crc_append, device encoder, AWGN, CASCLDecoder,
    errors over all K bits as the reference encoder's message_with_crc).
    Reference side: the reference's PolarEncoder(use_crc=True) frame loop,
    decoded by the oracle's CA-SCL restatement (the reference has no CA-SCL
    decoder: decoder.py:202-203,259); 16 384 frames per point, seeds fixed in
    make_ber_golden.py before any GPU run of this test."""
    from polarcode_and_ldpc_amd.harness.montecarlo import MonteCarlo, polar_round_fn
    from polarcode_and_ldpc_amd.polar import CASCLDecoder, construct_frozen_set
    N, K, L = 1024, 512, 32
    fr = construct_frozen_set(N, K, 2.0)
    dec = CASCLDecoder(N, K, L, frozen_bits=fr, crc_polynomial="CRC-8")
    dev = MonteCarlo(polar_round_fn(dec, seed=106, crc_polynomial="CRC-8"), info_bits=K,
                     batch=32768).run([snr], 65536, 10 ** 12)[0]
    r = _compare(dev, _ref_point(name, "cascl", snr), K, "CA-SCL L=32 CRC-8 N=1024 @ %g dB" % snr)
    assert r["fer_ref"] > 0.005
