"""GPU checks of the device channels, CRC append and the batched harness
(throughput_test.py / ber_simulation.py counterparts)."""
import json

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_crc_append_matches_host_crc_encode(gpu):
    from polarcode_and_ldpc_amd import _native
    from polarcode_and_ldpc_amd.polar.utils import CRC_POLYNOMIALS, crc_encode
    for name in ("CRC-8", "CRC-16", "CRC-24"):
        L = int(name.split("-")[1])
        msg = torch.empty((64, 100), dtype=torch.uint8, device="cuda")
        _native.random_bits(5, 0, msg)
        _native.crc_append(msg, 100 - L, L, CRC_POLYNOMIALS[name])
        m = msg.cpu().numpy().astype(int)
        for r in m[:16]:
            assert np.array_equal(crc_encode(r[:100 - L], name), r)


def test_device_bsc_and_rayleigh_statistics(gpu):
    from polarcode_and_ldpc_amd.channel import BSCChannel, RayleighFadingChannel
    B, n = 4096, 256
    flips = BSCChannel(0.1).transmit_batch_device(None, n, B, seed=3).double().mean().item()
    assert abs(flips - 0.1) < 0.003
    cw = torch.ones((B, n), dtype=torch.uint8, device="cuda")
    again = BSCChannel(0.1).transmit_batch_device(cw, n, B, seed=3)
    assert torch.equal(again, 1 - BSCChannel(0.1).transmit_batch_device(None, n, B, seed=3))
    ch = RayleighFadingChannel(2.0)
    llr = ch.llr_batch_device(None, n, B, seed=4)
    # E[LLR | s=+1] = 2 E[|h|^2] / sigma^2 = 2 / sigma^2 with E|h|^2 = 1
    assert abs(llr.mean().item() * ch.noise_std ** 2 / 2.0 - 1.0) < 0.01
    # frames are independent of the batch they are generated in
    part = ch.llr_batch_device(None, n, 8, seed=4, frame_offset=100)
    assert torch.equal(part, llr[100:108])


def test_throughput_harness_fields(gpu, tmp_path):
    from polarcode_and_ldpc_amd.harness.throughput import run_throughput_test
    r = run_throughput_test({"encoding": {"N": 256, "K": 128}},
                            {"encoding": {"n": 504, "k": 252}, "decoding": {"max_iterations": 20}},
                            tmp_path, num_iterations=512, snr_db=3.0)
    saved = json.load(open(tmp_path / "data" / "throughput_results.json"))
    for code in ("polar", "ldpc"):
        for key in ("encoding_time", "decoding_time", "end_to_end_time", "encoding_throughput",
                    "decoding_throughput", "end_to_end_throughput", "rate", "num_iterations"):
            assert key in saved[code] and saved[code][key] > 0
    assert r["ldpc"]["mean_iterations"] == 20.0  # the reference encoder's invalid codewords


def test_ber_harness_polar_and_ldpc(gpu, tmp_path):
    from polarcode_and_ldpc_amd.harness.ber import run_ber_simulation
    res = run_ber_simulation(np.array([-2.0, 6.0]), num_frames=8192, max_errors=50,
                             polar_config={"encoding": {"N": 256, "K": 128}},
                             ldpc_config={"encoding": {"n": 504, "k": 252}, "decoding": {"max_iterations": 20}},
                             output_dir=tmp_path, batch=4096)
    saved = json.load(open(tmp_path / "data" / "ber_simulation_results.json"))
    for code in ("polar", "ldpc"):
        ber, fer = saved[code]["self"]["ber"], saved[code]["self"]["fer"]
        assert len(ber) == 2 and ber[0] > ber[1] and fer[0] > 0.01 and fer[1] < 0.01
        pt = saved[code]["self"]["points"][0]
        assert pt["frame_errors"] >= 50 and pt["frames"] <= 8192  # max_errors stop, round granularity


def test_cascl_ber_beats_scl(gpu):
    """CA-SCL L=32 + CRC-8 (BASELINE config 4 shape) at -0.5 dB: FER below SCL's."""
    from polarcode_and_ldpc_amd.harness.ber import simulate_polar
    cfg = {"encoding": {"N": 1024, "K": 512}}
    _, f_scl, _ = simulate_polar([-0.5], 8192, 10 ** 9, cfg, list_size=32, crc_polynomial=None, batch=8192)
    _, f_ca, p = simulate_polar([-0.5], 8192, 10 ** 9, cfg, list_size=32, crc_polynomial="CRC-8", batch=8192)
    assert p[0].frames == 8192 and f_scl[0] > 0.0 and f_ca[0] < f_scl[0]


def test_ldpc_device_encoder_valid_codewords(gpu):
    """pl_gf2_encode: device codewords equal msg . G (mod 2) on the host, satisfy
    H, carry the message at info_positions, and decode back at high SNR."""
    from polarcode_and_ldpc_amd import _native
    from polarcode_and_ldpc_amd.channel import AWGNChannel
    from polarcode_and_ldpc_amd.ldpc import BPDecoder, LDPCEncoder
    enc = LDPCEncoder(504, 252, dv=3, dc=6, seed=42)
    B = 4096
    msg = torch.empty((B, 252), dtype=torch.uint8, device="cuda")
    _native.random_bits(7, 0, msg)
    cw = enc.encode_batch_device(msg)
    G, info = enc.valid_generator()
    m = msg.cpu().numpy().astype(np.int64)
    c = cw.cpu().numpy().astype(np.int64)
    assert np.array_equal(c, (m @ G.astype(np.int64)) % 2)
    assert not ((np.asarray(enc.H).astype(np.int64) @ c.T) % 2).any()
    assert np.array_equal(c[:, info], m)
    llr = AWGNChannel(5.0).llr_batch_device(cw, 504, B, seed=3)
    bits = BPDecoder(enc.H, 20).decode_batch(llr)  # device in, device out
    assert np.array_equal(bits.cpu().numpy()[:, info], m)


def test_ldpc_mc_random_codewords_match_zero_codeword(gpu):
    """BP is codeword-symmetric: the FER with random valid codewords (device
    encoder) agrees with the all-zero-codeword FER within Monte-Carlo error."""
    from polarcode_and_ldpc_amd.harness.montecarlo import MonteCarlo, ldpc_round_fn, wilson_interval
    from polarcode_and_ldpc_amd.ldpc import BPDecoder, LDPCEncoder
    enc = LDPCEncoder(504, 252, dv=3, dc=6, seed=42)
    dec = BPDecoder(enc.H, 20)
    res = {}
    for tag, e in (("zero", None), ("random", enc)):
        mc = MonteCarlo(ldpc_round_fn(dec, seed=11, info_bits=252, encoder=e), info_bits=252, batch=32768)
        p = mc.run([-1.0], 65536, 10 ** 9)[0]
        res[tag] = p
    fz, fr = res["zero"].fer, res["random"].fer
    assert 0.005 < fz < 0.9
    _, lo_z, hi_z = wilson_interval(res["zero"].frame_errors, res["zero"].frames, 0.999)
    _, lo_r, hi_r = wilson_interval(res["random"].frame_errors, res["random"].frames, 0.999)
    assert lo_z <= hi_r and lo_r <= hi_z, (fz, fr)


@pytest.mark.parametrize("width,ld,off", [(512, 512, 0), (512, 528, 16), (252, 252, 0), (504, 512, 0),
                                          (16, 16, 0), (1024, 1024, 0), (2048, 2048, 0), (8192, 8192, 0),
                                          (512, 512, 3), (7, 9, 1)])
def test_count_errors_vs_torch(gpu, width, ld, off):
    """pl_count_errors (16-byte chunk paths for aligned rows, byte path otherwise)
    against a torch count of low-bit mismatches; rows with 0, 1 and many errors."""
    from polarcode_and_ldpc_amd import _native
    B = 3001
    g = torch.Generator(device="cuda").manual_seed(width * 7 + off)
    base_r = torch.randint(0, 256, (B * ld + off + 64,), dtype=torch.uint8, device="cuda", generator=g)
    base_d = base_r.clone()
    flip = torch.rand((B, width), device="cuda", generator=g) < torch.rand((B, 1), device="cuda", generator=g) ** 4
    flip[::5] = False
    ref = base_r[off:off + B * ld].view(B, ld)[:, :width]
    dec = base_d[off:off + B * ld].view(B, ld)[:, :width]
    dec ^= flip.to(torch.uint8) | (torch.randint(0, 128, (B, width), dtype=torch.uint8, device="cuda",
                                                 generator=g) << 1)
    counts = torch.zeros(3, dtype=torch.int64, device="cuda")
    _native.count_errors(ref, dec, width, counts)
    e = ((ref & 1) != (dec & 1)).sum(dim=1)
    want = [int(e.sum()), int((e > 0).sum()), B]
    assert counts.tolist() == want


def test_awgn_vector_and_scalar_paths_agree(gpu):
    """the AWGN kernel's vector path (even n and ld, 16-byte aligned
    rows) and its scalar path (any other layout) read a codeword byte the same
    way (bit 0) and draw the same Philox stream: an odd-pitch, offset view gets
    exactly the LLRs of a contiguous one, also for bytes other than 0 / 1."""
    import torch
    from polarcode_and_ldpc_amd.channel import AWGNChannel
    B, n = 257, 64
    g = torch.Generator().manual_seed(3)
    cw = torch.randint(0, 256, (B, n), generator=g, dtype=torch.uint8).cuda()
    ch = AWGNChannel(1.5)
    a = ch.llr_batch_device(cw, n, B, seed=11, frame_offset=5)              # vector path
    big = torch.zeros((B, n + 1), dtype=torch.float64, device="cuda")
    b = ch.llr_batch_device(cw, n, B, seed=11, frame_offset=5, out=big[:, 1:])  # ld odd, unaligned: scalar
    c = ch.llr_batch_device((cw & 1).contiguous(), n, B, seed=11, frame_offset=5)
    torch.cuda.synchronize()
    assert torch.equal(a, b) and torch.equal(a, c)
