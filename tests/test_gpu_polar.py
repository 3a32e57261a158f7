"""Parity of the HIP polar decoders (through the C-ABI via the drop-in classes)
against (a) the reference's own outputs (golden fixtures, tests/golden/) and
(b) the C oracle on fresh seeded inputs.  Bar: bit-exact decoded bits."""
import ctypes

import numpy as np
import pytest
import torch

from conftest import golden

pytestmark = pytest.mark.gpu


def _P():
    import polarcode_and_ldpc_amd.polar as P
    return P


def _grid_waves(plan, fpw):
    """Resident wavefronts of a list plan's persistent grid: the smallest batch
    (in wavefronts) whose workspace is already the capped one."""
    cap = plan.workspace_bytes(1 << 22)
    hi = 1
    while plan.workspace_bytes(hi * fpw) < cap:
        hi *= 2
    lo = max(1, hi // 2)
    while lo < hi:
        mid = (lo + hi) // 2
        if plan.workspace_bytes(mid * fpw) < cap:
            lo = mid + 1
        else:
            hi = mid
    return lo


def _mismatch(a, b):
    a, b = np.asarray(a), np.asarray(b)
    assert a.shape == b.shape, (a.shape, b.shape)
    return int((a != b).any(axis=1).sum())


def test_native_library_loaded(gpu):
    from polarcode_and_ldpc_amd import _native
    assert _native.lib is not None and _native.LIB_PATH.endswith("libpolarldpc.so")


def test_sc_p1_throughput_frames(gpu):
    """BASELINE config 1: N=256 K=128 SC, the 100 frames of throughput_test.py."""
    d = golden("polar_p1.npz")
    dec = _P().SCDecoder(256, 128, frozen_bits=d["frozen"])
    assert _mismatch(dec.decode_batch(d["llr"]), d["sc"]) == 0
    # single-frame API == reference .decode
    for b in range(5):
        out = dec.decode(d["llr"][b])
        assert out.dtype == np.int64 and out.shape == (128,)
        assert np.array_equal(out, d["sc"][b])


@pytest.mark.parametrize("L", [1, 2, 4, 8])
def test_scl_p1_frames(gpu, L):
    d = golden("polar_p1.npz")
    dec = _P().SCLDecoder(256, 128, list_size=L, frozen_bits=d["frozen"])
    assert _mismatch(dec.decode_batch(d["llr"][:32]), d["scl_L%d" % L]) == 0


@pytest.mark.parametrize("tag", ["default", "bhatta"])
def test_sc_1024(gpu, tag):
    d = golden("polar_sc_1024.npz")
    dec = _P().SCDecoder(1024, 512, frozen_bits=d[tag + "_frozen"])
    assert _mismatch(dec.decode_batch(d[tag + "_llr"]), d[tag + "_sc"]) == 0


def test_scl_1024_l8(gpu):
    d = golden("polar_scl_1024_l8.npz")
    dec = _P().SCLDecoder(1024, 512, list_size=8, frozen_bits=d["frozen"])
    assert _mismatch(dec.decode_batch(d["llr"]), d["scl"]) == 0
    dec = _P().SCLDecoder(1024, 512, list_size=8, frozen_bits=d["default_frozen"])
    assert _mismatch(dec.decode_batch(d["default_llr"]), d["default_scl"]) == 0


def test_scl_1024_l32(gpu):
    d = golden("polar_scl_1024_l32.npz")
    dec = _P().SCLDecoder(1024, 512, list_size=32, frozen_bits=d["frozen"])
    assert _mismatch(dec.decode_batch(d["llr"]), d["scl"]) == 0


def test_scl_4096_l8(gpu):
    d = golden("polar_scl_4096_l8.npz")
    dec = _P().SCLDecoder(4096, 2048, list_size=8, frozen_bits=d["frozen"])
    assert _mismatch(dec.decode_batch(d["llr"]), d["scl"]) == 0


def test_small_cases_all_list_sizes(gpu):
    """Small N, K extremes (1, N-1), odd list sizes, LLRs with exact +-0,
    denormal-scale and large values."""
    d = golden("polar_small.npz")
    P = _P()
    bad = []
    for c in range(int(d["ncases"])):
        p = "c%d_" % c
        N, K, fr, llr = int(d[p + "N"]), int(d[p + "K"]), d[p + "frozen"], d[p + "llr"]
        if _mismatch(P.SCDecoder(N, K, frozen_bits=fr).decode_batch(llr), d[p + "sc"]):
            bad.append((c, "sc"))
        for L in (1, 2, 3, 4, 5, 6, 8, 16):
            if _mismatch(P.SCLDecoder(N, K, list_size=L, frozen_bits=fr).decode_batch(llr), d[p + "scl_L%d" % L]):
                bad.append((c, L))
    assert not bad, bad


def test_kat_n16(gpu):
    """docs/SCL_DECODER_README.md:115-128 known-answer test."""
    d = golden("polar_kat16.npz")
    P = _P()
    for L in (1, 2, 4, 8):
        out = P.SCLDecoder(16, 8, list_size=L, frozen_bits=d["frozen"]).decode(d["llr"])
        assert np.array_equal(out, d["scl_L%d" % L])
        assert np.array_equal(out, d["msg"])  # [0 1 0 0 0 1 0 0]


@pytest.mark.parametrize("N,L", [(64, 1), (64, 32), (256, 2), (256, 16), (512, 4), (1024, 1), (1024, 8),
                                 (2048, 8), (128, 32)])
def test_vs_oracle_random(gpu, oracle, N, L):
    """Fresh seeded AWGN frames (random messages, bit-reversed Bhattacharyya
    set) at low/medium SNR: HIP vs the C oracle, bit-exact."""
    P = _P()
    rng = np.random.RandomState(N * 100 + L)
    K = N // 2
    fr = P.construct_frozen_set(N, K, 1.0)
    enc = P.PolarEncoder(N, K, frozen_bits=fr)
    B = 48 if N * L <= 8192 else 16
    msg = rng.randint(0, 2, (B, K))
    cw = enc.encode_batch(msg)
    snr = rng.uniform(-1.0, 3.0, size=(B, 1))
    sigma = np.sqrt(1.0 / (2.0 * 10 ** (snr / 10.0)))
    llr = 2.0 * ((1.0 - 2.0 * cw) + sigma * rng.randn(B, N)) / sigma ** 2
    want_sc = oracle.sc_decode(N, fr, llr, threads=8)
    assert _mismatch(P.SCDecoder(N, K, frozen_bits=fr).decode_batch(llr), want_sc) == 0
    want = oracle.scl_decode(N, L, fr, llr, threads=8)
    got = P.SCLDecoder(N, K, list_size=L, frozen_bits=fr).decode_batch(llr)
    assert _mismatch(got, want) == 0


def test_device_batch_path_and_fused_depths(gpu, oracle):
    """Device-tensor API, and every fused-top depth F=1..4 gives identical bits."""
    from polarcode_and_ldpc_amd import _native
    P = _P()
    d = golden("polar_scl_1024_l8.npz")
    llr = torch.from_numpy(d["llr"]).cuda()
    mask = np.zeros(1024, np.uint8)
    mask[d["frozen"]] = 1
    for F in (1, 2, 3, 4):
        plan = _native.polar_plan(1024, 512, mask, 8, flags=F)
        assert plan.info.fused_top == F
        out = torch.empty((llr.shape[0], 512), dtype=torch.uint8, device="cuda")
        plan.decode(llr, out)
        assert _mismatch(out.cpu().numpy(), d["scl"]) == 0, F
        plan = _native.polar_plan(1024, 512, mask, 0, flags=F)
        plan.decode(llr, out)
        assert _mismatch(out.cpu().numpy(), oracle.sc_decode(1024, d["frozen"], d["llr"])) == 0, F
    dec = P.SCLDecoder(1024, 512, list_size=8, frozen_bits=d["frozen"])
    out = dec.decode_batch(llr)
    assert out.is_cuda and out.dtype == torch.uint8
    assert _mismatch(out.cpu().numpy(), d["scl"]) == 0


def test_full_batch_noiseless_roundtrip(gpu):
    """BASELINE config 2 size (B=65536, N=1024, L=8): encode -> noiseless BPSK
    LLR -> decode must return the message for every frame (size-independent
    property), and frames are independent of batch position."""
    from polarcode_and_ldpc_amd import _native
    P = _P()
    N, K, B = 1024, 512, 65536
    fr = P.construct_frozen_set(N, K, 2.0)
    dec = P.SCLDecoder(N, K, list_size=8, frozen_bits=fr)
    msg = torch.empty((B, K), dtype=torch.uint8, device="cuda")
    _native.random_bits(7, 0, msg)
    cw = torch.empty((B, N), dtype=torch.uint8, device="cuda")
    _native.polar_encode(dec.plan, msg, cw)
    llr = (1.0 - 2.0 * cw.to(torch.float64)) * 8.0
    out = dec.decode_batch(llr)
    assert torch.equal(out, msg)
    # host encoder agrees with the device encoder
    enc = P.PolarEncoder(N, K, frozen_bits=fr)
    assert np.array_equal(enc.encode_batch(msg[:64].cpu().numpy()), cw[:64].cpu().numpy())


def test_reference_assertions(gpu):
    P = _P()
    with pytest.raises(AssertionError):
        P.SCDecoder(100, 50)
    with pytest.raises(AssertionError):
        P.SCDecoder(64, 64)
    with pytest.raises(AssertionError):
        P.SCLDecoder(64, 32, list_size=0)
    with pytest.raises(AssertionError):
        P.SCDecoder(64, 32).decode(np.zeros(63))


@pytest.mark.parametrize("snr", [0.0, 1.5, 3.0])
def test_tree_kernel_matches_lane_kernel(gpu, oracle, snr):
    """The v4 tree kernel (default for N=1024 L=8) against the lane kernel
    (flags=0x20) on 4096 noisy frames, and a sample against the oracle."""
    from polarcode_and_ldpc_amd import _native
    from polarcode_and_ldpc_amd.channel import AWGNChannel
    P = _P()
    N, K, L, B = 1024, 512, 8, 4096
    fr = P.construct_frozen_set(N, K, 2.0)
    mask = np.zeros(N, np.uint8)
    mask[fr] = 1
    tree = _native.polar_plan(N, K, mask, L)
    lane = _native.polar_plan(N, K, mask, L, flags=0x20)
    assert tree.info.reserved == 4 and lane.info.reserved == 3
    msg = torch.empty((B, K), dtype=torch.uint8, device="cuda")
    _native.random_bits(11, 0, msg)
    cw = torch.empty((B, N), dtype=torch.uint8, device="cuda")
    _native.polar_encode(tree, msg, cw)
    llr = AWGNChannel(snr).llr_batch_device(cw, N, B, seed=5)
    a = torch.empty((B, K), dtype=torch.uint8, device="cuda")
    b = torch.empty_like(a)
    tree.decode(llr, a)
    lane.decode(llr, b)
    assert torch.equal(a, b)
    ref = oracle.scl_decode(N, L, fr, llr[:48].cpu().numpy())
    assert _mismatch(a[:48].cpu().numpy(), ref) == 0


def test_tree_kernel_ragged_batch(gpu):
    """Batch sizes that leave partial frame groups and fewer waves than the
    persistent grid: every frame matches a full-batch decode of the same rows."""
    from polarcode_and_ldpc_amd import _native
    P = _P()
    d = golden("polar_scl_1024_l8.npz")
    mask = np.zeros(1024, np.uint8)
    mask[d["frozen"]] = 1
    plan = _native.polar_plan(1024, 512, mask, 8)
    llr = torch.from_numpy(d["llr"]).cuda()
    for B in sorted({1, 3, 7, 9, llr.shape[0] - 1}):
        out = torch.empty((B, 512), dtype=torch.uint8, device="cuda")
        plan.decode(llr[:B], out)
        assert _mismatch(out.cpu().numpy(), d["scl"][:B]) == 0, B


@pytest.mark.parametrize("N,L,crc,flags", [(1024, 32, "CRC-8", 0), (1024, 8, "CRC-16", 0), (1024, 8, "CRC-24", 0x20),
                                           (256, 4, "CRC-8", 0), (4096, 8, "CRC-16", 0), (256, 64, "CRC-8", 0),
                                           (256, 128, "CRC-8", 0), (1024, 256, "CRC-16", 0)])
def test_cascl_vs_oracle(gpu, oracle, N, L, crc, flags):
    """CRC-aided SCL (build-defined extension; the reference never applies its
    CRC, so parity is against the oracle's restatement of the same rule).  Frames
    near the waterfall so the CRC changes the pick; every frame bit-exact."""
    from polarcode_and_ldpc_amd import _native
    from polarcode_and_ldpc_amd.polar.utils import CRC_POLYNOMIALS, crc_check, crc_encode
    P = _P()
    K = N // 2
    fr = P.construct_frozen_set(N, K, 2.0)
    clen = int(crc.split("-")[1])
    rng = np.random.RandomState(N + L + clen)
    B = 48 if N < 4096 else 12
    msg = np.stack([crc_encode(rng.randint(0, 2, K - clen), crc) for _ in range(B)])
    cw = P.PolarEncoder(N, K, frozen_bits=fr).encode_batch(msg)
    snr = rng.uniform(0.0, 1.5, size=(B, 1))
    sigma = np.sqrt(1.0 / (2.0 * 10 ** (snr / 10.0)))
    llr = 2.0 * ((1.0 - 2.0 * cw) + sigma * rng.randn(B, N)) / sigma ** 2
    want = oracle.cascl_decode(N, L, fr, llr, crc, threads=8)
    mask = np.zeros(N, np.uint8)
    mask[fr] = 1
    plan = _native.polar_plan(N, K, mask, L, flags=flags)
    plan.set_crc(clen, CRC_POLYNOMIALS[crc])
    out = torch.empty((B, K), dtype=torch.uint8, device="cuda")
    plan.decode(torch.from_numpy(llr).cuda(), out)
    got = out.cpu().numpy().astype(np.int64)
    assert _mismatch(got, want) == 0
    # the CRC decides at least as many frames as plain SCL, and clearing it restores SCL
    scl = oracle.scl_decode(N, L, fr, llr, threads=8)
    assert sum(crc_check(r, crc) for r in got) >= sum(crc_check(r, crc) for r in scl)
    plan.set_crc(0, 0)
    plan.decode(torch.from_numpy(llr).cuda(), out)
    assert _mismatch(out.cpu().numpy(), scl) == 0


def test_cascl_decoder_class(gpu):
    """CASCLDecoder drop-in: noiseless CRC'd frames round-trip; SC plans refuse CRC."""
    from polarcode_and_ldpc_amd import _native
    P = _P()
    N, K = 1024, 512
    fr = P.construct_frozen_set(N, K, 2.0)
    enc = P.PolarEncoder(N, K, frozen_bits=fr, use_crc=True, crc_polynomial="CRC-16")
    dec = P.CASCLDecoder(N, K, list_size=8, frozen_bits=fr, crc_polynomial="CRC-16")
    rng = np.random.RandomState(3)
    data = rng.randint(0, 2, (16, K - 16))
    cw = np.stack([enc.encode(d) for d in data])
    out = dec.decode_batch(8.0 * (1.0 - 2.0 * cw))
    assert np.array_equal(out[:, :K - 16], data)
    assert np.array_equal(dec.decode(8.0 * (1.0 - 2.0 * cw[0]))[:K - 16], data[0])
    mask = np.zeros(N, np.uint8)
    mask[fr] = 1
    with pytest.raises(AssertionError):
        _native.polar_plan(N, K, mask, 0).set_crc(8, 0x1D)


@pytest.mark.parametrize("flags", [0, 0x20])
def test_erasures_and_saturation_golden(gpu, flags):
    """Erasures (LLR = 0), saturated LLRs, +-inf, signed zeros and denormals
    against the reference's own outputs (golden polar_erasures.npz), SC and
    SCL, on the tree (flags 0, where an instance exists) and lane (0x20)
    kernels.  BEC frames with +-inf: SC only (see make_golden)."""
    from polarcode_and_ldpc_amd import _native
    d = golden("polar_erasures.npz")
    for N in (256, 1024):
        fr, L = d["N%d_frozen" % N], int(d["N%d_L" % N])
        llr = torch.from_numpy(d["N%d_llr" % N]).cuda()
        mask = np.zeros(N, np.uint8)
        mask[fr] = 1
        for lsz, key in ((0, "sc"), (L, "scl")):
            plan = _native.polar_plan(N, N // 2, mask, lsz, flags=flags)
            out = torch.empty((llr.shape[0], N // 2), dtype=torch.uint8, device="cuda")
            plan.decode(llr, out)
            assert _mismatch(out.cpu().numpy(), d["N%d_%s" % (N, key)]) == 0, (N, key, plan.info.reserved)
        plan = _native.polar_plan(N, N // 2, mask, 0, flags=flags)  # +-inf BEC frames: SC only
        inf = torch.from_numpy(d["N%d_inf_llr" % N]).cuda()
        out = torch.empty((inf.shape[0], N // 2), dtype=torch.uint8, device="cuda")
        plan.decode(inf, out)
        assert _mismatch(out.cpu().numpy(), d["N%d_inf_sc" % N]) == 0, (N, "inf_sc", plan.info.reserved)


@pytest.mark.parametrize("L", [4, 8, 16, 32])
def test_large_list_ties_vs_oracle(gpu, oracle, L):
    """Erasure-heavy frames make path metrics tie (LLR = 0 gives m0 = m1), which
    sends the large-list kernels' strict-comparison ranking to its stable
    tie-break fallback: every frame must still match the oracle."""
    from polarcode_and_ldpc_amd import _native
    d = golden("polar_erasures.npz")
    fr, llr = d["N1024_frozen"], d["N1024_llr"]
    mask = np.zeros(1024, np.uint8)
    mask[fr] = 1
    want = oracle.scl_decode(1024, L, fr, llr, threads=8)
    plan = _native.polar_plan(1024, 512, mask, L)
    assert plan.info.reserved == 4
    out = torch.empty((llr.shape[0], 512), dtype=torch.uint8, device="cuda")
    plan.decode(torch.from_numpy(llr).cuda(), out)
    assert _mismatch(out.cpu().numpy(), want) == 0


@pytest.mark.parametrize("N,L", [(1024, 8), (1024, 16), (1024, 32), (4096, 8)])
def test_near_tie_metrics_vs_oracle(gpu, oracle, N, L):
    """Channel LLRs of (nearly) one magnitude, 5 +- 1e-7: competing path metrics
    differ far below fp32 resolution, so the tree kernel's fp32 strict ranks
    collide constantly and its exact fp64 fallback decides -- bits must match
    the oracle."""
    from polarcode_and_ldpc_amd import _native
    P = _P()
    K = N // 2
    fr = P.construct_frozen_set(N, K, 2.0)
    rng = np.random.RandomState(N + L)
    B = 16
    cw = P.PolarEncoder(N, K, frozen_bits=fr).encode_batch(rng.randint(0, 2, (B, K)))
    sign = (1.0 - 2.0 * cw) * np.where(rng.rand(B, N) < 0.12, -1.0, 1.0)  # ~12 % flipped
    llr = sign * (5.0 + 1e-7 * rng.rand(B, N))
    mask = np.zeros(N, np.uint8)
    mask[fr] = 1
    plan = _native.polar_plan(N, K, mask, L)
    assert plan.info.reserved == 4
    out = torch.empty((B, K), dtype=torch.uint8, device="cuda")
    plan.decode(torch.from_numpy(llr).cuda(), out)
    assert _mismatch(out.cpu().numpy(), oracle.scl_decode(N, L, fr, llr, threads=8)) == 0


def test_empty_batch(gpu):
    """A zero-frame batch decodes to an empty [0, K] result (SC, SCL tree and
    lane kernels) without launching."""
    P = _P()
    for dec in (P.SCDecoder(1024, 512), P.SCLDecoder(1024, 512, list_size=8), P.SCLDecoder(512, 256, list_size=4)):
        got = dec.decode_batch(np.zeros((0, dec.N)))
        assert got.shape == (0, dec.K)
        got = dec.decode_batch(torch.zeros((0, dec.N), dtype=torch.float64, device="cuda"))
        assert tuple(got.shape) == (0, dec.K)


@pytest.mark.parametrize("N,L", [(1024, 8), (1024, 32), (2048, 8), (4096, 8), (256, 16)])
def test_list_growth_at_multiword_walks(gpu, oracle, N, L):
    """The list grows (1 -> 2 -> 4 -> ...) at decode steps with many trailing
    ones, where the partial-sum walk goes through the multi-word workspace
    depths: lanes that stop shadowing slot 0 at such a step must write their
    own planes.  Frozen set: all-frozen prefix, then info bits at steps
    2^k - 1 first; noisy frames; tree kernel vs the C oracle, bit-exact."""
    P = _P()
    n = N.bit_length() - 1
    K = N // 2
    br = np.array([int(format(i, "0%db" % n)[::-1], 2) for i in range(N)])  # decode step -> u index
    first = [s for s in (N // 16 - 1, N // 8 - 1, N // 4 - 1, 3 * N // 8 - 1, N // 2 - 1) if s > 0]
    rest = [s for s in range(N - 1, -1, -1) if s not in first][:K - len(first)]
    info_steps = sorted(set(first) | set(rest))
    assert len(info_steps) == K
    fr = np.setdiff1d(np.arange(N), br[info_steps])
    rng = np.random.RandomState(N + L)
    B = 16
    snr = rng.uniform(0.0, 2.0, size=(B, 1))
    sigma = np.sqrt(1.0 / (2.0 * 10 ** (snr / 10.0)))
    llr = 2.0 * (1.0 + sigma * rng.randn(B, N)) / sigma ** 2
    want = oracle.scl_decode(N, L, fr, llr, threads=8)
    got = P.SCLDecoder(N, K, list_size=L, frozen_bits=fr).decode_batch(llr)
    assert _mismatch(got, want) == 0


@pytest.mark.parametrize("L", [3, 5, 6, 7, 12, 20])
def test_tree_list_sizes_below_capacity(gpu, oracle, L):
    """List sizes that are not a power of two run on the tree kernel of the next
    capacity (8, 16, 32): the extra lanes never become paths (with shadow lanes
    they follow slot 0 for the whole frame).  Noisy N=1024 frames vs the
    oracle, bit-exact."""
    from polarcode_and_ldpc_amd import _native
    P = _P()
    N, K = 1024, 512
    fr = P.construct_frozen_set(N, K, 1.5)
    mask = np.zeros(N, np.uint8)
    mask[fr] = 1
    rng = np.random.RandomState(100 + L)
    B = 24
    snr = rng.uniform(0.0, 2.5, size=(B, 1))
    sigma = np.sqrt(1.0 / (2.0 * 10 ** (snr / 10.0)))
    msg = rng.randint(0, 2, (B, K))
    cw = P.PolarEncoder(N, K, frozen_bits=fr).encode_batch(msg)
    llr = 2.0 * ((1.0 - 2.0 * cw) + sigma * rng.randn(B, N)) / sigma ** 2
    plan = _native.polar_plan(N, K, mask, L)
    assert plan.info.reserved == 4  # tree kernel
    out = torch.empty((B, K), dtype=torch.uint8, device="cuda")
    plan.decode(torch.from_numpy(llr).cuda(), out)
    assert _mismatch(out.cpu().numpy(), oracle.scl_decode(N, L, fr, llr, threads=8)) == 0


@pytest.mark.parametrize("pad,off", [(0, 0), (1, 0), (2, 0), (6, 1)])
def test_strided_and_unaligned_rows(gpu, pad, off):
    """Channel rows with a leading dimension N + pad and a base offset of `off`
    doubles: the tree kernel reads depth-0 pairs in place only for 16-byte
    aligned rows (even ld, aligned base) and stages them otherwise; both give
    the contiguous decode's bits."""
    from polarcode_and_ldpc_amd import _native
    d = golden("polar_scl_1024_l8.npz")
    mask = np.zeros(1024, np.uint8)
    mask[d["frozen"]] = 1
    plan = _native.polar_plan(1024, 512, mask, 8)
    llr = torch.from_numpy(d["llr"]).cuda()
    B = llr.shape[0]
    buf = torch.full((B * (1024 + pad) + off + 8,), float("nan"), dtype=torch.float64, device="cuda")
    view = buf[off:off + B * (1024 + pad)].view(B, 1024 + pad)[:, :1024]
    view.copy_(llr)
    out = torch.empty((B, 512), dtype=torch.uint8, device="cuda")
    plan.decode(view, out)
    assert _mismatch(out.cpu().numpy(), d["scl"]) == 0


@pytest.mark.parametrize("N,L", [(256, 2), (256, 4), (256, 8), (256, 16), (256, 32), (512, 8), (512, 16),
                                 (1024, 2)])
def test_small_code_tree_instances_vs_oracle(gpu, oracle, N, L):
    """Tree-kernel instances for N = 256 / 512 and L = 2 (the reference's
    sc_vs_scl / benchmark_scl sizes): noisy frames vs the oracle, bit-exact."""
    from polarcode_and_ldpc_amd import _native
    P = _P()
    K = N // 2
    fr = P.construct_frozen_set(N, K, 1.0)
    mask = np.zeros(N, np.uint8)
    mask[fr] = 1
    rng = np.random.RandomState(7 * N + L)
    B = 40
    snr = rng.uniform(-0.5, 3.0, size=(B, 1))
    sigma = np.sqrt(1.0 / (2.0 * 10 ** (snr / 10.0)))
    msg = rng.randint(0, 2, (B, K))
    cw = P.PolarEncoder(N, K, frozen_bits=fr).encode_batch(msg)
    llr = 2.0 * ((1.0 - 2.0 * cw) + sigma * rng.randn(B, N)) / sigma ** 2
    llr[0, ::9] = 0.0  # erasures: metric ties
    plan = _native.polar_plan(N, K, mask, L)
    assert plan.info.reserved == 4  # tree kernel
    out = torch.empty((B, K), dtype=torch.uint8, device="cuda")
    plan.decode(torch.from_numpy(llr).cuda(), out)
    assert _mismatch(out.cpu().numpy(), oracle.scl_decode(N, L, fr, llr, threads=8)) == 0


@pytest.mark.parametrize("L", [0, 8, 32])
def test_n128_tree_instances_vs_oracle(gpu, oracle, L):
    """N = 128 (the reference's throughput_test default size) on the tree
    kernel: SC and SCL L = 8 / 32 against the oracle, bit-exact."""
    from polarcode_and_ldpc_amd import _native
    P = _P()
    N, K = 128, 64
    fr = P.construct_frozen_set(N, K, 1.0)
    mask = np.zeros(N, np.uint8)
    mask[fr] = 1
    rng = np.random.RandomState(128 + L)
    B = 48
    snr = rng.uniform(-1.0, 3.0, size=(B, 1))
    sigma = np.sqrt(1.0 / (2.0 * 10 ** (snr / 10.0)))
    msg = rng.randint(0, 2, (B, K))
    cw = P.PolarEncoder(N, K, frozen_bits=fr).encode_batch(msg)
    llr = 2.0 * ((1.0 - 2.0 * cw) + sigma * rng.randn(B, N)) / sigma ** 2
    llr[1, ::5] = 0.0
    plan = _native.polar_plan(N, K, mask, L)
    assert plan.info.reserved == 4  # tree kernel
    out = torch.empty((B, K), dtype=torch.uint8, device="cuda")
    plan.decode(torch.from_numpy(llr).cuda(), out)
    want = oracle.sc_decode(N, fr, llr, threads=8) if L == 0 else oracle.scl_decode(N, L, fr, llr, threads=8)
    assert _mismatch(out.cpu().numpy(), want) == 0


# ---------------------------------------------------------------- round 2
LOW_SNR_FIXTURES = [("polar_scl_1024_l32_m20.npz", 1024, 32), ("polar_scl_1024_l32_m10.npz", 1024, 32),
                    ("polar_scl_1024_l32_m0.npz", 1024, 32), ("polar_scl_4096_l8_wf15.npz", 4096, 8),
                    ("polar_scl_4096_l8_wf10.npz", 4096, 8)]


@pytest.mark.parametrize("name,N,L", LOW_SNR_FIXTURES)
def test_low_snr_large_list_golden(gpu, name, N, L):
    """The reference's own outputs where path metrics sit closest: SCL L=32 at
    -2 / -1 / 0 dB (64 frames each; BASELINE config 4 sweeps from -2 dB) and
    N=4096 L=8 in its waterfall (-1.5 / -1.0 dB).  The lean fp64 metric differs
    from NumPy's in the last ulp at most; decisions must not."""
    d = golden(name)
    dec = _P().SCLDecoder(N, N // 2, list_size=L, frozen_bits=d["frozen"])
    assert _mismatch(dec.decode_batch(d["llr"]), d["scl"]) == 0


@pytest.mark.parametrize("snr", [-1.5, -1.0])
def test_full_batch_noisy_vs_oracle(gpu, oracle, snr):
    """BASELINE config 2 at its full batch (B = 65 536, N = 1024, L = 8) on noisy
    frames: 4 096 frames spread over the whole batch (every 16th, so every
    resident wave and every frame slot of a wave is sampled) against the C
    oracle, bit-exact."""
    from polarcode_and_ldpc_amd import _native
    from polarcode_and_ldpc_amd.channel import AWGNChannel
    P = _P()
    N, K, L, B = 1024, 512, 8, 65536
    fr = P.construct_frozen_set(N, K, 2.0)
    dec = P.SCLDecoder(N, K, list_size=L, frozen_bits=fr)
    msg = torch.empty((B, K), dtype=torch.uint8, device="cuda")
    _native.random_bits(21, 0, msg)
    cw = torch.empty((B, N), dtype=torch.uint8, device="cuda")
    _native.polar_encode(dec.plan, msg, cw)
    llr = AWGNChannel(snr).llr_batch_device(cw, N, B, seed=22)
    out = dec.decode_batch(llr)
    idx = torch.arange(0, B, 16, device="cuda")
    want = oracle.scl_decode(N, L, fr, llr[idx].cpu().numpy(), threads=16)
    assert _mismatch(out[idx].cpu().numpy(), want) == 0
    assert 0 < (out != msg).any(dim=1).sum().item() < B  # a noisy regime: some frames in error


@pytest.mark.parametrize("L", [8, 32])
def test_later_grid_passes_vs_oracle(gpu, oracle, L):
    """The persistent grid decodes a batch in passes (grid = CUs x waves per CU
    wavefronts, 64 / L frames each); every wavefront's later passes run on the
    workspace and LDS its earlier frames left behind.  Frames from the last pass
    of a noisy multi-pass batch (-2 dB) equal the oracle's, bit for bit."""
    import torch
    from polarcode_and_ldpc_amd import _native
    from polarcode_and_ldpc_amd.channel import AWGNChannel
    P = _P()
    N, K = 1024, 512
    fr = P.construct_frozen_set(N, K, 2.0)
    dec = P.SCLDecoder(N, K, L, frozen_bits=fr)
    per_pass = _grid_waves(dec.plan, 64 // L) * (64 // L)
    B = 2 * per_pass + 96  # a ragged third pass
    msg = torch.empty((B, K), dtype=torch.uint8, device="cuda")
    _native.random_bits(91, 0, msg)
    cw = torch.empty((B, N), dtype=torch.uint8, device="cuda")
    _native.polar_encode(dec.plan, msg, cw)
    llr = AWGNChannel(-2.0).llr_batch_device(cw, N, B, seed=92)
    out = torch.empty((B, K), dtype=torch.uint8, device="cuda")
    dec.plan.decode(llr, out)
    torch.cuda.synchronize()
    S = 256 if L == 32 else 1024
    idx = torch.cat([torch.arange(per_pass, per_pass + S // 2), torch.arange(B - S // 2, B)]).cuda()
    want = oracle.scl_decode(N, L, fr, llr[idx].cpu().numpy(), threads=16)
    assert _mismatch(out[idx].cpu().numpy(), want) == 0
    assert 0 < (out != msg).any(dim=1).sum().item() < B


@pytest.mark.parametrize("N,L,snr", [(4096, 8, 1.0), (2048, 8, 1.0), (1024, 8, 0.0), (1024, 32, -1.0), (1024, 16, 0.0),
                                       (1024, 4, 1.0), (512, 8, 1.0), (512, 16, 0.0)])
def test_small_batch_instances(gpu, oracle, monkeypatch, N, L, snr):
    """Batches that fit the device at 8 wavefronts per CU decode on the
    small-batch tree instance (one more LDS depth, 2-wave register budget,
    polar_tree.hip tree_table_small).  At its largest batch, one frame above it
    (the product instance) and a ragged small batch, the bits equal those of a
    plan without it (PL_TREE_SMALL=0), and a sample of frames equals the oracle."""
    import torch
    from polarcode_and_ldpc_amd import _native
    from polarcode_and_ldpc_amd.channel import AWGNChannel
    P = _P()
    K = N // 2
    fr = P.construct_frozen_set(N, K, 2.0)
    dec = P.SCLDecoder(N, K, L, frozen_bits=fr)
    S = dec.plan.small_batch_frames()
    assert S > 0 and S % (64 // L) == 0
    monkeypatch.setenv("PL_TREE_SMALL", "0")
    ref = P.SCLDecoder(N, K, L, frozen_bits=fr)
    assert ref.plan.small_batch_frames() == 0
    B = S + 1
    msg = torch.empty((B, K), dtype=torch.uint8, device="cuda")
    _native.random_bits(93, 0, msg)
    cw = torch.empty((B, N), dtype=torch.uint8, device="cuda")
    _native.polar_encode(dec.plan, msg, cw)
    llr = AWGNChannel(snr).llr_batch_device(cw, N, B, seed=94)
    for b in (S, B, 333):
        a = torch.empty((b, K), dtype=torch.uint8, device="cuda")
        r = torch.empty((b, K), dtype=torch.uint8, device="cuda")
        dec.plan.decode(llr[:b], a)
        ref.plan.decode(llr[:b], r)
        torch.cuda.synchronize()
        assert torch.equal(a, r), b
    idx = torch.cat([torch.arange(0, 16), torch.arange(S - 16, S)]).cuda()
    a = torch.empty((S, K), dtype=torch.uint8, device="cuda")
    dec.plan.decode(llr[:S], a)
    torch.cuda.synchronize()
    want = oracle.scl_decode(N, L, fr, llr[idx].cpu().numpy(), threads=16)
    assert _mismatch(a[idx].cpu().numpy(), want) == 0


@pytest.mark.parametrize("N,L", [(1024, 8), (1024, 32), (4096, 8), (512, 4), (256, 0)])
def test_one_plan_two_streams(gpu, N, L):
    """Plans are shared across streams (SURVEY §8 b ownership row): two batches
    decoded concurrently on two streams with one plan (each stream gets its own
    workspace) equal the serial decodes, tree and lane kernels alike."""
    from polarcode_and_ldpc_amd import _native
    from polarcode_and_ldpc_amd.channel import AWGNChannel
    P = _P()
    K = N // 2
    fr = P.construct_frozen_set(N, K, 1.0)
    mask = np.zeros(N, np.uint8)
    mask[fr] = 1
    plan = _native.polar_plan(N, K, mask, L)
    B = 4096 if N * max(L, 1) <= 8192 else 1024
    llr = [AWGNChannel(1.0).llr_batch_device(None, N, B, seed=s) for s in (31, 32)]
    want = []
    for x in llr:
        o = torch.empty((B, K), dtype=torch.uint8, device="cuda")
        plan.decode(x, o)
        want.append(o)
    torch.cuda.synchronize()
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    got = [torch.zeros((B, K), dtype=torch.uint8, device="cuda") for _ in range(2)]
    s1.wait_stream(torch.cuda.current_stream())
    s2.wait_stream(torch.cuda.current_stream())
    for _ in range(3):
        with torch.cuda.stream(s1):
            plan.decode(llr[0], got[0])
        with torch.cuda.stream(s2):
            plan.decode(llr[1], got[1])
    torch.cuda.synchronize()
    assert torch.equal(got[0], want[0]) and torch.equal(got[1], want[1])


def test_release_and_wrong_device(gpu):
    """Boundary hardening: pl_plan_release frees a stream's
    workspace (and the next decode regrows it with the same bits), and every
    call on a plan from a device other than the plan's is refused with PL_EINVAL
    (pl_debug_set_plan_device stands in for a second GPU)."""
    from polarcode_and_ldpc_amd import _native
    from polarcode_and_ldpc_amd.channel import AWGNChannel
    P = _P()
    N, K, L, B = 1024, 512, 8, 2048
    fr = P.construct_frozen_set(N, K, 2.0)
    mask = np.zeros(N, np.uint8)
    mask[fr] = 1
    plan = _native.polar_plan(N, K, mask, L)
    llr = AWGNChannel(1.0).llr_batch_device(None, N, B, seed=5)
    a = torch.empty((B, K), dtype=torch.uint8, device="cuda")
    plan.decode(llr, a)
    s1 = torch.cuda.Stream()
    s1.wait_stream(torch.cuda.current_stream())
    b = torch.zeros_like(a)
    with torch.cuda.stream(s1):
        plan.decode(llr, b)
    torch.cuda.synchronize()
    assert torch.equal(a, b)
    n, nbytes = plan.workspace_stats()
    assert n == 2 and nbytes >= 2 * plan.workspace_bytes(B)
    plan.release(s1)
    assert plan.workspace_stats() == (1, plan.workspace_bytes(B))
    plan.release()
    assert plan.workspace_stats() == (0, 0)
    plan.release()  # no workspace: no-op
    c = torch.zeros_like(a)
    plan.decode(llr, c)  # regrows
    torch.cuda.synchronize()
    assert torch.equal(a, c) and plan.workspace_stats()[0] == 1
    plan.reserve(0)  # reserve(0) = release
    assert plan.workspace_stats() == (0, 0)

    # the wrong-device refusal, through the diagnostic build's test hook (the
    # product library does not carry it: ADVICE r03)
    assert _native.lib.pl_debug_set_plan_device(plan.handle, 0) == _native.PL_EUNSUPPORTED
    D = _native.load_diag()
    if D is None:
        pytest.skip("diagnostic library not built (make -C polarcode_and_ldpc_amd/csrc diag)")
    h = ctypes.c_void_p()
    assert D.pl_polar_plan_create(N, K, mask.ctypes.data_as(ctypes.c_void_p), L, 0, ctypes.byref(h)) == 0
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    P_ = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    ws = torch.empty(plan.workspace_bytes(B), dtype=torch.uint8, device="cuda")
    cw = torch.empty((B, N), dtype=torch.uint8, device="cuda")
    cur = torch.cuda.current_device()
    assert D.pl_debug_set_plan_device(h, cur + 7) == 0
    calls = {
        "pl_decode": lambda: D.pl_decode(h, P_(llr), B, N, P_(c), None, st),
        "pl_plan_reserve": lambda: D.pl_plan_reserve(h, B, st),
        "pl_plan_release": lambda: D.pl_plan_release(h, st),
        "pl_polar_plan_set_crc": lambda: D.pl_polar_plan_set_crc(h, 8, 0x1D),
        "pl_decode_ws": lambda: D.pl_decode_ws(h, P_(llr), B, N, P_(c), None, P_(ws), ws.numel(), st),
        "pl_polar_encode": lambda: D.pl_polar_encode(h, P_(a), B, P_(cw), st),
    }
    for name, call in calls.items():
        assert call() == _native.PL_EINVAL, name
        assert b"not the plan's device" in D.pl_last_error(), name
    n_, b_ = ctypes.c_int64(), ctypes.c_int64()
    assert D.pl_plan_workspace_stats(h, ctypes.byref(n_), ctypes.byref(b_)) == 0
    assert (n_.value, b_.value) == (0, 0)  # nothing was allocated on the wrong device
    assert D.pl_debug_set_plan_device(h, cur) == 0
    c.zero_()
    assert D.pl_decode(h, P_(llr), B, N, P_(c), None, st) == 0
    torch.cuda.synchronize()
    assert torch.equal(a, c)
    assert D.pl_plan_destroy(h) == 0


def test_caller_workspace_and_lazy_sizing(gpu):
    """pl_decode_ws: any workspace of at least one unit decodes the same bits
    (fewer resident waves); pl_plan_workspace_bytes grows with the batch up to
    the persistent grid, so a one-frame decode needs one wave's slice."""
    from polarcode_and_ldpc_amd import _native
    d = golden("polar_scl_1024_l8.npz")
    mask = np.zeros(1024, np.uint8)
    mask[d["frozen"]] = 1
    plan = _native.polar_plan(1024, 512, mask, 8)
    unit = plan.workspace_bytes(1)
    assert unit > 0 and plan.workspace_bytes(8) == unit  # 8 frames per wave at L = 8
    slice_ = plan.workspace_bytes(9) - unit  # one more wavefront's slice (the NaN masks are fixed)
    assert slice_ > 0 and plan.workspace_bytes(17) == unit + 2 * slice_
    assert plan.workspace_bytes(1 << 20) == plan.workspace_bytes(1 << 22)  # capped at the grid
    llr = torch.from_numpy(d["llr"]).cuda()
    B = llr.shape[0]
    for nunits in (1, 2, 7):
        # garbage in the caller's buffer (NaN masks included) must not matter
        ws = torch.full((unit + (nunits - 1) * slice_,), 0xA5, dtype=torch.uint8, device="cuda")
        out = torch.empty((B, 512), dtype=torch.uint8, device="cuda")
        plan.decode(llr, out, ws=ws)
        assert _mismatch(out.cpu().numpy(), d["scl"]) == 0, nunits
    with pytest.raises(AssertionError):
        plan.decode(llr, out, ws=torch.empty(unit - 256, dtype=torch.uint8, device="cuda"))
    # a strided output view is refused instead of being written at the wrong pitch
    wide = torch.empty((B, 600), dtype=torch.uint8, device="cuda")
    with pytest.raises(AssertionError):
        plan.decode(llr, wide[:, :512])
    with pytest.raises(AssertionError):
        plan.decode(llr.cpu(), out)


def test_scl_default_frozen_set_vs_oracle(gpu, oracle):
    """The reference's default frozen set (generate_frozen_bits: leaves 0..511
    of the decode order frozen at N=1024, the set throughput_test.py runs and
    bench.py's `default_frozen_set` line measures): HIP vs the C oracle, with
    erasures and saturated LLRs mixed in."""
    P = _P()
    rng = np.random.RandomState(71)
    enc = P.PolarEncoder(1024, 512)
    B = 96
    cw = enc.encode_batch(rng.randint(0, 2, (B, 512)))
    snr = rng.uniform(-1.0, 3.0, size=(B, 1))
    sigma = np.sqrt(1.0 / (2.0 * 10 ** (snr / 10.0)))
    llr = 2.0 * ((1.0 - 2.0 * cw) + sigma * rng.randn(B, 1024)) / sigma ** 2
    llr[5, :40] = 0.0
    llr[6, 100:300] = np.inf
    llr[7, ::3] = -np.inf
    llr[8] = 0.0
    for L in (8, 32):
        want = oracle.scl_decode(1024, L, enc.frozen_bits, llr, threads=8)
        got = P.SCLDecoder(1024, 512, list_size=L).decode_batch(llr)
        assert _mismatch(got, want) == 0, L


def test_scl_large_lists_golden_and_oracle(gpu, oracle):
    """List sizes 33..1024 (lane kernel: one frame per wavefront up to 64, one
    frame per workgroup of L/64 wavefronts above, 16-bit path slots above 256):
    the reference's L=64/128/256/300/512/1024 fixtures, plus non-power-of-two
    sizes against the oracle; 1025 is refused."""
    P = _P()
    d = golden("polar_scl_l64.npz")
    for tag, N in (("N256", 256), ("N1024", 1024)):
        dec = P.SCLDecoder(N, N // 2, list_size=64, frozen_bits=d[tag + "_frozen"])
        assert _mismatch(dec.decode_batch(d[tag + "_llr"]), d[tag + "_scl"]) == 0, tag
    d = golden("polar_scl_l256.npz")
    for tag, N, L in (("N256_L128", 256, 128), ("N256_L256", 256, 256), ("N1024_L128", 1024, 128)):
        dec = P.SCLDecoder(N, N // 2, list_size=L, frozen_bits=d[tag + "_frozen"])
        assert _mismatch(dec.decode_batch(d[tag + "_llr"]), d[tag + "_scl"]) == 0, tag
    rng = np.random.RandomState(64)
    N, K = 256, 128
    fr = P.construct_frozen_set(N, K, 1.0)
    cw = P.PolarEncoder(N, K, frozen_bits=fr).encode_batch(rng.randint(0, 2, (40, K)))
    sigma = np.sqrt(1.0 / (2.0 * 10 ** (rng.uniform(-1.0, 2.0, size=(40, 1)) / 10.0)))
    llr = 2.0 * ((1.0 - 2.0 * cw) + sigma * rng.randn(40, N)) / sigma ** 2
    llr[3, :30] = 0.0
    for L in (33, 48, 64, 65, 100, 128, 200, 256):
        want = oracle.scl_decode(N, L, fr, llr, threads=8)
        assert _mismatch(P.SCLDecoder(N, K, list_size=L, frozen_bits=fr).decode_batch(llr), want) == 0, L
    fr64 = P.construct_frozen_set(64, 32, 1.0)
    cw = P.PolarEncoder(64, 32, frozen_bits=fr64).encode_batch(rng.randint(0, 2, (24, 32)))
    llr64 = 2.0 * ((1.0 - 2.0 * cw) + 1.2 * rng.randn(24, 64)) / 1.44
    want = oracle.scl_decode(64, 256, fr64, llr64, threads=8)  # list outgrows 2^K paths: never pruned early
    assert _mismatch(P.SCLDecoder(64, 32, list_size=256, frozen_bits=fr64).decode_batch(llr64), want) == 0
    # lists above 256: 16-bit path slots, one frame per workgroup of up to 16
    # wavefronts (reference fixture + oracle, incl. a non-power-of-two list)
    d = golden("polar_scl_l1024.npz")
    for tag, Nt, L in (("N64_L512", 64, 512), ("N64_L300", 64, 300), ("N128_L1024", 128, 1024)):
        fr_t = d[tag + "_frozen"]
        dec = P.SCLDecoder(Nt, Nt - len(fr_t), list_size=L, frozen_bits=fr_t)
        assert _mismatch(dec.decode_batch(d[tag + "_llr"]), d[tag + "_scl"]) == 0, tag
    want = oracle.scl_decode(64, 700, fr64, llr64[:6], threads=8)
    assert _mismatch(P.SCLDecoder(64, 32, list_size=700, frozen_bits=fr64).decode_batch(llr64[:6]), want) == 0
    want = oracle.scl_decode(N, 513, fr, llr[:4], threads=8)
    assert _mismatch(P.SCLDecoder(N, K, list_size=513, frozen_bits=fr).decode_batch(llr[:4]), want) == 0
    with pytest.raises(ValueError):  # PL_EUNSUPPORTED: lists above 65536 paths
        P.SCLDecoder(N, K, list_size=65537, frozen_bits=fr).decode_batch(llr)


def test_scl_lists_above_1024(gpu, oracle):
    """Lists of 1025..2048 paths (VERDICT r03 missing 4; the reference accepts any
    L): every frame through the exact single-workgroup decoder of polar_nan.hip --
    the reference's L=2048 (N=64) and L=1500 (N=32) fixtures, the oracle at
    L=1025 / 2048 on noisy N=128 frames, CA-SCL at L=1500 against the oracle's
    restatement, and a NaN frame."""
    from polarcode_and_ldpc_amd import _native
    from polarcode_and_ldpc_amd.polar.utils import CRC_POLYNOMIALS
    P = _P()
    d = golden("polar_scl_l2048.npz")
    for tag, Nt, L in (("N64_L2048", 64, 2048), ("N32_L1500", 32, 1500)):
        fr_t = d[tag + "_frozen"]
        dec = P.SCLDecoder(Nt, Nt - len(fr_t), list_size=L, frozen_bits=fr_t)
        assert dec.plan.info.reserved == 6  # the exact single-workgroup decoder
        assert _mismatch(dec.decode_batch(d[tag + "_llr"]), d[tag + "_scl"]) == 0, tag
    rng = np.random.RandomState(2048)
    N, K = 128, 64
    fr = P.construct_frozen_set(N, K, 1.0)
    cw = P.PolarEncoder(N, K, frozen_bits=fr).encode_batch(rng.randint(0, 2, (6, K)))
    llr = 2.0 * ((1.0 - 2.0 * cw) + 1.1 * rng.randn(6, N)) / 1.21
    llr[5, ::7] = np.inf
    llr[5, 1::7] = -np.inf
    for L in (1025, 2048):
        want = oracle.scl_decode(N, L, fr, llr, threads=8)
        assert _mismatch(P.SCLDecoder(N, K, list_size=L, frozen_bits=fr).decode_batch(llr), want) == 0, L
    # above 2048 paths the per-frame list state moves from LDS to the workspace
    # (VERDICT r04 missing 3): two noisy frames and the +-inf frame
    sel = [0, 1, 5]
    for L in (2049, 4096):
        want = oracle.scl_decode(N, L, fr, llr[sel], threads=8)
        dec = P.SCLDecoder(N, K, list_size=L, frozen_bits=fr)
        assert dec.plan.info.reserved == 6
        assert _mismatch(dec.decode_batch(llr[sel]), want) == 0, L
    mask = np.zeros(N, np.uint8)
    mask[fr] = 1
    plan = _native.polar_plan(N, K, mask, 1500)
    plan.set_crc(8, CRC_POLYNOMIALS["CRC-8"])
    out = torch.empty((6, K), dtype=torch.uint8, device="cuda")
    plan.decode(torch.from_numpy(llr).cuda(), out)
    assert _mismatch(out.cpu().numpy(), oracle.cascl_decode(N, 1500, fr, llr, "CRC-8", threads=8)) == 0


@pytest.mark.parametrize("N,L,K", [(1024, 0, 300), (1024, 8, 512), (1024, 8, 40), (1024, 32, 700), (4096, 8, 2048),
                                   (256, 4, 128), (128, 32, 16), (2048, 8, 1500), (512, 16, 256), (1024, 8, 1016)])
def test_random_frozen_sets_rate0_nodes(gpu, oracle, N, L, K):
    """Random frozen sets (every alignment and size of all-frozen runs in decode
    order, so the tree kernel's rate-0 node path meets pairs / quads / octets
    everywhere, next to long info runs) at low SNR: HIP vs the C oracle."""
    P = _P()
    rng = np.random.RandomState(N + 7 * L + K)
    fr = np.sort(rng.choice(N, N - K, replace=False))
    enc = P.PolarEncoder(N, K, frozen_bits=fr)
    B = 32 if N * max(L, 1) <= 8192 else 12
    msg = rng.randint(0, 2, (B, K))
    cw = enc.encode_batch(msg)
    snr = rng.uniform(-2.0, 2.0, size=(B, 1))
    sigma = np.sqrt(1.0 / (2.0 * 10 ** (snr / 10.0)))
    llr = 2.0 * ((1.0 - 2.0 * cw) + sigma * rng.randn(B, N)) / sigma ** 2
    if L == 0:
        want = oracle.sc_decode(N, fr, llr, threads=8)
        got = P.SCDecoder(N, K, frozen_bits=fr).decode_batch(llr)
    else:
        want = oracle.scl_decode(N, L, fr, llr, threads=8)
        got = P.SCLDecoder(N, K, list_size=L, frozen_bits=fr).decode_batch(llr)
    assert _mismatch(got, want) == 0


def _block_frozen_set(N, rng):
    """A frozen set made of aligned all-frozen blocks in DECODE order (leaf i
    decodes index bitrev(i)): nodes of every size from 2 to N/2, at random
    positions, plus scattered single frozen leaves -- the SC kernel's rate-0
    skip meets nodes at register depths, at the multi-word depths (>= 64
    leaves), as left and as right children, and at the frame's start."""
    n = N.bit_length() - 1
    m = np.zeros(N, bool)
    for _ in range(rng.randint(2, 8)):
        k = rng.randint(1, n)
        start = rng.randint(0, N >> k) << k
        m[start:start + (1 << k)] = True
    m |= rng.rand(N) < 0.15
    if rng.rand() < 0.5:
        m[:1 << rng.randint(3, n)] = True  # a frozen prefix node
    if m.all():
        m[-1] = False
    rev = np.array([int(format(i, "0%db" % n)[::-1], 2) for i in range(N)])
    return np.sort(rev[np.nonzero(m)[0]])


@pytest.mark.parametrize("N", [128, 256, 512, 1024, 2048, 4096])
def test_sc_rate0_node_skip_vs_oracle(gpu, oracle, N, monkeypatch):
    """SC skips every all-frozen node (any size) without decoding its leaves:
    random block-structured frozen sets, noisy frames, a persistent grid forced
    to a few waves so each wavefront decodes several passes of 64 frames over
    stale workspace (PL_POLAR_WAVES): bits equal the oracle's."""
    P = _P()
    rng = np.random.RandomState(N + 11)
    monkeypatch.setenv("PL_POLAR_WAVES", "3")
    for trial in range(3):
        fr = _block_frozen_set(N, rng)
        K = N - len(fr)
        enc = P.PolarEncoder(N, K, frozen_bits=fr)
        B = 3 * 64 * 2 + 37
        msg = rng.randint(0, 2, (B, K))
        snr = rng.uniform(-1.0, 3.0, size=(B, 1))
        sigma = np.sqrt(1.0 / (2.0 * 10 ** (snr / 10.0)))
        llr = 2.0 * ((1.0 - 2.0 * enc.encode_batch(msg)) + sigma * rng.randn(B, N)) / sigma ** 2
        dec = P.SCDecoder(N, K, frozen_bits=fr)
        assert dec.plan.info.reserved == 4  # the tree kernel
        got = dec.decode_batch(llr)
        assert _mismatch(got, oracle.sc_decode(N, fr, llr, threads=8)) == 0, (trial, K)


def _nan_frames(N, K, fr, B, seed):
    """Frames whose SCL metrics become NaN, in the four kinds of
    make_golden.job_polar_nan (+-inf BEC with erasures, all +-inf, AWGN with
    +-inf positions, AWGN with NaN inputs)."""
    P = _P()
    rng = np.random.RandomState(seed)
    msg = rng.randint(0, 2, (B, K))
    cw = P.PolarEncoder(N, K, frozen_bits=fr).encode_batch(msg)
    sigma = np.sqrt(1.0 / (2.0 * 10 ** 0.1))
    llr = 2.0 * ((1.0 - 2.0 * cw) + sigma * rng.randn(B, N)) / sigma ** 2
    for f in range(B):
        kind = f % 4
        sgn = np.where(llr[f] >= 0, 1.0, -1.0)
        if kind == 0:
            x = sgn * np.inf
            x[rng.rand(N) < 0.2 + 0.3 * rng.rand()] = 0.0
        elif kind == 1:
            x = sgn * np.inf
        elif kind == 2:
            x = llr[f].copy()
            idx = rng.choice(N, size=max(1, N // 16), replace=False)
            x[idx] = rng.choice([np.inf, -np.inf], size=len(idx))
        else:
            x = llr[f].copy()
            x[rng.choice(N, size=max(1, N // 64), replace=False)] = np.nan
        llr[f] = x
    return llr


def test_scl_nan_metrics_golden(gpu):
    """frames whose path metrics become NaN (+-inf meeting in
    a g, decoder.py:417; NaN inputs), decoded by the reference itself
    (make_golden.job_polar_nan).  The list kernels flag them and
    polar_nan.hip decodes them again in CPython's list.sort order with
    np.argmax's first NaN: bit-exact at N = 16..1024, L = 1..64 (tree and lane
    kernels; L = 32 / 64 reach CPython's run merging and galloping)."""
    d = golden("polar_nan.npz")
    for N in (16, 64, 256, 1024):
        fr, llr = d["N%d_frozen" % N], d["N%d_llr" % N]
        K = N - len(fr)
        for L in d["N%d_Ls" % N]:
            dec = _P().SCLDecoder(N, K, list_size=int(L), frozen_bits=fr)
            assert _mismatch(dec.decode_batch(llr), d["N%d_L%d" % (N, L)]) == 0, (N, L)


@pytest.mark.parametrize("N,L,flags", [(1024, 8, 0), (1024, 32, 0), (4096, 8, 0), (256, 16, 0), (1024, 8, 0x20),
                                       (128, 128, 0), (64, 300, 0)])
def test_scl_nan_frames_in_large_batches(gpu, oracle, N, L, flags):
    """NaN frames scattered over a multi-pass batch of ordinary frames: the masks
    name the right (wavefront, pass, frame) and every other frame keeps the fast
    kernel's bits (vs the oracle's CPython-order restatement, pinned by the
    reference fixtures)."""
    from polarcode_and_ldpc_amd import _native
    P = _P()
    K = N // 2
    fr = P.construct_frozen_set(N, K, 2.0)
    mask = np.zeros(N, np.uint8)
    mask[fr] = 1
    plan = _native.polar_plan(N, K, mask, L, flags=flags)
    fpw = max(1, 64 // (1 << (L - 1).bit_length()))
    B = min(2 * _grid_waves(plan, fpw) * fpw + 37, 40000 if N <= 1024 else 20000)
    rng = np.random.RandomState(N + L)
    msg = rng.randint(0, 2, (B, K))
    cw = P.PolarEncoder(N, K, frozen_bits=fr).encode_batch(msg)
    sigma = np.sqrt(1.0 / (2.0 * 10 ** 0.15))
    llr = 2.0 * ((1.0 - 2.0 * cw) + sigma * rng.randn(B, N)) / sigma ** 2
    nan_idx = np.unique(np.concatenate([rng.choice(B, 24, replace=False), [0, B - 1]]))
    llr[nan_idx] = _nan_frames(N, K, fr, len(nan_idx), seed=N * 7 + L)
    out = torch.empty((B, K), dtype=torch.uint8, device="cuda")
    plan.decode(torch.from_numpy(llr).cuda(), out)
    got = out.cpu().numpy().astype(np.int64)
    chk = np.unique(np.concatenate([nan_idx, rng.choice(B, 40, replace=False)]))
    want = oracle.scl_decode(N, L, fr, llr[chk], threads=8)
    assert _mismatch(got[chk], want) == 0
    # a second decode of ordinary frames on the same workspace: the masks were re-zeroed
    clean = np.delete(np.arange(B), nan_idx)[:4096]
    out2 = torch.empty((len(clean), K), dtype=torch.uint8, device="cuda")
    plan.decode(torch.from_numpy(llr[clean]).cuda(), out2)
    assert np.array_equal(out2.cpu().numpy(), got[clean])


@pytest.mark.parametrize("N,L,crc", [(1024, 8, "CRC-8"), (1024, 32, "CRC-16"), (256, 64, "CRC-8")])
def test_cascl_nan_frames_vs_oracle(gpu, oracle, N, L, crc):
    """CA-SCL on NaN frames: the build-defined order of the final paths is the
    one list.sort(key=metric, reverse=True) leaves (CPython's, with NaN keys),
    first CRC pass, else np.argmax -- the oracle's restatement."""
    from polarcode_and_ldpc_amd import _native
    from polarcode_and_ldpc_amd.polar.utils import CRC_POLYNOMIALS
    P = _P()
    K = N // 2
    fr = P.construct_frozen_set(N, K, 2.0)
    llr = _nan_frames(N, K, fr, 32, seed=5 + L)
    mask = np.zeros(N, np.uint8)
    mask[fr] = 1
    plan = _native.polar_plan(N, K, mask, L)
    clen = int(crc.split("-")[1])
    plan.set_crc(clen, CRC_POLYNOMIALS[crc])
    out = torch.empty((len(llr), K), dtype=torch.uint8, device="cuda")
    plan.decode(torch.from_numpy(llr).cuda(), out)
    want = oracle.cascl_decode(N, L, fr, llr, crc, threads=8)
    assert _mismatch(out.cpu().numpy(), want) == 0


# ---------------------------------------------------------------------------
# Round 6: a frame with exactly ONE +-inf / huge input stays
# on the tree kernel's fast path (polar_tree.hip: no g can meet two infinities,
# so no NaN metric), where paths can reach -inf metrics and tie there.  Pinned
# against the reference itself (make_golden.job_polar_single_inf) and the oracle.

def _single_extreme(N, fr, llr, rng):
    """One +-inf / +-1e300 / +-1.5e308 input per frame, some frames with
    erasures (the same kinds as make_golden.single_extreme_frames)."""
    kinds = [(np.inf, +1, 0.0), (np.inf, -1, 0.0), (1e300, -1, 0.0), (1.5e308, +1, 0.0),
             (np.inf, +1, 0.2), (np.inf, -1, 0.4), (1e300, +1, 0.3), (1.5e308, -1, 0.25)]
    info = np.setdiff1d(np.arange(N), fr)
    out = llr.copy()
    for f in range(len(out)):
        val, rel, er = kinds[f % len(kinds)]
        x = out[f]
        if er:
            x[rng.rand(N) < er] = 0.0
        p = int(rng.choice(fr if (f // len(kinds)) % 2 == 0 else info))
        x[p] = (1.0 if x[p] >= 0 else -1.0) * rel * val
    return out


def _diag_decode_flagged(N, K, fr, L, llr, crc=None):
    """Decode through the diagnostic library's pl_debug_polar_flagged: (bits,
    per-frame flagged-for-redo bytes, kernel id).  The decode is the product
    kernel; the hook only reads the NaN masks back before the redo pass."""
    from polarcode_and_ldpc_amd import _native
    D = _native.load_diag()
    if D is None:
        pytest.skip("diagnostic library not built (make -C polarcode_and_ldpc_amd/csrc diag)")
    mask = np.zeros(N, np.uint8)
    mask[fr] = 1
    h = ctypes.c_void_p()
    assert D.pl_polar_plan_create(N, K, mask.ctypes.data_as(ctypes.c_void_p), L, 0, ctypes.byref(h)) == 0
    try:
        info = _native.PlanInfo()
        assert D.pl_plan_get_info(h, ctypes.byref(info)) == 0
        if crc is not None:
            assert D.pl_polar_plan_set_crc(h, crc[0], crc[1]) == 0
        x = torch.from_numpy(np.ascontiguousarray(llr)).cuda()
        out = torch.empty((len(llr), K), dtype=torch.uint8, device="cuda")
        flagged = np.full(len(llr), 7, np.uint8)
        st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
        rc = D.pl_debug_polar_flagged(h, ctypes.c_void_p(x.data_ptr()), len(llr), N, ctypes.c_void_p(out.data_ptr()),
                                      flagged.ctypes.data_as(ctypes.c_void_p), st)
        assert rc == 0, D.pl_last_error()
        torch.cuda.synchronize()
        return out.cpu().numpy().astype(np.int64), flagged, int(info.reserved)
    finally:
        D.pl_plan_destroy(h)


def test_single_extreme_input_golden_fast_path(gpu):
    """Reference decodes of one-+-inf / one-huge-input frames (N=1024 L=8 / L=32,
    N=2048 / 4096 L=8): bit-exact, on the tree kernel, and NOT flagged for the
    redo decoder -- while a NaN frame and a two-inf frame in the same batch are
    (the hook's positive control)."""
    d = golden("polar_single_inf.npz")
    for N in (1024, 2048, 4096):
        fr, llr = d["N%d_frozen" % N], d["N%d_llr" % N]
        K = N - len(fr)
        ctrl = llr[:2].copy()
        ctrl[0, 3] = np.nan
        ctrl[1, [5, 9]] = [np.inf, -np.inf]
        for L in d["N%d_Ls" % N]:
            L = int(L)
            want = d["N%d_L%d" % (N, L)]
            dec = _P().SCLDecoder(N, K, list_size=L, frozen_bits=fr)
            assert dec.plan.info.reserved == 4, (N, L)  # the tree kernel
            assert _mismatch(dec.decode_batch(llr), want) == 0, (N, L)
            bits, flagged, kern = _diag_decode_flagged(N, K, fr, L, np.concatenate([llr, ctrl]))
            assert kern == 4
            assert _mismatch(bits[:len(llr)], want) == 0, (N, L)
            assert not flagged[:len(llr)].any(), (N, L, np.nonzero(flagged)[0])
            assert flagged[len(llr):].all(), (N, L)


@pytest.mark.parametrize("N,L,B", [(1024, 8, 65536), (1024, 32, 65536), (2048, 8, 32768), (4096, 8, 16384)])
def test_single_extreme_frames_in_large_batch(gpu, oracle, N, L, B):
    """Single-extreme-input frames scattered over a BASELINE-size batch of noisy
    frames (1 dB): plain SCL and CA-SCL (CRC-8) against the oracle, and none of
    them flagged."""
    from polarcode_and_ldpc_amd.polar.utils import CRC_POLYNOMIALS
    P = _P()
    K = N // 2
    fr = P.construct_frozen_set(N, K, 2.0)
    rng = np.random.RandomState(N + 3 * L)
    msg = rng.randint(0, 2, (B, K))
    cw = P.PolarEncoder(N, K, frozen_bits=fr).encode_batch(msg)
    sigma = np.sqrt(1.0 / (2.0 * 10 ** 0.1))
    llr = 2.0 * ((1.0 - 2.0 * cw) + sigma * rng.randn(B, N)) / sigma ** 2
    rows = np.unique(np.concatenate([rng.choice(B, 46, replace=False), [0, 1, B - 1]]))
    llr[rows] = _single_extreme(N, fr, llr[rows], rng)
    chk = np.unique(np.concatenate([rows, rng.choice(B, 24, replace=False)]))
    for crc in (None, "CRC-8"):
        c = None if crc is None else (8, CRC_POLYNOMIALS[crc])
        bits, flagged, kern = _diag_decode_flagged(N, K, fr, L, llr, crc=c)
        assert kern == 4 and not flagged.any(), np.nonzero(flagged)[0][:8]
        if crc is None:
            want = oracle.scl_decode(N, L, fr, llr[chk], threads=8)
        else:
            want = oracle.cascl_decode(N, L, fr, llr[chk], crc, threads=8)
        assert _mismatch(bits[chk], want) == 0, crc
        # the product library gives the same bits for the whole batch
        dec = P.SCLDecoder(N, K, list_size=L, frozen_bits=fr)
        if crc is not None:
            dec.plan.set_crc(*c)
        assert _mismatch(dec.decode_batch(llr), bits) == 0, crc
