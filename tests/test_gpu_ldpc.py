"""Parity of the HIP LDPC decoders (BP, Min-Sum) against the reference's own
outputs (golden fixtures) and the C oracle.  Bar: bit-exact hard decisions and
identical iteration counts."""
import numpy as np
import pytest
import torch

from conftest import golden

pytestmark = pytest.mark.gpu


def _L():
    import polarcode_and_ldpc_amd.ldpc as L
    return L


def _H(d):
    from polarcode_and_ldpc_amd.ldpc import csr_to_dense
    return csr_to_dense(d["row_ptr"], d["col_idx"], int(d["n"]))


def test_bp_harness_frames(gpu):
    """BASELINE config 3 frames (throughput_test.py:285-315 condition: invalid
    codewords, 20 iterations every frame)."""
    d = golden("ldpc_bp_504.npz")
    dec = _L().BPDecoder(_H(d), max_iter=20)
    bits, its = dec.decode_batch(d["harness_llr"], return_iterations=True)
    assert np.array_equal(bits, d["harness_bits"])
    assert np.array_equal(its, d["harness_iters"])
    b, i = dec.decode(d["harness_llr"][0], return_iterations=True)
    assert np.array_equal(b, d["harness_bits"][0]) and i == d["harness_iters"][0]


def test_bp_zero_codeword_snrs(gpu):
    d = golden("ldpc_bp_504.npz")
    L = _L()
    H = _H(d)
    bits, its = L.BPDecoder(H, max_iter=20).decode_batch(d["zero_llr"], return_iterations=True)
    assert np.array_equal(bits, d["zero_bits"]) and np.array_equal(its, d["zero_iters"])
    assert np.array_equal(L.BPDecoder(H, max_iter=5, early_stop=False).decode_batch(d["zero_llr"][:24]),
                          d["noes5_bits"])
    b, i = L.BPDecoder(H, max_iter=50).decode_batch(d["zero_llr"][:12], return_iterations=True)
    assert np.array_equal(b, d["es50_bits"]) and np.array_equal(i, d["es50_iters"])


@pytest.mark.parametrize("fpg", ["1", "2"])
def test_bp_frames_per_group(gpu, oracle, monkeypatch, fpg):
    """ldpc_bp_grp_kernel decoding 1 or 2 frames per workgroup (PL_BP_FPG):
    the golden frames in odd-sized batches (a last workgroup with one frame), and
    a batch mixing frames that stop early with frames that never converge (the
    workgroup's two frames end at different iterations), against the oracle."""
    monkeypatch.setenv("PL_BP_FPG", fpg)
    d = golden("ldpc_bp_504.npz")
    L = _L()
    H = _H(d)
    dec = L.BPDecoder(H, max_iter=20)
    assert dec.plan.info.reserved == 7
    for B in (1, 7, 23):
        bits, its = dec.decode_batch(d["harness_llr"][:B], return_iterations=True)
        assert np.array_equal(bits, d["harness_bits"][:B]) and np.array_equal(its, d["harness_iters"][:B])
    bits, its = dec.decode_batch(d["zero_llr"], return_iterations=True)
    assert np.array_equal(bits, d["zero_bits"]) and np.array_equal(its, d["zero_iters"])
    mix = np.empty((2 * 24 + 1, 504))
    mix[0::2] = np.resize(d["zero_llr"][24:], (25, 504))  # the higher-SNR all-zero frames (early stop)
    mix[1::2] = d["harness_llr"][:24]
    rp, ci = L.dense_to_csr(H)
    want_b, want_i = oracle.ldpc_decode(rp, ci, 504, mix, threads=8)
    bits, its = dec.decode_batch(mix, return_iterations=True)
    assert np.array_equal(bits, want_b) and np.array_equal(its, want_i)


def test_ms_504(gpu):
    d = golden("ldpc_ms_504.npz")
    L = _L()
    H = _H(d)
    for norm in (1.0, 0.75):
        assert np.array_equal(L.MSDecoder(H, max_iter=20, normalization=norm).decode_batch(d["llr"]),
                              d["ms_%g" % norm])
    assert np.array_equal(L.MSDecoder(H, max_iter=7, normalization=0.75, early_stop=False)
                          .decode_batch(d["llr"][:10]), d["ms_noes7"])
    b, i = L.BPDecoder(H, max_iter=20).decode_batch(d["llr"], return_iterations=True)
    assert np.array_equal(b, d["bp_bits"]) and np.array_equal(i, d["bp_iters"])


@pytest.mark.parametrize("kernel", ["default", "compact", "generic"])
def test_ms_8192(gpu, kernel, monkeypatch):
    """n=8192: T/C do not fit LDS.  Default: the (3,6)-regular min-sum kernel
    (ldpc_ms36_kernel, rebuild-ready check state); compact: the compressed check
    state kernel (ldpc_ms_compact_kernel); generic: T/C in a global workspace."""
    if kernel != "default":
        monkeypatch.setenv("PL_LDPC_KERNEL", kernel)
    d = golden("ldpc_ms_8192.npz")
    dec = _L().MSDecoder(_H(d), max_iter=20, normalization=0.75)
    if kernel == "generic":
        assert dec.plan.info.lds_bytes < 64 * 1024 and dec.plan.info.reserved == 1
    else:
        assert dec.plan.info.reserved == (8 if kernel == "default" else 5)
    assert np.array_equal(dec.decode_batch(d["llr"]), d["ms_0_75"])


def _special_llrs(rng, B, n):
    """Noisy all-zero-codeword LLRs with the special values of min-sum's check
    statistics: exact zeros (one or many per check), -0, +-inf, NaN (one, a few)."""
    snr = rng.uniform(0.5, 2.5, size=(B, 1))
    sigma = np.sqrt(1.0 / (2.0 * 10 ** (snr / 10.0)))
    llr = 2.0 * (1.0 + sigma * rng.randn(B, n)) / sigma ** 2
    llr[1, ::5] = 0.0
    llr[2, ::97] = -0.0
    llr[3, 7] = np.nan
    llr[4, 11], llr[4, 12] = np.inf, -np.inf
    llr[5, :3] = np.nan
    llr[6, rng.rand(n) < 0.3] = 0.0          # erasures: checks with 1, 2 or more zeros
    llr[7, rng.rand(n) < 0.02] = np.nan      # scattered NaN
    llr[8, rng.rand(n) < 0.1] = np.inf
    llr[8, rng.rand(n) < 0.1] = -np.inf
    llr[9, :] = np.where(rng.rand(n) < 0.5, 0.0, -0.0)
    return llr


@pytest.mark.parametrize("kernel", ["default", "compact"])
@pytest.mark.parametrize("norm,es", [(0.75, True), (1.0, False), (-0.5, True), (1.25, False), (0.0, True)])
def test_ms_compact_vs_oracle(gpu, oracle, monkeypatch, kernel, norm, es):
    """The LDS-state min-sum kernels on an n=8192 (3,6)-regular code against the
    oracle, including exact zeros, +-inf and NaN LLRs (edge cases of the check
    statistics) and normalizations outside (0, 1]."""
    if kernel != "default":
        monkeypatch.setenv("PL_LDPC_KERNEL", kernel)
    L = _L()
    H = L.regular_construction(8192, 3, 6, seed=1)
    rp, ci = L.dense_to_csr(H)
    rng = np.random.RandomState(17)
    llr = _special_llrs(rng, 24, 8192)
    want_b, want_i = oracle.ldpc_decode(rp, ci, 8192, llr, algo="ms", max_iter=20, early_stop=es, norm=norm,
                                        threads=8)
    dec = L.MSDecoder(H, 20, norm, es)
    assert dec.plan.info.reserved == (8 if kernel == "default" else 5)
    got_b, got_i = dec.decode_batch(llr, return_iterations=True)
    assert np.array_equal(got_b, want_b)
    assert np.array_equal(got_i, want_i)


@pytest.mark.parametrize("n", [2048, 4096])
def test_ms36_smaller_codes_vs_oracle(gpu, oracle, n):
    """ldpc_ms36_kernel's n = 2048 / 4096 instances (one / two checks per thread)."""
    L = _L()
    H = L.regular_construction(n, 3, 6, seed=n)
    rp, ci = L.dense_to_csr(H)
    llr = _special_llrs(np.random.RandomState(n), 16, n)
    for norm, es in ((0.75, True), (1.0, False)):
        want_b, want_i = oracle.ldpc_decode(rp, ci, n, llr, algo="ms", max_iter=20, early_stop=es, norm=norm,
                                            threads=8)
        dec = L.MSDecoder(H, 20, norm, es)
        assert dec.plan.info.reserved == 8
        got_b, got_i = dec.decode_batch(llr, return_iterations=True)
        assert np.array_equal(got_b, want_b) and np.array_equal(got_i, want_i), (norm, es)


def test_ms_degree1_raises_like_reference(gpu):
    d = golden("ldpc_bp_504.npz")  # seed-42 mackay H has degree-1 checks
    dec = _L().MSDecoder(_H(d), max_iter=20)
    with pytest.raises(ValueError):
        dec.decode(d["harness_llr"][0])


@pytest.mark.parametrize("algo,norm,es", [("bp", 1.0, True), ("bp", 1.0, False), ("ms", 0.75, True),
                                          ("ms", 1.0, False)])
def test_vs_oracle_random(gpu, oracle, algo, norm, es):
    L = _L()
    H = L.regular_construction(504, 3, 6, seed=3) if algo == "ms" else L.mackay_construction(504, 252, 3, 6, 42)
    rp, ci = L.dense_to_csr(H)
    rng = np.random.RandomState(11)
    B = 64
    snr = rng.uniform(-1.0, 3.0, size=(B, 1))
    sigma = np.sqrt(1.0 / (2.0 * 10 ** (snr / 10.0)))
    llr = 2.0 * (1.0 + sigma * rng.randn(B, 504)) / sigma ** 2
    llr[0, ::7] = 0.0  # exact zeros
    want_b, want_i = oracle.ldpc_decode(rp, ci, 504, llr, algo=algo, max_iter=20, early_stop=es, norm=norm,
                                        threads=8)
    dec = L.BPDecoder(H, 20, es) if algo == "bp" else L.MSDecoder(H, 20, norm, es)
    got_b, got_i = dec.decode_batch(llr, return_iterations=True)
    assert np.array_equal(got_b, want_b)
    if algo == "bp":
        assert np.array_equal(got_i, want_i)


def test_full_batch_bp_device(gpu):
    """BASELINE config 3 size: B=65536 frames of the all-zero codeword at 3 dB
    (device AWGN), decoded on device; a 64-frame sample matches the oracle."""
    from oracle import oracle as O
    L = _L()
    from polarcode_and_ldpc_amd.channel import AWGNChannel
    H = L.mackay_construction(504, 252, 3, 6, 42)
    rp, ci = L.dense_to_csr(H)
    dec = L.BPDecoder(H, max_iter=20)
    B = 65536
    llr = AWGNChannel(3.0).llr_batch_device(None, 504, B, seed=5)
    bits, its = dec.decode_batch(llr, return_iterations=True)
    torch.cuda.synchronize()
    idx = np.arange(0, B, B // 64)
    want_b, want_i = O.ldpc_decode(rp, ci, 504, llr[idx].cpu().numpy(), max_iter=20, threads=8)
    assert np.array_equal(bits[idx].cpu().numpy().astype(np.int64), want_b)
    assert np.array_equal(its[idx].cpu().numpy(), want_i)


def test_bp_lean_math_stress_vs_oracle(gpu, oracle):
    """The BP kernel's own fp64 tanh/atanh (ldpc.hip) against the oracle's libm on
    1024 frames around the waterfall (-1..2.5 dB), where messages hover near
    decision boundaries longest: every decision and iteration count equal."""
    L = _L()
    H = L.mackay_construction(504, 252, 3, 6, 42)
    rp, ci = L.dense_to_csr(H)
    rng = np.random.RandomState(2024)
    B = 1024
    snr = rng.uniform(-1.0, 2.5, size=(B, 1))
    sigma = np.sqrt(1.0 / (2.0 * 10 ** (snr / 10.0)))
    llr = 2.0 * (1.0 + sigma * rng.randn(B, 504)) / sigma ** 2
    want_b, want_i = oracle.ldpc_decode(rp, ci, 504, llr, algo="bp", max_iter=20, early_stop=True, threads=16)
    got_b, got_i = L.BPDecoder(H, 20, True).decode_batch(llr, return_iterations=True)
    assert np.array_equal(got_b, want_b)
    assert np.array_equal(got_i, want_i)


@pytest.mark.parametrize("algo", ["bp", "ms"])
@pytest.mark.parametrize("kernel", ["default", "generic"])
def test_special_values_golden(gpu, algo, kernel, monkeypatch):
    """NaN, +-inf, +-0 channel LLRs through both flooding kernels (the
    register-cached one and the generic one, PL_LDPC_KERNEL=generic) against the
    reference's own outputs (golden ldpc_special.npz): nan_to_num of the BP
    check output, NaN-propagating min-sum, np.sign(+-0) = 0."""
    if kernel == "generic":
        monkeypatch.setenv("PL_LDPC_KERNEL", "generic")
    L = _L()
    d = golden("ldpc_special.npz")
    H = L.csr_to_dense(d[algo + "_row_ptr"], d[algo + "_col_idx"], 504)
    dec = L.BPDecoder(H, 20, True) if algo == "bp" else L.MSDecoder(H, 20, 0.75, True)
    got_b, got_i = dec.decode_batch(d["llr"], return_iterations=True)
    assert np.array_equal(got_b, d[algo + "_bits"])
    if algo == "bp":
        assert np.array_equal(got_i, d["bp_iters"])


def test_empty_batch(gpu):
    """A zero-frame batch returns empty bits and iteration counts (BP and MS)."""
    d = golden("ldpc_bp_504.npz")
    L = _L()
    H = _H(d)
    for dec in (L.BPDecoder(H, max_iter=20), L.MSDecoder(_H(golden("ldpc_ms_504.npz")), max_iter=20),
                L.MSDecoder(_H(golden("ldpc_ms_8192.npz")), max_iter=20)):
        bits = dec.decode_batch(np.zeros((0, dec.n)))
        assert bits.shape == (0, dec.n)
    bits, its = L.BPDecoder(H, max_iter=20).decode_batch(np.zeros((0, 504)), return_iterations=True)
    assert bits.shape == (0, 504) and its.shape == (0,)


def test_global_workspace_two_streams(gpu, oracle):
    """BP on an n=8192 code keeps its messages in a per-stream global workspace:
    two streams sharing one plan (different batch sizes, so each stream's
    workspace is sized to its own batch and regrown) decode exactly as serial
    decodes, and a caller-supplied workspace of one frame gives the same bits."""
    L = _L()
    H = L.regular_construction(8192, 3, 6, seed=2)
    dec = L.BPDecoder(H, max_iter=8)
    plan = dec.plan
    assert plan.info.reserved == 1  # generic kernel, global workspace
    rng = np.random.RandomState(3)
    xs = [torch.from_numpy(2.0 * (1.0 + 0.9 * rng.randn(B, 8192)) / 0.81).cuda() for B in (40, 72)]
    want = [dec.decode_batch(x, return_iterations=True) for x in xs]
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    got = [(torch.empty((x.shape[0], 8192), dtype=torch.uint8, device="cuda"),
            torch.empty((x.shape[0],), dtype=torch.int32, device="cuda")) for x in xs]
    for s in (s1, s2):
        s.wait_stream(torch.cuda.current_stream())
    for _ in range(2):
        with torch.cuda.stream(s1):
            plan.decode(xs[0], *got[0])
        with torch.cuda.stream(s2):
            plan.decode(xs[1], *got[1])
    torch.cuda.synchronize()
    for (b, i), (wb, wi) in zip(got, want):
        assert torch.equal(b, wb) and torch.equal(i, wi)
    unit = plan.workspace_bytes(1)
    assert unit > 0 and plan.workspace_bytes(3) == 3 * unit
    ws = torch.empty(unit, dtype=torch.uint8, device="cuda")
    b, i = torch.empty_like(got[0][0]), torch.empty_like(got[0][1])
    plan.decode(xs[0][:5], b[:5], i[:5], ws=ws)
    assert torch.equal(b[:5], want[0][0][:5]) and torch.equal(i[:5], want[0][1][:5])
    rp, ci = L.dense_to_csr(H)
    wb, wi = oracle.ldpc_decode(rp, ci, 8192, xs[0][:4].cpu().numpy(), "bp", 8, True, 1.0, threads=4)
    assert np.array_equal(b[:4].cpu().numpy(), wb) and np.array_equal(i[:4].cpu().numpy(), wi)


@pytest.mark.parametrize("code,n,dv,dc", [("mackay", 504, 3, 6), ("mackay", 600, 3, 6), ("regular", 1000, 3, 6),
                                          ("regular", 480, 4, 8), ("regular", 720, 4, 8)])
def test_bp_grouped_variants_vs_oracle(gpu, oracle, code, n, dv, dc):
    """BP through ldpc_bp_grp_kernel at each of its (DV, EPT, VPT) instances
    (3,6,2), (3,12,4), (4,8,2), (4,16,4): irregular MacKay codes (check degrees
    0..15 around dc, so slots mix degrees and the plan pads checks up to their
    slots' largest degree; n = 600 has a degree-15 check) and regular ones,
    with and without early stop, bits and iteration counts against the oracle
    (src/ldpc/decoder.py:62-122,124-202)."""
    L = _L()
    H = (L.mackay_construction(n, n // 2, dv, dc, seed=n + dv) if code == "mackay"
         else L.regular_construction(n, dv, dc, seed=n + dv))
    rp, ci = L.dense_to_csr(H)
    degs = np.diff(rp)
    rng = np.random.RandomState(n * 10 + dv)
    B = 48
    snr = rng.uniform(-1.0, 3.0, size=(B, 1))
    sigma = np.sqrt(1.0 / (2.0 * 10 ** (snr / 10.0)))
    llr = 2.0 * (1.0 + sigma * rng.randn(B, n)) / sigma ** 2
    llr[1, ::5] = 0.0
    for es in (True, False):
        dec = L.BPDecoder(H, 20, es)
        assert degs.max() <= 15 and dec.plan.info.reserved == 7, (n, dv, int(degs.max()))
        want_b, want_i = oracle.ldpc_decode(rp, ci, n, llr, algo="bp", max_iter=20, early_stop=es, threads=8)
        got_b, got_i = dec.decode_batch(llr, return_iterations=True)
        assert np.array_equal(got_b, want_b), (n, dv, es)
        assert np.array_equal(got_i, want_i), (n, dv, es)
