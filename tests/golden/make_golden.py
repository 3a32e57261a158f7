#!/usr/bin/env python3
"""Generate the golden parity fixtures under tests/golden/ from the reference.

This script is the ONLY place the reference implementation is executed.  It
runs in the build container (where /root/reference exists), imports the
reference read-only (``sys.path.insert(0, <ref>/src)``), feeds it inputs and
stores *data* (inputs + the reference's outputs) as small .npz files.  The
reference never travels to the GPU box; only these vectors do.

Usage:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py [--ref /root/reference]

Fixture inventory:
  polar_p1.npz         F1  N=256 K=128 SC, 100 frames produced exactly in the
                           order of benchmarks/throughput_test.py:196-228
                           (AWGNChannel(3.0, seed=42), 10 warm-up frames first);
                           plus SCL L=1/2/4/8 on the first 32 frames.
  polar_sc_1024.npz    F2  SC N=1024 K=512, default + bit-reversed
                           Bhattacharyya(2 dB) frozen sets, 0/1/3 dB.
  polar_scl_1024_l8.npz F3 SCL N=1024 K=512 L=8 (bit-reversed Bhattacharyya)
                           at 0/1.5/3 dB, and the default set at 3 dB.
  polar_scl_1024_l32.npz F4 SCL N=1024 K=512 L=32.
  polar_scl_4096_l8.npz  F5 SCL N=4096 K=2048 L=8.
  polar_small.npz      SC/SCL over small N, odd list sizes (3, 5, 6), K
                           extremes (1, N-1) and LLR vectors with exact zeros.
  polar_kat16.npz      F8  docs/SCL_DECODER_README.md:115-128 KAT.
  ldpc_bp_504.npz      F6  BP on the seed-42 mackay (504,252) H: the
                           throughput_test.py:285-315 frames (invalid
                           codewords, always 20 iterations) + all-zero
                           codewords at -1/0.5/1/3 dB, with iteration counts.
  ldpc_ms_504.npz      F7  MS (norm 1.0 and 0.75) on a (504,252) H whose row
                           degrees are all >= 2, + BP on the same H.
  ldpc_ms_8192.npz     F7  MS-20 on an n=8192 (3,6)-regular H.
  crc.npz              F9  crc_encode vectors for CRC-8/16/24.
  polar_nan.npz        (round 4) SCL frames with NaN path metrics (+-inf / NaN
                           LLRs): CPython's list.sort order of NaN keys.
  polar_single_inf.npz (round 6) SCL frames with exactly one +-inf / huge input.
  host_api.npz         (round 6) every exported host function / method's
                           outputs + the reference's public name inventory.
"""
import argparse
import json
import os
import platform
import sys
import time
from multiprocessing import Pool

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference"


def _imp():
    sys.dont_write_bytecode = True
    if os.path.join(REF, "src") not in sys.path:
        sys.path.insert(0, os.path.join(REF, "src"))
    import polar, ldpc, channel  # noqa: F401
    return polar, ldpc, channel


def bitrev(i, n):
    r = 0
    for _ in range(n):
        r = (r << 1) | (i & 1)
        i >>= 1
    return r


def bitrev_bhatta_frozen(N, K, snr=2.0):
    polar, _, _ = _imp()
    n = int(np.log2(N))
    frozen, info = polar.construct_polar_code(N, K, "bhattacharyya", snr)
    fr = np.sort(np.array([bitrev(int(i), n) for i in frozen], dtype=np.int64))
    return fr


def csr_from_dense(H):
    m, n = H.shape
    row_ptr = [0]
    col = []
    for i in range(m):
        nz = np.nonzero(H[i])[0]
        col.extend(nz.tolist())
        row_ptr.append(len(col))
    return np.array(row_ptr, np.int32), np.array(col, np.int32)


def regular_36_H(n, seed):
    """(3,6)-regular H by a seeded socket permutation; no repeated edges.
    Every row has degree exactly 6 (so Min-Sum is defined on every check)."""
    m = n // 2
    rng = np.random.RandomState(seed)
    while True:
        sockets = np.repeat(np.arange(m), 6)
        rng.shuffle(sockets)
        cols = sockets.reshape(n, 3)
        if all(len(set(r)) == 3 for r in cols):
            H = np.zeros((m, n), dtype=np.int64)
            for v in range(n):
                H[cols[v], v] = 1
            return H


# --------------------------------------------------------------------------
def job_p1():
    polar, ldpc, channel = _imp()
    N, K = 256, 128
    enc = polar.PolarEncoder(N, K)
    dec = polar.SCDecoder(N, K, frozen_bits=enc.get_frozen_bits_positions())
    ch = channel.AWGNChannel(snr_db=3.0, seed=42)
    for _ in range(10):
        msg = np.random.randint(0, 2, K)
        cw = enc.encode(msg)
        llr = ch.transmit(cw, return_llr=True)
        dec.decode(llr)
    messages = [np.random.randint(0, 2, K) for _ in range(100)]
    llrs = []
    for msg in messages:
        llrs.append(ch.transmit(enc.encode(msg), return_llr=True))
    llrs = np.array(llrs)
    sc = np.array([dec.decode(l) for l in llrs])
    out = dict(N=N, K=K, frozen=np.asarray(enc.get_frozen_bits_positions(), np.int64),
               llr=llrs, msg=np.array(messages), sc=sc)
    for L in (1, 2, 4, 8):
        d = polar.SCLDecoder(N, K, list_size=L, frozen_bits=enc.get_frozen_bits_positions())
        out["scl_L%d" % L] = np.array([d.decode(l.copy()) for l in llrs[:32]])
    return "polar_p1.npz", out


def _polar_frames(N, K, frozen, snrs, frames, seed):
    polar, _, channel = _imp()
    enc = polar.PolarEncoder(N, K, frozen_bits=frozen)
    np.random.seed(seed)
    llr, msg, snr_col = [], [], []
    for s in snrs:
        ch = channel.AWGNChannel(snr_db=s)
        for _ in range(frames):
            m = np.random.randint(0, 2, K)
            llr.append(ch.transmit(enc.encode(m), return_llr=True))
            msg.append(m)
            snr_col.append(s)
    return np.array(llr), np.array(msg), np.array(snr_col)


def job_sc1024():
    polar, _, _ = _imp()
    N, K = 1024, 512
    out = dict(N=N, K=K)
    default_frozen, _ = polar.generate_frozen_bits(N, K)
    for tag, fr in (("default", np.asarray(default_frozen, np.int64)),
                    ("bhatta", bitrev_bhatta_frozen(N, K))):
        llr, msg, snr = _polar_frames(N, K, fr, (0.0, 1.0, 3.0), 24, 1000 + len(tag))
        dec = polar.SCDecoder(N, K, frozen_bits=fr)
        out[tag + "_frozen"] = fr
        out[tag + "_llr"] = llr
        out[tag + "_msg"] = msg
        out[tag + "_snr"] = snr
        out[tag + "_sc"] = np.array([dec.decode(l) for l in llr])
    return "polar_sc_1024.npz", out


def job_scl(N, K, L, snrs, frames, seed, name, frozen_kind="bhatta"):
    polar, _, _ = _imp()
    if frozen_kind == "bhatta":
        fr = bitrev_bhatta_frozen(N, K)
    else:
        fr = np.asarray(polar.generate_frozen_bits(N, K)[0], np.int64)
    llr, msg, snr = _polar_frames(N, K, fr, snrs, frames, seed)
    dec = polar.SCLDecoder(N, K, list_size=L, frozen_bits=fr)
    t = time.time()
    out_bits = np.array([dec.decode(l.copy()) for l in llr])
    dt = (time.time() - t) / len(llr)
    return name, dict(N=N, K=K, L=L, frozen=fr, llr=llr, msg=msg, snr=snr,
                      scl=out_bits, ref_s_per_frame=dt)


def job_scl1024_l8():
    a = job_scl(1024, 512, 8, (0.0, 1.5, 3.0), 20, 7, "x")[1]
    b = job_scl(1024, 512, 8, (3.0,), 12, 8, "x", frozen_kind="default")[1]
    out = {k: v for k, v in a.items()}
    for k in ("frozen", "llr", "msg", "snr", "scl"):
        out["default_" + k] = b[k]
    return "polar_scl_1024_l8.npz", out


def job_scl1024_l32():
    return job_scl(1024, 512, 32, (1.0, 2.5), 4, 9, "polar_scl_1024_l32.npz")


def job_scl4096_l8():
    return job_scl(4096, 2048, 8, (1.5,), 3, 10, "polar_scl_4096_l8.npz")


# Round 2: wider reference-held parity where last-ulp metric differences could
# flip a near-tie rank -- low SNR (config 4's sweep starts at -2 dB), large
# lists and long codes near the waterfall.  One job per SNR point so the pool
# runs them in parallel (the reference takes ~2.4 s per L=32 frame, ~8 s per
# N=4096 L=8 frame).
def _job_scl_l32_low(var, snr, seed):
    def job():
        name = "polar_scl_1024_l32_m%d.npz" % int(round(-snr * 10))
        return job_scl(1024, 512, 32, (snr,), 64, seed, name)
    job.__name__ = job.__qualname__ = var  # picklable by module attribute
    return job


def _job_scl4096_wf(var, snr, seed):
    def job():
        name = "polar_scl_4096_l8_wf%d.npz" % int(round(-snr * 10))
        return job_scl(4096, 2048, 8, (snr,), 8, seed, name)
    job.__name__ = job.__qualname__ = var
    return job


job_scl1024_l32_m20 = _job_scl_l32_low("job_scl1024_l32_m20", -2.0, 201)
job_scl1024_l32_m10 = _job_scl_l32_low("job_scl1024_l32_m10", -1.0, 202)
job_scl1024_l32_m00 = _job_scl_l32_low("job_scl1024_l32_m00", 0.0, 203)
job_scl4096_wf_a = _job_scl4096_wf("job_scl4096_wf_a", -1.5, 211)
job_scl4096_wf_b = _job_scl4096_wf("job_scl4096_wf_b", -1.0, 212)
ROUND2_JOBS = [job_scl1024_l32_m20, job_scl1024_l32_m10, job_scl1024_l32_m00, job_scl4096_wf_a, job_scl4096_wf_b]


def job_scl_l64():
    """Round 2: list size 64 (one frame per wavefront in the lane kernel), N=256
    at 0/1/2 dB and N=1024 at 1 dB, bit-reversed Bhattacharyya sets."""
    out = {}
    for tag, (N, K, snrs, frames, seed) in (("N256", (256, 128, (0.0, 1.0, 2.0), 8, 301)),
                                           ("N1024", (1024, 512, (1.0,), 4, 302))):
        d = job_scl(N, K, 64, snrs, frames, seed, "x")[1]
        for k in ("frozen", "llr", "msg", "snr", "scl", "ref_s_per_frame"):
            out[tag + "_" + k] = d[k]
    return "polar_scl_l64.npz", out


ROUND2_JOBS.append(job_scl_l64)


def job_scl_l256():
    """Round 2: list sizes 128 and 256 (one frame per multi-wavefront workgroup)."""
    out = {}
    for tag, (N, K, L, snrs, frames, seed) in (("N256_L128", (256, 128, 128, (0.0, 1.5), 4, 311)),
                                              ("N256_L256", (256, 128, 256, (0.5,), 3, 312)),
                                              ("N1024_L128", (1024, 512, 128, (1.0,), 2, 313))):
        d = job_scl(N, K, L, snrs, frames, seed, "x")[1]
        for k in ("frozen", "llr", "msg", "snr", "scl", "ref_s_per_frame"):
            out[tag + "_" + k] = d[k]
    return "polar_scl_l256.npz", out


ROUND2_JOBS.append(job_scl_l256)


def job_scl_l1024():
    """Round 3: list sizes above 256 (16-bit path slots, one frame per workgroup
    of up to 16 wavefronts): N=64 at L=512 and L=300 (a non-power-of-two list in
    a 512-lane group), N=128 at L=1024, low SNR so the lists fill."""
    out = {}
    for tag, (N, K, L, snrs, frames, seed) in (("N64_L512", (64, 32, 512, (0.0, 1.0), 3, 321)),
                                              ("N64_L300", (64, 40, 300, (0.5,), 3, 322)),
                                              ("N128_L1024", (128, 64, 1024, (0.5,), 2, 323))):
        d = job_scl(N, K, L, snrs, frames, seed, "x")[1]
        for k in ("frozen", "llr", "msg", "snr", "scl", "ref_s_per_frame"):
            out[tag + "_" + k] = d[k]
    return "polar_scl_l1024.npz", out


ROUND2_JOBS.append(job_scl_l1024)


def job_small():
    """Small N, odd list sizes, K extremes, zero LLRs (deterministic cases)."""
    polar, _, channel = _imp()
    cases = []
    np.random.seed(77)
    specs = [(8, 4), (16, 8), (32, 16), (64, 32), (128, 64), (64, 1), (64, 63),
             (128, 100), (32, 5), (256, 77)]
    for (N, K) in specs:
        for fk in ("default", "bhatta"):
            if fk == "default":
                fr = np.asarray(polar.generate_frozen_bits(N, K)[0], np.int64)
            else:
                fr = bitrev_bhatta_frozen(N, K, 1.0)
            enc = polar.PolarEncoder(N, K, frozen_bits=fr)
            llrs = []
            for snr in (0.0, 2.0):
                ch = channel.AWGNChannel(snr_db=snr)
                for _ in range(6):
                    llrs.append(ch.transmit(enc.encode(np.random.randint(0, 2, K)), return_llr=True))
            # exact zeros, tiny values and big magnitudes
            z = llrs[0].copy(); z[::3] = 0.0
            llrs.append(z)
            z = llrs[1].copy(); z[1::2] = -0.0
            llrs.append(z)
            llrs.append(np.zeros(N))
            t = llrs[2].copy(); t[::2] *= 1e-300
            llrs.append(t)
            llrs.append(llrs[3] * 1e3)
            llrs = np.array(llrs)
            rec = dict(N=N, K=K, frozen=fr, llr=llrs)
            rec["sc"] = np.array([polar.SCDecoder(N, K, frozen_bits=fr).decode(l) for l in llrs])
            for L in (1, 2, 3, 4, 5, 6, 8, 16):
                d = polar.SCLDecoder(N, K, list_size=L, frozen_bits=fr)
                rec["scl_L%d" % L] = np.array([d.decode(l.copy()) for l in llrs])
            cases.append(rec)
    out = {}
    for ci, rec in enumerate(cases):
        for k, v in rec.items():
            out["c%d_%s" % (ci, k)] = v
    out["ncases"] = len(cases)
    return "polar_small.npz", out


def job_kat16():
    polar, _, channel = _imp()
    N, K = 16, 8
    enc = polar.PolarEncoder(N, K)
    np.random.seed(42)
    message = np.random.randint(0, 2, K)
    codeword = enc.encode(message)
    ch = channel.AWGNChannel(2.0)
    llr = ch.transmit(codeword, return_llr=True)
    out = dict(N=N, K=K, frozen=np.asarray(enc.frozen_bits, np.int64), msg=message,
               codeword=codeword, llr=llr)
    for L in (1, 2, 4, 8):
        out["scl_L%d" % L] = polar.SCLDecoder(N, K, list_size=L, frozen_bits=enc.frozen_bits).decode(llr)
    out["sc"] = polar.SCDecoder(N, K, frozen_bits=enc.frozen_bits).decode(llr)
    return "polar_kat16.npz", out


def job_bp504():
    _, ldpc, channel = _imp()
    n, k = 504, 252
    enc = ldpc.LDPCEncoder(n, k, dv=3, dc=6, seed=42)
    dec = ldpc.BPDecoder(enc.H, max_iter=20)
    ch = channel.AWGNChannel(snr_db=3.0, seed=42)
    for _ in range(10):
        msg = np.random.randint(0, 2, k)
        dec.decode(ch.transmit(enc.encode(msg), return_llr=True))
    messages = [np.random.randint(0, 2, k) for _ in range(100)]
    cws = [enc.encode(m) for m in messages[:24]]
    llrs = np.array([ch.transmit(c, return_llr=True) for c in cws])
    rp, ci = csr_from_dense(enc.H)
    out = dict(m=enc.H.shape[0], n=n, k=k, row_ptr=rp, col_idx=ci,
               harness_llr=llrs, harness_msg=np.array(messages[:24]), harness_cw=np.array(cws))
    np.random.seed(99)
    extra = np.random.randint(0, 2, (64, k))
    out["enc_msg"] = extra
    out["enc_cw"] = np.array([enc.encode(m) for m in extra])
    bits, its = zip(*[dec.decode(l, return_iterations=True) for l in llrs])
    out["harness_bits"] = np.array(bits)
    out["harness_iters"] = np.array(its)
    # all-zero codeword at several SNRs
    np.random.seed(4242)
    zl, zs = [], []
    for s in (-1.0, 0.5, 1.0, 3.0):
        c = channel.AWGNChannel(snr_db=s)
        for _ in range(12):
            zl.append(c.transmit(np.zeros(n, dtype=int), return_llr=True))
            zs.append(s)
    zl = np.array(zl)
    out["zero_llr"] = zl
    out["zero_snr"] = np.array(zs)
    bits, its = zip(*[dec.decode(l, return_iterations=True) for l in zl])
    out["zero_bits"] = np.array(bits)
    out["zero_iters"] = np.array(its)
    # no early stop, max_iter=5; and max_iter=50 with early stop
    d2 = ldpc.BPDecoder(enc.H, max_iter=5, early_stop=False)
    out["noes5_bits"] = np.array([d2.decode(l) for l in zl[:24]])
    d3 = ldpc.BPDecoder(enc.H, max_iter=50, early_stop=True)
    b3, i3 = zip(*[d3.decode(l, return_iterations=True) for l in zl[:12]])
    out["es50_bits"] = np.array(b3)
    out["es50_iters"] = np.array(i3)
    return "ldpc_bp_504.npz", out


def job_ms504():
    _, ldpc, channel = _imp()
    n = 504
    H = regular_36_H(n, 5)
    rp, ci = csr_from_dense(H)
    np.random.seed(555)
    llr, snr = [], []
    for s in (0.0, 1.0, 2.0):
        c = channel.AWGNChannel(snr_db=s)
        for _ in range(10):
            llr.append(c.transmit(np.zeros(n, dtype=int), return_llr=True))
            snr.append(s)
    llr = np.array(llr)
    out = dict(m=H.shape[0], n=n, row_ptr=rp, col_idx=ci, llr=llr, snr=np.array(snr))
    for norm in (1.0, 0.75):
        d = ldpc.MSDecoder(H, max_iter=20, normalization=norm)
        out["ms_%g" % norm] = np.array([d.decode(l) for l in llr])
    d = ldpc.MSDecoder(H, max_iter=7, normalization=0.75, early_stop=False)
    out["ms_noes7"] = np.array([d.decode(l) for l in llr[:10]])
    d = ldpc.BPDecoder(H, max_iter=20)
    b, i = zip(*[d.decode(l, return_iterations=True) for l in llr])
    out["bp_bits"] = np.array(b)
    out["bp_iters"] = np.array(i)
    return "ldpc_ms_504.npz", out


def job_ms8192():
    _, ldpc, channel = _imp()
    n = 8192
    H = regular_36_H(n, 11)
    rp, ci = csr_from_dense(H)
    np.random.seed(8192)
    llr = []
    for s in (1.0, 1.5):
        c = channel.AWGNChannel(snr_db=s)
        for _ in range(3):
            llr.append(c.transmit(np.zeros(n, dtype=int), return_llr=True))
    llr = np.array(llr)
    d = ldpc.MSDecoder(H, max_iter=20, normalization=0.75)
    t = time.time()
    bits = np.array([d.decode(l) for l in llr])
    return "ldpc_ms_8192.npz", dict(m=H.shape[0], n=n, row_ptr=rp, col_idx=ci, llr=llr,
                                    ms_0_75=bits, ref_s_per_frame=(time.time() - t) / len(llr))


def job_crc():
    polar, _, _ = _imp()
    np.random.seed(31)
    out = {}
    for poly in ("CRC-8", "CRC-16", "CRC-24"):
        data = np.random.randint(0, 2, (16, 40))
        enc = np.array([polar.crc_encode(d, poly) for d in data])
        out[poly.replace("-", "") + "_data"] = data
        out[poly.replace("-", "") + "_enc"] = enc
        out[poly.replace("-", "") + "_check"] = np.array([polar.crc_check(e, poly) for e in enc])
    return "crc.npz", out




def job_ldpc_special():
    """NaN / +-inf / +-0 / denormal channel LLRs through the reference BP (seed-42
    mackay H) and MS (regular H, normalization 0.75): nan_to_num of the BP check
    output, NaN-propagating np.min, np.sign(+-0) = 0."""
    _, ldpc, _ = _imp()
    n, k = 504, 252
    Hb = ldpc.LDPCEncoder(n, k, dv=3, dc=6, seed=42).H
    Hm = regular_36_H(n, 3)
    rng = np.random.RandomState(29)
    B = 12
    llr = 2.0 * (1.0 + 0.8 * rng.randn(B, n)) / 0.64
    for f in range(B):
        idx = rng.choice(n, size=1 + f % 6, replace=False)
        llr[f, idx] = [np.nan, np.inf, -np.inf, 0.0, -0.0, 1e-300][: len(idx)]
    out = dict(n=n, llr=llr)
    for tag, H in (("bp", Hb), ("ms", Hm)):
        rp, ci = csr_from_dense(H)
        out[tag + "_row_ptr"], out[tag + "_col_idx"] = rp, ci
    d = ldpc.BPDecoder(Hb, max_iter=20)
    b, i = zip(*[d.decode(l, return_iterations=True) for l in llr])
    out["bp_bits"], out["bp_iters"] = np.array(b), np.array(i)
    d = ldpc.MSDecoder(Hm, max_iter=20, normalization=0.75)
    out["ms_bits"] = np.array([d.decode(l) for l in llr])
    return "ldpc_special.npz", out


def job_polar_erasures():
    """Erasures (LLR = 0), saturated LLRs, signed zeros and denormals through the
    reference SC and SCL decoders: BEC-like frames (noiseless codewords as +-40
    with 25-50 % erasures), AWGN frames with 20 % erasures, and mixed special
    values (+-inf, +-0, +-1e-300, 1e300 on 1/8 of the positions).  BEC frames
    with +-inf are kept for SC only: there the reference's g forms inf - inf =
    NaN (decoder.py:417), and in SCL NaN path metrics make its list.sort order
    an artefact of CPython's sort algorithm."""
    polar, _, _ = _imp()
    out = {}
    for N, K, L in ((256, 128, 4), (1024, 512, 8)):
        fr = bitrev_bhatta_frozen(N, K)
        llr, msg, _ = _polar_frames(N, K, fr, (2.0,), 16, 77 + N)
        rng = np.random.RandomState(N)
        inf_llr = []
        for f in range(len(llr)):
            kind = f % 4
            sgn = np.where(llr[f] >= 0, 1.0, -1.0)
            if kind == 0:    # BEC, saturated finite
                x = sgn * 40.0
                x[rng.rand(N) < 0.25 + 0.25 * rng.rand()] = 0.0
                llr[f] = x
            elif kind == 1:  # AWGN with 20 % erasures
                llr[f][rng.rand(N) < 0.2] = 0.0
            elif kind == 2:  # mixed specials
                idx = rng.choice(N, size=N // 8, replace=False)
                llr[f][idx] = rng.choice([np.inf, -np.inf, 0.0, -0.0, 1e-300, -1e-300, 1e300], size=len(idx))
            else:            # BEC with +-inf (SC only)
                x = sgn * np.inf
                x[rng.rand(N) < 0.25 + 0.25 * rng.rand()] = 0.0
                inf_llr.append(x)
                llr[f] = sgn * 40.0
        sc = polar.SCDecoder(N, K, frozen_bits=fr)
        scl = polar.SCLDecoder(N, K, list_size=L, frozen_bits=fr)
        inf_llr = np.array(inf_llr)
        out["N%d_frozen" % N] = fr
        out["N%d_llr" % N] = llr
        out["N%d_msg" % N] = msg
        out["N%d_L" % N] = L
        out["N%d_sc" % N] = np.array([sc.decode(l.copy()) for l in llr])
        out["N%d_scl" % N] = np.array([scl.decode(l.copy()) for l in llr])
        out["N%d_inf_llr" % N] = inf_llr
        out["N%d_inf_sc" % N] = np.array([sc.decode(l.copy()) for l in inf_llr])
    return "polar_erasures.npz", out


def job_polar_nan():
    """SCL frames whose path metrics become NaN (round 4):
    +-inf LLRs that meet in a g give inf - inf = NaN (decoder.py:417), the NaN
    LLR gives NaN metrics (:374-406), and list.sort(key=..., reverse=True)
    (:307) orders NaN keys as CPython's algorithm happens to leave them; the final
    np.argmax (:258) picks the first NaN.  Frame kinds: BEC with +-inf and
    erasures, all +-inf (no erasure), AWGN with 1/16 of the positions set to
    +-inf of a random sign, AWGN with a few NaN inputs.  Lists from 1 to 64
    (L = 32 and 64 reach CPython's merge / galloping code: 64 and 128 candidates)."""
    polar, _, _ = _imp()
    out = {}
    cases = [(16, 8, (1, 2, 3, 4, 8)), (64, 32, (2, 4, 8, 16, 32, 48)), (256, 128, (4, 8, 32, 64)),
             (1024, 512, (8, 32))]
    for N, K, Ls in cases:
        fr = bitrev_bhatta_frozen(N, K)
        nfr = 12 if N <= 256 else 4
        llr, msg, _ = _polar_frames(N, K, fr, (1.0,), nfr, 900 + N)
        rng = np.random.RandomState(9000 + N)
        for f in range(len(llr)):
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
        out["N%d_frozen" % N] = fr
        out["N%d_llr" % N] = llr
        out["N%d_msg" % N] = msg
        out["N%d_Ls" % N] = np.array(Ls)
        for L in Ls:
            d = polar.SCLDecoder(N, K, list_size=L, frozen_bits=fr)
            out["N%d_L%d" % (N, L)] = np.array([d.decode(l.copy()) for l in llr])
    return "polar_nan.npz", out


def job_scl_l2048():
    """Round 4: list sizes above 1024 (the exact single-workgroup decoder):
    N=64 at L=2048 and N=32 at L=1500 (a non-power-of-two list), low SNR so the
    lists fill."""
    out = {}
    for tag, (N, K, L, snrs, frames, seed) in (("N64_L2048", (64, 32, 2048, (0.0,), 2, 331)),
                                              ("N32_L1500", (32, 16, 1500, (0.5,), 3, 332))):
        d = job_scl(N, K, L, snrs, frames, seed, "x")[1]
        for k in ("frozen", "llr", "msg", "snr", "scl", "ref_s_per_frame"):
            out[tag + "_" + k] = d[k]
    return "polar_scl_l2048.npz", out


def single_extreme_frames(N, fr, llr, rng):
    """Round 6: frames with exactly ONE infinite or huge
    channel LLR, the case the tree kernel keeps on its fast path (no g can meet
    two infinities, so no NaN metric; paths can still reach -inf metrics and tie
    there).  Kinds cycle with the frame index: the value, the sign relative to
    the noisy LLR it replaces (+1 agrees, -1 contradicts) and the erasure
    fraction (LLR 0) added around it.  The channel position alternates between
    an index of the frozen set and one of the information set."""
    kinds = [(np.inf, +1, 0.0), (np.inf, -1, 0.0), (1e300, -1, 0.0), (1.5e308, +1, 0.0),
             (np.inf, +1, 0.2), (np.inf, -1, 0.4), (1e300, +1, 0.3), (1.5e308, -1, 0.25)]
    info = np.setdiff1d(np.arange(N), fr)
    out = llr.copy()
    pos = np.zeros(len(llr), np.int64)
    for f in range(len(llr)):
        val, rel, er = kinds[f % len(kinds)]
        x = out[f]
        if er:
            x[rng.rand(N) < er] = 0.0
        p = int(rng.choice(fr if (f // len(kinds)) % 2 == 0 else info))
        s = 1.0 if x[p] >= 0 else -1.0
        x[p] = s * rel * val
        pos[f] = p
    return out, pos


def job_polar_single_inf():
    """Reference SCL decodes of single-extreme-input frames (single_extreme_frames):
    N=1024 K=512 at L=8 and L=32 (16 frames each, the same frames), N=2048 K=1024
    and N=4096 K=2048 at L=8 (8 frames each), 1 dB, bit-reversed Bhattacharyya sets.
    Semantics: decoder.py:306-307 (stable sort of -inf ties), :374-406 (metrics
    of +-inf LLRs), :412-417 (g with one infinite operand)."""
    polar, _, _ = _imp()
    out = {}
    for N, K, Ls, nfr in ((1024, 512, (8, 32), 16), (2048, 1024, (8,), 8), (4096, 2048, (8,), 8)):
        fr = bitrev_bhatta_frozen(N, K)
        llr, msg, _ = _polar_frames(N, K, fr, (1.0,), nfr, 1600 + N // 256)
        llr, pos = single_extreme_frames(N, fr, llr, np.random.RandomState(1700 + N // 256))
        out["N%d_frozen" % N] = fr
        out["N%d_llr" % N] = llr
        out["N%d_msg" % N] = msg
        out["N%d_pos" % N] = pos
        out["N%d_Ls" % N] = np.array(Ls)
        for L in Ls:
            d = polar.SCLDecoder(N, K, list_size=L, frozen_bits=fr)
            out["N%d_L%d" % (N, L)] = np.array([d.decode(l.copy()) for l in llr])
    return "polar_single_inf.npz", out


def _public_names():
    """{module: [public top-level names]} and {module.Class: [public methods]}
    of the reference's src/ packages, read from the files' syntax trees."""
    import ast
    mods, meths = {}, {}
    src = os.path.join(REF, "src")
    for pkg in ("polar", "ldpc", "channel", "utils", "lib_wrappers"):
        for f in sorted(os.listdir(os.path.join(src, pkg))):
            if not f.endswith(".py") or f == "__init__.py":
                continue
            tree = ast.parse(open(os.path.join(src, pkg, f), encoding="utf-8").read())
            mod = "%s.%s" % (pkg, f[:-3])
            mods[mod] = [n.name for n in tree.body
                         if isinstance(n, (ast.FunctionDef, ast.ClassDef)) and not n.name.startswith("_")]
            for n in tree.body:
                if isinstance(n, ast.ClassDef):
                    meths[mod + "." + n.name] = [m.name for m in n.body
                                                 if isinstance(m, ast.FunctionDef) and not m.name.startswith("_")]
    return mods, meths


def job_host_api():
    """Round 6: outputs of every host-side function and
    method the reference's packages export (construction incl. the GA and
    default methods, transforms, CRC, encoders, H builders, Tanner graph,
    syndrome, channels with seeds, metrics), plus the public name inventory,
    so tests/test_host_api.py can check the drop-in modules name by name."""
    polar, ldpc, channel = _imp()
    import polar.construction as PC
    import polar.utils as PU
    import ldpc.matrix as LM
    import ldpc.utils as LU
    import utils.metrics as UM
    out = {}
    mods, meths = _public_names()
    out["names_json"] = np.array(json.dumps({"modules": mods, "methods": meths}))
    # polar construction: all three methods over sizes, rates and design SNRs
    for N in (8, 16, 64, 256, 1024, 4096):
        for K in sorted({1, N // 4, N // 2, (3 * N) // 4, N - 1}):
            for snr in (-2.0, 0.0, 2.0, 5.0):
                for meth in ("bhattacharyya", "gaussian_approximation", "default"):
                    fr, info = PC.construct_polar_code(N, K, meth, snr)
                    key = "cpc_%d_%d_%g_%s" % (N, K, snr, meth)
                    out[key + "_frozen"], out[key + "_info"] = fr, info
        for snr in (-2.0, 0.0, 3.0, 6.0):
            out["bb_%d_%g" % (N, snr)] = PC.bhattacharyya_bounds(N, snr)
            out["ga_%d_%g" % (N, snr)] = PC.gaussian_approximation(N, snr)
            out["cap_%d_%g" % (N, snr)] = PC.calculate_channel_capacities(N, snr)
    # polar utils
    rng = np.random.RandomState(606)
    for n in (0, 1, 3, 10):
        out["brev_%d" % n] = np.array([PU.bit_reverse(i, n) for i in range(1 << n)])
        arr = rng.randn(1 << n)
        out["brevarr_%d_in" % n], out["brevarr_%d" % n] = arr, PU.bit_reverse_array(arr, n)
    for N, K in ((16, 8), (64, 20), (256, 128)):
        cp = rng.rand(N)
        fr, info = PU.generate_frozen_bits(N, K, cp)
        out["gfb_cp_%d_%d_in" % (N, K)], out["gfb_cp_%d_%d_frozen" % (N, K)] = cp, fr
        out["gfb_cp_%d_%d_info" % (N, K)] = info
        fr, info = PU.generate_frozen_bits(N, K)
        out["gfb_%d_%d_frozen" % (N, K)], out["gfb_%d_%d_info" % (N, K)] = fr, info
    for N in (1, 2, 16, 128):
        for tag, u in (("bin", rng.randint(0, 2, N)), ("int", rng.randint(0, 5, N)),
                       ("flt", rng.randint(0, 2, N).astype(float))):
            out["pt_%d_%s_in" % (N, tag)] = u
            out["ptr_%d_%s" % (N, tag)] = PU.polar_transform_recursive(u.copy())
            out["pti_%d_%s" % (N, tag)] = PU.polar_transform_iterative(u.copy())
    # polar encoder, with and without CRC
    for N, K, crc, poly in ((16, 8, False, "CRC-8"), (64, 32, True, "CRC-8"), (256, 128, True, "CRC-16"),
                            (1024, 512, True, "CRC-24"), (128, 40, False, "CRC-8")):
        enc = polar.PolarEncoder(N, K, use_crc=crc, crc_polynomial=poly)
        msgs = rng.randint(0, 2, (4, enc.K_data))
        key = "penc_%d_%d_%d_%s" % (N, K, int(crc), poly)
        out[key + "_msg"] = msgs
        out[key + "_cw"] = np.array([enc.encode(m) for m in msgs])
        out[key + "_info"] = np.asarray(enc.get_info_bits_positions())
        out[key + "_frozen"] = np.asarray(enc.get_frozen_bits_positions())
        out[key + "_rate"] = np.array(enc.get_code_rate())
    # LDPC matrices, encoder, utils
    for (n, k, dv, dc, seed) in ((504, 252, 3, 6, 42), (96, 48, 3, 6, 7), (120, 60, 3, 6, None), (60, 20, 2, 3, 3)):
        key = "ldpc_%d_%d_%d_%d_%s" % (n, k, dv, dc, seed)
        np.random.seed(1234)
        H = LM.generate_ldpc_matrix(n, k, "mackay", dv, dc, seed)
        out[key + "_H"] = H
        np.random.seed(1234)
        enc = ldpc.LDPCEncoder(n, k, dv=dv, dc=dc, seed=seed)
        out[key + "_encH"] = enc.get_parity_check_matrix()
        out[key + "_rate"] = np.array(enc.get_code_rate())
        out[key + "_direct"] = np.array(enc.use_direct_solving)
        msgs = rng.randint(0, 2, (6, k))
        cws = np.array([enc.encode(m) for m in msgs])
        out[key + "_msg"], out[key + "_cw"] = msgs, cws
        out[key + "_valid"] = np.array([bool(enc.verify_codeword(c)) for c in cws])
        G, P = LM.create_systematic_generator(enc.H)
        out[key + "_hasG"] = np.array(G is not None)
        if G is not None:
            out[key + "_G"] = G
        out[key + "_rank"] = np.array(LM.check_matrix_rank(enc.H))
        out[key + "_girth"] = np.array(LM.calculate_girth(enc.H))
        cn, vn = LU.create_tanner_graph(enc.H)
        out[key + "_tanner_c"] = np.array(json.dumps([list(map(int, c)) for c in cn]))
        out[key + "_tanner_v"] = np.array(json.dumps([list(map(int, v)) for v in vn]))
        rx = cws ^ (rng.rand(*cws.shape) < 0.03)
        out[key + "_rx"] = rx
        out[key + "_syn"] = np.array([LU.calculate_syndrome(enc.H, r) for r in rx])
        out[key + "_synok"] = np.array([bool(LU.check_syndrome(enc.H, r)) for r in rx])
        out[key + "_errs"] = np.array([LU.count_errors(c, r) for c, r in zip(cws, rx)])
        out[key + "_ham"] = np.array([LU.hamming_distance(c, r) for c, r in zip(cws, rx)])
    for (n, k, dv) in ((24, 12, 3), (60, 30, 2), (50, 10, 4)):
        out["peg_%d_%d_%d" % (n, k, dv)] = LM.peg_construction(n, k, dv)
    np.random.seed(77)
    out["ldpc_random_H"] = LM.generate_ldpc_matrix(40, 20, "random", seed=5)
    # channels (seeded: the global legacy stream)
    bits = rng.randint(0, 2, 200)
    out["ch_bits"] = bits
    for snr in (-1.0, 0.0, 2.5):
        ch = channel.AWGNChannel(snr, seed=11)
        out["awgn_%g_llr" % snr] = ch.transmit(bits, return_llr=True)
        out["awgn_%g_sym" % snr] = ch.transmit(bits, return_llr=False)
        out["awgn_%g_mod" % snr] = ch.modulate_bpsk(bits)
        out["awgn_%g_hard" % snr] = ch.demodulate_bpsk_hard(ch.add_noise(ch.modulate_bpsk(bits)))
        out["awgn_%g_cap" % snr] = np.array(ch.get_capacity())
        out["awgn_%g_sigma" % snr] = np.array(ch.noise_std)
        ch.update_snr(snr + 1.0)
        out["awgn_%g_sigma_upd" % snr] = np.array(ch.noise_std)
        out["awgn_%g_llr_upd" % snr] = ch.symbols_to_llr(ch.modulate_bpsk(bits) * 0.7)
    for p in (0.0, 0.05, 0.3):
        out["bsc_%g" % p] = channel.BSCChannel(p, seed=12).transmit(bits)
    for snr in (0.0, 3.0):
        fc = channel.RayleighFadingChannel(snr, seed=13)
        out["ray_%g_llr" % snr] = fc.transmit(bits, return_llr=True)
        out["ray_%g_sym" % snr] = fc.transmit(bits, return_llr=False)
    # metrics
    a, b = rng.randint(0, 2, 500), rng.randint(0, 2, 500)
    out["met_a"], out["met_b"] = a, b
    out["met_ber"] = np.array(UM.calculate_ber(a, b))
    out["met_fer"] = np.array(UM.calculate_fer(list(a.reshape(50, 10)), list(b.reshape(50, 10))))
    out["met_thr"] = np.array([UM.calculate_throughput(12345, t) for t in (0.0, -1.0, 0.37, 2.0)])
    out["met_wilson"] = np.array([UM.calculate_ber_with_confidence(e, t, c) for e, t, c in
                                  ((0, 1000, 0.95), (17, 1000, 0.95), (999, 1000, 0.9), (5, 0, 0.95),
                                   (400, 100000, 0.99))])
    out["met_snr"] = np.array([UM.calculate_snr_from_ebn0(e, r) for e in (-1.0, 2.0) for r in (0.25, 0.5, 0.9)])
    out["met_ebn0"] = np.array([UM.calculate_ebn0_from_snr(e, r) for e in (-1.0, 2.0) for r in (0.25, 0.5, 0.9)])
    return "host_api.npz", out


JOBS = [job_scl4096_l8, job_scl1024_l8, job_ms8192, job_scl1024_l32, job_bp504,
        job_sc1024, job_ms504, job_small, job_p1, job_kat16, job_crc, job_ldpc_special, job_polar_erasures
        ] + ROUND2_JOBS + [job_polar_nan, job_scl_l2048, job_polar_single_inf, job_host_api]


def _run(fn):
    t = time.time()
    name, out = fn()
    np.savez_compressed(os.path.join(HERE, name), **out)
    return name, time.time() - t


def main():
    global REF
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default=REF)
    ap.add_argument("--only", default=None)
    ap.add_argument("-j", type=int, default=6)
    a = ap.parse_args()
    REF = a.ref
    jobs = [j for j in JOBS if a.only is None or j.__name__ in a.only.split(",")]
    with Pool(a.j) as p:
        for name, dt in p.imap_unordered(_run, jobs):
            print("wrote %s in %.1fs" % (name, dt), flush=True)
    meta = dict(numpy=np.__version__, python=platform.python_version(),
                machine=platform.machine(), processor=platform.processor(),
                generated=time.strftime("%Y-%m-%d %H:%M:%S"),
                note="outputs produced by the reference implementation at " + REF)
    with open(os.path.join(HERE, "META.json"), "w") as f:
        json.dump(meta, f, indent=1)


if __name__ == "__main__":
    main()
