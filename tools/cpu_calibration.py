"""Calibrate bench.py's CPU baseline (oracle/refnumpy.py) against the reference.

Build container only (it imports the reference read-only from /root/reference;
the GPU box has no reference).  On ONE pinned core, for the same frames of the
headline configuration (N=1024 K=512 SCL L=8, the bench's frozen set, 3 dB):
  * the reference's own SCLDecoder.decode (src/polar/decoder.py:225-262), timed
    frame by frame as benchmarks/throughput_test.py:230-237 times its decoder;
  * refnumpy.scl_frame (the restatement bench.py's cpu_baseline runs);
  * the C oracle (oracle/refcpu.c) on the same frames, one thread;
and checks that all three give the same bits.  Also records the CPU model, so
the GPU box's figure (its host CPU, in bench.py's cpu_baseline.host) can be
compared with BASELINE.md's survey-container number.

usage: python tools/cpu_calibration.py [--frames 8] [--core 0] [--out profiles/r05/cpu_calibration.json]
"""
import argparse
import json
import os
import platform
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference"


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or "unknown"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=8)
    ap.add_argument("--core", type=int, default=0)
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "r05", "cpu_calibration.json"))
    ap.add_argument("--default-set", action="store_true",
                    help="the reference's default frozen set (generate_frozen_bits), as BASELINE.md's figure")
    a = ap.parse_args()
    os.sched_setaffinity(0, {a.core})
    sys.dont_write_bytecode = True
    sys.path.insert(0, ROOT)
    from oracle import oracle, refnumpy
    from polarcode_and_ldpc_amd.polar import construct_frozen_set
    from polarcode_and_ldpc_amd.polar.encoder import PolarEncoder
    from polarcode_and_ldpc_amd.channel import AWGNChannel

    N, K, L, snr = 1024, 512, 8, 3.0
    if a.default_set:
        from polarcode_and_ldpc_amd.polar.utils import generate_frozen_bits
        fr = np.asarray(generate_frozen_bits(N, K)[0])
    else:
        fr = construct_frozen_set(N, K, 2.0)
    enc = PolarEncoder(N, K, frozen_bits=fr)
    ch = AWGNChannel(snr_db=snr, seed=42)
    rng = np.random.RandomState(7)
    llrs = np.array([ch.transmit(enc.encode(rng.randint(0, 2, K)), return_llr=True) for _ in range(a.frames)])
    info = np.setdiff1d(np.arange(N), fr)
    fset = set(int(x) for x in fr)

    sys.path.insert(0, os.path.join(REF, "src"))
    import polar as refpolar  # the reference package, read-only
    rdec = refpolar.SCLDecoder(N, K, list_size=L, frozen_bits=fr)
    rdec.decode(llrs[0])  # warm-up (throughput_test.py:200-205 warms its decoder)

    res = {}
    t0 = time.perf_counter()
    ref_bits = [np.asarray(rdec.decode(l)) for l in llrs]
    res["reference_SCLDecoder"] = (time.perf_counter() - t0) / a.frames
    refnumpy.scl_frame(llrs[0], N, L, fset, info)  # warm-up
    t0 = time.perf_counter()
    port_bits = [np.asarray(refnumpy.scl_frame(l, N, L, fset, info)) for l in llrs]
    res["refnumpy_scl_frame"] = (time.perf_counter() - t0) / a.frames
    t0 = time.perf_counter()
    c_bits = oracle.scl_decode(N, L, fr, llrs, threads=1)
    res["oracle_refcpu_c"] = (time.perf_counter() - t0) / a.frames

    same = all(np.array_equal(np.asarray(r).astype(np.int64), np.asarray(p).astype(np.int64))
               for r, p in zip(ref_bits, port_bits)) and np.array_equal(np.array(ref_bits).astype(np.int64), c_bits)
    out = dict(config="SCL N=1024 K=512 L=8, %s, 3 dB" % ("the reference's default frozen set (generate_frozen_bits)"
                                                          if a.default_set else "bench frozen set (construct_frozen_set 2 dB)"),
               frames=a.frames, core=a.core, cpu_model=cpu_model(), python=platform.python_version(),
               numpy=np.__version__, seconds_per_frame={k: round(v, 5) for k, v in res.items()},
               refnumpy_over_reference=round(res["refnumpy_scl_frame"] / res["reference_SCLDecoder"], 3),
               bits_identical=bool(same),
               info_mbps_single_core={k: round(K / v / 1e6, 6) for k, v in res.items()})
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
