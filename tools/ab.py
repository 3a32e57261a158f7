"""A/B timing of experimental builds of libpolarldpc.so (diagnostic).

usage: python tools/ab.py [--cases polar_l8,ldpc_bp] [--reps 3] LIB[@VAR=VAL,...] [...]

Each LIB is loaded in its own process (PL_LIB_PATH); libs alternate `reps`
times.  Per case: median kernel time over 10 launches (HIP events, after 2
warmups) and a digest of the decoded bits, which must equal the first LIB's.
Build a variant with e.g.
  make -C polarcode_and_ldpc_amd/csrc OUT=$PWD/build/lib_x.so OBJDIR=$PWD/build/obj_x EXTRA=-DPL_EXP_X
"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CASES = ("enc_1024", "enc_4096", "awgn_1024", "awgn_8192", "lane_2048_l32", "lane_1024_l64", "lane_512_l4", "lane_8192_l8", "lane_1024_l128", "polar_l8_128k", "polar_l32_64k", "polar_4096_128k", "polar_2048", "polar_l16", "polar_sc128", "polar_sc512", "polar_sc2048", "polar_sc4096", "polar_l8", "ldpc_bp", "ldpc_bp_valid", "polar_l32", "polar_4096", "ms_8192", "ms_8192_es", "ms_504", "polar_sc", "polar_sc_def", "polar_sc_def_128k", "polar_sc_def_256k",
         "polar_sc256", "cascl_l32", "polar_4096_8k", "polar_2048_16k", "polar_l8_16k", "polar_l32_4k",
         "polar_l16_8k", "polar_l4_32k", "polar_512_16k", "polar_512_l16_8k")


def worker(cases):
    sys.path.insert(0, ROOT)
    import numpy as np
    import torch
    from polarcode_and_ldpc_amd import _native
    from polarcode_and_ldpc_amd.channel import AWGNChannel
    from polarcode_and_ldpc_amd.polar import construct_frozen_set
    torch.cuda.set_device(0)
    res = {}

    def timeit(fn):
        for _ in range(2):
            fn()
        ts = []
        for _ in range(10):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            fn()
            b.record()
            torch.cuda.synchronize()
            ts.append(a.elapsed_time(b))
        return float(np.median(ts))

    def digest(t):
        x = t.to(torch.int64).flatten()
        w = torch.arange(1, x.numel() + 1, device=x.device, dtype=torch.int64) % 1000003
        return int((x * w).sum().item())

    for case in cases:
        if case.startswith("polar") or case.startswith("lane"):
            N, L, B, snr = {"polar_l8": (1024, 8, 65536, 3.0), "polar_l32": (1024, 32, 16384, 1.0), "polar_l32_64k": (1024, 32, 65536, 1.0),
                            "polar_l8_128k": (1024, 8, 131072, 3.0),
                            "lane_2048_l32": (2048, 32, 16384, 1.0), "lane_1024_l64": (1024, 64, 8192, 1.0),
                            "lane_512_l4": (512, 4, 65536, 2.0), "lane_8192_l8": (8192, 8, 8192, 2.0),
                            "lane_1024_l128": (1024, 128, 4096, 1.0),
                            "polar_4096_128k": (4096, 8, 131072, 3.0), "polar_l16": (1024, 16, 32768, 1.0), "polar_2048": (2048, 8, 32768, 1.0),
                            "polar_4096": (4096, 8, 16384, 1.0), "polar_sc": (1024, 0, 65536, 3.0),
                            "polar_4096_8k": (4096, 8, 8192, 1.0), "polar_2048_16k": (2048, 8, 16384, 1.0),
                            "polar_l8_16k": (1024, 8, 16384, 3.0), "polar_l32_4k": (1024, 32, 4096, 1.0),
                            "polar_l16_8k": (1024, 16, 8192, 1.0), "polar_l4_32k": (1024, 4, 32768, 2.0),
                            "polar_512_16k": (512, 8, 16384, 2.0), "polar_512_l16_8k": (512, 16, 8192, 1.0),
                            "polar_sc_def": (1024, 0, 65536, 3.0), "polar_sc_def_128k": (1024, 0, 131072, 3.0), "polar_sc_def_256k": (1024, 0, 262144, 3.0), "polar_sc256": (256, 0, 65536, 3.0),
                            "polar_sc128": (128, 0, 65536, 3.0), "polar_sc512": (512, 0, 65536, 3.0),
                            "polar_sc2048": (2048, 0, 32768, 3.0), "polar_sc4096": (4096, 0, 32768, 3.0)}[case]
            K = N // 2
            if case.startswith("polar_sc_def"):  # the reference's default set (generate_frozen_bits)
                from polarcode_and_ldpc_amd.polar import SCDecoder
                fr = SCDecoder(N, K).frozen_bits
            else:
                fr = construct_frozen_set(N, K, 2.0)
            mask = np.zeros(N, np.uint8)
            mask[fr] = 1
            plan = _native.polar_plan(N, K, mask, L)
            msg = torch.empty((B, K), dtype=torch.uint8, device="cuda")
            _native.random_bits(42, 0, msg)
            cw = torch.empty((B, N), dtype=torch.uint8, device="cuda")
            _native.polar_encode(plan, msg, cw)
            llr = AWGNChannel(snr).llr_batch_device(cw, N, B, seed=42)
            out = torch.empty((B, K), dtype=torch.uint8, device="cuda")
            ms = timeit(lambda: plan.decode(llr, out))
            res[case] = dict(ms=ms, digest=digest(out), errors=int((out != msg).any(dim=1).sum().item()))
        elif case == "cascl_l32":  # the bench's cascl_l32 key: CRC-8 messages, seed 44, 1 dB
            from polarcode_and_ldpc_amd.polar import CASCLDecoder
            from polarcode_and_ldpc_amd.polar.utils import CRC_POLYNOMIALS
            N, K, L, B = 1024, 512, 32, 65536
            fr = construct_frozen_set(N, K, 2.0)
            dec = CASCLDecoder(N, K, list_size=L, frozen_bits=fr, crc_polynomial="CRC-8")
            msg = torch.empty((B, K), dtype=torch.uint8, device="cuda")
            _native.random_bits(44, 0, msg)
            _native.crc_append(msg, K - 8, 8, CRC_POLYNOMIALS["CRC-8"])
            cw = torch.empty((B, N), dtype=torch.uint8, device="cuda")
            _native.polar_encode(dec.plan, msg, cw)
            llr = AWGNChannel(1.0).llr_batch_device(cw, N, B, seed=44)
            out = torch.empty((B, K), dtype=torch.uint8, device="cuda")
            ms = timeit(lambda: dec.plan.decode(llr, out))
            res[case] = dict(ms=ms, digest=digest(out))
        elif case == "ldpc_bp_valid":
            from polarcode_and_ldpc_amd.ldpc import BPDecoder, LDPCEncoder
            enc = LDPCEncoder(504, 252, dv=3, dc=6, seed=42)
            plan = BPDecoder(enc.H, max_iter=20).plan
            B = 65536
            llr = AWGNChannel(3.0).llr_batch_device(None, 504, B, seed=4243)
            out = torch.empty((B, 504), dtype=torch.uint8, device="cuda")
            its = torch.empty((B,), dtype=torch.int32, device="cuda")
            ms = timeit(lambda: plan.decode(llr, out, its))
            res[case] = dict(ms=ms, digest=digest(out) ^ digest(its), mean_it=float(its.double().mean().item()))
        elif case == "ldpc_bp":
            from polarcode_and_ldpc_amd.ldpc import BPDecoder, LDPCEncoder
            enc = LDPCEncoder(504, 252, dv=3, dc=6, seed=42)
            plan = BPDecoder(enc.H, max_iter=20).plan
            B = 65536
            base = enc.encode_batch(np.random.RandomState(42).randint(0, 2, (4096, 252)))
            cw = torch.from_numpy(np.tile(base, (B // 4096, 1)).astype(np.uint8)).cuda()
            llr = AWGNChannel(3.0).llr_batch_device(cw, 504, B, seed=4242)
            out = torch.empty((B, 504), dtype=torch.uint8, device="cuda")
            its = torch.empty((B,), dtype=torch.int32, device="cuda")
            ms = timeit(lambda: plan.decode(llr, out, its))
            res[case] = dict(ms=ms, digest=digest(out) ^ digest(its))
        elif case.startswith("enc_"):
            N = int(case.split("_")[1])
            K, B = N // 2, 65536 if N <= 1024 else 16384
            fr = construct_frozen_set(N, K, 2.0)
            mask = np.zeros(N, np.uint8)
            mask[fr] = 1
            plan = _native.polar_plan(N, K, mask, 8)
            msg = torch.empty((B, K), dtype=torch.uint8, device="cuda")
            _native.random_bits(3, 0, msg)
            cw = torch.empty((B, N), dtype=torch.uint8, device="cuda")
            ms = timeit(lambda: _native.polar_encode(plan, msg, cw))
            res[case] = dict(ms=ms, digest=digest(cw))
        elif case.startswith("awgn_"):
            n = int(case.split("_")[1])
            B = 65536 if n <= 1024 else 16384
            cw = torch.empty((B, n), dtype=torch.uint8, device="cuda")
            _native.random_bits(5, 0, cw)
            ch = AWGNChannel(1.0)
            llr = torch.empty((B, n), dtype=torch.float64, device="cuda")
            ms = timeit(lambda: ch.llr_batch_device(cw, n, B, seed=9, out=llr))
            res[case] = dict(ms=ms, digest=int(llr.view(torch.int64).sum().item()))
        elif case == "ms_8192_es":  # the bench's long_ms key: early stop at 1.5 dB, all-zero codeword
            from polarcode_and_ldpc_amd.ldpc import MSDecoder
            from polarcode_and_ldpc_amd.ldpc.matrix import regular_construction
            H = regular_construction(8192, 3, 6, seed=11)
            plan = MSDecoder(H, max_iter=20, early_stop=True).plan
            B = 16384
            llr = AWGNChannel(1.5).llr_batch_device(None, 8192, B, seed=47)
            out = torch.empty((B, 8192), dtype=torch.uint8, device="cuda")
            its = torch.empty((B,), dtype=torch.int32, device="cuda")
            ms = timeit(lambda: plan.decode(llr, out, its))
            res[case] = dict(ms=ms, digest=digest(out) ^ digest(its), mean_it=float(its.double().mean().item()))
        elif case == "ms_504":  # min-sum, (3,6)-regular n=504 (ldpc_reg_kernel; the seed-42 H has degree-1 checks), early stop, 1 dB
            from polarcode_and_ldpc_amd.ldpc import MSDecoder
            from polarcode_and_ldpc_amd.ldpc.matrix import regular_construction
            plan = MSDecoder(regular_construction(504, 3, 6, seed=5), max_iter=20, early_stop=True).plan
            B = 65536
            llr = AWGNChannel(1.0).llr_batch_device(None, 504, B, seed=48)
            out = torch.empty((B, 504), dtype=torch.uint8, device="cuda")
            its = torch.empty((B,), dtype=torch.int32, device="cuda")
            ms = timeit(lambda: plan.decode(llr, out, its))
            res[case] = dict(ms=ms, digest=digest(out) ^ digest(its), mean_it=float(its.double().mean().item()))
        elif case == "ms_8192":
            from polarcode_and_ldpc_amd.ldpc import MSDecoder
            from polarcode_and_ldpc_amd.ldpc.matrix import regular_construction
            H = regular_construction(8192, 3, 6, seed=11)
            plan = MSDecoder(H, max_iter=20, early_stop=False).plan
            B = 16384
            llr = AWGNChannel(1.0).llr_batch_device(None, 8192, B, seed=46)  # many frames fail: nonzero bits
            out = torch.empty((B, 8192), dtype=torch.uint8, device="cuda")
            its = torch.empty((B,), dtype=torch.int32, device="cuda")
            ms = timeit(lambda: plan.decode(llr, out, its))
            res[case] = dict(ms=ms, digest=digest(out))
    print(json.dumps(res), flush=True)


def main():
    args = sys.argv[1:]
    if args and args[0] == "--worker":
        worker(args[1].split(","))
        return
    cases, reps = ["polar_l8", "ldpc_bp"], 3
    libs = []
    i = 0
    while i < len(args):
        if args[i] == "--cases":
            cases = args[i + 1].split(",")
            i += 2
        elif args[i] == "--reps":
            reps = int(args[i + 1])
            i += 2
        else:
            libs.append(args[i])
            i += 1
    table = {lib: {c: [] for c in cases} for lib in libs}
    ref = {}
    for r in range(reps):
        for lib in libs:
            path, _, extra = lib.partition("@")
            env = dict(os.environ, PL_LIB_PATH=os.path.abspath(path))
            for kv in filter(None, extra.split(",")):
                k, _, v = kv.partition("=")
                env[k] = v
            p = subprocess.run([sys.executable, os.path.abspath(__file__), "--worker", ",".join(cases)], env=env,
                               capture_output=True, text=True, timeout=600)
            if p.returncode != 0:
                print("FAIL", lib, p.stderr[-3000:], flush=True)
                sys.exit(p.returncode)
            res = json.loads(p.stdout.strip().splitlines()[-1])
            for c, v in res.items():
                table[lib][c].append(v["ms"])
                if c not in ref:
                    ref[c] = v["digest"]
                elif v["digest"] != ref[c]:
                    print("MISMATCH", os.path.basename(lib), c, flush=True)
            print("rep %d %s %s" % (r, os.path.basename(lib), json.dumps(res)), flush=True)
    print("%-40s %s" % ("lib", "  ".join("%12s" % c for c in cases)))
    for lib in libs:
        print("%-40s %s" % (os.path.relpath(lib.partition("@")[0], ROOT)[-40:], "  ".join("%12.3f" % min(table[lib][c]) for c in cases)))


if __name__ == "__main__":
    main()
