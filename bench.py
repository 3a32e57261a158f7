#!/usr/bin/env python3
"""Benchmark: decoded info-Mbps of the MI355X decoders (BASELINE.json metric).

Headline (`value`): Polar N=1024 K=512 SCL L=8, 65 536 AWGN frames per GPU
(BASELINE.json configs[1]); a step = one batched decode of the resident LLR
matrix + on-device error count (+ one all-reduce of the counters when N > 1).
Secondary (`ldpc`): LDPC (504,252) BP max_iter=20 (configs[2]) on the
reference harness's frames (benchmarks/throughput_test.py:285-315: its encoder's
invalid codewords, so every frame runs all 20 iterations); `ldpc.valid_codewords`
is the same decode on valid (all-zero) codewords with early stop.
`end_to_end`: the polar Monte-Carlo step with fresh device messages, encoding and
AWGN inside the timed region (SURVEY §8 d "end-to-end MC").

info-Mbps = frames * K_info / t / 1e6 (throughput_test.py:217, :304).
Usage: python bench.py [--gpus N --steps K --warmup W]; N > 1 under torchrun.
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "decoded info-Mbps: polar N=1024 SCL L=8 & LDPC(504,252) BP, 1/2/4/8 GPUs"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def timed_steps(step, steps, warmup, world):
    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    return dt


class KernelTimer:
    """HIP events around the decode launch, on the stream it is launched on."""

    def __init__(self):
        self.pairs = []

    def __call__(self, fn):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        fn()
        e.record()
        self.pairs.append((s, e))

    def reset(self):
        self.pairs = []

    def mean_ms(self):
        torch.cuda.synchronize()
        return float(np.mean([s.elapsed_time(e) for s, e in self.pairs])) if self.pairs else float("nan")


def load_traffic(name):
    p = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if not os.path.exists(p):
        return None
    try:
        t = json.load(open(p)).get(name)
        return None if t is None else float(t["bytes_per_launch"])
    except Exception:
        return None


def load_valu(name):
    p = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        return float(json.load(open(p))[name]["valu_instr_per_launch"])
    except Exception:
        return None


def _valu_rate(roof, name, cus, clock_ghz=2.4):
    """VALU issue against its ceiling: SQ_INSTS_VALU (PMC, per launch) over the
    live kernel time.  A CU issues at most one wave64 fp64 VALU instruction per
    cycle (4 SIMDs, 4 cycles each), so peak = CUs x clock."""
    v = load_valu(name)
    if v is None:
        return
    rate = v / (roof["kernel_ms"] / 1e3) / 1e9  # G wave-instructions / s
    peak = cus * clock_ghz
    roof["valu"] = dict(instr_per_launch=v, achieved=rate, peak=peak, unit="G wave-instr/s (fp64 VALU)",
                        frac=rate / peak, source="profiles/pmc_traffic.json (SQ_INSTS_VALU)")


def traffic_source(name):
    p = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        return json.load(open(p))[name]["source"]
    except Exception:
        return None


def _traffic_rate(roof):
    """Measured HBM-side bytes per launch (PMC) over the live kernel time: the
    bandwidth the kernel actually draws, beside the algorithmic-bytes roofline."""
    if roof.get("traffic"):
        gbs = roof["traffic"] / (roof["kernel_ms"] / 1e3) / 1e9
        roof["traffic_GBps"] = gbs
        roof["traffic_frac"] = gbs / HBM_PEAK_GBS


def cpu_threads():
    n = len(os.sched_getaffinity(0))
    return max(1, min(16, n))


def bench_polar(args, rank, world):
    from polarcode_and_ldpc_amd import _native
    from polarcode_and_ldpc_amd.channel import AWGNChannel
    from polarcode_and_ldpc_amd.polar import SCLDecoder, construct_frozen_set

    N, K, L, B = 1024, 512, args.list_size, args.batch
    frozen = construct_frozen_set(N, K, 2.0)
    dec = SCLDecoder(N, K, list_size=L, frozen_bits=frozen)
    plan = dec.plan
    off = rank * B
    msg = torch.empty((B, K), dtype=torch.uint8, device="cuda")
    _native.random_bits(42, off, msg)
    cw = torch.empty((B, N), dtype=torch.uint8, device="cuda")
    _native.polar_encode(plan, msg, cw)
    llr = AWGNChannel(args.snr).llr_batch_device(cw, N, B, seed=42, frame_offset=off)
    out = torch.empty((B, K), dtype=torch.uint8, device="cuda")
    counts = torch.zeros(3, dtype=torch.int64, device="cuda")
    kt = KernelTimer()

    sc = torch.zeros(3, dtype=torch.int64, device="cuda")  # this step's counters

    def step():
        kt(lambda: plan.decode(llr, out))
        sc.zero_()
        _native.count_errors(msg, out, K, sc)
        if world > 1:
            dist.all_reduce(sc)
        counts.add_(sc)

    dt = timed_steps(step, args.steps, args.warmup, world)
    kms = kt.mean_ms()  # includes warmup launches; steady state
    kt.reset()
    for _ in range(3):
        kt(lambda: plan.decode(llr, out))
    kms = kt.mean_ms()
    frames = B * world * args.steps
    value = frames * K / dt / 1e6
    bytes_per_frame = 8 * N + K
    achieved = B * bytes_per_frame / (kms / 1e3) / 1e9
    res = dict(value=value, ms_per_step=dt / args.steps * 1e3, kernel_ms=kms, B=B,
               roofline=dict(bound="hbm", achieved=achieved, peak=HBM_PEAK_GBS, unit="GB/s",
                             frac=achieved / HBM_PEAK_GBS, traffic=load_traffic("polar_scl_1024_l8"),
                             traffic_unit="HBM bytes per launch (2*FETCH_SIZE+WRITE_SIZE, rocprofv3 PMC)",
                             traffic_source=traffic_source("polar_scl_1024_l8"),
                             algorithmic_bytes_per_frame=bytes_per_frame, frames_per_launch=B,
                             kernel=("polar_tree_kernel<n=10,LCAP=%d,SCL,F=%d>" % (L, plan.info.fused_top)
                                     if plan.info.reserved == 4 else "polar_lane_kernel (generation %d)"
                                     % plan.info.reserved),
                             kernel_ms=kms),
               plan=dict(lds_bytes=plan.info.lds_bytes, fused_top=plan.info.fused_top))
    _traffic_rate(res["roofline"])
    _valu_rate(res["roofline"], "polar_scl_1024_l8", torch.cuda.get_device_properties(0).multi_processor_count)
    c = counts.cpu().numpy()
    res["ber"] = float(c[0]) / max(1, c[2] * K)
    res["fer"] = float(c[1]) / max(1, c[2])

    if args.skip_extra:
        return res
    # End-to-end Monte Carlo (SURVEY §8 d): each step draws fresh messages,
    # encodes, adds AWGN and decodes on the device, then counts errors.
    ch = AWGNChannel(args.snr)
    e2e_counts = torch.zeros(3, dtype=torch.int64, device="cuda")
    e2e_step_no = [0]
    msg2, cw2, out2 = torch.empty_like(msg), torch.empty_like(cw), torch.empty_like(out)
    llr2 = torch.empty_like(llr)

    def e2e_step():
        o = off + e2e_step_no[0] * B * world  # fresh global frame indices every step
        e2e_step_no[0] += 1
        _native.random_bits(43, o, msg2)
        _native.polar_encode(plan, msg2, cw2)
        ch.llr_batch_device(cw2, N, B, seed=43, frame_offset=o, out=llr2)
        plan.decode(llr2, out2)
        sc.zero_()
        _native.count_errors(msg2, out2, K, sc)
        if world > 1:
            dist.all_reduce(sc)
        e2e_counts.add_(sc)

    edt = timed_steps(e2e_step, args.steps, args.warmup, world)
    ec = e2e_counts.cpu().numpy()
    res["end_to_end"] = dict(value=B * world * args.steps * K / edt / 1e6, unit="info-Mbps",
                             ms_per_step=edt / args.steps * 1e3,
                             what="per step: device random messages + polar encode + AWGN LLRs (Philox) + "
                                  "SCL decode + error count (+ all-reduce)",
                             ber=float(ec[0]) / max(1, ec[2] * K), fer=float(ec[1]) / max(1, ec[2]))
    if rank == 0 and world == 1 and not args.skip_cpu:
        from oracle import oracle as O
        S = args.cpu_frames
        th = cpu_threads()
        llr_h = llr[:S].cpu().numpy()
        t0 = time.perf_counter()
        ref = O.scl_decode(N, L, frozen, llr_h, threads=th)
        ct = time.perf_counter() - t0
        got = out[:S].cpu().numpy().astype(np.int64)
        res["cpu_baseline"] = dict(value=S * K / ct / 1e6, unit="info-Mbps", cores=th, kind="port",
                                   sample="first %d frames of the same LLR batch, oracle/refcpu.c SCL L=%d "
                                          "(loop-faithful C restatement, OpenMP %d threads), %.1f s" % (S, L, th, ct),
                                   mismatching_frames_vs_gpu=int((ref != got).any(axis=1).sum()))
        S1 = max(1, S // 16)  # single-core figure, same frames
        t0 = time.perf_counter()
        O.scl_decode(N, L, frozen, llr_h[:S1], threads=1)
        c1 = time.perf_counter() - t0
        res["cpu_baseline"]["single_core"] = dict(value=S1 * K / c1 / 1e6, unit="info-Mbps", cores=1,
                                                  sample="first %d frames, 1 thread, %.1f s" % (S1, c1))
    return res


def bench_ldpc(args, rank, world):
    from polarcode_and_ldpc_amd.channel import AWGNChannel
    from polarcode_and_ldpc_amd.ldpc import BPDecoder, LDPCEncoder

    n, k, B = 504, 252, args.batch
    enc = LDPCEncoder(n, k, dv=3, dc=6, seed=42)  # throughput_test.py:285 (rank-251 H, direct solving)
    dec = BPDecoder(enc.H, max_iter=20)
    plan = dec.plan
    rs = np.random.RandomState(42 + rank)
    U = 4096  # distinct messages, tiled; every frame gets its own noise
    base = enc.encode_batch(rs.randint(0, 2, (U, k)))
    cw = torch.from_numpy(np.tile(base, (B // U + 1, 1))[:B].astype(np.uint8)).cuda()
    llr = AWGNChannel(args.snr).llr_batch_device(cw, n, B, seed=4242, frame_offset=rank * B)
    out = torch.empty((B, n), dtype=torch.uint8, device="cuda")
    its = torch.empty((B,), dtype=torch.int32, device="cuda")
    counts = torch.zeros(3, dtype=torch.int64, device="cuda")
    kt = KernelTimer()

    sc = torch.zeros(3, dtype=torch.int64, device="cuda")

    def step():
        kt(lambda: plan.decode(llr, out, its))
        sc.zero_()
        _native_count(cw, out, k, sc)
        if world > 1:
            dist.all_reduce(sc)
        counts.add_(sc)

    from polarcode_and_ldpc_amd._native import count_errors as _native_count
    dt = timed_steps(step, args.steps, args.warmup, world)
    kt.reset()
    for _ in range(3):
        kt(lambda: plan.decode(llr, out, its))
    kms = kt.mean_ms()
    value = B * world * args.steps * k / dt / 1e6
    bpf = 9 * n
    achieved = B * bpf / (kms / 1e3) / 1e9
    mean_it = float(its.double().mean().item())
    res = dict(metric="decoded info-Mbps, LDPC (504,252) BP max_iter=20, reference-harness frames @ %.1f dB" % args.snr,
               value=value, unit="info-Mbps", ms_per_step=dt / args.steps * 1e3, kernel_ms=kms,
               mean_iterations=mean_it, vs_published=value / 7.95e-5,
               roofline=dict(bound="hbm", achieved=achieved, peak=HBM_PEAK_GBS, unit="GB/s",
                             frac=achieved / HBM_PEAK_GBS, traffic=load_traffic("ldpc_bp_504"),
                             traffic_unit="HBM bytes per launch (2*FETCH_SIZE+WRITE_SIZE, rocprofv3 PMC)",
                             traffic_source=traffic_source("ldpc_bp_504"),
                             algorithmic_bytes_per_frame=bpf, frames_per_launch=B, kernel_ms=kms,
                             kernel={2: "ldpc_reg_kernel<BP,DV=3>", 1: "ldpc_decode_kernel<BP>",
                                     3: "ldpc_check_kernel<BP>"}.get(plan.info.reserved, "?")))
    _traffic_rate(res["roofline"])
    _valu_rate(res["roofline"], "ldpc_bp_504", torch.cuda.get_device_properties(0).multi_processor_count)
    res["roofline"]["limit"] = "VALU issue (fp64 transcendentals), see roofline.valu; HBM fields are the algorithmic view"
    if args.skip_extra:
        return res
    # Second frame source (SURVEY §8 d): valid codewords (all-zero; BP is
    # codeword-symmetric) at the same SNR, early stop on.
    llr0 = AWGNChannel(args.snr).llr_batch_device(None, n, B, seed=4243, frame_offset=rank * B)
    out0 = torch.empty_like(out)
    its0 = torch.empty_like(its)

    def step0():
        plan.decode(llr0, out0, its0)

    dt0 = timed_steps(step0, args.steps, args.warmup, world)
    res["valid_codewords"] = dict(value=B * world * args.steps * k / dt0 / 1e6, unit="info-Mbps",
                                  ms_per_step=dt0 / args.steps * 1e3,
                                  mean_iterations=float(its0.double().mean().item()),
                                  bit_errors=int(out0.sum().item()),
                                  what="all-zero codeword frames (device AWGN), BP max_iter=20, early stop")
    if rank == 0 and world == 1 and not args.skip_cpu:
        from oracle import oracle as O
        from polarcode_and_ldpc_amd.ldpc import dense_to_csr
        S = args.cpu_frames_ldpc
        th = cpu_threads()
        rp, ci = dense_to_csr(enc.H)
        llr_h = llr[:S].cpu().numpy()
        t0 = time.perf_counter()
        rb, ri = O.ldpc_decode(rp, ci, n, llr_h, "bp", 20, True, 1.0, threads=th)
        ct = time.perf_counter() - t0
        got = out[:S].cpu().numpy().astype(np.int64)
        res["cpu_baseline"] = dict(value=S * k / ct / 1e6, unit="info-Mbps", cores=th, kind="port",
                                   sample="first %d frames of the same batch, oracle/refcpu.c BP-20, %d threads, "
                                          "%.1f s" % (S, th, ct),
                                   mismatching_frames_vs_gpu=int((rb != got).any(axis=1).sum()))
        S1 = max(1, S // 16)
        t0 = time.perf_counter()
        O.ldpc_decode(rp, ci, n, llr_h[:S1], "bp", 20, True, 1.0, threads=1)
        c1 = time.perf_counter() - t0
        res["cpu_baseline"]["single_core"] = dict(value=S1 * k / c1 / 1e6, unit="info-Mbps", cores=1,
                                                  sample="first %d frames, 1 thread, %.1f s" % (S1, c1))
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--batch", type=int, default=65536)
    ap.add_argument("--list-size", type=int, default=8)
    ap.add_argument("--snr", type=float, default=3.0)
    ap.add_argument("--cpu-frames", type=int, default=8192)
    ap.add_argument("--cpu-frames-ldpc", type=int, default=65536)
    ap.add_argument("--skip-cpu", action="store_true")
    ap.add_argument("--skip-ldpc", action="store_true")
    ap.add_argument("--skip-extra", action="store_true",
                    help="only the headline decodes (no end-to-end / valid-codeword runs): profiling passes")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    pol = bench_polar(args, rank, world)
    ldp = None if args.skip_ldpc else bench_ldpc(args, rank, world)
    if rank == 0:
        line = {
            "metric": METRIC, "value": pol["value"], "unit": "info-Mbps", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": pol["ms_per_step"],
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f64",
            "data": "synthetic: random messages, device polar encoder, device AWGN (Philox) at %.1f dB Es/N0" % args.snr,
            "config": {"workload": "polar N=1024 K=512 SCL L=%d decode, bit-reversed Bhattacharyya(2 dB) frozen set"
                                   % args.list_size,
                       "global_batch": args.batch * world, "frames_per_gpu": args.batch,
                       "parallelism": "frame-sharded x%d (one RCCL all-reduce of error counters per step)" % world},
            "roofline": pol["roofline"],
            "cpu_baseline": pol.get("cpu_baseline"),
            "ber": pol["ber"], "fer": pol["fer"], "plan": pol["plan"],
            "end_to_end": pol.get("end_to_end"),
        }
        if ldp is not None:
            line["ldpc"] = ldp
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
