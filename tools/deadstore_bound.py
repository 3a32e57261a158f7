"""Dead-store bound of the headline SCL kernel.

usage: python tools/deadstore_bound.py [--batch 65536] [--reps 10]
Diagnostic library (PL_LIB_PATH).  The bench's headline frames (N=1024 K=512
L=8, frozen set construct_frozen_set(2 dB), 3 dB, device messages / encoder /
AWGN as bench.py makes them).  Mode 1 decodes once recording which workspace
pool arrays (depths F..DL-1 = 3..6) a right child's g reads and which were
stored; mode 2 replays the same frames skipping every store of an array that
was never read -- the same bits by construction (checked) -- and both are
timed against the product kernel on the same box (HIP events, median).  The
saving is measured between two runs of the same replay instance: with the
recorded mask (dead stores skipped) and with every array marked read (every
store kept).  It is an upper bound on what any predictor of dead stores could
buy, since a real predictor has to decide at store time without the future."""
import argparse
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("PL_LIB_PATH", os.path.join(ROOT, "polarcode_and_ldpc_amd", "_lib", "diag", "libpolarldpc_diag.so"))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from polarcode_and_ldpc_amd import _native  # noqa: E402
from polarcode_and_ldpc_amd.channel import AWGNChannel  # noqa: E402
from polarcode_and_ldpc_amd.polar import SCLDecoder, construct_frozen_set  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--batch", type=int, default=65536)
ap.add_argument("--reps", type=int, default=10)
a = ap.parse_args()
torch.cuda.set_device(0)
N, K, L, B = 1024, 512, 8, a.batch
dec = SCLDecoder(N, K, list_size=L, frozen_bits=construct_frozen_set(N, K, 2.0))
plan = dec.plan
msg = torch.empty((B, K), dtype=torch.uint8, device="cuda")
_native.random_bits(1234, 0, msg)
cw = torch.empty((B, N), dtype=torch.uint8, device="cuda")
_native.polar_encode(plan, msg, cw)
llr = AWGNChannel(3.0).llr_batch_device(cw, N, B, seed=1234)
F, DL = plan.info.fused_top, 7
DSW = ((1 << DL) - (1 << F)) * 2
groups = (B + 7) // 8
mask = torch.zeros((groups, 2, DSW), dtype=torch.int32, device="cuda")
P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
S = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
ref = torch.empty((B, K), dtype=torch.uint8, device="cuda")
out = torch.empty_like(ref)


def ds(mode):
    _native.check(_native.lib.pl_debug_polar_deadstore(plan.handle, P(llr), B, N, P(out), P(mask), mode, S),
                  "pl_debug_polar_deadstore")


def timeit(fn):
    for _ in range(2):
        fn()
    ts = []
    for _ in range(a.reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    return float(np.median(ts)), [round(t, 4) for t in ts]


plan.decode(llr, ref)
ds(1)
torch.cuda.synchronize()
same_record = bool(torch.equal(out, ref))
m = mask.cpu().numpy().view(np.uint32)


def popcount(x):
    return int(np.unpackbits(x.view(np.uint8)).sum())


read_bits, stored_bits = popcount(m[:, 0]), popcount(m[:, 1])
per_depth = {}
off = 0
for d in range(F, DL):
    w = (1 << d) * 2
    per_depth[d] = dict(stored=popcount(m[:, 1, off:off + w]), read=popcount(m[:, 0, off:off + w] & m[:, 1, off:off + w]))
    per_depth[d]["read_frac"] = round(per_depth[d]["read"] / max(1, per_depth[d]["stored"]), 4)
    off += w
ds(2)
torch.cuda.synchronize()
same_replay = bool(torch.equal(out, ref))
t_prod, ts_prod = timeit(lambda: plan.decode(llr, ref))
t_rep, ts_rep = timeit(lambda: ds(2))
# the same replay instance with every array marked read: every store kept, the
# same instruction stream and register allocation as the dead-store replay
# (whose mask lookups cost time of their own), so the two differ only in the
# dead stores' traffic
saved_mask = mask.clone()
mask.fill_(-1)
t_all, ts_all = timeit(lambda: ds(2))
ds(2)
torch.cuda.synchronize()
same_all = bool(torch.equal(out, ref))
mask.copy_(saved_mask)
t_prod2, ts_prod2 = timeit(lambda: plan.decode(llr, ref))
# bytes: every stored pool array of depth d is 2^(n-d) doubles per plane
n = 10
stored_bytes = sum(per_depth[d]["stored"] * (1 << (n - d)) * 8 for d in per_depth)
dead_bytes = sum((per_depth[d]["stored"] - per_depth[d]["read"]) * (1 << (n - d)) * 8 for d in per_depth)
t_base = min(t_prod, t_prod2)
print(json.dumps({
    "config": "SCL N=1024 K=512 L=8, 3 dB, %d frames, F=%d, DL=%d" % (B, F, DL),
    "bits_equal": {"record": same_record, "replay": same_replay, "replay_all_stores": same_all},
    "pool_arrays": {"stored": stored_bits, "read": read_bits, "read_frac": round(read_bits / max(1, stored_bits), 4),
                    "per_depth": per_depth},
    "pool_store_bytes_per_launch": stored_bytes, "dead_store_bytes_per_launch": dead_bytes,
    "ms": {"product": t_prod, "replay_dead_stores_skipped": t_rep, "replay_all_stores_kept": t_all,
           "product_again": t_prod2},
    "saving_upper_bound": round(1.0 - t_rep / t_all, 4),
    "replay_overhead_vs_product": round(t_all / t_base - 1.0, 4),
    "samples_ms": {"product": ts_prod, "replay": ts_rep, "replay_all": ts_all, "product_again": ts_prod2}},
    indent=1))
