"""The frame-per-wavefront SCL prototype (polar_fpw.hip, diagnostic library)
against the product's lane-per-path tree kernel at the headline configuration
(N=1024 K=512 L=8, 65 536 AWGN frames at 3 dB): kernel times (HIP events,
median of 5), decoded bits compared frame by frame, and the prototype's
per-phase cycles per leaf.

usage (GPU box): PL_LIB_PATH=$PWD/polarcode_and_ldpc_amd/_lib/diag/libpolarldpc_diag.so \\
                 python tools/fpw_proto.py [--batch 65536] [--snr 3.0]"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from polarcode_and_ldpc_amd import _native
from polarcode_and_ldpc_amd.channel import AWGNChannel
from polarcode_and_ldpc_amd.polar import construct_frozen_set

ap = argparse.ArgumentParser()
ap.add_argument("--batch", type=int, default=65536)
ap.add_argument("--snr", type=float, default=3.0)
ap.add_argument("--reps", type=int, default=5)
a = ap.parse_args()
N, K, L, B = 1024, 512, 8, a.batch
fr = construct_frozen_set(N, K, 2.0)
mask = np.zeros(N, np.uint8)
mask[fr] = 1
plan = _native.polar_plan(N, K, mask, L)
msg = torch.empty((B, K), dtype=torch.uint8, device="cuda")
_native.random_bits(7, 0, msg)
cw = torch.empty((B, N), dtype=torch.uint8, device="cuda")
_native.polar_encode(plan, msg, cw)
llr = AWGNChannel(a.snr).llr_batch_device(cw, N, B, seed=8)
out_p = torch.empty((B, K), dtype=torch.uint8, device="cuda")
out_f = torch.empty((B, K), dtype=torch.uint8, device="cuda")


def timed(fn):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(a.reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    return float(np.median(ts))


ms_p = timed(lambda: plan.decode(llr, out_p))
ms_f = timed(lambda: plan.decode_fpw(llr, out_f))
st = torch.zeros(5, dtype=torch.int64, device="cuda")
plan.decode_fpw(llr, out_f, st)
torch.cuda.synchronize()
s = st.cpu().numpy().astype(float)
names = ["descent", "metric", "prune", "partial_sums", "output"]
mism = int((out_p != out_f).any(dim=1).sum().item())
print(json.dumps({
    "config": "N=1024 K=512 L=8, %d frames, %.1f dB" % (B, a.snr),
    "product_tree_kernel_ms": ms_p, "frame_per_wave_ms": ms_f, "ratio": ms_f / ms_p,
    "frames_mismatching_product": mism,
    "fer_product": float((out_p != msg).any(dim=1).float().mean().item()),
    "fpw_cycles_per_leaf_per_wave": s.sum() / B / N,
    "fpw_cycles_per_leaf_by_phase": {k: round(v / B / N, 1) for k, v in zip(names, s)},
    "fpw_share": {k: round(v / s.sum(), 4) for k, v in zip(names, s)},
}))
