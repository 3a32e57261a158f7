"""Throughput of the SCL tree kernel when a fraction of frames hold infinite
LLRs (such frames are flagged on their inputs and decoded again by
the single-workgroup NaN-order redo kernel).

usage: python tools/nan_cost.py [--batch 65536]
Headline configuration (N=1024 K=512 L=8, 3 dB); in the chosen fraction of
frames one channel LLR is set to +inf (an erasure-style known bit).  Prints the
decode time per fraction; bits of a sample of flagged frames are checked
against the same frames decoded alone (the redo path is exact: tests/test_gpu_polar.py)."""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from polarcode_and_ldpc_amd import _native  # noqa: E402
from polarcode_and_ldpc_amd.channel import AWGNChannel  # noqa: E402
from polarcode_and_ldpc_amd.polar import SCLDecoder, construct_frozen_set  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--batch", type=int, default=65536)
a = ap.parse_args()
torch.cuda.set_device(0)
N, K, B = 1024, 512, a.batch
dec = SCLDecoder(N, K, list_size=8, frozen_bits=construct_frozen_set(N, K, 2.0))
msg = torch.empty((B, K), dtype=torch.uint8, device="cuda")
_native.random_bits(77, 0, msg)
cw = torch.empty((B, N), dtype=torch.uint8, device="cuda")
_native.polar_encode(dec.plan, msg, cw)
base = AWGNChannel(3.0).llr_batch_device(cw, N, B, seed=77)
out = torch.empty((B, K), dtype=torch.uint8, device="cuda")
res = []
for frac in (0.0, 1e-4, 1e-3, 1e-2):
    llr = base.clone()
    nflag = int(round(frac * B))
    rows = torch.arange(nflag, device="cuda") * (B // max(1, nflag)) if nflag else None
    if nflag:
        llr[rows, 5] = float("inf")
    dec.plan.decode(llr, out)  # warm-up
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    dec.plan.decode(llr, out)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1)
    ok = None
    if nflag:  # a flagged frame decoded alone gives the same bits
        r = int(rows[0].item())
        one = torch.empty((1, K), dtype=torch.uint8, device="cuda")
        dec.plan.decode(llr[r:r + 1].contiguous(), one)
        ok = bool(torch.equal(one[0], out[r]))
    res.append(dict(flagged_fraction=frac, flagged_frames=nflag, ms=round(ms, 3),
                    info_mbps=round(B * K / ms / 1e3, 1), sample_bits_equal_alone=ok))
print(json.dumps({"config": "SCL N=1024 K=512 L=8, 3 dB, %d frames, one +inf LLR in flagged frames" % B,
                  "points": res}, indent=1))
