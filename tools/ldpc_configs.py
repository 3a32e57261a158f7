"""LDPC kernel timing at the BASELINE.json LDPC configurations (diagnostic):
(504,252) BP-20 on reference-harness frames and on valid frames, n=8192 MS-20
(regular dv=3, dc=6 H: every check degree >= 2, as MSDecoder needs)."""
import json, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from polarcode_and_ldpc_amd.channel import AWGNChannel
from polarcode_and_ldpc_amd.ldpc import BPDecoder, MSDecoder, regular_construction


def run(dec, n, B, snr, label, k):
    llr = AWGNChannel(snr).llr_batch_device(None, n, B, seed=7)
    out = torch.empty((B, n), dtype=torch.uint8, device="cuda")
    its = torch.empty((B,), dtype=torch.int32, device="cuda")
    dec.plan.decode(llr, out, its); torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(3):
        dec.plan.decode(llr, out, its)
    e1.record(); torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 3
    print(json.dumps({"config": label, "B": B, "ms": round(ms, 3), "info_mbps": round(B * k / ms / 1e3, 1),
                      "mean_iter": float(its.double().mean()), "lds": dec.plan.info.lds_bytes}), flush=True)


H = regular_construction(8192, 3, 6, seed=1)
run(MSDecoder(H, max_iter=20), 8192, 16384, 2.0, "n=8192 MS-20 early-stop @2dB", 4096)
run(MSDecoder(H, max_iter=20, early_stop=False), 8192, 16384, 2.0, "n=8192 MS-20 no early stop", 4096)
run(BPDecoder(H, max_iter=20, early_stop=False), 8192, 16384, 2.0, "n=8192 BP-20 no early stop", 4096)
H5 = regular_construction(504, 3, 6, seed=3)
run(MSDecoder(H5, max_iter=20, early_stop=False), 504, 65536, 3.0, "n=504 MS-20 no early stop", 252)
