"""Kernel time and info-Mbps of the polar decoder at every BASELINE.json polar
configuration (tree kernel vs lane kernel).  Diagnostic; one JSON line each."""
import json, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from polarcode_and_ldpc_amd import _native
from polarcode_and_ldpc_amd.channel import AWGNChannel
from polarcode_and_ldpc_amd.polar import construct_frozen_set

CONFIGS = [(256, 0, 65536), (1024, 0, 65536), (4096, 0, 65536), (1024, 4, 65536), (1024, 8, 65536),
           (2048, 8, 32768), (1024, 16, 32768), (1024, 32, 16384), (4096, 8, 16384)]
if len(sys.argv) > 1:  # e.g. "256:8:65536,512:8:65536"
    CONFIGS = [tuple(int(x) for x in c.split(":")) for c in sys.argv[1].split(",")]
for N, L, B in CONFIGS:
    K = N // 2
    fr = construct_frozen_set(N, K, 2.0)
    mask = np.zeros(N, np.uint8); mask[fr] = 1
    for flags in (0, 0x20):
        plan = _native.polar_plan(N, K, mask, L, flags=flags)
        msg = torch.empty((B, K), dtype=torch.uint8, device="cuda"); _native.random_bits(42, 0, msg)
        cw = torch.empty((B, N), dtype=torch.uint8, device="cuda"); _native.polar_encode(plan, msg, cw)
        llr = AWGNChannel(3.0).llr_batch_device(cw, N, B, seed=42)
        out = torch.empty((B, K), dtype=torch.uint8, device="cuda")
        plan.decode(llr, out); torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(3):
            plan.decode(llr, out)
        e1.record(); torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / 3
        print(json.dumps({"N": N, "L": L, "B": B, "kernel": plan.info.reserved, "ms": round(ms, 3),
                          "info_mbps": round(B * K / ms / 1e3, 1)}), flush=True)
        plan.close()
