"""Per-phase cycle shares of the polar list decoder (diagnostic build path).
usage: python tools/polar_stamps.py [--list-size 8] [--batch 65536] [--fused F]"""
import argparse, json, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from polarcode_and_ldpc_amd import _native
from polarcode_and_ldpc_amd.channel import AWGNChannel
from polarcode_and_ldpc_amd.polar import construct_frozen_set

ap = argparse.ArgumentParser()
ap.add_argument("--list-size", type=int, default=8)
ap.add_argument("--N", type=int, default=1024)
ap.add_argument("--batch", type=int, default=65536)
ap.add_argument("--fused", type=int, default=0)
ap.add_argument("--snr", type=float, default=3.0)
a = ap.parse_args()
N, K = a.N, a.N // 2
fr = construct_frozen_set(N, K, 2.0)
mask = np.zeros(N, np.uint8); mask[fr] = 1
plan = _native.polar_plan(N, K, mask, a.list_size, flags=a.fused)
msg = torch.empty((a.batch, K), dtype=torch.uint8, device="cuda"); _native.random_bits(42, 0, msg)
cw = torch.empty((a.batch, N), dtype=torch.uint8, device="cuda"); _native.polar_encode(plan, msg, cw)
llr = AWGNChannel(a.snr).llr_batch_device(cw, N, a.batch, seed=42)
out = torch.empty((a.batch, K), dtype=torch.uint8, device="cuda")
st = torch.zeros(16, dtype=torch.int64, device="cuda")
plan.decode_stamped(llr, out, st); torch.cuda.synchronize(); st.zero_()
t = time.perf_counter(); plan.decode_stamped(llr, out, st); torch.cuda.synchronize(); dt = time.perf_counter() - t
s_all = st.cpu().numpy().astype(float)
s, mc = s_all[:8], s_all[8:12]
ok = bool(torch.equal(out, msg)) if a.snr > 20 else None
names = ["fused_top", "ws_chains", "lds_chain", "metrics", "prune_clone", "beta_walk", "final", "ws_sync"] if plan.info.reserved == 4 else ["llr_update", "metrics", "prune_clone", "beta_walk", "final"]
print(json.dumps({"N": N, "L": a.list_size, "fused": plan.info.fused_top, "lds": plan.info.lds_bytes,
                  "stamped_ms": dt * 1e3, "cycles_per_frame": s.sum() / a.batch,
                  "share": {k: round(v / s.sum(), 4) for k, v in zip(names, s)},
                  # tree kernel: per-wave path_metrics_fast calls, those with a lane needing
                  # log1p(e^-x), such lanes and active lanes (stamps[8..11])
                  "metric_calls": mc[0], "metric_calls_evaluating": mc[1],
                  "metric_lanes_evaluating": mc[2], "metric_lanes_active": mc[3],
                  "wave_eval_fraction": round(mc[1] / max(1.0, mc[0]), 4),
                  "lane_eval_fraction_of_active": round(mc[2] / max(1.0, mc[3]), 4)}))
