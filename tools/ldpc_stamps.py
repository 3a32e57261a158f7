"""Per-phase cycle shares of the degree-grouped BP kernel (diagnostic build).

usage: python tools/ldpc_stamps.py [--batch 65536]
Loads the diagnostic library (PL_LIB_PATH), decodes the bench's BP-20 frames
(the reference harness's invalid codewords of the seed-42 (504,252) code at
3 dB) through pl_debug_ldpc_stamps and prints, per wavefront index of the
workgroup (= per SIMD: wavefront w of every frame runs on SIMD w), the cycle
share of each phase and the mean cycles per frame-iteration."""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("PL_LIB_PATH", os.path.join(ROOT, "polarcode_and_ldpc_amd", "_lib", "diag", "libpolarldpc_diag.so"))
sys.path.insert(0, ROOT)
import argparse  # noqa: E402

import numpy as np  # noqa: E402
import torch  # noqa: E402

from polarcode_and_ldpc_amd import _native  # noqa: E402
from polarcode_and_ldpc_amd.channel import AWGNChannel  # noqa: E402
from polarcode_and_ldpc_amd.ldpc import BPDecoder, LDPCEncoder  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--batch", type=int, default=65536)
a = ap.parse_args()
torch.cuda.set_device(0)
enc = LDPCEncoder(504, 252, dv=3, dc=6, seed=42)
plan = BPDecoder(enc.H, max_iter=20).plan
B = a.batch
base = enc.encode_batch(np.random.RandomState(42).randint(0, 2, (4096, 252)))
cw = torch.from_numpy(np.tile(base, ((B + 4095) // 4096, 1))[:B].astype(np.uint8)).cuda()
llr = AWGNChannel(3.0).llr_batch_device(cw, 504, B, seed=4242)
out = torch.empty((B, 504), dtype=torch.uint8, device="cuda")
its = torch.empty((B,), dtype=torch.int32, device="cuda")
st = torch.zeros((4, 8), dtype=torch.int64, device="cuda")
P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
S = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def run():
    _native.check(_native.lib.pl_debug_ldpc_stamps(plan.handle, P(llr), B, 504, P(out), P(its), P(st), S),
                  "pl_debug_ldpc_stamps")


run()
torch.cuda.synchronize()
ref = out.clone()
plan.decode(llr, out, its)
torch.cuda.synchronize()
same = bool(torch.equal(ref, out))
st.zero_()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
run()
e1.record()
torch.cuda.synchronize()
s = st.cpu().numpy().astype(float)
names = ["init", "vote", "check_pass", "check_barrier", "variable_pass", "tanh_list", "end_barrier", "output"]
iters = float(its.double().mean().item())
print(json.dumps({"batch": B, "stamped_ms": e0.elapsed_time(e1), "bits_equal_product": same, "mean_iters": iters,
                  "per_wave": [{k: round(v / row.sum(), 4) for k, v in zip(names, row)} for row in s],
                  "cycles_per_frame_iter_per_wave": [round(row.sum() / B / iters, 1) for row in s],
                  "all_waves": {k: round(v / s.sum(), 4) for k, v in zip(names, s.sum(0))}}, indent=1))
