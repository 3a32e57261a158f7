"""PC-sampling target (diagnostic): the headline SCL decode (N=1024 K=512 L=8,
65 536 frames at 3 dB), a few launches.  usage: python tools/pcsample_polar.py [reps] [N L B]"""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from polarcode_and_ldpc_amd.channel import AWGNChannel
from polarcode_and_ldpc_amd.polar import SCLDecoder, construct_frozen_set

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
N, L, B = (int(x) for x in sys.argv[2:5]) if len(sys.argv) > 4 else (1024, 8, 65536)
K = N // 2
torch.cuda.set_device(0)
fr = construct_frozen_set(N, K, 2.0)
dec = SCLDecoder(N, K, list_size=L, frozen_bits=fr)
cw = torch.zeros((B, N), dtype=torch.uint8, device="cuda")
llr = AWGNChannel(3.0).llr_batch_device(cw, N, B, seed=7)
for _ in range(reps):
    out = dec.decode_batch(llr)
torch.cuda.synchronize()
print("decoded", out.shape, int(out.sum().item()))
