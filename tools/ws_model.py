"""Modelled memory traffic of the polar tree kernel (polar_tree.hip), per frame,
to attribute the PMC bytes (2*FETCH_SIZE + WRITE_SIZE) to its sources.

usage: python tools/ws_model.py [N K L F DL]      (default 1024 512 8 3 7)

Counts, for the headline frozen set (bit-reversed Bhattacharyya at 2 dB), the
bytes each decode step moves between the CUs and L2 when every access misses
(an upper bound per source; the PMC counters see what misses L2):
  pools   workspace LLR depths F..DL-1: the streaming descend stores every
          depth it recomputes (N/2^d values per active path) and the g of a
          right child reads its parent's pairs;
  fused   the fused top's reads of the staged depth D0 (channel in place, or
          the staged f(ch) / f(f(ch))), once per frame (de-duplicated);
  stage   staging writes of f(ch), f(f(ch)) + the channel read that makes them;
  beta    multi-word partial sums (workspace) read by g / fused top and written
          by the walk, plus the walk buffers.
Inactive list slots (shadow lanes) move no bytes of their own.
"""
import sys

import numpy as np


def bitrev(i, n):
    r = 0
    for _ in range(n):
        r = (r << 1) | (i & 1)
        i >>= 1
    return r


def frozen_set(N, K, snr=2.0):
    import os
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from polarcode_and_ldpc_amd.polar.construction import construct_frozen_set
    return construct_frozen_set(N, K, snr)


def model(N=1024, K=512, L=8, F=3, DL=7):
    n = N.bit_length() - 1
    NB = n - 6
    fr = set(int(x) for x in frozen_set(N, K))
    frozen_dec = [bitrev(i, n) in fr for i in range(N)]
    NS = min(F - 1, 3)
    b = dict(pools_w=0, pools_r=0, fused=0, stage=0, beta=0)
    b["stage"] = 8 * N + 8 * sum(N >> d for d in range(1, NS + 1))  # channel read + staged writes
    nact = 1
    for i in range(N):
        dstart = 1 if i == 0 else n - ((i & -i).bit_length() - 1)
        if dstart <= F:
            right = [0] + [(i >> (n - d)) & 1 for d in range(1, F + 1)]
            D0 = 0
            for d0 in range(min(NS, F), 0, -1):
                if not any(right[1:d0 + 1]):
                    D0 = d0
                    break
            b["fused"] += 8 * (N >> D0)
            b["beta"] += 4 * nact * sum((N >> d) // 32 for d in range(1, min(F, NB) + 1) if right[d])
            lo = F
        else:
            p = dstart - 1
            if F <= p < DL:
                b["pools_r"] += 8 * nact * (N >> p)
            if dstart <= NB:
                b["beta"] += 4 * nact * max(1, (N >> dstart) // 32)
            lo = dstart
        for d in range(max(lo, F), DL):
            b["pools_w"] += 8 * nact * (N >> d)
        if not frozen_dec[i]:
            nact = min(2 * nact, L)
        # walk through multi-word depths: trailing ones of i beyond 5 levels
        to = ((~i) & -(~i)).bit_length() - 1
        steps = min(to, n)
        if steps > 5:
            for k in range(5, steps):
                b["beta"] += 4 * nact * 3 * (1 << (k - 5))
    return b


if __name__ == "__main__":
    args = [int(x) for x in sys.argv[1:]] or [1024, 512, 8, 3, 7]
    b = model(*args)
    tot = sum(b.values())
    for k, v in b.items():
        print("%-8s %9.1f KB/frame  %5.1f %%  %6.2f GB per 65 536 frames" % (k, v / 1e3, 100 * v / tot,
                                                                           v * 65536 / 1e9))
    print("%-8s %9.1f KB/frame          %6.2f GB per 65 536 frames" % ("total", tot / 1e3, tot * 65536 / 1e9))
