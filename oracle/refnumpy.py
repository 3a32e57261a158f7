"""NumPy restatement of the reference's per-frame decode loops -- TEST
INFRASTRUCTURE and CPU BASELINE ONLY.

Why it exists: BASELINE.json's north_star asks for "the reference NumPy CPU
path timed on the host cores in the same run".  The reference itself cannot
travel to the GPU box, so this module restates its hot loops with the same
NumPy scalar/array operations, in the same order, on the same data layout
(full (N, n+1) float64 LLR / bit matrices per path, full list snapshots per
information bit, list-of-check Python loops for BP).  It is therefore as slow
as the reference by construction, and bit-exact with it (tests/test_oracle_
golden.py pins it to the reference-generated fixtures).  `bench.py` times it
over a pool of worker processes on the first frames of the benchmark batch
(cpu_baseline, kind "port").  The shipped package never imports it.

Restated from (reference paths under /root/reference):
  sc_frame   src/polar/decoder.py:38-71   (_update_llrs :73-94, _update_bits :96-115,
                                           f :121-127, g :129-144, levels :146-170)
  scl_frame  src/polar/decoder.py:225-262 (frozen :264-281, info :283-339,
                                           per-path updates :341-372, metric :374-406)
  bp_frame   src/ldpc/decoder.py:124-202  (check node :62-96, variable node :98-122)
  ms_frame   src/ldpc/decoder.py:257-352
"""
from __future__ import annotations

import os

import numpy as np


# ---------------------------------------------------------------- polar
def _bitrev(i: int, n: int) -> int:  # src/polar/utils.py:11-26
    r = 0
    for _ in range(n):
        r = (r << 1) | (i & 1)
        i >>= 1
    return r


def _lead_zeros_plus1(i: int, n: int) -> int:  # decoder.py:146-157 (first 1 from the MSB)
    c = 1
    m = 1 << (n - 1)
    while c <= n and not (m & i):
        c += 1
        m >>= 1
    return min(c, n)


def _lead_ones_plus1(i: int, n: int) -> int:  # decoder.py:159-170 (first 0 from the MSB)
    c = 1
    m = 1 << (n - 1)
    while c <= n and (m & i):
        c += 1
        m >>= 1
    return min(c, n)


def _f(a, b):  # min-sum f, decoder.py:121-127 / :408-410
    return np.sign(a) * np.sign(b) * min(abs(a), abs(b))


def _g(btm, top, b):  # decoder.py:129-144 / :412-417
    return btm + top if b == 0 else btm - top


def _llr_pass(Lm, Bm, l, N, n):
    """The LLR update towards leaf l on one (N, n+1) matrix pair."""
    for s in range(n - _lead_zeros_plus1(l, n), n):
        blk = 2 << s
        half = blk >> 1
        for j in range(l, N, blk):
            if j % blk < half:
                Lm[j, s + 1] = _f(Lm[j, s], Lm[j + half, s])
            else:
                Lm[j, s + 1] = _g(Lm[j, s], Lm[j - half, s], Bm[j - half, s + 1])


def _bit_pass(Bm, l, N, n):
    """Partial-sum propagation after leaf l's decision."""
    if l < N / 2:
        return
    for s in range(n, n - _lead_ones_plus1(l, n), -1):
        blk = 1 << s
        half = blk >> 1
        for j in range(l, -1, -blk):
            if j % blk >= half:
                Bm[j - half, s - 1] = int(Bm[j, s]) ^ int(Bm[j - half, s])
                Bm[j, s - 1] = Bm[j, s]


def _path_ll(lam, bit):  # decoder.py:374-406, same branches and ufunc calls
    if bit == 0:
        return -np.log1p(np.exp(-lam)) if lam >= 0 else lam - np.log1p(np.exp(lam))
    return -lam - np.log1p(np.exp(-lam)) if lam >= 0 else -np.log1p(np.exp(lam))


def sc_frame(llr, N, frozen, info):
    """One SC decode; frozen = set of frozen u indices, info = ascending info indices."""
    n = N.bit_length() - 1
    Lm = np.full((N, n + 1), np.nan)
    Bm = np.full((N, n + 1), np.nan)
    Lm[:, 0] = np.asarray(llr, dtype=np.float64)
    for i in range(N):
        l = _bitrev(i, n)
        _llr_pass(Lm, Bm, l, N, n)
        Bm[l, n] = 0 if (l in frozen or Lm[l, n] >= 0) else 1
        _bit_pass(Bm, l, N, n)
    return Bm[:, n].astype(int)[info]


def scl_frame(llr, N, Lsz, frozen, info):
    """One SCL decode with the reference's list bookkeeping (metrics of every leaf,
    stable descending candidate sort, full snapshots, first-max argmax)."""
    n = N.bit_length() - 1
    LP = np.full((Lsz, N, n + 1), np.nan)
    BP = np.full((Lsz, N, n + 1), np.nan)
    pm = np.full(Lsz, -np.inf)
    act = np.zeros(Lsz, dtype=bool)
    act[0] = True
    pm[0] = 0.0
    x = np.asarray(llr, dtype=np.float64)
    for p in range(Lsz):
        LP[p, :, 0] = x
    for i in range(N):
        l = _bitrev(i, n)
        if l in frozen:
            for p in range(Lsz):
                if act[p]:
                    _llr_pass(LP[p], BP[p], l, N, n)
                    BP[p, l, n] = 0
                    pm[p] += _path_ll(LP[p, l, n], 0)
                    _bit_pass(BP[p], l, N, n)
            continue
        live = np.where(act)[0]
        zeros, ones = [], []
        for p in live:
            _llr_pass(LP[p], BP[p], l, N, n)
            lam = LP[p, l, n]
            zeros.append((pm[p] + _path_ll(lam, 0), p, 0))
            ones.append((pm[p] + _path_ll(lam, 1), p, 1))
        cand = zeros + ones
        cand.sort(key=lambda c: c[0], reverse=True)  # stable: ties keep list order
        keep = cand[:min(len(cand), Lsz)]
        snapL, snapB = LP.copy(), BP.copy()
        _ = pm.copy()  # the reference snapshots the metrics too (unused)
        act[:] = False
        pm[:] = -np.inf
        for k, (met, par, bit) in enumerate(keep):
            LP[k] = snapL[par].copy()
            BP[k] = snapB[par].copy()
            BP[k, l, n] = bit
            pm[k] = met
            act[k] = True
            _bit_pass(BP[k], l, N, n)
    best = np.argmax(pm)
    return BP[best, :, n].astype(int)[info]


# ---------------------------------------------------------------- LDPC
class Tanner:
    """Neighbour lists of a dense H in the reference's ascending scan order
    (decoder.py:35-60), plus flat edge indices for the two message stores."""

    def __init__(self, H):
        H = np.asarray(H)
        self.H = H
        self.m, self.n = H.shape
        self.chk = [np.nonzero(H[c] == 1)[0] for c in range(self.m)]
        self.var = [np.nonzero(H[:, v] == 1)[0] for v in range(self.n)]
        # message store: one slot per (check, position); var_slots[v] lists the
        # slots of v's checks in ascending check order
        self.cstart = np.concatenate([[0], np.cumsum([len(c) for c in self.chk])]).astype(np.int64)
        self.var_slots = []
        for v in range(self.n):
            self.var_slots.append(np.array([self.cstart[c] + int(np.searchsorted(self.chk[c], v))
                                            for c in self.var[v]], dtype=np.int64))


def _bp_check(msgs):  # decoder.py:62-96
    d = len(msgs)
    out = np.zeros(d)
    t = np.clip(np.tanh(msgs / 2.0), -0.999999, 0.999999)
    for i in range(d):
        p = np.clip(np.prod(t[np.arange(d) != i]), -0.999999, 0.999999)
        out[i] = 2.0 * np.arctanh(p)
    return np.nan_to_num(out, nan=0.0, posinf=20.0, neginf=-20.0)


def _ms_check(msgs, norm):  # decoder.py:257-287
    d = len(msgs)
    out = np.zeros(d)
    sg = np.sign(msgs)
    mg = np.abs(msgs)
    for i in range(d):
        keep = np.arange(d) != i
        out[i] = np.prod(sg[keep]) * np.min(mg[keep]) * norm
    return out


def _flood(tg: Tanner, llr, max_iter, early_stop, check_fn):
    """Flooding schedule shared by BP and MS (decoder.py:124-202, :289-352):
    v2c[slot] holds the variable-to-check message on that edge, c2v[slot] the
    reply."""
    llr = np.asarray(llr, dtype=np.float64)
    v2c = np.zeros(int(tg.cstart[-1]))
    c2v = np.zeros_like(v2c)
    for v in range(tg.n):
        v2c[tg.var_slots[v]] = llr[v]
    its = max_iter
    decoded = np.zeros(tg.n, dtype=int)
    for it in range(max_iter):
        for c in range(tg.m):
            a, b = tg.cstart[c], tg.cstart[c + 1]
            c2v[a:b] = check_fn(np.array(list(v2c[a:b])))
        total = np.zeros(tg.n)
        for v in range(tg.n):
            sl = tg.var_slots[v]
            msgs = [c2v[s] for s in sl]
            tv = llr[v] + np.sum(msgs)
            total[v] = tv
            for k, s in enumerate(sl):
                v2c[s] = tv - msgs[k]
        decoded = (total <= 0).astype(int)
        if early_stop and np.all((tg.H @ decoded) % 2 == 0):
            its = it + 1
            break
    return decoded, its


def bp_frame(tg: Tanner, llr, max_iter=50, early_stop=True):
    return _flood(tg, llr, max_iter, early_stop, _bp_check)


def ms_frame(tg: Tanner, llr, max_iter=50, normalization=1.0, early_stop=True):
    if any(len(c) == 1 for c in tg.chk):
        raise ValueError("zero-size array to reduction operation minimum which has no identity")
    return _flood(tg, llr, max_iter, early_stop, lambda m: _ms_check(m, normalization))[0]


# ---------------------------------------------------------------- batch drivers
# A task is (spec, row): spec names the decoder set-up by value (small: the
# frozen indices, or H as CSR), and each worker builds it once and caches it.
_CACHE = {}


def _built(spec):
    if spec not in _CACHE:
        if spec[0] == "polar":
            _, N, Lsz, frozen = spec
            fr = set(frozen)
            _CACHE[spec] = (N, Lsz, fr, np.setdiff1d(np.arange(N), np.asarray(frozen, dtype=np.int64)))
        else:
            _, m, n, rp, ci = spec[:5]
            H = np.zeros((m, n), dtype=int)
            for c in range(m):
                H[c, list(ci[rp[c]:rp[c + 1]])] = 1
            _CACHE[spec] = Tanner(H)
    return _CACHE[spec]


def _task(job):
    spec, row = job
    st = _built(spec)
    if spec[0] == "polar":
        N, Lsz, fr, info = st
        return sc_frame(row, N, fr, info) if Lsz <= 0 else scl_frame(row, N, Lsz, fr, info)
    algo, max_iter, early_stop, norm = spec[5:]
    if algo == "bp":
        return bp_frame(st, row, max_iter, early_stop)
    return ms_frame(st, row, max_iter, norm, early_stop), max_iter


def _run(spec, llr, pool):
    jobs = [(spec, r) for r in np.atleast_2d(np.asarray(llr, dtype=np.float64))]
    return pool.map(_task, jobs, chunksize=1) if pool is not None else [_task(j) for j in jobs]


def polar_batch(N, list_size, frozen, llr, pool=None):
    """[B, N] -> int64 [B, K] (list_size <= 0: SC)."""
    spec = ("polar", int(N), int(list_size), tuple(sorted(int(x) for x in frozen)))
    res = _run(spec, llr, pool)
    return np.array(res, dtype=np.int64).reshape(len(res), -1)


def ldpc_batch(H, llr, algo="bp", max_iter=20, early_stop=True, normalization=1.0, pool=None):
    """[B, n] -> (int64 [B, n], int64 [B] iterations; MS reports max_iter)."""
    H = np.asarray(H)
    m, n = H.shape
    rp, ci = [0], []
    for c in range(m):
        nz = np.nonzero(H[c] == 1)[0].tolist()
        ci.extend(nz)
        rp.append(len(ci))
    spec = ("ldpc", m, n, tuple(rp), tuple(ci), algo, int(max_iter), bool(early_stop), float(normalization))
    res = _run(spec, llr, pool)
    return np.array([r[0] for r in res], dtype=np.int64), np.array([r[1] for r in res], dtype=np.int64)


def make_pool(processes):
    """Spawn-context worker pool.  bench.py creates it BEFORE any GPU call, so no
    process holding a HIP runtime is ever forked."""
    import multiprocessing as mp
    return mp.get_context("spawn").Pool(processes)
