"""ctypes front-end of the C oracle (oracle/refcpu.c) -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this
module.  The shipped package (polarcode_and_ldpc_amd) never does.

Functions return exactly what the reference's `.decode` returns:
  sc_decode / scl_decode  -> int64 [B, K]  (u_hat[info_bits], ascending index)
                             src/polar/decoder.py:69-71, :258-262
  bp_decode / ms_decode   -> int64 [B, n]  (+ iterations for BP)
                             src/ldpc/decoder.py:190-202, :343-352
"""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_SO = os.path.join(_HERE, "_build", "liboracle.so")
_lib = None

ORC_EDEGREE = -4


def build():
    subprocess.check_call(["make", "-s", "-C", _HERE], stdout=subprocess.DEVNULL)


def lib():
    global _lib
    if _lib is None:
        srcs = [os.path.join(_HERE, f) for f in ("refcpu.c", "pysort.h")]
        if not os.path.exists(_SO) or os.path.getmtime(_SO) < max(os.path.getmtime(f) for f in srcs):
            build()
        L = ctypes.CDLL(_SO)
        P = ctypes.c_void_p
        L.orc_polar_decode_batch.argtypes = [ctypes.c_int, ctypes.c_int, P, P, ctypes.c_int64,
                                             ctypes.c_int64, P, ctypes.c_int]
        L.orc_ldpc_decode_batch.argtypes = [ctypes.c_int, ctypes.c_int, P, P, ctypes.c_int, ctypes.c_int,
                                            ctypes.c_int, ctypes.c_double, P, ctypes.c_int64,
                                            ctypes.c_int64, P, P, ctypes.c_int]
        L.orc_cascl_decode_batch.argtypes = [ctypes.c_int, ctypes.c_int, P, P, ctypes.c_int64, ctypes.c_int64, P,
                                             ctypes.c_int, ctypes.c_int, ctypes.c_uint32]
        L.orc_crc.argtypes = [P, ctypes.c_int, ctypes.c_int, ctypes.c_uint32]
        L.orc_crc.restype = ctypes.c_uint32
        L.orc_pysort_desc.argtypes = [P, ctypes.c_int, P]
        _lib = L
    return _lib


def _ptr(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def frozen_mask(N, frozen_bits):
    m = np.zeros(N, np.uint8)
    m[np.asarray(frozen_bits, np.int64)] = 1
    return m


def polar_decode_u(N, list_size, frozen_bits, llr, threads=1):
    """Full u_hat [B, N] (uint8).  list_size <= 0 -> SC."""
    llr = np.ascontiguousarray(np.atleast_2d(np.asarray(llr, np.float64)))
    B = llr.shape[0]
    assert llr.shape[1] == N
    mask = frozen_mask(N, frozen_bits)
    u = np.zeros((B, N), np.uint8)
    rc = lib().orc_polar_decode_batch(N, int(list_size), _ptr(mask), _ptr(llr), B, N, _ptr(u), int(threads))
    if rc:
        raise RuntimeError("oracle polar decode failed: %d" % rc)
    return u


def _info(N, frozen_bits):
    return np.setdiff1d(np.arange(N), np.asarray(frozen_bits, np.int64))


def sc_decode(N, frozen_bits, llr, threads=1):
    return polar_decode_u(N, 0, frozen_bits, llr, threads)[:, _info(N, frozen_bits)].astype(np.int64)


def scl_decode(N, L, frozen_bits, llr, threads=1):
    return polar_decode_u(N, L, frozen_bits, llr, threads)[:, _info(N, frozen_bits)].astype(np.int64)


CRC_POLY = {"CRC-8": (8, 0x1D), "CRC-16": (16, 0x1021), "CRC-24": (24, 0x1864CFB)}  # src/polar/utils.py:99-103


def cascl_decode(N, L, frozen_bits, llr, crc_polynomial="CRC-8", threads=1):
    """CRC-aided SCL (build-defined extension; the reference has none): u_hat[info]
    of the first path in descending-metric order passing crc_check, else argmax."""
    crc_len, poly = CRC_POLY.get(crc_polynomial, CRC_POLY["CRC-8"])
    llr = np.ascontiguousarray(np.atleast_2d(np.asarray(llr, np.float64)))
    B = llr.shape[0]
    mask = frozen_mask(N, frozen_bits)
    u = np.zeros((B, N), np.uint8)
    rc = lib().orc_cascl_decode_batch(N, int(L), _ptr(mask), _ptr(llr), B, N, _ptr(u), int(threads), crc_len,
                                      poly & 0xFFFFFFFF)
    if rc:
        raise RuntimeError("oracle CA-SCL decode failed: %d" % rc)
    return u[:, _info(N, frozen_bits)].astype(np.int64)


def ldpc_decode(row_ptr, col_idx, n, llr, algo="bp", max_iter=20, early_stop=True, norm=1.0, threads=1):
    row_ptr = np.ascontiguousarray(row_ptr, np.int32)
    col_idx = np.ascontiguousarray(col_idx, np.int32)
    m = len(row_ptr) - 1
    llr = np.ascontiguousarray(np.atleast_2d(np.asarray(llr, np.float64)))
    B = llr.shape[0]
    bits = np.zeros((B, n), np.uint8)
    its = np.zeros(B, np.int32)
    rc = lib().orc_ldpc_decode_batch(m, n, _ptr(row_ptr), _ptr(col_idx), 0 if algo == "bp" else 1,
                                     int(max_iter), int(bool(early_stop)), float(norm), _ptr(llr), B, n,
                                     _ptr(bits), _ptr(its), int(threads))
    if rc == ORC_EDEGREE:
        raise ValueError("zero-size array to reduction operation minimum which has no identity")
    if rc:
        raise RuntimeError("oracle ldpc decode failed: %d" % rc)
    return bits.astype(np.int64), its


def crc(bits, crc_len, poly):
    b = np.ascontiguousarray(np.asarray(bits, np.uint8))
    return lib().orc_crc(_ptr(b), len(b), crc_len, poly)


def pysort_desc(keys):
    """Permutation that CPython 3.10's list.sort(key=..., reverse=True) applies to
    a list whose keys are `keys` (float64, NaN allowed): oracle/pysort.h."""
    k = np.ascontiguousarray(np.asarray(keys, np.float64))
    perm = np.zeros(len(k), np.int32)
    if lib().orc_pysort_desc(_ptr(k), len(k), _ptr(perm)):
        raise RuntimeError("oracle pysort failed")
    return perm
