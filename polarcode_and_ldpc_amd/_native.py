"""ctypes binding of libpolarldpc.so (include/polarldpc.h).

The HIP library is the only compute path: if it is missing or cannot be
loaded this module raises at import time -- there is no CPU fallback.
PyTorch (ROCm) is used only to own device buffers and streams: it is imported
first so that the library binds to the same HIP runtime instance as torch.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np
import torch  # noqa: F401  (loads torch's libamdhip64 first; our .so reuses it)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("PL_LIB_PATH", os.path.join(_HERE, "_lib", "libpolarldpc.so"))

PL_OK, PL_EINVAL, PL_ENOMEM, PL_EHIP, PL_EUNSUPPORTED = 0, -1, -2, -3, -4
PL_LDPC_BP, PL_LDPC_MS = 0, 1

EXPORTS = (
    "pl_polar_plan_create", "pl_ldpc_plan_create", "pl_decode", "pl_plan_reserve", "pl_plan_get_info",
    "pl_plan_destroy", "pl_last_error", "pl_random_bits", "pl_polar_encode", "pl_awgn_llr",
    "pl_count_errors", "pl_debug_polar_stamps", "pl_debug_ldpc_stamps", "pl_debug_polar_deadstore", "pl_polar_plan_set_crc", "pl_crc_append",
    "pl_rayleigh_llr", "pl_bsc", "pl_gf2_encode", "pl_decode_ws", "pl_plan_workspace_bytes",
    "pl_plan_release", "pl_plan_workspace_stats", "pl_debug_set_plan_device", "pl_debug_polar_fpw",
    "pl_debug_polar_flagged", "pl_polar_plan_small_batch",
)


class PlanInfo(ctypes.Structure):
    _fields_ = [("kind", ctypes.c_int32), ("n_in", ctypes.c_int32), ("n_out", ctypes.c_int32),
                ("list_size", ctypes.c_int32), ("lds_bytes", ctypes.c_int32), ("fused_top", ctypes.c_int32),
                ("frames_per_block", ctypes.c_int32), ("reserved", ctypes.c_int32)]


def _load(path=LIB_PATH):
    if not os.path.exists(path):
        raise ImportError(
            "polarcode_and_ldpc_amd: native library %s not found -- build it with "
            "`python -c 'import __graft_entry__ as g; g.build()'` (make -C polarcode_and_ldpc_amd/csrc). "
            "There is no CPU fallback." % path)
    L = ctypes.CDLL(path)
    P, I32, I64, D = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_double
    PP = ctypes.POINTER(ctypes.c_void_p)
    L.pl_polar_plan_create.argtypes = [I32, I32, P, I32, I32, PP]
    L.pl_ldpc_plan_create.argtypes = [I32, I32, P, P, I32, I32, I32, D, I32, PP]
    L.pl_decode.argtypes = [P, P, I64, I64, P, P, P]
    L.pl_plan_reserve.argtypes = [P, I64, P]
    L.pl_decode_ws.argtypes = [P, P, I64, I64, P, P, P, I64, P]
    L.pl_plan_workspace_bytes.argtypes = [P, I64, ctypes.POINTER(ctypes.c_int64)]
    L.pl_plan_release.argtypes = [P, P]
    L.pl_plan_workspace_stats.argtypes = [P, ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_int64)]
    L.pl_debug_set_plan_device.argtypes = [P, I32]
    L.pl_plan_get_info.argtypes = [P, ctypes.POINTER(PlanInfo)]
    L.pl_polar_plan_small_batch.argtypes = [P, ctypes.POINTER(ctypes.c_int64)]
    L.pl_plan_destroy.argtypes = [P]
    L.pl_last_error.restype = ctypes.c_char_p
    L.pl_random_bits.argtypes = [ctypes.c_uint64, I64, I64, I32, P, P]
    L.pl_polar_encode.argtypes = [P, P, I64, P, P]
    L.pl_awgn_llr.argtypes = [P, I32, I64, D, ctypes.c_uint64, I64, P, I64, P]
    L.pl_count_errors.argtypes = [P, I64, P, I64, I32, I64, P, P]
    L.pl_debug_polar_stamps.argtypes = [P, P, I64, I64, P, P, P]
    L.pl_debug_polar_fpw.argtypes = [P, P, I64, I64, P, P, I32, P]
    L.pl_debug_ldpc_stamps.argtypes = [P, P, I64, I64, P, P, P, P]
    L.pl_debug_polar_deadstore.argtypes = [P, P, I64, I64, P, P, I32, P]
    L.pl_debug_polar_flagged.argtypes = [P, P, I64, I64, P, P, P]
    L.pl_polar_plan_set_crc.argtypes = [P, I32, ctypes.c_uint32]
    L.pl_crc_append.argtypes = [P, I64, I64, I32, I32, ctypes.c_uint32, P]
    L.pl_rayleigh_llr.argtypes = [P, I32, I64, D, ctypes.c_uint64, I64, P, I64, P]
    L.pl_bsc.argtypes = [P, I32, I64, D, ctypes.c_uint64, I64, P, I64, P]
    L.pl_gf2_encode.argtypes = [P, I32, I32, P, I64, I64, P, I64, P]
    for name in EXPORTS:
        getattr(L, name).restype = ctypes.c_int if name != "pl_last_error" else ctypes.c_char_p
    return L


lib = _load()
_BUILD_ID = None
DIAG_LIB_PATH = os.path.join(_HERE, "_lib", "diag", "libpolarldpc_diag.so")


def load_diag():
    """The diagnostic build (make diag: stamped kernels, test hooks), bound like
    the product library, or None if it was not built.  Tests and tools only."""
    return _load(DIAG_LIB_PATH) if os.path.exists(DIAG_LIB_PATH) else None


def build_id() -> str:
    """Digest of the loaded libpolarldpc.so (keys resumable result logs to the
    decoder build that produced them)."""
    global _BUILD_ID
    if _BUILD_ID is None:
        import hashlib
        with open(LIB_PATH, "rb") as f:
            _BUILD_ID = hashlib.sha1(f.read()).hexdigest()[:16]
    return _BUILD_ID


class NativeError(RuntimeError):
    pass


def check(rc: int, what: str):
    if rc == PL_OK:
        return
    msg = (lib.pl_last_error() or b"").decode(errors="replace")
    if rc == PL_EINVAL:
        raise AssertionError("%s: %s" % (what, msg))
    if rc == PL_EUNSUPPORTED:
        raise ValueError("%s: %s" % (what, msg))
    raise NativeError("%s failed (%d): %s" % (what, rc, msg))


def _stream(stream=None) -> int:
    if stream is None:
        stream = torch.cuda.current_stream()
    return int(stream.cuda_stream) if hasattr(stream, "cuda_stream") else int(stream)


def _ld(t: "torch.Tensor") -> int:
    """Row pitch in elements; a single row may carry any stride (e.g. 0 from a
    NumPy newaxis view), so it is normalised to the row length."""
    return int(t.stride(0)) if t.shape[0] > 1 else int(t.shape[1])


def _dptr(t: "torch.Tensor"):
    assert t.is_cuda and (t.dim() < 2 or t.stride(-1) == 1), "device tensor must have unit inner stride"
    return ctypes.c_void_p(t.data_ptr())


def require_gpu():
    if not torch.cuda.is_available():
        raise RuntimeError("polarcode_and_ldpc_amd: no HIP device visible (the decoders run on MI355X only)")


class Plan:
    """Owner of a pl_plan*.  The plan holds device constants; decode workspace is
    per stream (grown lazily by the library) or caller-supplied (decode(ws=...))."""

    def __init__(self, handle: ctypes.c_void_p):
        self._h = handle
        info = PlanInfo()
        check(lib.pl_plan_get_info(self._h, ctypes.byref(info)), "pl_plan_get_info")
        self.info = info

    @property
    def handle(self):
        return self._h

    def reserve(self, max_batch: int, stream=None):
        """Pre-size `stream`'s workspace (default: torch's current stream)."""
        check(lib.pl_plan_reserve(self._h, int(max_batch), ctypes.c_void_p(_stream(stream))), "pl_plan_reserve")

    def release(self, stream=None):
        """Free `stream`'s workspace (default: torch's current stream)."""
        check(lib.pl_plan_release(self._h, ctypes.c_void_p(_stream(stream))), "pl_plan_release")

    def workspace_stats(self):
        """(streams with a workspace, their total bytes)."""
        n, b = ctypes.c_int64(), ctypes.c_int64()
        check(lib.pl_plan_workspace_stats(self._h, ctypes.byref(n), ctypes.byref(b)), "pl_plan_workspace_stats")
        return int(n.value), int(b.value)

    def small_batch_frames(self) -> int:
        """Largest batch decoded on the small-batch tree instance (0: none)."""
        b = ctypes.c_int64()
        check(lib.pl_polar_plan_small_batch(self._h, ctypes.byref(b)), "pl_polar_plan_small_batch")
        return int(b.value)

    def workspace_bytes(self, batch: int) -> int:
        b = ctypes.c_int64()
        check(lib.pl_plan_workspace_bytes(self._h, int(batch), ctypes.byref(b)), "pl_plan_workspace_bytes")
        return int(b.value)

    def _check(self, llr, bits, iters):
        # the kernels write bits at row pitch n_out and iters densely; llr rows
        # may carry any pitch >= n_in but unit inner stride
        assert isinstance(llr, torch.Tensor) and llr.is_cuda, "llr must be a device tensor"
        assert llr.dtype == torch.float64 and llr.dim() == 2 and llr.stride(1) == 1 and llr.shape[1] >= self.info.n_in
        assert bits.is_cuda and bits.dtype == torch.uint8 and bits.shape == (llr.shape[0], self.info.n_out)
        assert bits.is_contiguous(), "bits must be contiguous [B, n_out] (row pitch n_out)"
        if iters is not None:
            assert iters.is_cuda and iters.dtype == torch.int32 and iters.shape == (llr.shape[0],) \
                and iters.is_contiguous(), "iters must be a contiguous int32 [B] device tensor"

    def decode(self, llr: "torch.Tensor", bits: "torch.Tensor", iters: "torch.Tensor | None" = None, stream=None,
               ws: "torch.Tensor | None" = None):
        """llr fp64 [B, >=n_in] device, bits uint8 [B, n_out] contiguous, iters int32 [B]
        or None; ws: optional caller-owned uint8 device workspace (pl_decode_ws)."""
        self._check(llr, bits, iters)
        B = llr.shape[0]
        it = ctypes.c_void_p(iters.data_ptr()) if iters is not None else None
        st = ctypes.c_void_p(_stream(stream))
        if ws is None:
            check(lib.pl_decode(self._h, ctypes.c_void_p(llr.data_ptr()), B, _ld(llr),
                                ctypes.c_void_p(bits.data_ptr()), it, st), "pl_decode")
        else:
            assert ws.is_cuda and ws.is_contiguous()
            check(lib.pl_decode_ws(self._h, ctypes.c_void_p(llr.data_ptr()), B, _ld(llr),
                                   ctypes.c_void_p(bits.data_ptr()), it, ctypes.c_void_p(ws.data_ptr()),
                                   ws.numel() * ws.element_size(), st), "pl_decode_ws")

    def decode_stamped(self, llr: "torch.Tensor", bits: "torch.Tensor", stamps: "torch.Tensor", stream=None):
        """Diagnostic decode accumulating per-phase cycle totals into stamps (int64 [5])."""
        check(lib.pl_debug_polar_stamps(self._h, ctypes.c_void_p(llr.data_ptr()), llr.shape[0], _ld(llr),
                                        _dptr(bits), _dptr(stamps), ctypes.c_void_p(_stream(stream))),
              "pl_debug_polar_stamps")

    def decode_fpw(self, llr: "torch.Tensor", bits: "torch.Tensor", stamps=None, grid: int = 0, stream=None):
        """Diagnostic: the frame-per-wavefront prototype (pl_debug_polar_fpw, N=1024 L=8)."""
        check(lib.pl_debug_polar_fpw(self._h, ctypes.c_void_p(llr.data_ptr()), llr.shape[0], _ld(llr),
                                     _dptr(bits), _dptr(stamps) if stamps is not None else None, int(grid),
                                     ctypes.c_void_p(_stream(stream))), "pl_debug_polar_fpw")

    def set_crc(self, crc_len: int, poly: int):
        """CRC-aided list selection (pl_polar_plan_set_crc); crc_len 0 = off."""
        check(lib.pl_polar_plan_set_crc(self._h, int(crc_len), ctypes.c_uint32(int(poly) & 0xFFFFFFFF)),
              "pl_polar_plan_set_crc")

    def close(self):
        if getattr(self, "_h", None):
            lib.pl_plan_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def polar_plan(N: int, K: int, frozen_mask: np.ndarray, list_size: int, flags: int = 0) -> Plan:
    require_gpu()
    mask = np.ascontiguousarray(frozen_mask, dtype=np.uint8)
    h = ctypes.c_void_p()
    check(lib.pl_polar_plan_create(int(N), int(K), mask.ctypes.data_as(ctypes.c_void_p), int(list_size),
                                   int(flags), ctypes.byref(h)), "pl_polar_plan_create")
    return Plan(h)


def ldpc_plan(row_ptr: np.ndarray, col_idx: np.ndarray, n: int, algo: int, max_iter: int, early_stop: bool,
              normalization: float = 1.0) -> Plan:
    require_gpu()
    rp = np.ascontiguousarray(row_ptr, dtype=np.int32)
    ci = np.ascontiguousarray(col_idx, dtype=np.int32)
    h = ctypes.c_void_p()
    check(lib.pl_ldpc_plan_create(len(rp) - 1, int(n), rp.ctypes.data_as(ctypes.c_void_p),
                                  ci.ctypes.data_as(ctypes.c_void_p), int(algo), int(max_iter),
                                  int(bool(early_stop)), float(normalization), 0, ctypes.byref(h)),
          "pl_ldpc_plan_create")
    return Plan(h)


def random_bits(seed: int, frame_offset: int, bits: "torch.Tensor", stream=None):
    B, k = bits.shape
    check(lib.pl_random_bits(ctypes.c_uint64(seed & (2**64 - 1)), int(frame_offset), B, k, _dptr(bits),
                             ctypes.c_void_p(_stream(stream))), "pl_random_bits")


def polar_encode(plan: Plan, msg: "torch.Tensor", codeword: "torch.Tensor", stream=None):
    check(lib.pl_polar_encode(plan.handle, _dptr(msg), msg.shape[0], _dptr(codeword),
                              ctypes.c_void_p(_stream(stream))), "pl_polar_encode")


def awgn_llr(codeword: "torch.Tensor | None", n: int, batch: int, snr_db: float, seed: int, frame_offset: int,
             llr: "torch.Tensor", stream=None):
    cw = _dptr(codeword) if codeword is not None else None
    check(lib.pl_awgn_llr(cw, int(n), int(batch), float(snr_db), ctypes.c_uint64(seed & (2**64 - 1)),
                          int(frame_offset), _dptr(llr), _ld(llr), ctypes.c_void_p(_stream(stream))),
          "pl_awgn_llr")


def count_errors(ref: "torch.Tensor", dec: "torch.Tensor", width: int, counts: "torch.Tensor", stream=None):
    check(lib.pl_count_errors(_dptr(ref), _ld(ref), _dptr(dec), _ld(dec), int(width), ref.shape[0],
                              _dptr(counts), ctypes.c_void_p(_stream(stream))), "pl_count_errors")


def crc_append(msg: "torch.Tensor", k_data: int, crc_len: int, poly: int, stream=None):
    """msg uint8 [B, >= k_data+crc_len]: write the CRC bits of msg[:, :k_data] after them."""
    check(lib.pl_crc_append(_dptr(msg), _ld(msg), msg.shape[0], int(k_data), int(crc_len),
                            ctypes.c_uint32(int(poly) & 0xFFFFFFFF), ctypes.c_void_p(_stream(stream))),
          "pl_crc_append")


def rayleigh_llr(codeword, n: int, batch: int, snr_db: float, seed: int, frame_offset: int, llr, stream=None):
    cw = _dptr(codeword) if codeword is not None else None
    check(lib.pl_rayleigh_llr(cw, int(n), int(batch), float(snr_db), ctypes.c_uint64(seed & (2**64 - 1)),
                              int(frame_offset), _dptr(llr), _ld(llr), ctypes.c_void_p(_stream(stream))),
          "pl_rayleigh_llr")


def bsc(codeword, n: int, batch: int, crossover_prob: float, seed: int, frame_offset: int, out, stream=None):
    cw = _dptr(codeword) if codeword is not None else None
    check(lib.pl_bsc(cw, int(n), int(batch), float(crossover_prob), ctypes.c_uint64(seed & (2**64 - 1)),
                     int(frame_offset), _dptr(out), _ld(out), ctypes.c_void_p(_stream(stream))), "pl_bsc")


def gf2_encode(g_packed: "torch.Tensor", k: int, n: int, msg: "torch.Tensor", cw: "torch.Tensor", stream=None):
    """cw = msg . G (GF(2)); g_packed int32 [ceil(k/32), n] device (pack_gf2_columns)."""
    assert g_packed.dtype == torch.int32 and g_packed.is_contiguous() and g_packed.shape == ((k + 31) // 32, n)
    check(lib.pl_gf2_encode(_dptr(g_packed), int(k), int(n), _dptr(msg), _ld(msg), msg.shape[0], _dptr(cw), _ld(cw),
                            ctypes.c_void_p(_stream(stream))), "pl_gf2_encode")


def pack_gf2_columns(G: np.ndarray) -> np.ndarray:
    """k x n 0/1 matrix -> int32 [ceil(k/32), n]: bit i of [w, j] = G[32 w + i, j]."""
    G = (np.asarray(G) & 1).astype(np.uint64)
    k, n = G.shape
    kw = (k + 31) // 32
    Gp = np.zeros((kw * 32, n), np.uint64)
    Gp[:k] = G
    w = (Gp.reshape(kw, 32, n) << np.arange(32, dtype=np.uint64)[None, :, None]).sum(axis=1)
    return w.astype(np.uint32).view(np.int32)
