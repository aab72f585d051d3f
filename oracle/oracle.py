"""ctypes view of oracle/liboracle.so -- TEST INFRASTRUCTURE ONLY.

The CPU restatement of the reference decoder (oracle/qec_oracle.c).  Only
tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this
module, and only as the checker / the timed CPU baseline; the product package
qec_ldpc_amd never imports it.
"""
import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "liboracle.so")

STOP = {"ref": 0, "fixed": 1, "syndrome": 2}


class Stats(ctypes.Structure):
    _fields_ = [(k, ctypes.c_uint32) for k in
                ("tested", "withX", "withZ", "weight", "corrected", "synX", "synZ", "logical", "convX", "convZ")]

    def as_dict(self):
        return {k: int(getattr(self, k)) for k, _ in self._fields_}


_lib = None


def build():
    """Compile the restatement (gcc, -ffp-contract=off: reference float semantics)."""
    import subprocess
    subprocess.check_call(["make", "-s", "-C", _HERE])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        vp, i, f, u8p = ctypes.c_void_p, ctypes.c_int, ctypes.c_float, ctypes.c_void_p
        L.oc_code_load.restype = vp
        L.oc_code_load.argtypes = [ctypes.c_char_p]
        L.oc_code_free.argtypes = [vp]
        L.oc_code_info.argtypes = [vp, ctypes.c_void_p]
        L.oc_decode_batch.restype = i
        L.oc_decode_batch.argtypes = [vp, u8p, u8p, ctypes.c_long, f, i, i, u8p, u8p, u8p, vp, vp, i]
        L.oc_syndrome_batch.argtypes = [vp, i, u8p, ctypes.c_long, u8p]
        L.oc_sample_fixed_weight.argtypes = [ctypes.c_uint32, i, ctypes.c_long, i, u8p, u8p]
        L.oc_get_statistics.restype = i
        L.oc_get_statistics.argtypes = [vp, i, ctypes.c_long, f, i, ctypes.c_uint32, i, ctypes.POINTER(Stats)]
        L.oc_check_logical.restype = i
        L.oc_check_logical.argtypes = [vp, ctypes.c_void_p]
        _lib = L
    return _lib


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p) if a is not None else None


class OracleCode:
    """Quantum_LDPC_Code as the oracle loads it (QEC_LDPC/Quantum_LDPC_Code.h:26-80)."""

    def __init__(self, path):
        self._h = lib().oc_code_load(os.fsencode(path))
        if not self._h:
            raise FileNotFoundError("Unable to find code file " + str(path))
        info = np.zeros(9, dtype=np.int32)
        lib().oc_code_info(self._h, _p(info))
        self.J, self.K, self.L, self.P, self.sigma, self.tau, self.n, self.mX, self.mZ = map(int, info)

    def __del__(self):
        if getattr(self, "_h", None):
            lib().oc_code_free(self._h)
            self._h = None

    def syndrome(self, sector, e):
        e = np.ascontiguousarray(e, dtype=np.uint8)
        B = e.shape[0]
        m = self.mZ if sector else self.mX
        s = np.empty((B, m), dtype=np.uint8)
        lib().oc_syndrome_batch(self._h, int(sector), _p(e), B, _p(s))
        return s

    def decode_batch(self, sX, sZ, p, max_iter, stop="ref", want_q=False, nthreads=0):
        sX = np.ascontiguousarray(sX, dtype=np.uint8)
        sZ = np.ascontiguousarray(sZ, dtype=np.uint8)
        B = sX.shape[0]
        eX = np.empty((B, self.n), dtype=np.uint8)
        eZ = np.empty((B, self.n), dtype=np.uint8)
        flags = np.empty(B, dtype=np.uint8)
        iters = np.empty((B, 2), dtype=np.int32)
        q = np.empty((B, (self.mX + self.mZ) * self.L), dtype=np.float32) if want_q else None
        rc = lib().oc_decode_batch(self._h, _p(sX), _p(sZ), B, float(p), int(max_iter), STOP[stop],
                                   _p(eX), _p(eZ), _p(flags), _p(iters), _p(q), int(nthreads))
        if rc:
            raise RuntimeError("oracle decode failed (irregular code?)")
        return eX, eZ, flags, iters, q

    def sample_fixed_weight(self, seed, W, count):
        x = np.empty((count, self.n), dtype=np.uint8)
        z = np.empty((count, self.n), dtype=np.uint8)
        lib().oc_sample_fixed_weight(seed & 0xFFFFFFFF, W, count, self.n, _p(x), _p(z))
        return x, z

    def check_logical(self, ex, ez):
        errs = np.concatenate([ex, ez]).astype(np.int32)
        return bool(lib().oc_check_logical(self._h, _p(errs)))

    def get_statistics(self, W, tested, p, max_iter, seed, nthreads=0):
        st = Stats()
        lib().oc_get_statistics(self._h, W, tested, float(p), max_iter, seed & 0xFFFFFFFF, nthreads,
                                ctypes.byref(st))
        return st.as_dict()
