"""qec_ldpc_amd -- Python view of libqecldpc.so, the MI355X belief-propagation
decoder for quasi-cyclic CSS quantum LDPC codes.

Mirrors the reference's interface (cantwellc/QEC_LDPC):
  * Quantum_LDPC_Code.createFromFile / GetSyndromeX / GetSyndromeZ / CheckLogicalError
    (QEC_LDPC/Quantum_LDPC_Code.h:26-142)
  * QC_LDPC_CSS(J, K, L, P, sigma, tau) generator (QEC_LDPC/QEC_LDPC_CSS.cu:5-131)
  * DecoderGPU(code).Decode / GetStatistics (QEC_LDPC/Decoder.h:40-47, DecoderGPU.h:117-280)
plus the batched entry points the GPU engine is built around (decode_batch,
decode_batch_dev).  Every call goes through the C ABI declared in
include/qec_ldpc.h; there is no CPU decoding path in this package.  If the
shared object is missing the import of the library fails loudly.
"""
import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libqecldpc.so")

SUCCESS = 0
SYNDROME_FAIL_X = 1
SYNDROME_FAIL_Z = 2
CONVERGENCE_FAIL_X = 4
CONVERGENCE_FAIL_Z = 8
STOP = {"ref": 0, "fixed": 1, "syndrome": 2}
ENGINE = {"auto": 0, "circulant": 1, "sparse": 2, "cpu": 3}
OPTION = {"hard_paths": 1, "cycle_jump": 2, "schedule": 3, "sector_split": 4, "phase_stats": 5, "triage": 6,
          "last_path": 7, "mc_decode_time": 8}
# QEC_PATH_* bits of QEC_OPT_LAST_PATH (include/qec_ldpc.h): the launch sequence of the last decode call
PATH = {"ordered": 1, "sector_order": 2, "split_waves": 4, "sector_launches": 8, "triage": 16, "bit_rows": 32,
        "sparse": 64, "records": 128}

# every symbol include/qec_ldpc.h declares
EXPORTS = (
    "qec_last_error", "qec_abi_version", "qec_build_id",
    "qec_code_load", "qec_code_generate", "qec_code_free", "qec_code_params", "qec_code_exponents",
    "qec_code_pcm", "qec_code_describe", "qec_code_syndrome", "qec_code_check_logical",
    "qec_decoder_create", "qec_decoder_create_engine", "qec_decoder_create_multi", "qec_decoder_destroy",
    "qec_decoder_num_parts", "qec_decoder_part", "qec_decoder_device", "qec_decoder_describe",
    "qec_decoder_set_option", "qec_decoder_get_option",
    "qec_decode_batch", "qec_decode_batch_dev", "qec_decode_batch_packed", "qec_decode_batch_packed_dev",
    "qec_decode_bits_packed_dev",
    "qec_sample_fixed_weight", "qec_get_statistics",
    "qec_sample_depolarizing_dev", "qec_sample_syndrome_dev", "qec_syndrome_dev", "qec_statistics_dev",
    "qec_statistics_packed_dev", "qec_pack_decisions_dev",
    "qec_monte_carlo",
)
MC_COUNTERS = ("withX", "withZ", "synX", "synZ", "logical", "corrected", "convX", "convZ")
MC_COUNTERS_ALL = MC_COUNTERS + ("iterationsX", "iterationsZ")


def record_bytes(n):
    """Bytes of one packed decision record (QEC_RECORD_BYTES): eX bits, eZ bits, flags byte."""
    return 2 * ((n + 7) // 8) + 1


class QecError(RuntimeError):
    pass


class Stats(ctypes.Structure):
    """qec_stats == CodeStatistics counters (QEC_LDPC/CodeStatistics.h:5-20)."""
    _fields_ = [("randSeed", ctypes.c_uint32), ("numErrorsTested", ctypes.c_uint32),
                ("numXErrorsTested", ctypes.c_uint32), ("numZErrorsTested", ctypes.c_uint32),
                ("errorWeight", ctypes.c_uint32), ("corrected", ctypes.c_uint32),
                ("syndromeErrorsX", ctypes.c_uint32), ("syndromeErrorsZ", ctypes.c_uint32),
                ("logicalErrors", ctypes.c_uint32), ("convergenceFailX", ctypes.c_uint32),
                ("convergenceFailZ", ctypes.c_uint32), ("durationMicroSeconds", ctypes.c_int64)]

    def as_dict(self):
        return {k: int(getattr(self, k)) for k, _ in self._fields_}


class MCResult(ctypes.Structure):
    """qec_mc_result: a device Monte-Carlo run's counters and timings."""
    _fields_ = [(k, ctypes.c_uint64) for k in ("tested", "withX", "withZ", "synX", "synZ", "logical", "corrected",
                                               "convX", "convZ", "iterationsX", "iterationsZ")] + \
               [("decodeSeconds", ctypes.c_double), ("totalSeconds", ctypes.c_double)]

    def as_dict(self):
        return {k: (float(getattr(self, k)) if t is ctypes.c_double else int(getattr(self, k)))
                for k, t in self._fields_}


_lib = None


def lib():
    """The loaded libqecldpc.so (raises if it was not built)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise QecError("libqecldpc.so not built (%s); run `make` or __graft_entry__.build()" % LIB_PATH)
        # One HIP runtime per process: torch ships its own libamdhip64 (soname .so.7, file name
        # .so).  Loaded first, it also serves this library's libamdhip64.so.7; loaded after
        # /opt/rocm's copy, it is a second runtime in the process and torch then sees no GPU.
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        L = ctypes.CDLL(LIB_PATH)
        vp, i, f, sz = ctypes.c_void_p, ctypes.c_int, ctypes.c_float, ctypes.c_size_t
        sig = {
            "qec_last_error": (ctypes.c_char_p, []),
            "qec_abi_version": (i, []),
            "qec_build_id": (ctypes.c_char_p, []),
            "qec_code_load": (vp, [ctypes.c_char_p]),
            "qec_code_generate": (vp, [i, i, i, i, i, i]),
            "qec_code_free": (i, [vp]),
            "qec_code_params": (i, [vp, vp]),
            "qec_code_exponents": (i, [vp, i, vp]),
            "qec_code_pcm": (i, [vp, i, vp]),
            "qec_code_describe": (i, [vp, ctypes.c_char_p, sz]),
            "qec_code_syndrome": (i, [vp, i, vp, sz, vp]),
            "qec_code_check_logical": (i, [vp, vp, vp, sz, vp]),
            "qec_decoder_create": (vp, [vp, i, sz]),
            "qec_decoder_create_engine": (vp, [vp, i, sz, i]),
            "qec_decoder_create_multi": (vp, [vp, vp, i, sz]),
            "qec_decoder_destroy": (i, [vp]),
            "qec_decoder_num_parts": (i, [vp]),
            "qec_decoder_part": (vp, [vp, i]),
            "qec_decoder_device": (i, [vp]),
            "qec_decoder_describe": (i, [vp, ctypes.c_char_p, sz]),
            "qec_decoder_set_option": (i, [vp, i, i]),
            "qec_decoder_get_option": (i, [vp, i, vp]),
            "qec_decode_batch": (i, [vp, vp, vp, sz, f, i, i, vp, vp, vp, vp, vp]),
            "qec_decode_batch_dev": (i, [vp, vp, vp, sz, f, i, i, vp, vp, vp, vp, vp, vp]),
            "qec_decode_batch_packed": (i, [vp, vp, vp, sz, f, i, i, vp, vp]),
            "qec_decode_batch_packed_dev": (i, [vp, vp, vp, sz, f, i, i, vp, vp, vp, vp]),
            "qec_decode_bits_packed_dev": (i, [vp, vp, vp, sz, f, i, i, vp, vp, vp, vp]),
            "qec_sample_fixed_weight": (i, [ctypes.c_uint32, i, sz, i, vp, vp]),
            "qec_get_statistics": (i, [vp, i, i, f, i, ctypes.c_uint32, i, ctypes.POINTER(Stats)]),
            "qec_sample_depolarizing_dev": (i, [vp, ctypes.c_uint64, ctypes.c_uint64, sz, f, vp, vp, vp]),
            "qec_sample_syndrome_dev": (i, [vp, ctypes.c_uint64, ctypes.c_uint64, sz, f, vp, vp, vp, vp]),
            "qec_syndrome_dev": (i, [vp, vp, vp, sz, vp, vp, vp]),
            "qec_statistics_dev": (i, [vp, vp, vp, vp, vp, vp, sz, vp, vp]),
            "qec_statistics_packed_dev": (i, [vp, vp, vp, vp, sz, vp, vp]),
            "qec_pack_decisions_dev": (i, [vp, vp, vp, vp, sz, vp, vp]),
            "qec_monte_carlo": (i, [vp, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64, f, i, i, sz,
                                    ctypes.POINTER(MCResult)]),
        }
        for name, (res, args) in sig.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def last_error():
    return lib().qec_last_error().decode()


def build_id():
    """Hash of the sources and flags the loaded library was built from (Makefile BUILD_ID)."""
    return lib().qec_build_id().decode()


def _check(rc, what):
    if rc != 0:
        raise QecError("%s failed (%d): %s" % (what, rc, last_error()))


def _ptr(a):
    if a is None:
        return None
    return a.ctypes.data_as(ctypes.c_void_p)


def syndrome_bytes(s):
    """Integer syndrome entries to the ABI's bytes, keeping both of the reference's readings of an
    entry: its truthiness in the check update (DecoderCPU.h:178) and its exact value in the
    syndrome comparison (:381) -- 0 -> 0, 1 -> 1, anything else -> 2 (as include/Decoder.h)."""
    s = np.asarray(s)
    return np.where(s == 0, 0, np.where(s == 1, 1, 2)).astype(np.uint8)


def _u8(a, shape):
    a = np.ascontiguousarray(a, dtype=np.uint8)
    if a.shape != shape:
        a = a.reshape(shape)
    return a


class Quantum_LDPC_Code:
    """Code model (QEC_LDPC/Quantum_LDPC_Code.h:7-150)."""

    def __init__(self, handle):
        if not handle:
            raise QecError(last_error())
        self._h = ctypes.c_void_p(handle)
        v = np.zeros(9, dtype=np.int32)
        _check(lib().qec_code_params(self._h, _ptr(v)), "qec_code_params")
        (self.J, self.K, self.L, self.P, self.sigma, self.tau, self.n, self.numEqsX,
         self.numEqsZ) = (int(x) for x in v)

    @staticmethod
    def createFromFile(path):
        h = lib().qec_code_load(os.fsencode(path))
        if not h:
            raise QecError(last_error())
        return Quantum_LDPC_Code(h)

    load = createFromFile

    def __del__(self):
        h = getattr(self, "_h", None)
        if h and _lib is not None:
            _lib.qec_code_free(h)
            self._h = None

    @property
    def handle(self):
        return self._h

    def describe(self):
        buf = ctypes.create_string_buffer(256)
        _check(lib().qec_code_describe(self._h, buf, 256), "qec_code_describe")
        return buf.value.decode()

    __str__ = describe

    def exponents(self, sector):
        R = self.K if sector else self.J
        e = np.zeros((R, self.L), dtype=np.int32)
        _check(lib().qec_code_exponents(self._h, int(sector), _ptr(e)), "qec_code_exponents")
        return e

    def pcm(self, sector):
        m = self.numEqsZ if sector else self.numEqsX
        h = np.zeros((m, self.n), dtype=np.uint8)
        _check(lib().qec_code_pcm(self._h, int(sector), _ptr(h)), "qec_code_pcm")
        return h

    @property
    def pcmX(self):
        return self.pcm(0)

    @property
    def pcmZ(self):
        return self.pcm(1)

    def syndrome(self, sector, errors):
        """Batched GetSyndromeX/Z: errors [B, n] -> [B, m]."""
        e = np.atleast_2d(np.ascontiguousarray(errors, dtype=np.uint8))
        m = self.numEqsZ if sector else self.numEqsX
        s = np.empty((e.shape[0], m), dtype=np.uint8)
        _check(lib().qec_code_syndrome(self._h, int(sector), _ptr(e), e.shape[0], _ptr(s)), "qec_code_syndrome")
        return s

    def GetSyndromeX(self, errors):
        return self.syndrome(0, errors)[0]

    def GetSyndromeZ(self, errors):
        return self.syndrome(1, errors)[0]

    def check_logical(self, ex, ez):
        ex = np.atleast_2d(np.ascontiguousarray(ex, dtype=np.uint8))
        ez = np.atleast_2d(np.ascontiguousarray(ez, dtype=np.uint8))
        out = np.empty(ex.shape[0], dtype=np.uint8)
        _check(lib().qec_code_check_logical(self._h, _ptr(ex), _ptr(ez), ex.shape[0], _ptr(out)),
               "qec_code_check_logical")
        return out.astype(bool)

    def CheckLogicalError(self, errors):
        errors = np.asarray(errors)
        return bool(self.check_logical(errors[: self.n], errors[self.n:])[0])


def QC_LDPC_CSS(J, K, L, P, sigma, tau):
    """Generated code (QEC_LDPC/QEC_LDPC_CSS.cu:5-131); carries no I-P matrix."""
    h = lib().qec_code_generate(J, K, L, P, sigma, tau)
    if not h:
        raise QecError(last_error())
    return Quantum_LDPC_Code(h)


def sample_fixed_weight(seed, W, count, n):
    """The reference's fixed-weight sampler stream (DecoderCPU.h:448-459)."""
    x = np.empty((count, n), dtype=np.uint8)
    z = np.empty((count, n), dtype=np.uint8)
    _check(lib().qec_sample_fixed_weight(seed & 0xFFFFFFFF, W, count, n, _ptr(x), _ptr(z)),
           "qec_sample_fixed_weight")
    return x, z


class DecoderGPU:
    """MI355X BP engine behind the reference's DecoderGPU slot (QEC_LDPC/DecoderGPU.h).

    engine: "auto" (wave-circulant kernel when the code has one, else sparse-graph),
    "circulant" or "sparse" (include/qec_ldpc.h, QEC_ENGINE_*).
    max_batch: sizes the device-pointer workspace so the *_dev decodes allocate nothing for
    batches up to it (graph capture); larger batches grow it on demand.
    devices: a list of HIP device ordinals for a multi-device decoder (qec_decoder_create_multi):
    the host-buffer calls, GetStatistics and monte_carlo shard their samples over the devices;
    the *_dev calls go to one of parts()."""

    def __init__(self, code, device=0, engine="auto", max_batch=0, devices=None, _handle=None):
        self.code = code
        self._owned = _handle is None
        if _handle is not None:
            h = _handle
        elif devices is not None:
            devs = (ctypes.c_int * len(devices))(*[int(x) for x in devices])
            h = lib().qec_decoder_create_multi(code.handle, devs, len(devices), int(max_batch))
        else:
            h = lib().qec_decoder_create_engine(code.handle, int(device), int(max_batch), ENGINE[engine])
        if not h:
            raise QecError(last_error())
        self._h = ctypes.c_void_p(h)
        self.device = int(lib().qec_decoder_device(self._h))
        self.num_parts = int(lib().qec_decoder_num_parts(self._h))

    def __del__(self):
        h = getattr(self, "_h", None)
        if h and _lib is not None and getattr(self, "_owned", False):
            _lib.qec_decoder_destroy(h)
        self._h = None

    def parts(self):
        """Single-device views of a multi-device decoder's parts (or [self])."""
        if self.num_parts == 1:
            return [self]
        out = []
        for k in range(self.num_parts):
            h = lib().qec_decoder_part(self._h, k)
            if not h:
                raise QecError(last_error())
            p = DecoderGPU(self.code, _handle=h)
            p._parent = self  # keeps the group (the owner of the part) alive
            out.append(p)
        return out

    def describe(self):
        buf = ctypes.create_string_buffer(256)
        _check(lib().qec_decoder_describe(self._h, buf, 256), "qec_decoder_describe")
        return buf.value.decode()

    def set_option(self, name, value):
        """qec_decoder_set_option (include/qec_ldpc.h): e.g. set_option("hard_paths", 0)."""
        _check(lib().qec_decoder_set_option(self._h, OPTION[name], int(value)), "qec_decoder_set_option")

    def get_option(self, name):
        v = ctypes.c_int(0)
        _check(lib().qec_decoder_get_option(self._h, OPTION[name], ctypes.byref(v)), "qec_decoder_get_option")
        return v.value

    def last_path(self):
        """The launch sequence of this handle's last decode call (QEC_OPT_LAST_PATH) as a set of
        PATH names, e.g. {"bit_rows", "records", "ordered", "sector_order", "sector_launches"}."""
        v = self.get_option("last_path")
        return {k for k, b in PATH.items() if v & b}

    def record_bytes(self):
        """Bytes of one packed decision record: 2 ceil(n/8) + 1."""
        return record_bytes(self.code.n)

    # ---- host buffers ------------------------------------------------------------------
    def decode_batch(self, sX, sZ, p, max_iter, stop="ref", want_iters=False, want_q=False):
        """Host-buffer batch decode -> (eX, eZ, flags, iters|None, q|None)."""
        c = self.code
        sX = np.atleast_2d(sX)
        B = sX.shape[0]
        sX = _u8(sX, (B, c.numEqsX))
        sZ = _u8(sZ, (B, c.numEqsZ))
        eX = np.empty((B, c.n), dtype=np.uint8)
        eZ = np.empty((B, c.n), dtype=np.uint8)
        flags = np.empty(B, dtype=np.uint8)
        iters = np.empty((B, 2), dtype=np.int32) if want_iters else None
        q = np.empty((B, (c.numEqsX + c.numEqsZ) * c.L), dtype=np.float32) if want_q else None
        _check(lib().qec_decode_batch(self._h, _ptr(sX), _ptr(sZ), B, float(p), int(max_iter), STOP[stop],
                                      _ptr(eX), _ptr(eZ), _ptr(flags), _ptr(iters), _ptr(q)), "qec_decode_batch")
        return eX, eZ, flags, iters, q

    def decode_batch_packed(self, sX, sZ, p, max_iter, stop="ref", want_iters=False):
        """Host-buffer batch decode to packed decision records -> (records [B, record_bytes()], iters|None)."""
        c = self.code
        sX = np.atleast_2d(sX)
        B = sX.shape[0]
        sX = _u8(sX, (B, c.numEqsX))
        sZ = _u8(sZ, (B, c.numEqsZ))
        rec = np.empty((B, self.record_bytes()), dtype=np.uint8)
        iters = np.empty((B, 2), dtype=np.int32) if want_iters else None
        _check(lib().qec_decode_batch_packed(self._h, _ptr(sX), _ptr(sZ), B, float(p), int(max_iter), STOP[stop],
                                             _ptr(rec), _ptr(iters)), "qec_decode_batch_packed")
        return rec, iters

    # ---- device buffers (torch tensors on this decoder's GPU) ---------------------------
    _binding = False

    def _issue(self, name, args):
        """Calls the C entry point, or (inside bind) returns it with its checked arguments."""
        fn = getattr(lib(), name)
        if self._binding:
            return fn, args, name
        _check(fn(*args), name)

    def bind(self, method, *args, **kw):
        """A zero-argument callable that re-issues one device-buffer decode call (decode_batch_dev,
        decode_batch_packed_dev or decode_bits_packed_dev) with these arguments: the tensors are
        validated and their pointers taken once, so each call is only the C ABI call (for launch-bound
        loops over the same buffers; the tensors must stay alive and unmoved)."""
        self._binding = True
        try:
            fn, cargs, name = method(*args, **kw)
        finally:
            self._binding = False

        def call():
            rc = fn(*cargs)
            if rc != 0:
                raise QecError("%s failed (%d): %s" % (name, rc, last_error()))
        return call

    def _stream(self, stream):
        if stream is None:
            import torch
            return torch.cuda.current_stream(self.device).cuda_stream
        return stream if isinstance(stream, int) else stream.cuda_stream

    def _t(self, t, name, dtype, shape, optional=False):
        """Device pointer of tensor t after checking it is what the C ABI will read or write."""
        if t is None:
            if optional:
                return None
            raise QecError("%s: tensor required" % name)
        import torch
        if not isinstance(t, torch.Tensor):
            raise QecError("%s: expected a torch tensor, got %s" % (name, type(t).__name__))
        if not t.is_cuda or t.device.index != self.device:
            raise QecError("%s: must be on cuda:%d (the decoder's device), is on %s" % (name, self.device, t.device))
        if t.dtype != dtype:
            raise QecError("%s: dtype must be %s, is %s" % (name, dtype, t.dtype))
        if not t.is_contiguous():
            raise QecError("%s: must be contiguous" % name)
        if tuple(t.shape) != tuple(shape):
            raise QecError("%s: shape must be %s, is %s" % (name, tuple(shape), tuple(t.shape)))
        return t.data_ptr()

    def _single(self, what):
        if self.num_parts != 1:
            raise QecError("%s: device buffers live on one GPU; call it on one of parts()" % what)

    def decode_batch_dev(self, sX, sZ, p, max_iter, stop, eX, eZ, flags, iters=None, q=None, stream=None):
        """Device-buffer batch decode on torch tensors, async on `stream` (a torch.cuda.Stream, a raw
        hipStream_t int, or None = torch's current stream on the decoder's device)."""
        import torch
        self._single("decode_batch_dev")
        c = self.code
        B = sX.shape[0]
        u8 = torch.uint8
        args = (self._t(sX, "sX", u8, (B, c.numEqsX)), self._t(sZ, "sZ", u8, (B, c.numEqsZ)),
                B, float(p), int(max_iter), STOP[stop],
                self._t(eX, "eX", u8, (B, c.n)), self._t(eZ, "eZ", u8, (B, c.n)), self._t(flags, "flags", u8, (B,)),
                self._t(iters, "iters", torch.int32, (B, 2), True),
                self._t(q, "q", torch.float32, (B, (c.numEqsX + c.numEqsZ) * c.L), True))
        return self._issue("qec_decode_batch_dev", (self._h, *args, ctypes.c_void_p(self._stream(stream))))

    def decode_batch_packed_dev(self, sX, sZ, p, max_iter, stop, records, iters=None, q=None, stream=None):
        """Device-buffer batch decode into packed decision records [B, record_bytes()] (uint8)."""
        import torch
        self._single("decode_batch_packed_dev")
        c = self.code
        B = sX.shape[0]
        u8 = torch.uint8
        args = (self._t(sX, "sX", u8, (B, c.numEqsX)), self._t(sZ, "sZ", u8, (B, c.numEqsZ)),
                B, float(p), int(max_iter), STOP[stop],
                self._t(records, "records", u8, (B, self.record_bytes())),
                self._t(iters, "iters", torch.int32, (B, 2), True),
                self._t(q, "q", torch.float32, (B, (c.numEqsX + c.numEqsZ) * c.L), True))
        return self._issue("qec_decode_batch_packed_dev", (self._h, *args, ctypes.c_void_p(self._stream(stream))))

    def decode_bits_packed_dev(self, sXbits, sZbits, p, max_iter, stop, records, iters=None, q=None, stream=None):
        """Device-buffer decode of bit-row syndromes (int32 [B, ceil(m/32)] words, bit c of a row =
        check c) into packed decision records [B, record_bytes()] (uint8)."""
        import torch
        self._single("decode_bits_packed_dev")
        c = self.code
        B = sXbits.shape[0]
        args = (self._t(sXbits, "sXbits", torch.int32, (B, (c.numEqsX + 31) // 32)),
                self._t(sZbits, "sZbits", torch.int32, (B, (c.numEqsZ + 31) // 32)),
                B, float(p), int(max_iter), STOP[stop],
                self._t(records, "records", torch.uint8, (B, self.record_bytes())),
                self._t(iters, "iters", torch.int32, (B, 2), True),
                self._t(q, "q", torch.float32, (B, (c.numEqsX + c.numEqsZ) * c.L), True))
        return self._issue("qec_decode_bits_packed_dev", (self._h, *args, ctypes.c_void_p(self._stream(stream))))

    def sample_depolarizing_dev(self, seed, start, p, x, z, stream=None):
        """Device depolarising errors (the gap walk over Philox4x32-10 words, include/qec_ldpc.h)
        for samples [start, start + x.shape[0])."""
        import torch
        self._single("sample_depolarizing_dev")
        B, n = x.shape[0], self.code.n
        _check(lib().qec_sample_depolarizing_dev(self._h, seed & (2 ** 64 - 1), start, B, float(p),
                                                 self._t(x, "x", torch.uint8, (B, n)),
                                                 self._t(z, "z", torch.uint8, (B, n)),
                                                 ctypes.c_void_p(self._stream(stream))),
               "qec_sample_depolarizing_dev")

    def sample_syndrome_dev(self, seed, start, p, sX, sZ, errp=None, stream=None):
        """Fused front end: syndromes of the depolarising errors of samples [start, start + B)
        (the sample_depolarizing_dev stream), optionally the errors bit-packed (errp [B, 2 ceil(n/8)])."""
        import torch
        self._single("sample_syndrome_dev")
        c = self.code
        B = sX.shape[0]
        _check(lib().qec_sample_syndrome_dev(self._h, seed & (2 ** 64 - 1), start, B, float(p),
                                             self._t(sX, "sX", torch.uint8, (B, c.numEqsX)),
                                             self._t(sZ, "sZ", torch.uint8, (B, c.numEqsZ)),
                                             self._t(errp, "errp", torch.uint8, (B, 2 * ((c.n + 7) // 8)), True),
                                             ctypes.c_void_p(self._stream(stream))), "qec_sample_syndrome_dev")

    def syndrome_dev(self, x, z, sX, sZ, stream=None):
        import torch
        self._single("syndrome_dev")
        c = self.code
        B = x.shape[0]
        u8 = torch.uint8
        _check(lib().qec_syndrome_dev(self._h, self._t(x, "x", u8, (B, c.n)), self._t(z, "z", u8, (B, c.n)), B,
                                      self._t(sX, "sX", u8, (B, c.numEqsX)), self._t(sZ, "sZ", u8, (B, c.numEqsZ)),
                                      ctypes.c_void_p(self._stream(stream))), "qec_syndrome_dev")

    def statistics_dev(self, x, z, eX, eZ, flags, counters, stream=None):
        """Adds the batch's CodeStatistics counters into the int64 device tensor counters[8]
        (order: MC_COUNTERS)."""
        import torch
        self._single("statistics_dev")
        c = self.code
        B = x.shape[0]
        u8 = torch.uint8
        _check(lib().qec_statistics_dev(self._h, self._t(x, "x", u8, (B, c.n)), self._t(z, "z", u8, (B, c.n)),
                                        self._t(eX, "eX", u8, (B, c.n)), self._t(eZ, "eZ", u8, (B, c.n)),
                                        self._t(flags, "flags", u8, (B,)), B,
                                        self._t(counters, "counters", torch.int64, (len(MC_COUNTERS),)),
                                        ctypes.c_void_p(self._stream(stream))), "qec_statistics_dev")

    def statistics_packed_dev(self, errp, records, counters, iters=None, stream=None):
        """Adds the counters of packed errors + packed decision records into counters (int64 device
        tensor: [8] = MC_COUNTERS, or [10] = MC_COUNTERS_ALL when iters [B, 2] is given)."""
        import torch
        self._single("statistics_packed_dev")
        c = self.code
        B = errp.shape[0]
        nc = len(MC_COUNTERS_ALL) if iters is not None else len(MC_COUNTERS)
        _check(lib().qec_statistics_packed_dev(self._h, self._t(errp, "errp", torch.uint8, (B, 2 * ((c.n + 7) // 8))),
                                               self._t(records, "records", torch.uint8, (B, self.record_bytes())),
                                               self._t(iters, "iters", torch.int32, (B, 2), True), B,
                                               self._t(counters, "counters", torch.int64, (nc,)),
                                               ctypes.c_void_p(self._stream(stream))), "qec_statistics_packed_dev")

    def pack_decisions_dev(self, eX, eZ, flags, out, stream=None):
        """Bit-packs a decoded device batch into out [B, record_bytes()] (uint8 device tensor)."""
        import torch
        self._single("pack_decisions_dev")
        c = self.code
        B = eX.shape[0]
        u8 = torch.uint8
        _check(lib().qec_pack_decisions_dev(self._h, self._t(eX, "eX", u8, (B, c.n)), self._t(eZ, "eZ", u8, (B, c.n)),
                                            self._t(flags, "flags", u8, (B,)), B,
                                            self._t(out, "out", u8, (B, self.record_bytes())),
                                            ctypes.c_void_p(self._stream(stream))), "qec_pack_decisions_dev")

    # ---- Monte-Carlo ---------------------------------------------------------------------
    def monte_carlo(self, seed, start, count, p, max_iter, stop="syndrome", batch=1 << 20):
        """Device Monte-Carlo run (sample -> syndrome -> decode -> statistics); returns a dict."""
        r = MCResult()
        _check(lib().qec_monte_carlo(self._h, seed & (2 ** 64 - 1), start, count, float(p), int(max_iter),
                                     STOP[stop], batch, ctypes.byref(r)), "qec_monte_carlo")
        return r.as_dict()

    def Decode(self, syndromeX, syndromeZ, errorProbability, maxIterations):
        """Decoder::Decode for one syndrome pair -> (ErrorCode, outErrorsX, outErrorsZ)."""
        eX, eZ, flags, _, _ = self.decode_batch(syndrome_bytes(syndromeX)[None], syndrome_bytes(syndromeZ)[None],
                                                errorProbability, maxIterations, "ref")
        return int(flags[0]), eX[0].astype(np.int32), eZ[0].astype(np.int32)

    def GetStatistics(self, errorWeight, numErrors, errorProbability, maxIterations, seed=None, nThreads=1):
        if seed is None:
            seed = int.from_bytes(os.urandom(4), "little")
        st = Stats()
        _check(lib().qec_get_statistics(self._h, errorWeight, numErrors, float(errorProbability), maxIterations,
                                        seed & 0xFFFFFFFF, nThreads, ctypes.byref(st)), "qec_get_statistics")
        return st.as_dict()


class DecoderCPU(DecoderGPU):
    """The reference's DecoderCPU slot (QEC_LDPC/DecoderCPU.h): the library's CPU engine
    (device -1; host threads, bit-identical decisions).  Host-buffer entry points and
    GetStatistics only."""

    def __init__(self, code):
        super().__init__(code, device=-1, engine="cpu")

    def GetStatistics(self, errorWeight, numErrors, errorProbability, maxIterations, seed=None, nThreads=None):
        # the reference tests (numErrors / threads) * threads samples with its OpenMP thread count
        return super().GetStatistics(errorWeight, numErrors, errorProbability, maxIterations, seed,
                                     nThreads if nThreads is not None else 1)


def format_statistics(code, st):
    """CodeStatistics operator<< text block (QEC_LDPC/CodeStatistics.h:22-37)."""
    return ("Code: %s\nRand Seed: %d\nDuration(micro-s): %d\nErrors Tested: %d\nErrors With X: %d\n"
            "Errors With Z: %d\nError Weight: %d\nCorrected: %d\nSyndrome Errors X: %d\n"
            "Syndrome Errors Z: %d\nLogical Errors: %d\nConvergence Fail X: %d\nConvergence Fail Z: %d\n"
            % (code.describe(), st["randSeed"], st["durationMicroSeconds"], st["numErrorsTested"],
               st["numXErrorsTested"], st["numZErrorsTested"], st["errorWeight"], st["corrected"],
               st["syndromeErrorsX"], st["syndromeErrorsZ"], st["logicalErrors"], st["convergenceFailX"],
               st["convergenceFailZ"]))
