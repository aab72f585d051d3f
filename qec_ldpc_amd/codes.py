"""Locations of the code files the reference ships (QEC_LDPC's J_*_K_*... text files).

The repository keeps them gzip-compressed under tests/golden/codes/ (data
fixtures); `code_path(name)` returns a plain-text copy the C loader can read,
materialised once per process in a temp directory.
"""
import gzip
import os
import tempfile

_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CODE_DIR = os.path.join(_ROOT, "tests", "golden", "codes")
P7 = "J_3_K_3_L_6_P_7_s_2_t_3"
P61 = "J_4_K_5_L_10_P_61_s_9_t_49"
_cache = {}


def code_path(name):
    if name in _cache and os.path.exists(_cache[name]):
        return _cache[name]
    src = os.path.join(CODE_DIR, name + ".txt.gz")
    d = tempfile.mkdtemp(prefix="qec_codes_")
    dst = os.path.join(d, name + ".txt")
    with gzip.open(src, "rb") as f, open(dst, "wb") as g:
        g.write(f.read())
    _cache[name] = dst
    return dst


def write_code_file(path, J, K, L, P, sigma, tau, HX, HZ, IMP=None):
    """Write a code in the reference's 4-line text format (Quantum_LDPC_Code.h:26-80):
    "J K L P sigma tau" / HX row-major / HZ row-major / I-P row-major (zeros if None)."""
    import numpy as np

    n = HX.shape[1]
    if IMP is None:
        IMP = np.zeros((2 * n, 2 * n), dtype=np.uint8)

    def row(a):
        return " ".join(map(str, np.asarray(a, dtype=np.uint8).ravel().tolist()))

    with open(path, "w") as f:
        f.write("%d %d %d %d %d %d\n" % (J, K, L, P, sigma, tau))
        f.write(row(HX) + "\n")
        f.write(row(HZ) + "\n")
        f.write(row(IMP) + "\n")
    return path
