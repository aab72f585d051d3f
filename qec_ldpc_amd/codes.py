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
