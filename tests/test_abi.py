"""The C-ABI shared object loads and exports every symbol include/qec_ldpc.h declares
(no GPU compute here)."""
import ctypes
import os
import re
import subprocess

import pytest

import qec_ldpc_amd as q

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    txt = open(os.path.join(ROOT, "include", "qec_ldpc.h")).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(qec_[a-z_0-9]+)\s*\(", txt)))


def test_every_declared_symbol_is_exported():
    lib = ctypes.CDLL(q.LIB_PATH)
    syms = declared_symbols()
    assert len(syms) >= 18
    missing = [s for s in syms if not hasattr(lib, s)]
    assert not missing, missing
    assert set(syms) == set(q.EXPORTS)


def test_exports_are_c_linkage():
    out = subprocess.run(["nm", "-D", "--defined-only", q.LIB_PATH], capture_output=True, text=True).stdout
    for s in declared_symbols():
        assert re.search(r"\bT %s$" % s, out, flags=re.M), s


def test_abi_version_and_error_text():
    assert q.lib().qec_abi_version() == 4
    assert q.lib().qec_code_load(b"/nonexistent/code.txt") is None
    assert "Unable to find code file" in q.last_error()


def test_no_oracle_in_product():
    """The product library never links the oracle."""
    out = subprocess.run(["ldd", q.LIB_PATH], capture_output=True, text=True).stdout
    assert "oracle" not in out
    src = open(os.path.join(ROOT, "qec_ldpc_amd", "__init__.py")).read()
    assert "oracle" not in src.split('"""', 2)[2]


def test_cli_built():
    assert os.access(os.path.join(ROOT, "tools", "qec_ldpc"), os.X_OK)


def test_headers_compile_as_cpp(tmp_path):
    """The C++ mirror of the reference interface compiles against the C ABI."""
    src = tmp_path / "t.cpp"
    src.write_text('#include "Decoder.h"\n#include "DecoderGPU.h"\n#include "QC_LDPC_CSS.h"\n'
                   '#include "RandomErrorGenerator.h"\nint main(){ return 0; }\n')
    r = subprocess.run(["g++", "-std=c++17", "-fsyntax-only", "-I", os.path.join(ROOT, "include"), str(src)],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr


@pytest.mark.skipif(os.path.exists("/dev/kfd"), reason="a GPU may be present")
def test_decoder_create_without_gpu_fails_loudly(code_paths):
    c = q.Quantum_LDPC_Code.createFromFile(code_paths["P61"])
    with pytest.raises(q.QecError, match="HIP"):
        q.DecoderGPU(c)


def test_build_id_matches_sources():
    """qec_build_id() is the Makefile's hash of the library sources: the loaded library was built
    from this tree (a stale .so, or one built from other sources, fails here)."""
    import glob
    import hashlib
    csrc = os.path.join(ROOT, "qec_ldpc_amd", "csrc")
    srcs = sorted(glob.glob(os.path.join(csrc, "*.hip")) + glob.glob(os.path.join(csrc, "*.cpp"))
                  + glob.glob(os.path.join(csrc, "*.h")))
    srcs += [os.path.join(ROOT, "include", "qec_ldpc.h"), os.path.join(ROOT, "include", "HostDeviceArray.h"),
             os.path.join(ROOT, "Makefile")]
    h = hashlib.sha256(b"".join(open(s, "rb").read() for s in srcs)).hexdigest()[:16]
    assert q.build_id() == h
