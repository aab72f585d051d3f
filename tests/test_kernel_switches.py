"""The decode kernels keep only the compile-time switches some build uses in both states (VERDICT round 5,
item 5: every experiment switch measured slower was removed in round 6, its measurement kept under
profiles/).  This test pins that list and checks that the kernel source compiles (semantic analysis
of every instantiated kernel, -fsyntax-only) in each state of each remaining switch.  The product build
(Makefile) compiles the translation-unit selectors and QEC_PHASE_STATS both ways for real."""
import os
import re
import shutil
import subprocess

import pytest

from conftest import ROOT

SRC = os.path.join(ROOT, "qec_ldpc_amd", "csrc", "bp_decode.hip")
HIPCC = "/opt/rocm/bin/hipcc"

# switch -> the build that uses its non-default state
ALLOWED = {
    "QEC_PHASE_STATS": "bp_decode_phase.hip (the instrumented kernels of QEC_OPT_PHASE_STATS)",
    "QEC_P61_MINREG_TU": "bp_decode_p61.hip (the iterative-minreg translation unit)",
    "QEC_PHASE_TU": "bp_decode_phase.hip",
    "QEC_KBENCH_MINIMAL": "tools/kbench/build_variants.sh, spills.sh (shipped-code kernels only)",
}


def test_only_listed_switches():
    text = open(SRC).read()
    found = set(re.findall(r"#\s*(?:ifndef|ifdef|if|elif)\s+(?:defined\()?\s*(QEC_[A-Z0-9_]+)", text))
    found |= set(re.findall(r"defined\((QEC_[A-Z0-9_]+)\)", text))
    assert found <= set(ALLOWED), sorted(found - set(ALLOWED))


@pytest.mark.skipif(not shutil.which(HIPCC) and not os.path.exists(HIPCC), reason="no hipcc")
@pytest.mark.parametrize("defines", [[], ["-DQEC_KBENCH_MINIMAL"], ["-DQEC_PHASE_STATS=1", "-DQEC_PHASE_TU=1"],
                                     ["-DQEC_P61_MINREG_TU=1"]])
def test_compiles_in_each_state(defines):
    r = subprocess.run([HIPCC, "--offload-arch=gfx950", "-std=c++17", "-fsyntax-only", "-ffp-contract=off",
                        "-Wno-unused-command-line-argument", *defines, SRC], capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
