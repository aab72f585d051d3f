"""The CLI's flags on the CPU (tools/qec_ldpc, main.cu's loop: QEC_LDPC/main.cu:43-118; SURVEY.md
section 5 "Config / flags"): --engine cpu runs DecoderCPU (the library's host engine, no GPU) and
writes the reference's results blocks; inconsistent flags exit with status 2 before any decoder
exists.  The GPU side (--engine gpu, --rng philox) is tests/test_gpu_kat.py."""
import os
import re
import subprocess

import pytest

from conftest import ROOT

CLI = os.path.join(ROOT, "tools", "qec_ldpc")


def _run(tmp_path, flags, code=None, line="1 2 2000 30 0.02"):
    (tmp_path / "results").mkdir(exist_ok=True)
    if code:
        (tmp_path / "init.txt").write_text("%s %s\n" % (code, line))
    return subprocess.run([CLI] + flags + ["init.txt"], cwd=tmp_path, capture_output=True, text=True, timeout=120)


def test_cli_cpu_engine(tmp_path, code_paths):
    r = _run(tmp_path, ["--engine", "cpu"], code_paths["P7"])
    assert r.returncode == 0, r.stderr
    assert "Engine: CPU" in r.stdout
    files = sorted(os.listdir(tmp_path / "results"))
    assert files == ["[J=3,K=3,L=6,P=7,s=2,t=3][[n=42,k=0]]_W_1_MAX_30_p_0.02.txt",
                     "[J=3,K=3,L=6,P=7,s=2,t=3][[n=42,k=0]]_W_2_MAX_30_p_0.02.txt"]
    hw = os.cpu_count() or 1
    for f in files:
        fields = dict(re.findall(r"^([A-Za-z ()\-]+): (.*)$", (tmp_path / "results" / f).read_text(), flags=re.M))
        tested = int(fields["Errors Tested"])
        assert tested == (2000 // hw) * hw  # DecoderCPU.h:420-440: numErrors / nThreads per thread
        # every tested sample is either corrected, a syndrome fail, or a logical error
        assert int(fields["Corrected"]) + int(fields["Logical Errors"]) <= tested
        assert int(fields["Errors With X"]) <= tested and int(fields["Errors With Z"]) <= tested
    assert "Run complete." in (tmp_path / "output_log.txt").read_text()


@pytest.mark.parametrize("flags", [
    ["--engine", "tpu"],
    ["--engine", "cpu", "--gpus", "2"],
    ["--engine", "cpu", "--rng", "philox"],
    ["--rng", "mt"],
    ["--stop", "fixed"],           # GetStatistics keeps the reference stop rule
    ["--batch", "1024"],
    ["--rng", "philox", "--stop", "never"],
    ["--rng", "philox", "--batch", "0"],
    ["--rng", "philox", "--batch", "x"],
    ["--frobnicate", "1"],
])
def test_cli_refuses_bad_flags(tmp_path, code_paths, flags):
    r = _run(tmp_path, flags, code_paths["P7"])
    assert r.returncode == 2, (flags, r.stdout, r.stderr)
    assert "usage: qec_ldpc" in r.stderr
    assert os.listdir(tmp_path / "results") == []
