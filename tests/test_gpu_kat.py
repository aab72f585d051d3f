"""End-to-end known-answer tests on the GPU: DecoderGPU::GetStatistics (errors from
the reference's mt19937(seed) stream, GPU decode with the reference stop rule,
I-P logical check) reproduces the reference's published CodeStatistics counters,
and the CLI (main.cu's loop) writes results blocks in the reference format."""
import os
import re
import subprocess

import pytest

import qec_ldpc_amd as q
from conftest import COUNTERS, code_key, kat_subset

pytestmark = pytest.mark.gpu

MAP = {"tested": "numErrorsTested", "withX": "numXErrorsTested", "withZ": "numZErrorsTested",
       "corrected": "corrected", "synX": "syndromeErrorsX", "synZ": "syndromeErrorsZ",
       "logical": "logicalErrors", "convX": "convergenceFailX", "convZ": "convergenceFailZ"}


@pytest.fixture(scope="module")
def decoders(code_paths):
    out = {}
    for k, p in code_paths.items():
        c = q.Quantum_LDPC_Code.createFromFile(p)
        out[k] = q.DecoderGPU(c, 0)
    return out


@pytest.mark.parametrize("idx", range(10))
def test_gpu_reproduces_published_counters(idx, kat_records, decoders):
    rec = kat_subset(kat_records)[idx]
    st = decoders[code_key(rec)].GetStatistics(rec["W"], rec["tested"], rec["p_run"], rec["MAX"], rec["seed"])
    got = {k: st[MAP[k]] for k in COUNTERS}
    assert got == {k: rec[k] for k in COUNTERS}, (rec["file"], rec["block"])
    assert st["randSeed"] == rec["seed"] and st["errorWeight"] == rec["W"]


def test_cli_drop_in(tmp_path, code_paths):
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    (tmp_path / "results").mkdir()
    (tmp_path / "init.txt").write_text("%s 1 2 2000 30 0.02\n" % code_paths["P7"])
    r = subprocess.run([os.path.join(root, "tools", "qec_ldpc"), "init.txt"], cwd=tmp_path,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    files = sorted(os.listdir(tmp_path / "results"))
    assert files == ["[J=3,K=3,L=6,P=7,s=2,t=3][[n=42,k=0]]_W_1_MAX_30_p_0.02.txt",
                     "[J=3,K=3,L=6,P=7,s=2,t=3][[n=42,k=0]]_W_2_MAX_30_p_0.02.txt"]
    txt = (tmp_path / "results" / files[1]).read_text()
    fields = dict(re.findall(r"^([A-Za-z ()\-]+): (.*)$", txt, flags=re.M))
    assert fields["Code"] == "[J=3,K=3,L=6,P=7,s=2,t=3][[n=42,k=0]]"
    assert int(fields["Errors Tested"]) == 2000 and int(fields["Error Weight"]) == 2
    assert "Run complete." in (tmp_path / "output_log.txt").read_text()
