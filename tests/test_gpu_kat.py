"""End-to-end known-answer tests on the GPU: DecoderGPU::GetStatistics (errors from the
reference's mt19937(seed) stream, GPU decode with the reference stop rule, I-P logical check)
reproduces the reference's published CodeStatistics counters -- every block of
QEC_LDPC/results/** (tests/golden/kat.json) -- and the CLI (main.cu's loop) writes results
blocks in the reference format.

The archived blocks (QEC_LDPC/results/archive/*) come from two generations of the reference
(SURVEY.md section 4).  tests/golden/kat_archive.json, made by the ORACLE
(tests/golden/classify_archive.py), says which counter mapping each follows:
  full        every counter as published;
  no_logical  written before logical-error detection existed: published Corrected =
              Corrected + Logical of the current code, every other counter as published;
  unmatched   neither (excluded here, with the reason in the skip message).
"""
import json
import os
import re
import subprocess

import pytest

import qec_ldpc_amd as q
from conftest import COUNTERS, GOLDEN, ROOT, code_key

pytestmark = pytest.mark.gpu

MAP = {"tested": "numErrorsTested", "withX": "numXErrorsTested", "withZ": "numZErrorsTested",
       "corrected": "corrected", "synX": "syndromeErrorsX", "synZ": "syndromeErrorsZ",
       "logical": "logicalErrors", "convX": "convergenceFailX", "convZ": "convergenceFailZ"}


def _records():
    with open(os.path.join(GOLDEN, "kat.json")) as f:
        recs = json.load(f)
    cls = {}
    path = os.path.join(GOLDEN, "kat_archive.json")
    if os.path.exists(path):
        with open(path) as f:
            cls = {(r["set"], r["file"], r["block"]): r["class"] for r in json.load(f)}
    out = []
    for r in recs:
        c = "full" if r["set"] not in ("archive", ".") else cls.get((r["set"], r["file"], r["block"]), "unclassified")
        out.append((r, c))
    return out


RECORDS = _records()


def _id(rc):
    r, c = rc
    m = re.search(r"_W_(\d+)_MAX_(\d+)_p_([0-9.]+)", r["file"])
    return "%s-%s-W%s-MAX%s-p%s-b%d" % (r["set"].strip("[]").replace(",", "_")[:12], code_key(r), m.group(1),
                                        m.group(2), m.group(3), r["block"])


@pytest.fixture(scope="module")
def decoders(code_paths):
    out = {}
    for k, p in code_paths.items():
        c = q.Quantum_LDPC_Code.createFromFile(p)
        out[k] = q.DecoderGPU(c, 0)
    return out


@pytest.mark.parametrize("rc", RECORDS, ids=[_id(x) for x in RECORDS])
def test_gpu_reproduces_published_counters(rc, decoders):
    rec, cls = rc
    if cls in ("unmatched", "unclassified"):
        pytest.skip("archive block %s: the oracle (CPU restatement of the current DecoderCPU) reproduces it "
                    "under neither known counter mapping" % cls)
    st = decoders[code_key(rec)].GetStatistics(rec["W"], rec["tested"], rec["p_run"], rec["MAX"], rec["seed"])
    got = {k: st[MAP[k]] for k in COUNTERS}
    if cls == "no_logical":
        got["corrected"] += got["logical"]
        got["logical"] = 0
    assert got == {k: rec[k] for k in COUNTERS}, (rec["file"], rec["block"], cls)
    assert st["randSeed"] == rec["seed"] and st["errorWeight"] == rec["W"]


def test_every_archive_block_classified():
    """The fixture classifies every archived block, and every one of them reproduces."""
    arch = [c for r, c in RECORDS if r["set"] in ("archive", ".")]
    assert len(arch) == 89 and "unclassified" not in arch and "unmatched" not in arch


def test_getstats_through_cpp_interface(code_paths, kat_records):
    """DecoderGPU::GetStats (QEC_LDPC/DecoderGPU.h:193-228) on the flat error arrays of a
    published block equals GetStatistics on its seed, on one device and on a two-part decoder."""
    rec = [r for r in kat_records if r["set"] == "[2,3,6,7,2,3]" and r["file"].endswith("_W_5_MAX_100_p_0.02.txt")][0]
    for devs in ("0", "0,0"):
        r = subprocess.run([os.path.join(ROOT, "tools", "getstats_check"), code_paths["P7"], str(rec["W"]), "20000",
                            str(rec["MAX"]), "0.02", str(rec["seed"]), "--devices", devs],
                           capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, r.stdout + r.stderr
        out = json.loads(r.stdout.strip().splitlines()[-1])
        assert out["getstats"] == out["getstatistics"] and out["getstats"][0] == 20000


@pytest.mark.parametrize("flags", [[], ["--gpus", "1"], ["--devices", "0,0"]])
def test_cli_drop_in(tmp_path, code_paths, flags):
    (tmp_path / "results").mkdir()
    (tmp_path / "init.txt").write_text("%s 1 2 2000 30 0.02\n" % code_paths["P7"])
    r = subprocess.run([os.path.join(ROOT, "tools", "qec_ldpc")] + flags + ["init.txt"], cwd=tmp_path,
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



@pytest.mark.parametrize("stop,flags", [("syndrome", []), ("ref", ["--devices", "0,0"]), ("fixed", ["--batch", "4096"])])
def test_cli_philox_runs(tmp_path, code_paths, decoders, stop, flags):
    """--rng philox: COUNT depolarising samples at p (qec_monte_carlo) -> one results block whose
    counters equal the library's Monte-Carlo run on the same Philox stream, for every stop rule,
    device list and batch size."""
    (tmp_path / "results").mkdir()
    (tmp_path / "init.txt").write_text("%s 1 1 20000 30 0.02\n" % code_paths["P7"])
    r = subprocess.run([os.path.join(ROOT, "tools", "qec_ldpc"), "--rng", "philox", "--stop", stop,
                        "--seed", "0x51EC0DE"] + flags + ["init.txt"],
                       cwd=tmp_path, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    files = os.listdir(tmp_path / "results")
    assert files == ["[J=3,K=3,L=6,P=7,s=2,t=3][[n=42,k=0]]_DEPOLARIZING_MAX_30_p_0.02_%s.txt" % stop]
    fields = dict(re.findall(r"^([A-Za-z ()\-]+): (.*)$", (tmp_path / "results" / files[0]).read_text(), flags=re.M))
    want = decoders["P7"].monte_carlo(0x51EC0DE, 0, 20000, 0.02, 30, stop)
    names = {"tested": "Errors Tested", "withX": "Errors With X", "withZ": "Errors With Z",
             "corrected": "Corrected", "synX": "Syndrome Errors X", "synZ": "Syndrome Errors Z",
             "logical": "Logical Errors", "convX": "Convergence Fail X", "convZ": "Convergence Fail Z",
             "iterationsX": "Iterations X", "iterationsZ": "Iterations Z"}
    assert {k: int(fields[v]) for k, v in names.items()} == {k: want[k] for k in names}
    assert want["tested"] == 20000 and fields["Stop Rule"] == stop
