"""The oracle (oracle/qec_oracle.c, CPU restatement of DecoderCPU) reproduces the
reference's published CodeStatistics blocks counter-for-counter.

Pin: QEC_LDPC/results/** blocks (seed -> 8 counters), extracted into
tests/golden/kat.json by tests/golden/make_kat.py.  The errors are re-drawn from
mt19937(seed) through VS2015's uniform_int_distribution (DecoderCPU.h:394-459),
decoded with the reference stop rule, and counted as DecoderCPU.h:464-521 does.
"""
import pytest

from conftest import COUNTERS, code_key, kat_subset
from oracle.oracle import OracleCode


@pytest.fixture(scope="module")
def oracle_codes(code_paths):
    return {k: OracleCode(v) for k, v in code_paths.items()}


def test_kat_fixture_well_formed(kat_records):
    assert len(kat_records) > 250
    for r in kat_records:
        assert r["tested"] > 0 and r["W"] == r["weight"]
        assert r["corrected"] + r["logical"] <= r["tested"]


@pytest.mark.parametrize("idx", range(10))
def test_oracle_reproduces_published_counters(idx, kat_records, oracle_codes):
    rec = kat_subset(kat_records)[idx]
    st = oracle_codes[code_key(rec)].get_statistics(rec["W"], rec["tested"], rec["p_run"], rec["MAX"], rec["seed"])
    got = {k: st[k] for k in COUNTERS}
    exp = {k: rec[k] for k in COUNTERS}
    assert got == exp, (rec["file"], rec["block"])


def test_oracle_p61_p001_label_needs_p002(kat_records, oracle_codes):
    """the P61 '_p_0.01' files only reproduce with errorProbability 0.02."""
    rec = [r for r in kat_subset(kat_records) if r["file"].endswith("_W_10_MAX_100_p_0.01.txt")][0]
    st = oracle_codes["P61"].get_statistics(rec["W"], 2000, 0.01, rec["MAX"], rec["seed"])
    st2 = oracle_codes["P61"].get_statistics(rec["W"], 2000, 0.02, rec["MAX"], rec["seed"])
    assert st != st2


def _archive(cls, k):
    import json
    import os
    from conftest import GOLDEN
    with open(os.path.join(GOLDEN, "kat_archive.json")) as f:
        arch = {(r["set"], r["file"], r["block"]): r["class"] for r in json.load(f)}
    with open(os.path.join(GOLDEN, "kat.json")) as f:
        recs = [r for r in json.load(f) if r["set"] == "archive" and "_P_7_" in r["code"]
                and arch[(r["set"], r["file"], r["block"])] == cls]
    return recs[k]


@pytest.mark.parametrize("cls,k", [("full", 0), ("full", 2), ("no_logical", 0), ("no_logical", 5)])
def test_oracle_archive_mapping(cls, k, oracle_codes):
    """The archive classification the GPU KAT test relies on (tests/golden/kat_archive.json,
    made by classify_archive.py) holds for a sample of P7 archive blocks: "no_logical" blocks
    were written before logical-error detection (published Corrected = Corrected + Logical)."""
    rec = _archive(cls, k)
    st = oracle_codes["P7"].get_statistics(rec["W"], rec["tested"], rec["p_run"], rec["MAX"], rec["seed"])
    if cls == "no_logical":
        assert st["logical"] > 0 and rec["logical"] == 0
        st["corrected"] += st["logical"]
        st["logical"] = 0
    assert {k2: st[k2] for k2 in COUNTERS} == {k2: rec[k2] for k2 in COUNTERS}
