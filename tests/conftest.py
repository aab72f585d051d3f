import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run on the GPU box with -m gpu)")


@pytest.fixture(scope="session")
def code_paths():
    from qec_ldpc_amd.codes import P7, P61, code_path
    return {"P7": code_path(P7), "P61": code_path(P61)}


@pytest.fixture(scope="session")
def kat_records():
    with open(os.path.join(GOLDEN, "kat.json")) as f:
        return json.load(f)


def kat_subset(records, quick=True):
    """A fast, representative selection of published blocks."""
    want = [
        # P7, 100 000 samples each, MAX 100, p 0.02
        ("[2,3,6,7,2,3]", "_W_1_MAX_100_p_0.02.txt", 0),
        ("[2,3,6,7,2,3]", "_W_3_MAX_100_p_0.02.txt", 0),
        ("[2,3,6,7,2,3]", "_W_3_MAX_1000_p_0.02.txt", 1),
        ("[2,3,6,7,2,3]", "_W_11_MAX_100_p_0.02.txt", 1),
        # P61, 1 000 samples, MAX 100, p 0.02
        ("[4,5,10,61,9,49]", "_W_1_MAX_100_p_0.02.txt", 0),
        ("[4,5,10,61,9,49]", "_W_15_MAX_100_p_0.02.txt", 0),
        ("[4,5,10,61,9,49]", "_W_30_MAX_100_p_0.02.txt", 0),
        ("[4,5,10,61,9,49]", "_W_45_MAX_100_p_0.02.txt", 0),
        ("[4,5,10,61,9,49]", "_W_60_MAX_100_p_0.02.txt", 0),
        # P61 file labelled p_0.01 that was produced with 0.02 (10 000 samples)
        ("[4,5,10,61,9,49]", "_W_10_MAX_100_p_0.01.txt", 0),
    ]
    if not quick:
        want += [
            ("[2,3,6,7,2,3]", "_W_5_MAX_1000_p_0.02.txt", 0),
            ("[4,5,10,61,9,49]", "_W_60_MAX_1000_p_0.02.txt", 0),
        ]
    out = []
    for s, suffix, blk in want:
        for r in records:
            if r["set"] == s and r["file"].endswith(suffix) and r["block"] == blk:
                out.append(r)
    return out


COUNTERS = ["tested", "withX", "withZ", "corrected", "synX", "synZ", "logical", "convX", "convZ"]


def code_key(rec):
    return "P7" if "_P_7_" in rec["code"] else "P61"
