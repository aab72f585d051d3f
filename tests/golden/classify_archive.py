"""Classify the reference's archived results blocks (QEC_LDPC/results/archive/*, and the
top-level results file) by re-running them through the ORACLE (CPU restatement of
DecoderCPU), so the GPU known-answer test knows which counter mapping each block follows.

SURVEY.md section 4: the archive holds blocks from two generations of the reference:
  * "full"        -- every counter matches the current DecoderCPU::GetStatistics;
  * "no_logical"  -- written by a version without logical-error detection: Errors-With,
                     Syndrome-fail and Convergence-fail counters match, and the published
                     Corrected equals Corrected + Logical of the current code (Logical 0);
  * "unmatched"   -- neither (kept in the fixture, excluded from the GPU test with this reason).

Run in the build container (no GPU needed):  python tests/golden/classify_archive.py [threads]
Writes tests/golden/kat_archive.json: [{"file", "block", "class", "oracle": {counters}}].
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from conftest import COUNTERS, code_key  # noqa: E402
from oracle.oracle import OracleCode  # noqa: E402
from qec_ldpc_amd.codes import P7, P61, code_path  # noqa: E402

OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "kat_archive.json")


def classify(rec, st):
    if all(st[k] == rec[k] for k in COUNTERS):
        return "full"
    same = ("tested", "withX", "withZ", "synX", "synZ", "convX", "convZ")
    if all(st[k] == rec[k] for k in same) and rec["logical"] == 0 and \
            rec["corrected"] == st["corrected"] + st["logical"]:
        return "no_logical"
    return "unmatched"


def main():
    threads = int(sys.argv[1]) if len(sys.argv) > 1 else 0
    with open(os.path.join(ROOT, "tests", "golden", "kat.json")) as f:
        recs = [r for r in json.load(f) if r["set"] in ("archive", ".")]
    codes = {"P7": OracleCode(code_path(P7)), "P61": OracleCode(code_path(P61))}
    done = {}
    if os.path.exists(OUT):
        with open(OUT) as f:
            done = {(r["set"], r["file"], r["block"]): r for r in json.load(f)}
    # quick ones first (P7), so a partial run is already useful
    recs.sort(key=lambda r: (code_key(r) != "P7", r["tested"], r["W"]))
    for r in recs:
        key = (r["set"], r["file"], r["block"])
        if key in done:
            continue
        t = time.time()
        st = codes[code_key(r)].get_statistics(r["W"], r["tested"], r["p_run"], r["MAX"], r["seed"], nthreads=threads)
        done[key] = {"set": r["set"], "file": r["file"], "block": r["block"], "class": classify(r, st),
                     "oracle": {k: st[k] for k in COUNTERS}}
        print("%-8s %-70s %s %.1fs" % (code_key(r), r["file"][-40:], done[key]["class"], time.time() - t), flush=True)
        with open(OUT, "w") as f:
            json.dump(sorted(done.values(), key=lambda d: (d["set"], d["file"], d["block"])), f, indent=0)


if __name__ == "__main__":
    main()
