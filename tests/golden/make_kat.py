"""Extract known-answer fixtures from the reference's published results files.

Run in the build container (where /root/reference exists):
    python tests/golden/make_kat.py

The reference's QEC_LDPC/results/**.txt files are CodeStatistics text blocks
(format: QEC_LDPC/CodeStatistics.h:22-37) written by main.cu's loop
(QEC_LDPC/main.cu:91-104) with the seed of each run.  Each block becomes one
record: (code, W, MAX, p from the file name, seed, tested) -> the 8 counters.
Only data is extracted; nothing from the reference's sources is kept.

`p_run` is the errorProbability the block was actually produced with.  The P=61
files of results/[4,5,10,61,9,49]/ whose names say p_0.01 reproduce only with 0.02
(SURVEY.md section 4), so their p_run is 0.02; everything else, the top-level P=61
p_0.01 file included (it reproduces with 0.01), uses the file-name value.
"""
import json
import os
import re
import sys

REF = "/root/reference/QEC_LDPC/results"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "kat.json")

FIELDS = [
    ("Rand Seed", "seed"),
    ("Duration(micro-s)", "duration_us"),
    ("Errors Tested", "tested"),
    ("Errors With X", "withX"),
    ("Errors With Z", "withZ"),
    ("Error Weight", "weight"),
    ("Corrected", "corrected"),
    ("Syndrome Errors X", "synX"),
    ("Syndrome Errors Z", "synZ"),
    ("Logical Errors", "logical"),
    ("Convergence Fail X", "convX"),
    ("Convergence Fail Z", "convZ"),
]

NAME_RE = re.compile(r"\[J=(\d+),K=(\d+),L=(\d+),P=(\d+),s=(\d+),t=(\d+)\]\[\[n=\d+,k=-?\d+\]\]_W_(\d+)_MAX_(\d+)_p_([0-9.]+)\.txt$")


def parse_blocks(text):
    blocks, cur = [], {}
    for line in text.splitlines():
        line = line.strip()
        if line.startswith("Code:"):
            if cur:
                blocks.append(cur)
            cur = {}
            continue
        for label, key in FIELDS:
            if line.startswith(label + ":"):
                cur[key] = int(line.split(":", 1)[1])
    if cur:
        blocks.append(cur)
    return blocks


def main():
    if not os.path.isdir(REF):
        sys.exit("reference results not present; the committed kat.json is the fixture")
    recs = []
    for sub in ["[2,3,6,7,2,3]", "[4,5,10,61,9,49]", "archive", "."]:
        d = os.path.join(REF, sub)
        for fn in sorted(os.listdir(d)):
            m = NAME_RE.search(fn)
            if not m:
                continue
            J, K, L, P, s, t, W, MAX = map(int, m.groups()[:8])
            p_file = float(m.group(9))
            code = "J_%d_K_%d_L_%d_P_%d_s_%d_t_%d" % (J, K, L, P, s, t)
            p_run = 0.02 if (sub == "[4,5,10,61,9,49]" and P == 61 and p_file == 0.01) else p_file
            with open(os.path.join(d, fn)) as f:
                blocks = parse_blocks(f.read())
            for bi, b in enumerate(blocks):
                rec = {"set": sub, "file": fn, "block": bi, "code": code, "W": W, "MAX": MAX,
                       "p_file": p_file, "p_run": p_run}
                rec.update(b)
                recs.append(rec)
    with open(OUT, "w") as f:
        json.dump(recs, f, indent=0)
    print("wrote %d records to %s" % (len(recs), OUT))


if __name__ == "__main__":
    main()
