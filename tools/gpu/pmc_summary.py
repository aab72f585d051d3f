"""Reduce rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of `bench.py --no-cpu` into
profiles/pmc_<code>.json, which bench.py reads for roofline.traffic.

HBM bytes per decode launch = 2 x FETCH_SIZE + WRITE_SIZE (both reported in KiB),
following MI355X_MICROARCH.md 'HBM [CDNA4]': on gfx950 FETCH_SIZE counts half the
bytes of a coalesced streaming read, WRITE_SIZE counts the bytes.  Only the BP
decode kernel's dispatches are used (the sampler/syndrome kernels run before the
timed region and are excluded).

Usage: python tools/gpu/pmc_summary.py --fetch DIR --write DIR --code p61
       --batch 65536 --iters 50 --stop fixed --out profiles/pmc_p61.json
"""
import argparse
import csv
import glob
import json
import os


def counter_values(d, name, kernel_substr="bp_decode_kernel"):
    vals, kname = [], None
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if row.get("Counter_Name") == name and kernel_substr in row.get("Kernel_Name", ""):
                    vals.append(float(row["Counter_Value"]))
                    kname = row["Kernel_Name"]
    return vals, kname


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write", required=True)
    ap.add_argument("--code", required=True)
    ap.add_argument("--batch", type=int, required=True)
    ap.add_argument("--iters", type=int, required=True)
    ap.add_argument("--stop", default="fixed")
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    fv, kname = counter_values(a.fetch, "FETCH_SIZE")
    wv, _ = counter_values(a.write, "WRITE_SIZE")
    if not fv or not wv:
        raise SystemExit("no FETCH_SIZE/WRITE_SIZE rows for the decode kernel under %s / %s" % (a.fetch, a.write))
    fetch = sum(fv) / len(fv) * 1024.0
    write = sum(wv) / len(wv) * 1024.0
    out = {
        "code": a.code, "batch": a.batch, "iters": a.iters, "stop": a.stop, "kernel": kname,
        "dispatches": {"fetch": len(fv), "write": len(wv)},
        "fetch_size_bytes_raw": round(fetch), "write_size_bytes": round(write),
        "hbm_bytes_per_launch": round(2.0 * fetch + write),
        "correction": "2 x FETCH_SIZE + WRITE_SIZE (MI355X_MICROARCH.md, HBM [CDNA4]: gfx950 FETCH_SIZE counts half)",
    }
    with open(a.out, "w") as fh:
        json.dump(out, fh, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
