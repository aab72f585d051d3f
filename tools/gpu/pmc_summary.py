"""Reduce one tools/gpu/run_profile.sh directory (a rocprofv3 --kernel-trace --stats pass and
the --pmc passes of `bench.py --no-extras`) into profiles/pmc_<code>.json, which bench.py
reads for its VALU-issue roofline and `traffic`.

For the BP decode kernels (Kernel_Name contains bp_decode_kernel), per decode step (one launch,
or the X and Z launches of the sector-launch shape, summed):
  * HBM bytes = 2 x FETCH_SIZE + WRITE_SIZE (both reported in KiB), following
    MI355X_MICROARCH.md 'HBM [CDNA4]': on gfx950 FETCH_SIZE counts half the bytes of a
    coalesced streaming read, WRITE_SIZE counts the bytes;
  * SQ_INSTS_VALU / _LDS / _SALU: wave instructions issued; SQ_WAVES; SQ_WAIT_ANY,
    SQ_ACTIVE_INST_ANY, SQ_WAVE_CYCLES (quad-cycles), GRBM_GUI_ACTIVE (cycles);
  * duration: the kernel-trace pass's average (the PMC passes serialise and slow kernels);
  * VALU issue fraction = SQ_INSTS_VALU x 2 cycles / (1024 SIMDs x 2.4 GHz x duration).
Per-syndrome values (÷ the launch's batch) let bench.py price other batch sizes of the same
workload.

Usage: python tools/gpu/pmc_summary.py --dir gpurun_out/prof_TAG/p61 --code p61
       --bench gpurun_out/prof_TAG/p61/bench_trace.json --out profiles/pmc_p61.json
(tools/gpu/run_profile.sh runs the passes and this summary per workload).
"""
import argparse
import csv
import glob
import hashlib
import json
import os
import sys

KERNEL = "bp_decode_kernel"


def counter_rows(d):
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            yield from csv.DictReader(fh)


def per_dispatch(d, kernel=KERNEL):
    """{counter: {kernel name: [value per dispatch]}} and each decode kernel's metadata.  A decode step
    may be several launches (the sector launches: an X kernel, then a Z kernel), so values are kept
    per kernel name and a step is the sum over the names of their per-dispatch averages."""
    per, names, meta = {}, {}, {}
    for row in counter_rows(d):
        name = row.get("Kernel_Name", "")
        if kernel not in name:
            continue
        key = (row["Dispatch_Id"], row["Counter_Name"])
        per[key] = per.get(key, 0.0) + float(row["Counter_Value"])
        names[row["Dispatch_Id"]] = name
        meta[name] = {"vgpr": int(row["VGPR_Count"]), "sgpr": int(row["SGPR_Count"]),
                      "scratch_bytes_per_lane": int(row["Scratch_Size"]), "lds_bytes": int(row["LDS_Block_Size"]),
                      "workgroup": int(row["Workgroup_Size"])}
    vals = {}
    for (disp, counter), v in per.items():
        vals.setdefault(counter, {}).setdefault(names[disp], []).append(v)
    return vals, meta


def per_step(vals):
    """{counter: value per decode step}: per kernel name the average over its dispatches, summed."""
    return {c: sum(sum(v) / len(v) for v in by_name.values()) for c, by_name in vals.items()}


def trace_duration_ns(d, kernel=KERNEL):
    """Decode time per step: per kernel name the average duration, summed; and the dispatch count."""
    durs = {}
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if kernel in row.get("Kernel_Name", ""):
                    durs.setdefault(row["Kernel_Name"], []).append(int(row["End_Timestamp"]) - int(row["Start_Timestamp"]))
    if not durs:
        return None, 0
    return sum(sum(v) / len(v) for v in durs.values()), sum(len(v) for v in durs.values())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dir", required=True)
    ap.add_argument("--code", required=True)
    ap.add_argument("--bench", required=True, help="bench.py JSON line of the trace pass (workload)")
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    with open(a.bench) as f:
        line = [x for x in f.read().splitlines() if x.startswith("{")][-1]
    b = json.loads(line)
    batch = b["config"]["per_gpu_batch"]
    vals, meta = {}, {}
    for sub in sorted(glob.glob(os.path.join(a.dir, "pmc*"))):
        if os.path.isdir(sub):
            v, m = per_dispatch(sub)
            vals.update(v)
            meta.update(m)
    if "SQ_INSTS_VALU" not in vals:
        raise SystemExit("no SQ_INSTS_VALU rows for the decode kernel under %s" % a.dir)
    avg = per_step(vals)
    dur_ns, ndisp = trace_duration_ns(os.path.join(a.dir, "trace"))
    kernels = sorted(meta)
    out = {"code": a.code, "batch": batch, "iters": b["config"]["bp_iters"], "stop": b["config"]["stop"],
           "p": b["config"]["p"], "output": b["config"].get("output"), "hard_paths": b["config"].get("hard_paths", 1),
           "input": b["config"].get("input", "bytes"),
           "kernel": " + ".join(kernels), "launches_per_step": len(kernels),
           "vgpr": max(m["vgpr"] for m in meta.values()), "sgpr": max(m["sgpr"] for m in meta.values()),
           "scratch_bytes_per_lane": max(m["scratch_bytes_per_lane"] for m in meta.values()),
           "lds_bytes": max(m["lds_bytes"] for m in meta.values()), "workgroup": meta[kernels[0]]["workgroup"],
           "kernels": meta,
           "dispatches": {k: sum(len(x) for x in v.values()) for k, v in vals.items()},
           "kernel_trace_avg_ns": dur_ns, "kernel_trace_dispatches": ndisp,
           "timing_basis": "per step: each decode kernel's average over its dispatches, summed over the kernels"}
    per_launch = {k: round(v) for k, v in avg.items()}
    out["per_launch"] = per_launch
    # the library the counters were collected on: bench.py uses this profile only for that binary
    root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    lib = os.path.join(root, "qec_ldpc_amd", "libqecldpc.so")
    with open(lib, "rb") as fh:
        out["library_sha256"] = hashlib.sha256(fh.read()).hexdigest()
    sys.path.insert(0, root)
    import qec_ldpc_amd
    out["build_id"] = qec_ldpc_amd.build_id()
    if "FETCH_SIZE" in avg and "WRITE_SIZE" in avg:
        hbm = 2.0 * avg["FETCH_SIZE"] * 1024.0 + avg["WRITE_SIZE"] * 1024.0
        out["hbm_bytes_per_launch"] = round(hbm)
        out["hbm_bytes_per_syndrome"] = hbm / batch
        out["hbm_correction"] = "2 x FETCH_SIZE + WRITE_SIZE, KiB -> B (MI355X_MICROARCH.md, HBM [CDNA4])"
    out["valu_insts_per_launch"] = round(avg["SQ_INSTS_VALU"])
    out["valu_insts_per_syndrome"] = avg["SQ_INSTS_VALU"] / batch
    if dur_ns:
        issue_s = avg["SQ_INSTS_VALU"] * 2 / (1024 * 2.4e9)
        out["valu_issue_frac"] = round(issue_s / (dur_ns * 1e-9), 4)
        out["valu_issue_basis"] = "SQ_INSTS_VALU x 2 cycles / (1024 SIMDs x 2.4 GHz x kernel-trace duration)"
    # cost-weighted VALU issue (profiles/r03/valu_probe.json, event throughput at 32 waves per SIMD
    # requested: v_mul / v_add / v_fma 2.1-2.4 cycles, v_rcp_f32 8.1, i.e. a transcendental holds the
    # SIMD's VALU for four plain slots) and LDS issue (ds_bpermute_b32 24.2 SIMD-cycles, the CU's LDS
    # shared by 4 SIMDs: 6 CU-cycles per wave instruction, an upper price for the cheaper ds_read/write)
    if dur_ns and "SQ_INSTS_VALU_TRANS_F32" in avg:
        trans = avg["SQ_INSTS_VALU_TRANS_F32"]
        slots = avg["SQ_INSTS_VALU"] - trans + 4 * trans
        out["valu_trans_per_launch"] = round(trans)
        out["valu_weighted_slots_per_syndrome"] = slots / batch
        out["valu_weighted_issue_frac"] = round(slots * 2 / (1024 * 2.4e9) / (dur_ns * 1e-9), 4)
        out["valu_mix_per_launch"] = {k[len("SQ_INSTS_VALU_"):]: round(avg[k]) for k in avg
                                      if k.startswith("SQ_INSTS_VALU_") and k != "SQ_INSTS_VALU_TRANS_F32"}
    if dur_ns and "SQ_INSTS_LDS" in avg:
        out["lds_issue_frac"] = round(avg["SQ_INSTS_LDS"] * 6 / (256 * 2.4e9) / (dur_ns * 1e-9), 4)
        out["lds_issue_basis"] = "SQ_INSTS_LDS x 6 CU-cycles (ds_bpermute_b32 price) / (256 CUs x 2.4 GHz x duration)"
    if avg.get("SQ_ACTIVE_INST_LDS") and "SQ_LDS_BANK_CONFLICT" in avg:
        # extra LDS cycles from bank conflicts over the cycles with an LDS instruction active
        out["lds_bank_conflict_share"] = round(avg["SQ_LDS_BANK_CONFLICT"] / avg["SQ_ACTIVE_INST_LDS"], 4)
    if "SQ_WAIT_ANY" in avg and "SQ_ACTIVE_INST_ANY" in avg:
        out["wait_over_issue"] = round(avg["SQ_WAIT_ANY"] / max(avg["SQ_ACTIVE_INST_ANY"], 1), 4)
    with open(a.out, "w") as fh:
        json.dump(out, fh, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
