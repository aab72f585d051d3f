"""Reduce one p of tools/gpu/run_mc_profile.sh (a kernel-trace pass and five PMC passes of
`tools/psweep.py --stop S --ps P --reps 1`: 2^20 samples in one batch) into profiles/pmc_mc_p61_p<P>.json
(syndrome stop) or profiles/pmc_mc_p61_<S>_p<P>.json (other stop rules), which
tools/psweep.py reads for the roofline of its lines.

Per kernel of the Monte-Carlo call (fused sampler/triage kernel, list-mode decode, survivor statistics,
or the front end / ordered decode / statistics above p = 0.01): its average dispatch time (trace pass),
the counters per dispatch (PMC passes, averaged over the dispatches), and
  * VALU issue fraction = SQ_INSTS_VALU x 2 cycles / (1024 SIMDs x 2.4 GHz x dispatch time);
  * LDS issue fraction  = SQ_INSTS_LDS x 6 CU-cycles / (256 CUs x 2.4 GHz x dispatch time) (the
    ds_bpermute_b32 price, an upper price for the cheaper LDS instructions);
  * wait / issue = SQ_WAIT_ANY / SQ_ACTIVE_INST_ANY; LDS bank-conflict share of the LDS-active cycles;
  * HBM bytes = 2 x FETCH_SIZE + WRITE_SIZE (KiB -> B; MI355X_MICROARCH.md, HBM [CDNA4]).
Usage: python tools/gpu/mc_pmc_summary.py --dir gpurun_out/mc_TAG/p0.002 --p 0.002 --out pmc.json
"""
import argparse
import csv
import glob
import json
import os
import re
import sys


def short(name):
    base = name.split("(")[0]
    base = re.sub(r"^void ", "", base)
    kern = base.split("<")[0].replace("qec::", "")
    mode = re.search(r", (\d)>$", base)
    if kern == "bp_decode_kernel" and mode:
        return "bp_decode_kernel[mode %s]" % mode.group(1)
    return kern


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dir", required=True)
    ap.add_argument("--p", type=float, required=True)
    ap.add_argument("--stop", default="syndrome", choices=["syndrome", "fixed", "ref"])
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    durs = {}
    for f in glob.glob(os.path.join(a.dir, "trace", "**", "*kernel_trace.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            durs.setdefault(short(row["Kernel_Name"]), []).append(int(row["End_Timestamp"]) - int(row["Start_Timestamp"]))
    per = {}
    meta = {}
    for f in glob.glob(os.path.join(a.dir, "pmc*", "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            k = short(row["Kernel_Name"])
            key = (k, row["Dispatch_Id"], row["Counter_Name"])
            per[key] = per.get(key, 0.0) + float(row["Counter_Value"])
            meta[k] = {"vgpr": int(row["VGPR_Count"]), "scratch_bytes_per_lane": int(row["Scratch_Size"]),
                       "lds_bytes": int(row["LDS_Block_Size"]), "workgroup": int(row["Workgroup_Size"])}
    vals = {}
    for (k, disp, c), v in per.items():
        vals.setdefault(k, {}).setdefault(c, []).append(v)
    root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    sys.path.insert(0, root)
    import qec_ldpc_amd
    out = {"p": a.p, "samples": 1 << 20, "batch": 1 << 20, "stop": a.stop, "iters": 50,
           "code": "J_4_K_5_L_10_P_61_s_9_t_49", "build_id": qec_ldpc_amd.build_id(),
           "source": "tools/gpu/run_mc_profile.sh (rocprofv3 kernel trace + 5 PMC passes of tools/psweep.py --stop %s "
                     "--ps P --reps 1)" % a.stop,
           "kernels": {}}
    for k, d in sorted(durs.items()):
        if k.startswith("__amd_rocclr"):
            continue
        ns = sum(d) / len(d)
        e = {"avg_ns": round(ns), "trace_dispatches": len(d), **meta.get(k, {})}
        c = {n: sum(v) / len(v) for n, v in vals.get(k, {}).items()}
        e["counters_per_dispatch"] = {n: round(v) for n, v in sorted(c.items())}
        if "SQ_INSTS_VALU" in c:
            e["valu_issue_frac"] = round(c["SQ_INSTS_VALU"] * 2 / (1024 * 2.4e9) / (ns * 1e-9), 4)
        if "SQ_INSTS_LDS" in c:
            e["lds_issue_frac"] = round(c["SQ_INSTS_LDS"] * 6 / (256 * 2.4e9) / (ns * 1e-9), 4)
        if c.get("SQ_ACTIVE_INST_ANY"):
            e["wait_over_issue"] = round(c.get("SQ_WAIT_ANY", 0.0) / c["SQ_ACTIVE_INST_ANY"], 4)
        if c.get("SQ_ACTIVE_INST_LDS") and "SQ_LDS_BANK_CONFLICT" in c:
            e["lds_bank_conflict_share"] = round(c["SQ_LDS_BANK_CONFLICT"] / c["SQ_ACTIVE_INST_LDS"], 4)
        if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
            hbm = 2.0 * c["FETCH_SIZE"] * 1024 + c["WRITE_SIZE"] * 1024
            e["hbm_bytes"] = round(hbm)
            e["hbm_GBps"] = round(hbm / (ns * 1e-9) / 1e9, 1)
        out["kernels"][k] = e
    dom = max(out["kernels"], key=lambda k: out["kernels"][k]["avg_ns"])
    out["dominant"] = dom
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1)
    print("p=%g dominant %s %.1f us" % (a.p, dom, out["kernels"][dom]["avg_ns"] / 1e3),
          {k: (round(v["avg_ns"] / 1e3, 1), v.get("valu_issue_frac"), v.get("lds_issue_frac"), v.get("wait_over_issue"))
           for k, v in out["kernels"].items()})


if __name__ == "__main__":
    main()
