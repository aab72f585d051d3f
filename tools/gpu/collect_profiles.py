"""Copy the PMC summaries of tools/gpu/run_profile.sh runs into profiles/ under the names bench.py
looks for (pmc_<code>[_<batch>][_hp0].json; the 2^20 workloads without the batch), after checking
that each was taken on this tree's library build, and with --rocprof DIR each workload's
kernel-trace --stats summary as DIR/<name>_kernel_stats.csv.

    python tools/gpu/collect_profiles.py [--rocprof profiles/rNN/rocprof] gpurun_out/prof_TAG [gpurun_out/prof_TAG2 ...]
"""
import glob
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def target_name(pm):
    sfx = "" if int(pm.get("hard_paths", 1)) else "_hp0"
    if pm["batch"] == 1 << 20:
        return "pmc_%s%s.json" % (pm["code"], sfx)
    return "pmc_%s_%d%s.json" % (pm["code"], pm["batch"], sfx)


def main():
    import argparse
    import qec_ldpc_amd as q
    ap = argparse.ArgumentParser()
    ap.add_argument("--rocprof", default=None, help="also copy each workload's kernel-trace summary here")
    ap.add_argument("dirs", nargs="+")
    a = ap.parse_args()
    bid = q.build_id()
    for d in a.dirs:
        for f in sorted(glob.glob(os.path.join(d, "pmc_*.json"))):
            with open(f) as fh:
                pm = json.load(fh)
            if pm.get("build_id") != bid:
                print("skip %s: build %s, this tree %s" % (f, pm.get("build_id"), bid))
                continue
            dst = os.path.join(ROOT, "profiles", target_name(pm))
            shutil.copyfile(f, dst)
            name = os.path.basename(f)[len("pmc_"):-len(".json")]
            stats = os.path.join(d, name, "trace", "run_kernel_stats.csv")
            if a.rocprof and os.path.exists(stats):
                os.makedirs(a.rocprof, exist_ok=True)
                shutil.copyfile(stats, os.path.join(a.rocprof, "%s_kernel_stats.csv" % name))
            print("%s -> %s (frac %.4f / %.4f weighted, %.1f B per syndrome)" % (
                f, os.path.relpath(dst, ROOT), pm.get("valu_issue_frac") or 0, pm.get("valu_weighted_issue_frac") or 0,
                pm.get("hbm_bytes_per_syndrome") or 0))


if __name__ == "__main__":
    main()
