# Per-dispatch PMC counts (instruction mix, waits, i-cache) of build/variants/<name> libraries
# on one P61 batch: V="a b" bash tools/gpu/pmc_variants.sh
set -o pipefail
R="$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; cd /tmp
timeout -k 10 60 rocprofv3 -L > "$R/gpurun_out/counters.txt" 2>&1 || echo "list rc=$?"
grep -o "SQC_ICACHE[A-Z_]*\|SQ_IFETCH[A-Z_]*\|SQ_INSTS_BRANCH\|SQ_WAIT_INST_ANY\|SQ_INST_CYCLES_VMEM\|SQ_INSTS_SMEM" "$R/gpurun_out/counters.txt" | sort -u
V="${V:-nmin shortall}"
i=0
for grp in "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES" "SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -k 10 -s KILL 120 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d "$R/gpurun_out/pmcv/pmc$i" -o run -- \
     python3 "$R/tools/kbench/compare.py" --code p61 --batch 262144 --reps 1 $V > "$R/gpurun_out/pmcv_pmc$i.txt" 2>&1 || { echo "pmc$i failed"; tail -5 "$R/gpurun_out/pmcv_pmc$i.txt"; exit 1; }
done
if grep -q "SQC_ICACHE_MISSES" "$R/gpurun_out/counters.txt"; then
  timeout -k 10 -s KILL 120 rocprofv3 --kernel-trace --pmc SQC_ICACHE_MISSES SQC_ICACHE_HITS --output-format csv -d "$R/gpurun_out/pmcv/pmc3" -o run -- \
     python3 "$R/tools/kbench/compare.py" --code p61 --batch 262144 --reps 1 $V > "$R/gpurun_out/pmcv_pmc3.txt" 2>&1 || echo "pmc3 failed"
fi
python3 - "$R/gpurun_out/pmcv" <<'PY'
import csv, glob, sys, collections
rows = collections.defaultdict(dict)
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "bp_decode" not in r["Kernel_Name"]: continue
        key = (f.split("/pmc")[1][0], int(r["Dispatch_Id"]))
        rows[key][r["Counter_Name"]] = rows[key].get(r["Counter_Name"], 0) + float(r["Counter_Value"])
for k in sorted(rows): print(k, {c: int(v) for c, v in sorted(rows[k].items())})
PY
