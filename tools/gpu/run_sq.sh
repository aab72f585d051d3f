# SQ stall-breakdown passes (one rocprofv3 --pmc run per group, kernel-trace only beside it)
#   bash tools/gpu/run_sq.sh TAG CODE
set -o pipefail
R="$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-sq}; CODE=${2:-p61}
OUT="$R/gpurun_out/sq_$TAG"; mkdir -p "$OUT"; cd /tmp
timeout -s KILL 60 rocprofv3 -L > "$OUT/counters.txt" 2>&1 || true
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
           "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_SCA SQ_INSTS_BRANCH GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d "$OUT/p$i" -o run -- \
      python3 "$R/bench.py" --no-cpu --no-full-arith --steps 2 --warmup 1 --code "$CODE" > "$OUT/p$i.json" 2> "$OUT/p$i.err"
  rc=$?; echo "pass $i rc=$rc"
  if [ $rc -ne 0 ]; then tail -3 "$OUT/p$i.err"; exit $rc; fi
done
python3 - "$OUT" <<'PY'
import csv, glob, sys, json
out = {}
for f in glob.glob(sys.argv[1] + "/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "bp_decode" in r["Kernel_Name"]:
            out.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
print(json.dumps({k: sum(v) / len(v) for k, v in sorted(out.items())}))
PY
