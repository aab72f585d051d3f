# Monte-Carlo (config 5) evidence: the p-sweep, its kernel-trace summary and two PMC passes of
# one sweep point (front end, decode, statistics kernels).
#   bash tools/gpu/run_mc_profile.sh TAG [p]
set -o pipefail
R="$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-r02}; P=${2:-0.002}
OUT="$R/gpurun_out/mc_$TAG"
mkdir -p "$OUT"
cd "$R"
timeout -k 10 300 python tools/psweep.py --out "$OUT/psweep.json" > "$OUT/psweep.txt" 2>&1 || { tail -5 "$OUT/psweep.txt"; exit 1; }
tail -1 "$OUT/psweep.txt"
python -c "
import json
for l in json.load(open('$OUT/psweep.json')): print('p=%-6g %12.1f syn/s  decode %.4f s of %.4f s' % (l['p'], l['syndromes_per_s'], l['decode_seconds'], l['seconds']))"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- \
    python3 "$R/tools/psweep.py" --ps $P > /dev/null 2> "$OUT/trace.err" || { tail -5 "$OUT/trace.err"; exit 1; }
cat "$OUT/trace/run_kernel_stats.csv"
i=0
for grp in "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES" "SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -k 10 -s KILL 180 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d "$OUT/pmc$i" -o run -- \
      python3 "$R/tools/psweep.py" --ps $P --total 262144 > /dev/null 2> "$OUT/pmc$i.err"
  rc=$?; echo "pmc$i rc=$rc"; if [ $rc -ne 0 ]; then tail -5 "$OUT/pmc$i.err"; exit $rc; fi
done
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
out = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(out + "/pmc*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0][-40:]
        agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in agg.items():
    print(k, {c: round(sum(v) / len(v)) for c, v in sorted(d.items())})
PY
