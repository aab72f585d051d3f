# P7 order pass: staged vs direct histogram and chunk sizes (environment overrides), kernel trace
# of the P7 bench workload per setting.   bash tools/gpu/run_hist_ab.sh TAG
set -o pipefail
R="$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-x}
OUT="$R/gpurun_out/hist_$TAG"; mkdir -p "$OUT"; cd /tmp
for cfg in ${CFGS:-0:1024 1:1024 1:2048 1:4096 1:8192}; do
  st=${cfg%%:*}; ch=${cfg#*:}
  QEC_HIST_STAGED=$st QEC_HIST_CHUNK=$ch timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/s${st}c$ch" -o run -- \
      python3 "$R/bench.py" --code p7 --no-cpu --no-extras --steps 20 > "$OUT/s${st}c$ch.json" 2> "$OUT/s${st}c$ch.err" || { tail -5 "$OUT/s${st}c$ch.err"; exit 1; }
  python3 -c "
import csv, json
d = json.loads(open('$OUT/s${st}c$ch.json').read().splitlines()[-1])
t = {r['Name'][:30]: float(r['AverageNs']) / 1e3 for r in csv.DictReader(open('$OUT/s${st}c$ch/run_kernel_stats.csv')) if 'schedule' in r['Name']}
print('staged=$st chunk=$ch', round(d['value'] / 1e9, 3), 'G/s', {k: round(v, 1) for k, v in t.items()})"
done
