# p-sweep points with the dispatch-order pass on/off (QEC_OPT_SCHEDULE via psweep --opt).
#   bash tools/gpu/run_sched_ab.sh TAG p...
set -o pipefail
R="$GRAFT_REPO_ROOT"
TAG=${1:-x}; shift
OUT="$R/gpurun_out/sched_$TAG"; mkdir -p "$OUT"
for s in 1 0; do
  timeout -k 10 300 python "$R/tools/psweep.py" --ps $* --opt schedule=$s --out "$OUT/s$s.json" > "$OUT/s$s.txt" 2>&1 || { tail -5 "$OUT/s$s.txt"; exit 1; }
  python3 -c "
import json
for l in json.load(open('$OUT/s$s.json')): print('schedule=$s p=%-6g %12.1f syn/s  decode %.4f s of %.4f s' % (l['p'], l['syndromes_per_s'], l['decode_seconds'], l['seconds']))"
done
