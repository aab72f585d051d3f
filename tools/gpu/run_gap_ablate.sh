# mc_gap_kernel ablations (timing only): QEC_GAP_ABLATE = 0 full, 1 no write-out, 2 no walk.
#   bash tools/gpu/run_gap_ablate.sh TAG [p] [spw]
set -o pipefail
R="$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-x}; P=${2:-0.002}; SPW=${3:-16}
OUT="$R/gpurun_out/abl_$TAG"
mkdir -p "$OUT"
cd /tmp
for ab in 0 1 2; do
  QEC_GAP_SPW=$SPW QEC_GAP_ABLATE=$ab timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/a$ab" -o run -- \
      python3 "$R/tools/psweep.py" --ps $P > "$OUT/a$ab.txt" 2> "$OUT/a$ab.err" || { tail -5 "$OUT/a$ab.err"; exit 1; }
  python3 -c "
import csv
for r in csv.DictReader(open('$OUT/a$ab/run_kernel_stats.csv')):
    print('ablate=$ab', r['Name'][:36], r['AverageNs'])" | grep -E "gap|statistics"
done
