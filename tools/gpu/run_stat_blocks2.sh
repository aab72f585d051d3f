# statistics kernels' grid cap (QEC_STAT_BLOCKS) on one 2^20-sample sweep point.
#   bash tools/gpu/run_stat_blocks2.sh TAG p blocks...
set -o pipefail
R="$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=$1; P=$2; shift 2
OUT="$R/gpurun_out/stb2_$TAG"; mkdir -p "$OUT"; cd /tmp
for nb in "$@"; do
  QEC_STAT_BLOCKS=$nb timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/b$nb" -o run -- \
      python3 "$R/tools/psweep.py" --ps $P > "$OUT/b$nb.txt" 2> "$OUT/b$nb.err" || { tail -5 "$OUT/b$nb.err"; exit 1; }
  python3 -c "
import csv
for r in csv.DictReader(open('$OUT/b$nb/run_kernel_stats.csv')):
    if 'statistics' in r['Name']: print('blocks=$nb', r['Calls'], r['AverageNs'])"
done
