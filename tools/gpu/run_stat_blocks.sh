# statistics_packed_kernel grid size (QEC_STAT_BLOCKS) at one sweep point, kernel-trace per setting.
#   bash tools/gpu/run_stat_blocks.sh TAG p blocks...
set -o pipefail
R="$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=$1; P=$2; shift 2
OUT="$R/gpurun_out/stb_$TAG"; mkdir -p "$OUT"; cd /tmp
for nb in "$@"; do
  QEC_STAT_BLOCKS=$nb timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/b$nb" -o run -- \
      python3 "$R/tools/psweep.py" --ps $P > "$OUT/b$nb.txt" 2> "$OUT/b$nb.err" || { tail -5 "$OUT/b$nb.err"; exit 1; }
  python3 -c "
import csv
for r in csv.DictReader(open('$OUT/b$nb/run_kernel_stats.csv')):
    if 'statistics' in r['Name']: print('blocks=$nb', r['AverageNs'])"
done
