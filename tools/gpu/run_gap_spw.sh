# Monte-Carlo front end: samples per wave of mc_gap_kernel (QEC_GAP_SPW) at one sweep point,
# kernel-trace summaries per setting.
#   bash tools/gpu/run_gap_spw.sh TAG [p] [spw...]
set -o pipefail
R="$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-x}; P=${2:-0.002}; shift 2
OUT="$R/gpurun_out/spw_$TAG"
mkdir -p "$OUT"
cd /tmp
for spw in ${*:-8 16 32 64}; do
  QEC_GAP_SPW=$spw timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/s$spw" -o run -- \
      python3 "$R/tools/psweep.py" --ps $P > "$OUT/s$spw.txt" 2> "$OUT/s$spw.err" || { tail -5 "$OUT/s$spw.err"; exit 1; }
  echo "== spw=$spw $(tail -1 $OUT/s$spw.txt)"
  grep -E "mc_gap|statistics_packed" "$OUT/s$spw/run_kernel_stats.csv" | cut -d, -f1-4
done
