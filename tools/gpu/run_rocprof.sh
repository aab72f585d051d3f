# rocprofv3 kernel-trace summary of the bench (no PMC in this pass)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
R="$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-r01}
CODE=${2:-p61}
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_$TAG" -o run -- python3 "$R/bench.py" --no-cpu --no-full-arith --steps 10 --warmup 2 --code "$CODE" > "$R/gpurun_out/bench_prof_$TAG.json" 2> "$R/gpurun_out/bench_prof_$TAG.err"
echo "rocprof rc=$?"
find "$R/gpurun_out/prof_$TAG" -name "*stats*" | head
for f in $(find "$R/gpurun_out/prof_$TAG" -name "*kernel_stats.csv"); do cat "$f"; done
cat "$R/gpurun_out/bench_prof_$TAG.json"
