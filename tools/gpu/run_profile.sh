# rocprofv3 evidence for bench.py's roofline: one kernel-trace --stats pass and two
# PMC passes (FETCH_SIZE, WRITE_SIZE: separate runs, --kernel-trace only beside --pmc)
# per code; then the per-launch HBM-byte summary that bench.py reads for `traffic`.
#   bash tools/gpu/run_profile.sh TAG [codes...]
set -o pipefail
R="$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-r01}; shift
CODES=${*:-p61 p7}
OUT="$R/gpurun_out/prof_$TAG"
mkdir -p "$OUT"; cd /tmp
for code in $CODES; do
  mkdir -p "$OUT/$code"
  if [ "$code" = "p7" ]; then IT=20; else IT=50; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/$code/trace" -o run -- \
      python3 "$R/bench.py" --no-cpu --no-full-arith --steps 10 --warmup 2 --code "$code" > "$OUT/$code/bench_trace.json" 2> "$OUT/$code/trace.err"
  rc=$?; echo "$code trace rc=$rc"; cat "$OUT/$code/bench_trace.json"
  if [ $rc -ne 0 ]; then tail -5 "$OUT/$code/trace.err"; exit $rc; fi
  for ctr in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 -s KILL 120 rocprofv3 --kernel-trace --pmc $ctr --output-format csv -d "$OUT/$code/$ctr" -o run -- \
        python3 "$R/bench.py" --no-cpu --no-full-arith --steps 3 --warmup 1 --code "$code" > "$OUT/$code/bench_$ctr.json" 2> "$OUT/$code/$ctr.err"
    rc=$?; echo "$code $ctr rc=$rc"
    if [ $rc -ne 0 ]; then tail -5 "$OUT/$code/$ctr.err"; exit $rc; fi
  done
  python3 "$R/tools/gpu/pmc_summary.py" --fetch "$OUT/$code/FETCH_SIZE" --write "$OUT/$code/WRITE_SIZE" \
      --code "$code" --batch 65536 --iters $IT --stop fixed --out "$OUT/pmc_$code.json" || exit 1
done
find "$OUT" -name "*kernel_stats.csv" -exec sh -c 'echo "== $1"; cat "$1"' _ {} \;
