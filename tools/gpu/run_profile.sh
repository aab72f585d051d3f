# rocprofv3 evidence for bench.py's roofline, per code: one kernel-trace --stats pass and four
# PMC passes (each counter group in its own run, --kernel-trace only beside --pmc), then the
# per-launch / per-syndrome summary bench.py reads (profiles/pmc_<code>.json).
#   bash tools/gpu/run_profile.sh TAG [codes...]
# EXTRA="--global-batch 65536" profiles another workload of bench.py (same per-code layout).
set -o pipefail
R="$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-r02}; shift
CODES=${*:-p61 p7}
OUT="$R/gpurun_out/prof_$TAG"
mkdir -p "$OUT"; cd /tmp
for code in $CODES; do
  mkdir -p "$OUT/$code"
  BENCH="$R/bench.py --no-cpu --no-extras --code $code $EXTRA"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/$code/trace" -o run -- \
      python3 $BENCH --steps 10 --warmup 2 > "$OUT/$code/bench_trace.json" 2> "$OUT/$code/trace.err"
  rc=$?; echo "$code trace rc=$rc"; cat "$OUT/$code/bench_trace.json"
  if [ $rc -ne 0 ]; then tail -5 "$OUT/$code/trace.err"; exit $rc; fi
  i=0
  for grp in "FETCH_SIZE" "WRITE_SIZE" "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES" \
             "SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES GRBM_GUI_ACTIVE" \
             "SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_INT32 SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT"; do
    i=$((i+1))
    timeout -k 10 -s KILL 180 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d "$OUT/$code/pmc$i" -o run -- \
        python3 $BENCH --steps 2 --warmup 1 > "$OUT/$code/bench_pmc$i.json" 2> "$OUT/$code/pmc$i.err"
    rc=$?; echo "$code pmc$i ($grp) rc=$rc"
    if [ $rc -ne 0 ]; then tail -5 "$OUT/$code/pmc$i.err"; exit $rc; fi
  done
  python3 "$R/tools/gpu/pmc_summary.py" --dir "$OUT/$code" --code "$code" --bench "$OUT/$code/bench_trace.json" \
      --out "$OUT/pmc_$code.json" || exit 1
done
find "$OUT" -name "*kernel_stats.csv" -exec sh -c 'echo "== $1"; cat "$1"' _ {} \;
