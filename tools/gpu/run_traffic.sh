# roofline.traffic: FETCH_SIZE and WRITE_SIZE of the decode kernel, one rocprofv3 --pmc
# pass each (kernel-trace only beside it), reduced by pmc_summary.py into
# gpurun_out/pmc_<code>.json (copy to profiles/ to make bench.py report it).
#   bash tools/gpu/run_traffic.sh TAG CODE
set -o pipefail
R="$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-traffic}; CODE=${2:-p61}
OUT="$R/gpurun_out/traffic_${TAG}_$CODE"; mkdir -p "$OUT"; cd /tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $c --output-format csv -d "$OUT/$c" -o run -- \
      python3 "$R/bench.py" --no-cpu --no-full-arith --steps 3 --warmup 1 --code "$CODE" > "$OUT/$c.json" 2> "$OUT/$c.err"
  rc=$?; echo "pmc $c rc=$rc"
  if [ $rc -ne 0 ]; then tail -3 "$OUT/$c.err"; exit $rc; fi
done
case $CODE in p61) IT=50;; p7) IT=20;; esac
python3 "$R/tools/gpu/pmc_summary.py" --fetch "$OUT/FETCH_SIZE" --write "$OUT/WRITE_SIZE" --code "$CODE" \
    --batch 65536 --iters $IT --stop fixed --out "$R/gpurun_out/pmc_$CODE.json"
