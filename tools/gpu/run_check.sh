# Full GPU check: all -m gpu tests, the headline bench, then optional variant comparisons.
#   bash tools/gpu/run_check.sh TAG [p7 variants...]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-run}; shift
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/pytest_gpu_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu_$TAG.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err; brc=$?
echo "bench rc=$brc"; cat gpurun_out/bench_$TAG.json
[ $brc -ne 0 ] && { tail -5 gpurun_out/bench_$TAG.err; exit $brc; }
if [ $# -gt 0 ]; then
  timeout -k 10 300 python tools/kbench/compare.py --code p7 --reps 5 "$@" > gpurun_out/cmp_p7_$TAG.txt 2>&1
  echo "p7 compare rc=$?"; grep "syn/s" gpurun_out/cmp_p7_$TAG.txt
fi
