# GPU check of the tree: the -m gpu suite, then the default bench line.
#   bash tools/gpu/run_check.sh TAG [pytest args...]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-x}; shift
echo "start $(date)"
timeout -k 10 900 python -u -m pytest tests -m gpu -q --maxfail=20 --timeout 300 --timeout-method thread \
    -p no:cacheprovider "$@" > gpurun_out/pytest_gpu_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -40 gpurun_out/pytest_gpu_$TAG.log | grep -v "^\.\+ *\[" 
if [ $rc -eq 0 ] || [ $rc -eq 1 ]; then
  timeout -k 10 400 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
  echo "bench rc=$?"; cat gpurun_out/bench_$TAG.json; tail -5 gpurun_out/bench_$TAG.err
fi
