set -o pipefail
cd "$GRAFT_REPO_ROOT"
echo "start $(date)"; nproc; rocm-smi --showproductname 2>&1 | head -8
timeout -k 10 900 python -m pytest tests -m gpu -q --maxfail=30 -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -30 gpurun_out/pytest_gpu.log
if [ $rc -eq 0 ] || [ $rc -eq 1 ]; then
  timeout -k 10 400 python bench.py > gpurun_out/bench1.json 2> gpurun_out/bench1.err; echo "bench rc=$?"; cat gpurun_out/bench1.json; tail -5 gpurun_out/bench1.err
fi
