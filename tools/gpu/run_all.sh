# GPU tests, headline bench, and the p-sweep (config 5 shape, 1 GPU)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-run}
echo "start $(date)"
timeout -k 10 900 python -m pytest tests -m gpu -q --maxfail=30 -p no:cacheprovider > gpurun_out/pytest_gpu_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -25 gpurun_out/pytest_gpu_$TAG.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err; brc=$?
echo "bench rc=$brc"; cat gpurun_out/bench_$TAG.json; tail -3 gpurun_out/bench_$TAG.err
if [ $brc -ne 0 ]; then exit $brc; fi
timeout -k 10 400 python tools/psweep.py --total 262144 --out gpurun_out/psweep_$TAG.json > gpurun_out/psweep_$TAG.log 2>&1
echo "psweep rc=$?"; cat gpurun_out/psweep_$TAG.log | tail -12
