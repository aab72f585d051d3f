# The N > 1 bench path rehearsed on one GPU: two ranks sharing GPU 0 over gloo (RCCL needs one GPU
# per rank), strong scaling of the 2^20 batch, gather timed alone and end to end.
#   bash tools/gpu/run_rehearse.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r02}
QEC_BENCH_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 2 --no-extras \
    > gpurun_out/bench_2rank_$TAG.json 2> gpurun_out/bench_2rank_$TAG.err
rc=$?; echo "2-rank rc=$rc"; grep "^{" gpurun_out/bench_2rank_$TAG.json | tail -1; tail -3 gpurun_out/bench_2rank_$TAG.err
exit $rc
