set -o pipefail
cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python bench.py --stop ref --no-cpu > gpurun_out/bench_ref_s7g.json 2> gpurun_out/bench_ref_s7g.err || exit $?
cat gpurun_out/bench_ref_s7g.json | cut -c1-300
timeout -k 10 400 python tools/psweep.py --total 262144 --out gpurun_out/psweep_s7g.json > gpurun_out/psweep_s7g.log 2>&1 || exit $?
tail -10 gpurun_out/psweep_s7g.log
QEC_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 5 --warmup 2 > gpurun_out/bench_2rank_s7g.json 2> gpurun_out/bench_2rank_s7g.err || exit $?
cat gpurun_out/bench_2rank_s7g.json
