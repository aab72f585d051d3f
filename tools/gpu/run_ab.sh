# A/B timings of bench.py variants on one box, then the rocprof evidence.
#   bash tools/gpu/run_ab.sh TAG "label:bench args" ...
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=$1; shift
for k in 1 2; do
  for v in "$@"; do
    name=${v%%:*}; a=${v#*:}
    timeout -k 10 150 python bench.py --no-cpu --no-extras $a > gpurun_out/ab_${TAG}_${name}_$k.json 2>gpurun_out/ab_${TAG}.err || { tail -5 gpurun_out/ab_${TAG}.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/ab_${TAG}_${name}_$k.json')); print('%-12s %14.1f syn/s  decode %.4f ms' % ('$name', d['value'], d['decode_ms']))"
  done
done
