# Variant comparisons on several workloads in one call:
#   bash tools/gpu/run_cmp.sh TAG variant...   (P61 @ p=0.01 and 0.05, P7 @ 0.02)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=$1; shift
for w in "p61:" "p61_p05:--p 0.05" "p7:"; do
  name=${w%%:*}; extra=${w#*:}; code=${name%%_*}
  timeout -k 10 300 python tools/kbench/compare.py --code $code $extra --reps 5 "$@" > gpurun_out/cmp_${TAG}_$name.txt 2>&1 \
    || { tail -5 gpurun_out/cmp_${TAG}_$name.txt; exit 1; }
  echo "== $name"; grep "syn/s" gpurun_out/cmp_${TAG}_$name.txt
done
