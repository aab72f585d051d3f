# Variant comparisons (tools/kbench/build_variants.sh builds) on several workloads in one call:
#   bash tools/gpu/run_cmp.sh TAG variant...
# P61 fixed 50 @ p=0.01 (2^20 and 131 072), @ p=0.05, syndrome stop @ p=0.002, P7 fixed 20 @ 0.02.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=$1; shift
for w in "p61:--batch 1048576" "p61_131k:--batch 131072" "p61_p05:--p 0.05 --batch 262144" \
         "p61_syn:--p 0.002 --stop 2 --batch 262144" "p7:--batch 1048576"; do
  name=${w%%:*}; extra=${w#*:}; code=${name%%_*}
  timeout -k 10 300 python tools/kbench/compare.py --code $code $extra --reps 5 "$@" > gpurun_out/cmp_${TAG}_$name.txt 2>&1 \
    || { tail -5 gpurun_out/cmp_${TAG}_$name.txt; exit 1; }
  echo "== $name"; grep "syn/s" gpurun_out/cmp_${TAG}_$name.txt
done
