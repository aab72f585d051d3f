# P7 decode of build/variants/<name> libraries: fixed 20 at p = 0.02 (2^20 and 65 536), syndrome
# stop at p = 0.02:  bash tools/gpu/run_p7_variants.sh TAG variant...
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=$1; shift
for w in "p7:--batch 1048576" "p7_65k:--batch 65536" "p7_ref:--batch 1048576 --stop 0" "p7_syn:--batch 1048576 --stop 2 --iters 50"; do
  name=${w%%:*}; extra=${w#*:}
  timeout -k 10 300 python tools/kbench/compare.py --code p7 $extra --reps 5 "$@" > gpurun_out/p7v_${TAG}_$name.txt 2>&1 \
    || { tail -5 gpurun_out/p7v_${TAG}_$name.txt; exit 1; }
  echo "== $name"; grep "syn/s" gpurun_out/p7v_${TAG}_$name.txt
done
