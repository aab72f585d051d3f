# Time build/variants/<name> libraries against each other on the standard workloads (P61 fixed
# @ p=0.01 2^20 and @ p=0.05, P61 syndrome stop @ p=0.002, P7 fixed): V="a b c" bash tools/gpu/run_variants.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"
V="${V:-cur nmin}"
for w in "p61:--batch 1048576" "p61_p05:--p 0.05 --batch 262144" "p61_syn:--p 0.002 --stop 2 --batch 262144" "p7:--batch 1048576"; do
  name=${w%%:*}; extra=${w#*:}; code=${name%%_*}
  timeout -k 10 300 python tools/kbench/compare.py --code $code $extra --reps 5 $V > gpurun_out/var_$name.txt 2>&1 \
    || { tail -5 gpurun_out/var_$name.txt; exit 1; }
  echo "== $name"; grep "syn/s" gpurun_out/var_$name.txt
done
