# iterative-minreg scheduling vs default across stop rules and codes
set -o pipefail
cd "$GRAFT_REPO_ROOT"
for spec in "p61_fix:--code p61 --stop 1" "p61_syn:--code p61 --stop 2" "p61_ref:--code p61 --stop 0" "p7_fix:--code p7 --stop 1" "p7_syn:--code p7 --stop 2" "p7_ref:--code p7 --stop 0"; do
  name=${spec%%:*}; extra=${spec#*:}
  timeout -k 10 200 python tools/kbench/compare.py $extra --reps 7 cur minreg cur minreg > gpurun_out/cmp_s7v_$name.txt 2>&1 || { tail -5 gpurun_out/cmp_s7v_$name.txt; exit 1; }
  echo "== $name"; grep "syn/s" gpurun_out/cmp_s7v_$name.txt
done
