# P61 per-variant tuning check: fixed stop (old vs new tuning), syndrome and reference stop
set -o pipefail
cd "$GRAFT_REPO_ROOT"
for spec in "fix01:--stop 1" "fix05:--stop 1 --p 0.05" "syn01:--stop 2" "syn05:--stop 2 --p 0.05" "ref01:--stop 0"; do
  name=${spec%%:*}; extra=${spec#*:}
  timeout -k 10 200 python tools/kbench/compare.py --code p61 $extra --reps 5 old cur synm1 > gpurun_out/cmp_s7n_$name.txt 2>&1 || { tail -5 gpurun_out/cmp_s7n_$name.txt; exit 1; }
  echo "== $name"; grep "syn/s" gpurun_out/cmp_s7n_$name.txt
done
