# syndrome-stop occupancy (P61 4 vs 3 waves/SIMD) at three error rates
set -o pipefail
cd "$GRAFT_REPO_ROOT"
for pp in 0.01 0.03 0.05; do
  timeout -k 10 200 python tools/kbench/compare.py --code p61 --stop 2 --p $pp --reps 5 cur syn3 cur > gpurun_out/cmp_s7t_syn_$pp.txt 2>&1 || { tail -5 gpurun_out/cmp_s7t_syn_$pp.txt; exit 1; }
  echo "== $pp"; grep "syn/s" gpurun_out/cmp_s7t_syn_$pp.txt
done
