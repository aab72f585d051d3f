# P61 fixed stop under the minreg scheduler at 4 / 5 (cur) / 6 waves per SIMD
set -o pipefail
cd "$GRAFT_REPO_ROOT"
for pp in 0.01 0.05; do
  timeout -k 10 200 python tools/kbench/compare.py --code p61 --p $pp --reps 7 cur mw4 mw6 cur > gpurun_out/cmp_s7y_$pp.txt 2>&1 || { tail -5 gpurun_out/cmp_s7y_$pp.txt; exit 1; }
  echo "== $pp"; grep "syn/s" gpurun_out/cmp_s7y_$pp.txt
done
