# Syndrome-stop decode (config 5's kernel) of build/variants/<name> libraries at several p, P61
# and P7:  bash tools/gpu/run_syn_variants.sh TAG variant...
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=$1; shift
for w in "p61_002:--p 0.002" "p61_01:--p 0.01" "p61_05:--p 0.05" "p61_1:--p 0.1 --batch 65536" "p7_02:--p 0.02 --batch 1048576" "p7_1:--p 0.1 --batch 1048576"; do
  name=${w%%:*}; extra=${w#*:}; code=${name%%_*}
  timeout -k 10 300 python tools/kbench/compare.py --code $code --stop 2 --iters 50 --batch 262144 $extra --reps 5 "$@" \
      > gpurun_out/syn_${TAG}_$name.txt 2>&1 || { tail -5 gpurun_out/syn_${TAG}_$name.txt; exit 1; }
  echo "== $name"; grep "syn/s" gpurun_out/syn_${TAG}_$name.txt
done
