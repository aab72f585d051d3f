# experiment call: variant comparison, then (optionally) PMC passes
set -o pipefail
R="$GRAFT_REPO_ROOT"
cd "$R"
TAG=$1; shift
CODE=$1; shift
PMC=$1; shift
timeout -k 10 400 python tools/kbench/compare.py --code "$CODE" --reps 5 "$@" > gpurun_out/cmp_$TAG.txt 2>&1
rc=$?; echo "compare rc=$rc"; cat gpurun_out/cmp_$TAG.txt | tail -12
if [ $rc -ne 0 ]; then exit $rc; fi
if [ "$PMC" = "pmc" ]; then bash tools/gpu/run_pmc.sh "$TAG" "$CODE"; fi
