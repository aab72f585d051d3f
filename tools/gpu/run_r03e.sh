# round 3, call e: gpu tests (triage gated by p), P7 column groups at 2^20, profiles: headline (with
# the VALU-mix pass), P7 configs[1], the Monte-Carlo pipeline at p = 0.002.
set -o pipefail
R="$GRAFT_REPO_ROOT"
O="$R/gpurun_out/r03e"
mkdir -p "$O"
cd "$R"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$O/pytest.log" 2>&1
rc=$?; tail -5 "$O/pytest.log"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/kbench/compare.py --code p7 --batch 1048576 --reps 5 cur cg2 cg3 > "$O/cmp_p7_2e20.txt" 2>&1 || { tail "$O/cmp_p7_2e20.txt"; exit 1; }
cat "$O/cmp_p7_2e20.txt"
timeout -k 10 600 bash tools/gpu/run_profile.sh r03e p61 || exit 1
EXTRA="--global-batch 65536" timeout -k 10 400 bash tools/gpu/run_profile.sh r03e7 p7 || exit 1
timeout -k 10 600 bash tools/gpu/run_mc_profile.sh r03e 0.002 || exit 1
