# round 3, call m: one-launch cooperative order pass (QEC_OPT_SCHEDULE 1/2 vs 4 = two launches); gpu suite.
set -o pipefail
R="$GRAFT_REPO_ROOT"
O="$R/gpurun_out/r03m"
mkdir -p "$O"
cd "$R"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$O/pytest.log" 2>&1
rc=$?; tail -3 "$O/pytest.log"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/kbench/compare.py --code p7 --batch 65536 --reps 11 cur cur:schedule=4 cur:schedule=0 > "$O/cmp_p7_65536.txt" 2>&1 || { tail "$O/cmp_p7_65536.txt"; exit 1; }
cat "$O/cmp_p7_65536.txt"
timeout -k 10 300 python tools/kbench/compare.py --code p61 --batch 65536 --reps 9 cur cur:schedule=4 cur:schedule=0 > "$O/cmp_p61_65536.txt" 2>&1 || { tail "$O/cmp_p61_65536.txt"; exit 1; }
cat "$O/cmp_p61_65536.txt"
timeout -k 10 300 python tools/kbench/compare.py --code p7 --batch 262144 --reps 7 cur cur:schedule=4 > "$O/cmp_p7_262144.txt" 2>&1 || { tail "$O/cmp_p7_262144.txt"; exit 1; }
cat "$O/cmp_p7_262144.txt"
timeout -k 10 120 python bench.py --code p7 --global-batch 65536 --no-cpu --no-extras > "$O/bench_p7_65536.json" 2> "$O/bench_p7.err" || { tail "$O/bench_p7.err"; exit 1; }
cat "$O/bench_p7_65536.json"
