# round 3, call v: one-launch bucket-form dispatch order (P7) vs the two-launch counting sort; gpu suite.
set -o pipefail
R="$GRAFT_REPO_ROOT"
O="$R/gpurun_out/r03v"
mkdir -p "$O"
cd "$R"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$O/pytest.log" 2>&1
rc=$?; tail -3 "$O/pytest.log"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/kbench/compare.py --code p7 --batch 65536 --reps 15 cur cur:schedule=4 cur:schedule=0 > "$O/cmp_p7_65536.txt" 2>&1 || { tail "$O/cmp_p7_65536.txt"; exit 1; }
cat "$O/cmp_p7_65536.txt"
timeout -k 10 300 python tools/kbench/compare.py --code p7 --batch 262144 --reps 9 cur cur:schedule=4 > "$O/cmp_p7_262144.txt" 2>&1 || { tail "$O/cmp_p7_262144.txt"; exit 1; }
cat "$O/cmp_p7_262144.txt"
timeout -k 10 120 python bench.py --code p7 --global-batch 65536 --no-cpu --no-extras > "$O/bench_p7_65536.json" 2> "$O/bench_p7.err" || { tail "$O/bench_p7.err"; exit 1; }
python -c "import json; d=json.load(open('$O/bench_p7_65536.json')); print('bench p7 65536', d['value'], d['ms_per_step'], d['decode_ms'])"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/p7_trace" -o run -- \
    python3 "$R/bench.py" --code p7 --global-batch 65536 --no-cpu --no-extras --steps 20 > /dev/null 2> "$O/p7trace.err" || { tail -5 "$O/p7trace.err"; exit 1; }
cat "$O/p7_trace/run_kernel_stats.csv" | cut -c1-150
