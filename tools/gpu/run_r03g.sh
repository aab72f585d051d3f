# round 3, call g: lane statistics kernel, compile-time triage, P7 order-pass buckets; the gpu suite.
set -o pipefail
R="$GRAFT_REPO_ROOT"
O="$R/gpurun_out/r03g"
mkdir -p "$O"
cd "$R"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$O/pytest.log" 2>&1
rc=$?; tail -3 "$O/pytest.log"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python bench.py --code p7 --global-batch 65536 --no-cpu --no-extras > "$O/bench_p7_65536.json" 2> "$O/bench_p7.err" || { tail "$O/bench_p7.err"; exit 1; }
cat "$O/bench_p7_65536.json"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/mc_trace" -o run -- \
    python3 "$R/tools/psweep.py" --ps 0.001 0.002 0.005 0.01 > "$O/psweep.txt" 2> "$O/trace.err" || { tail -5 "$O/trace.err"; exit 1; }
cat "$O/psweep.txt"
cat "$O/mc_trace/run_kernel_stats.csv"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/p7_trace" -o run -- \
    python3 "$R/bench.py" --code p7 --global-batch 65536 --no-cpu --no-extras --steps 20 > /dev/null 2> "$O/p7trace.err" || { tail -5 "$O/p7trace.err"; exit 1; }
cat "$O/p7_trace/run_kernel_stats.csv"
