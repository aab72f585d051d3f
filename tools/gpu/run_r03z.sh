# round 3, call z: 16-byte rows in the Monte-Carlo pipeline (statistics kernel with 16-byte loads); gpu suite.
set -o pipefail
R="$GRAFT_REPO_ROOT"
O="$R/gpurun_out/r03z"
mkdir -p "$O"
cd "$R"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$O/pytest.log" 2>&1
rc=$?; tail -3 "$O/pytest.log"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python tools/psweep.py --ps 0.001 0.002 0.005 0.01 0.05 --reps 5 > "$O/psweep.txt" 2>&1 || { tail "$O/psweep.txt"; exit 1; }
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/trace" -o run -- \
    python3 "$R/tools/psweep.py" --ps 0.002 > /dev/null 2> "$O/trace.err" || { tail -5 "$O/trace.err"; exit 1; }
cut -d, -f1-4 "$O/trace/run_kernel_stats.csv" | cut -c1-120
