# round 3, call b: the gpu test suite (new: launcher, non-binary syndromes, full-batch Monte-Carlo,
# wider oracle slices), the probe with event timing, configs[1] after the order-pass change, and the
# headline with the new extras.
set -o pipefail
R="$GRAFT_REPO_ROOT"
O="$R/gpurun_out/r03b"
mkdir -p "$O"
cd "$R"
timeout -k 10 120 tools/kbench/valu_probe > "$O/valu_probe.json" || exit 1
cat "$O/valu_probe.json"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$O/pytest.log" 2>&1
rc=$?; tail -15 "$O/pytest.log"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python bench.py --code p7 --global-batch 65536 --no-cpu > "$O/bench_p7_65536.json" 2> "$O/bench_p7.err" || { tail "$O/bench_p7.err"; exit 1; }
cat "$O/bench_p7_65536.json"
timeout -k 10 300 python bench.py --no-cpu > "$O/bench_p61.json" 2> "$O/bench_p61.err" || { tail "$O/bench_p61.err"; exit 1; }
cat "$O/bench_p61.json"
timeout -k 10 300 python tools/psweep.py --out "$O/psweep.json" > "$O/psweep.log" 2>&1 || { tail "$O/psweep.log"; exit 1; }
cat "$O/psweep.log"
