# round 3, call d: counter list, probe (event throughput), gpu tests, headline + P7 configs[1] bench,
# config-5 sweep with the triage, A/B of soft-iteration options.
set -o pipefail
R="$GRAFT_REPO_ROOT"
O="$R/gpurun_out/r03d"
mkdir -p "$O"
cd "$R"
export TMPDIR=/tmp
timeout -k 10 60 rocprofv3 --list-avail > "$O/list_avail.txt" 2>&1; echo "list-avail rc=$?"
timeout -k 10 200 tools/kbench/valu_probe > "$O/valu_probe.json" || exit 1
cat "$O/valu_probe.json"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$O/pytest.log" 2>&1
rc=$?; tail -15 "$O/pytest.log"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python bench.py --code p7 --global-batch 65536 --no-cpu > "$O/bench_p7_65536.json" 2> "$O/bench_p7.err" || { tail "$O/bench_p7.err"; exit 1; }
cat "$O/bench_p7_65536.json"
timeout -k 10 300 python tools/psweep.py --out "$O/psweep.json" > "$O/psweep.log" 2>&1 || { tail "$O/psweep.log"; exit 1; }
cat "$O/psweep.log"
timeout -k 10 300 python bench.py --no-cpu > "$O/bench_p61.json" 2> "$O/bench_p61.err" || { tail "$O/bench_p61.err"; exit 1; }
cat "$O/bench_p61.json"
timeout -k 10 400 python tools/kbench/compare.py --code p61 --batch 1048576 --reps 5 cur gg tr3 pipe3 cg2 > "$O/cmp_headline.txt" 2>&1 || { tail "$O/cmp_headline.txt"; exit 1; }
cat "$O/cmp_headline.txt"
timeout -k 10 300 python tools/kbench/compare.py --code p7 --batch 65536 --reps 7 cur pipe3 pipe5 cg2 cg3 > "$O/cmp_p7_65536.txt" 2>&1 || { tail "$O/cmp_p7_65536.txt"; exit 1; }
cat "$O/cmp_p7_65536.txt"
