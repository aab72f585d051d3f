# round 3, call f: triage (compile-time tables) + row statistics (32 samples per wave) kernel
# times at p = 0.002, P7 configs[1] launch-shape options, gpu triage/montecarlo tests.
set -o pipefail
R="$GRAFT_REPO_ROOT"
O="$R/gpurun_out/r03f"
mkdir -p "$O"
cd "$R"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_triage.py tests/test_gpu_montecarlo.py tests/test_gpu_packed.py -x -q --timeout 300 --timeout-method thread > "$O/pytest.log" 2>&1
rc=$?; tail -3 "$O/pytest.log"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/kbench/compare.py --code p7 --batch 65536 --reps 9 cur cur:sector_split=0 cur:schedule=0 cur:sector_split=0,schedule=0 cg3 cg3:sector_split=0 > "$O/cmp_p7_65536.txt" 2>&1 || { tail "$O/cmp_p7_65536.txt"; exit 1; }
cat "$O/cmp_p7_65536.txt"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/mc_trace" -o run -- \
    python3 "$R/tools/psweep.py" --ps 0.002 0.005 0.01 > "$O/psweep.txt" 2> "$O/trace.err" || { tail -5 "$O/trace.err"; exit 1; }
cat "$O/psweep.txt"
cat "$O/mc_trace/run_kernel_stats.csv"
