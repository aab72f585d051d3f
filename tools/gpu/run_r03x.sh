# round 3, call x: list-mode decode grid (QEC_LIST_ROUNDS) after the triage's per-workgroup atomics.
set -o pipefail
R="$GRAFT_REPO_ROOT"
O="$R/gpurun_out/r03x"
mkdir -p "$O"
cd "$R"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_triage.py -x -q --timeout 300 --timeout-method thread > "$O/pytest.log" 2>&1
rc=$?; tail -2 "$O/pytest.log"; [ $rc -ne 0 ] && exit $rc
cd /tmp
for r in 1 2 4 8; do
  QEC_LIST_ROUNDS=$r timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/trace$r" -o run -- \
      python3 "$R/tools/psweep.py" --ps 0.002 0.005 0.01 --reps 3 > "$O/psweep$r.txt" 2> "$O/trace$r.err" || { tail -5 "$O/trace$r.err"; exit 1; }
  echo "rounds $r"; grep -h "bp_decode\|triage" "$O/trace$r/run_kernel_stats.csv" | cut -d, -f1-4 | cut -c1-40,200-
done
