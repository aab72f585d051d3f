# round 3, call t: the P61 row barrier (Tune::kRowBarrier) against none on every P61 stop rule; gpu suite.
set -o pipefail
R="$GRAFT_REPO_ROOT"
O="$R/gpurun_out/r03t"
mkdir -p "$O"
cd "$R"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$O/pytest.log" 2>&1
rc=$?; tail -3 "$O/pytest.log"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python tools/kbench/compare.py --code p61 --batch 1048576 --reps 9 rb0 cur > "$O/cmp_p61.txt" 2>&1 || { tail "$O/cmp_p61.txt"; exit 1; }
cat "$O/cmp_p61.txt"
timeout -k 10 300 python tools/kbench/compare.py --code p61 --batch 1048576 --reps 3 --stop 2 --p 0.05 rb0 cur > "$O/cmp_p61_syn005.txt" 2>&1 || { tail "$O/cmp_p61_syn005.txt"; exit 1; }
cat "$O/cmp_p61_syn005.txt"
timeout -k 10 300 python tools/kbench/compare.py --code p61 --batch 1048576 --reps 3 --stop 0 rb0 cur > "$O/cmp_p61_ref.txt" 2>&1 || { tail "$O/cmp_p61_ref.txt"; exit 1; }
cat "$O/cmp_p61_ref.txt"
timeout -k 10 300 python tools/kbench/compare.py --code p61 --batch 65536 --reps 9 rb0 cur > "$O/cmp_p61_65536.txt" 2>&1 || { tail "$O/cmp_p61_65536.txt"; exit 1; }
cat "$O/cmp_p61_65536.txt"
