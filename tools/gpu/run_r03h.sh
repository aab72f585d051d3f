# round 3, call h: issue priority for long-running waves (QEC_LONG_PRIO) and the one-launch local order
# (QEC_OPT_SCHEDULE = 3) on P7 configs[1] and 2^20, P61 configs[2]; the schedule tests.
set -o pipefail
R="$GRAFT_REPO_ROOT"
O="$R/gpurun_out/r03h"
mkdir -p "$O"
cd "$R"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -k "schedule or split" --timeout 200 --timeout-method thread > "$O/pytest.log" 2>&1
rc=$?; tail -3 "$O/pytest.log"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/kbench/compare.py --code p7 --batch 65536 --reps 11 cur cur:schedule=3 cur:schedule=0 lp2 lp4 lp6 lp9 lp4:schedule=3 > "$O/cmp_p7_65536.txt" 2>&1 || { tail "$O/cmp_p7_65536.txt"; exit 1; }
cat "$O/cmp_p7_65536.txt"
timeout -k 10 300 python tools/kbench/compare.py --code p7 --batch 1048576 --reps 5 cur lp2 lp4 lp6 lp9 > "$O/cmp_p7_2e20.txt" 2>&1 || { tail "$O/cmp_p7_2e20.txt"; exit 1; }
cat "$O/cmp_p7_2e20.txt"
timeout -k 10 300 python tools/kbench/compare.py --code p61 --batch 65536 --reps 7 cur lp4 lp6 lp9 > "$O/cmp_p61_65536.txt" 2>&1 || { tail "$O/cmp_p61_65536.txt"; exit 1; }
cat "$O/cmp_p61_65536.txt"
