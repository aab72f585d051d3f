# round 3, call y: the first var pass that tests for the hard state (QEC_TRACK_FROM 1 / 2 / 3).
set -o pipefail
R="$GRAFT_REPO_ROOT"
O="$R/gpurun_out/r03y"
mkdir -p "$O"
cd "$R"
export TMPDIR=/tmp
timeout -k 10 400 python tools/kbench/compare.py --code p61 --batch 1048576 --reps 7 cur tr1 tr3 > "$O/cmp_p61.txt" 2>&1 || { tail "$O/cmp_p61.txt"; exit 1; }
cat "$O/cmp_p61.txt"
timeout -k 10 300 python tools/kbench/compare.py --code p7 --batch 65536 --reps 15 cur tr1 tr3 > "$O/cmp_p7_65536.txt" 2>&1 || { tail "$O/cmp_p7_65536.txt"; exit 1; }
cat "$O/cmp_p7_65536.txt"
timeout -k 10 300 python tools/kbench/compare.py --code p7 --batch 1048576 --reps 5 cur tr1 > "$O/cmp_p7_2e20.txt" 2>&1 || { tail "$O/cmp_p7_2e20.txt"; exit 1; }
cat "$O/cmp_p7_2e20.txt"
