# round 3, call o: P7 launch-shape knobs after the scaled division (min waves, pipelining, column groups).
set -o pipefail
R="$GRAFT_REPO_ROOT"
O="$R/gpurun_out/r03o"
mkdir -p "$O"
cd "$R"
export TMPDIR=/tmp
timeout -k 10 300 python tools/kbench/compare.py --code p7 --batch 65536 --reps 15 cur mw7 mw6 p1 p3 cg2 cg6 > "$O/cmp_p7_65536.txt" 2>&1 || { tail "$O/cmp_p7_65536.txt"; exit 1; }
cat "$O/cmp_p7_65536.txt"
timeout -k 10 300 python tools/kbench/compare.py --code p7 --batch 1048576 --reps 5 cur mw7 mw6 p1 p3 cg2 cg6 > "$O/cmp_p7_2e20.txt" 2>&1 || { tail "$O/cmp_p7_2e20.txt"; exit 1; }
cat "$O/cmp_p7_2e20.txt"
timeout -k 10 300 python tools/kbench/compare.py --code p61 --batch 1048576 --reps 5 cur p1 p3 > "$O/cmp_p61.txt" 2>&1 || { tail "$O/cmp_p61.txt"; exit 1; }
cat "$O/cmp_p61.txt"
