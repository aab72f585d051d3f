# round 3, call q: straight-line scaled var passes with a scheduling barrier per column group
# (QEC_ASSUME_SCALED + QEC_COL_BARRIER), spill-free.
set -o pipefail
R="$GRAFT_REPO_ROOT"
O="$R/gpurun_out/r03q"
mkdir -p "$O"
cd "$R"
export TMPDIR=/tmp
timeout -k 10 400 python tools/kbench/compare.py --code p61 --batch 1048576 --reps 7 cur asb asbcg2 b cur:hard_paths=0 asb:hard_paths=0 asbcg2:hard_paths=0 > "$O/cmp_p61.txt" 2>&1 || { tail "$O/cmp_p61.txt"; exit 1; }
cat "$O/cmp_p61.txt"
timeout -k 10 300 python tools/kbench/compare.py --code p7 --batch 65536 --reps 15 cur asb asbcg2 b > "$O/cmp_p7_65536.txt" 2>&1 || { tail "$O/cmp_p7_65536.txt"; exit 1; }
cat "$O/cmp_p7_65536.txt"
timeout -k 10 300 python tools/kbench/compare.py --code p7 --batch 1048576 --reps 5 cur asb asbcg2 b > "$O/cmp_p7_2e20.txt" 2>&1 || { tail "$O/cmp_p7_2e20.txt"; exit 1; }
cat "$O/cmp_p7_2e20.txt"
timeout -k 10 300 python tools/kbench/compare.py --code p61 --batch 1048576 --reps 3 --stop 2 --p 0.05 cur asb b > "$O/cmp_p61_syn005.txt" 2>&1 || { tail "$O/cmp_p61_syn005.txt"; exit 1; }
cat "$O/cmp_p61_syn005.txt"
