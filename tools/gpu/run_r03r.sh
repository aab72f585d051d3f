# round 3, call r: confirm the per-column scheduling barrier (QEC_COL_BARRIER) on the headline, full
# arithmetic, configs[2] and the syndrome stop.
set -o pipefail
R="$GRAFT_REPO_ROOT"
O="$R/gpurun_out/r03r"
mkdir -p "$O"
cd "$R"
export TMPDIR=/tmp
timeout -k 10 400 python tools/kbench/compare.py --code p61 --batch 1048576 --reps 9 cur b bcg2 bp1 cur:hard_paths=0 b:hard_paths=0 bcg2:hard_paths=0 > "$O/cmp_p61.txt" 2>&1 || { tail "$O/cmp_p61.txt"; exit 1; }
cat "$O/cmp_p61.txt"
timeout -k 10 300 python tools/kbench/compare.py --code p61 --batch 65536 --reps 9 cur b bcg2 > "$O/cmp_p61_65536.txt" 2>&1 || { tail "$O/cmp_p61_65536.txt"; exit 1; }
cat "$O/cmp_p61_65536.txt"
timeout -k 10 300 python tools/kbench/compare.py --code p61 --batch 1048576 --reps 3 --stop 2 --p 0.02 cur b > "$O/cmp_p61_syn002.txt" 2>&1 || { tail "$O/cmp_p61_syn002.txt"; exit 1; }
cat "$O/cmp_p61_syn002.txt"
timeout -k 10 300 python tools/kbench/compare.py --code p61 --batch 1048576 --reps 3 --stop 0 cur b > "$O/cmp_p61_ref.txt" 2>&1 || { tail "$O/cmp_p61_ref.txt"; exit 1; }
cat "$O/cmp_p61_ref.txt"
