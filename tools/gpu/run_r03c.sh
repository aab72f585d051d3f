# round 3, call c: A/B of soft-iteration options on the P61 headline (2^20 @ 50 fixed) and its
# full-arithmetic form (hard paths off), interleaved in one process, outputs checked identical.
set -o pipefail
R="$GRAFT_REPO_ROOT"
O="$R/gpurun_out/r03c"
mkdir -p "$O"
cd "$R"
timeout -k 10 400 python tools/kbench/compare.py --code p61 --batch 1048576 --reps 5 cur gg tr3 pipe3 cg2 > "$O/cmp_headline.txt" 2>&1 || { tail "$O/cmp_headline.txt"; exit 1; }
cat "$O/cmp_headline.txt"
timeout -k 10 600 python tools/kbench/compare.py --code p61 --batch 262144 --reps 3 cur:hard_paths=0 gg:hard_paths=0 pipe3:hard_paths=0 cg2:hard_paths=0 > "$O/cmp_full.txt" 2>&1 || { tail "$O/cmp_full.txt"; exit 1; }
cat "$O/cmp_full.txt"
