# round 3, call p: config-5 profile at p = 0.002 (trace + PMC of front end, triage, list decode, statistics)
# and the scaled division without its per-column branch (QEC_ASSUME_SCALED experiment).
set -o pipefail
R="$GRAFT_REPO_ROOT"
O="$R/gpurun_out/r03p"
mkdir -p "$O"
cd "$R"
export TMPDIR=/tmp
timeout -k 10 300 python tools/kbench/compare.py --code p61 --batch 1048576 --reps 5 cur as ascg1 cur:hard_paths=0 as:hard_paths=0 > "$O/cmp_p61.txt" 2>&1 || { tail "$O/cmp_p61.txt"; exit 1; }
cat "$O/cmp_p61.txt"
timeout -k 10 300 python tools/kbench/compare.py --code p7 --batch 65536 --reps 15 cur as ascg1 > "$O/cmp_p7_65536.txt" 2>&1 || { tail "$O/cmp_p7_65536.txt"; exit 1; }
cat "$O/cmp_p7_65536.txt"
timeout -k 10 300 python tools/kbench/compare.py --code p7 --batch 1048576 --reps 5 cur as ascg1 > "$O/cmp_p7_2e20.txt" 2>&1 || { tail "$O/cmp_p7_2e20.txt"; exit 1; }
cat "$O/cmp_p7_2e20.txt"
bash tools/gpu/run_mc_profile.sh r03 0.002
