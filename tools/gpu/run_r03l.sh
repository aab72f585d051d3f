# round 3, call l: straight-line soft var passes (QEC_SOFT_STRAIGHT 0/1/2) and gather pipelining depth.
set -o pipefail
R="$GRAFT_REPO_ROOT"
O="$R/gpurun_out/r03l"
mkdir -p "$O"
cd "$R"
export TMPDIR=/tmp
timeout -k 10 400 python tools/kbench/compare.py --code p61 --batch 1048576 --reps 5 ss0 cur ss2 ss2p3 ss2p1 ss0:hard_paths=0 cur:hard_paths=0 ss2:hard_paths=0 > "$O/cmp_p61.txt" 2>&1 || { tail "$O/cmp_p61.txt"; exit 1; }
cat "$O/cmp_p61.txt"
timeout -k 10 300 python tools/kbench/compare.py --code p7 --batch 65536 --reps 11 ss0 cur ss2 ss2p3 ss2p1 > "$O/cmp_p7_65536.txt" 2>&1 || { tail "$O/cmp_p7_65536.txt"; exit 1; }
cat "$O/cmp_p7_65536.txt"
timeout -k 10 300 python tools/kbench/compare.py --code p7 --batch 1048576 --reps 5 ss0 cur ss2 ss2p3 > "$O/cmp_p7_2e20.txt" 2>&1 || { tail "$O/cmp_p7_2e20.txt"; exit 1; }
cat "$O/cmp_p7_2e20.txt"
timeout -k 10 300 python tools/kbench/compare.py --code p61 --batch 1048576 --reps 3 --stop 2 --p 0.05 ss0 cur ss2 > "$O/cmp_p61_syn005.txt" 2>&1 || { tail "$O/cmp_p61_syn005.txt"; exit 1; }
cat "$O/cmp_p61_syn005.txt"
