# round 3, call k: guard-free scaled short division (QEC_SCALED_DIV) -- gpu suite, A/B against the
# previous revision (base), without the scaling (noscale), and P7 without column groups (cg1).
set -o pipefail
R="$GRAFT_REPO_ROOT"
O="$R/gpurun_out/r03k"
mkdir -p "$O"
cd "$R"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$O/pytest.log" 2>&1
rc=$?; tail -3 "$O/pytest.log"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python tools/kbench/compare.py --code p61 --batch 1048576 --reps 5 base cur noscale base:hard_paths=0 cur:hard_paths=0 noscale:hard_paths=0 > "$O/cmp_p61.txt" 2>&1 || { tail "$O/cmp_p61.txt"; exit 1; }
cat "$O/cmp_p61.txt"
timeout -k 10 300 python tools/kbench/compare.py --code p7 --batch 65536 --reps 11 base cur noscale cg1 > "$O/cmp_p7_65536.txt" 2>&1 || { tail "$O/cmp_p7_65536.txt"; exit 1; }
cat "$O/cmp_p7_65536.txt"
timeout -k 10 300 python tools/kbench/compare.py --code p7 --batch 1048576 --reps 5 base cur cg1 base:hard_paths=0 cur:hard_paths=0 cg1:hard_paths=0 > "$O/cmp_p7_2e20.txt" 2>&1 || { tail "$O/cmp_p7_2e20.txt"; exit 1; }
cat "$O/cmp_p7_2e20.txt"
timeout -k 10 300 python tools/kbench/compare.py --code p61 --batch 1048576 --reps 3 --stop 2 --p 0.05 base cur > "$O/cmp_p61_syn005.txt" 2>&1 || { tail "$O/cmp_p61_syn005.txt"; exit 1; }
cat "$O/cmp_p61_syn005.txt"
