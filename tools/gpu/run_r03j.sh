# round 3, call j: guard ballots without integer round trips, no hardness tracking in full-arithmetic
# launches (A/B against the previous revision), P7 waves per workgroup; parity suite.
set -o pipefail
R="$GRAFT_REPO_ROOT"
O="$R/gpurun_out/r03j"
mkdir -p "$O"
cd "$R"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_packed.py -x -q --timeout 300 --timeout-method thread > "$O/pytest.log" 2>&1
rc=$?; tail -3 "$O/pytest.log"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python tools/kbench/compare.py --code p61 --batch 1048576 --reps 5 base cur base:hard_paths=0 cur:hard_paths=0 > "$O/cmp_p61.txt" 2>&1 || { tail "$O/cmp_p61.txt"; exit 1; }
cat "$O/cmp_p61.txt"
timeout -k 10 300 python tools/kbench/compare.py --code p7 --batch 65536 --reps 11 base cur wpb2 wpb4 > "$O/cmp_p7_65536.txt" 2>&1 || { tail "$O/cmp_p7_65536.txt"; exit 1; }
cat "$O/cmp_p7_65536.txt"
timeout -k 10 300 python tools/kbench/compare.py --code p7 --batch 1048576 --reps 5 base cur base:hard_paths=0 cur:hard_paths=0 > "$O/cmp_p7_2e20.txt" 2>&1 || { tail "$O/cmp_p7_2e20.txt"; exit 1; }
cat "$O/cmp_p7_2e20.txt"
