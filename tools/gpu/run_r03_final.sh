# round 3 final evidence: gpu suite, smoke, bench lines, rocprofv3 trace + PMC of the bench workloads
# (profiles/pmc_*.json stamped with this build's id), config-5 profile and sweeps.
set -o pipefail
R="$GRAFT_REPO_ROOT"
O="$R/gpurun_out/final"
mkdir -p "$O"
cd "$R"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$O/pytest.log" 2>&1
rc=$?; tail -3 "$O/pytest.log"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 || { tail "$O/smoke.log"; exit 1; }
cat "$O/smoke.log"
bash tools/gpu/run_profile.sh final p61 p7 > "$O/profile.log" 2>&1 || { tail "$O/profile.log"; exit 1; }
EXTRA="--global-batch 65536" bash tools/gpu/run_profile.sh final_65536 p7 > "$O/profile_65536.log" 2>&1 || { tail "$O/profile_65536.log"; exit 1; }
grep -E "rc=" "$O/profile.log" "$O/profile_65536.log" | tr '\n' ' '; echo
