# round 3 evidence, part 2: rocprofv3 kernel trace + PMC passes of the bench workloads (configs[3] P61,
# P7 2^20, P7 configs[1]) -> profiles/pmc_*.json stamped with the library's build id.
set -o pipefail
R="$GRAFT_REPO_ROOT"
cd "$R"
bash tools/gpu/run_profile.sh r03 p61 p7 || exit 1
EXTRA="--global-batch 65536" bash tools/gpu/run_profile.sh r03_65536 p7 || exit 1
