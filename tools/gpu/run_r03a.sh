# round 3, call a: VALU/LDS instruction pricing (valu_probe) and the P7 configs[1] profile
# (65 536 syndromes, 20 fixed iterations): kernel trace + PMC passes.
set -o pipefail
R="$GRAFT_REPO_ROOT"
mkdir -p "$R/gpurun_out/r03"
timeout -k 10 120 "$R/tools/kbench/valu_probe" > "$R/gpurun_out/r03/valu_probe.json" || exit 1
cat "$R/gpurun_out/r03/valu_probe.json"
EXTRA="--global-batch 65536" timeout -k 10 500 bash "$R/tools/gpu/run_profile.sh" r03a p7
