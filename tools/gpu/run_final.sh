# Round-end evidence of the tree: -m gpu suite, smoke(), default bench line, rocprofv3 kernel
# stats + PMC summaries of the bench workloads, and the config-5 p-sweep profile.
#   bash tools/gpu/run_final.sh TAG
set -o pipefail
R="$GRAFT_REPO_ROOT"
TAG=${1:-final}
cd "$R"
bash tools/gpu/run_check.sh "$TAG" || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1; rc=$?
echo "smoke rc=$rc"; tail -2 gpurun_out/smoke_$TAG.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu/run_profile.sh "$TAG" p61 p7 > gpurun_out/profile_$TAG.log 2>&1 || { tail -5 gpurun_out/profile_$TAG.log; exit 1; }
echo "profile ok"
bash tools/gpu/run_mc_profile.sh "$TAG" > gpurun_out/mcprofile_$TAG.log 2>&1 || { tail -5 gpurun_out/mcprofile_$TAG.log; exit 1; }
echo "mc profile ok"
