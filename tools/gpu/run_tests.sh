# GPU pytest run with per-test timeouts: bash tools/gpu/run_tests.sh TAG [pytest args...]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-run}; shift
timeout -k 10 1000 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider "$@" \
    > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|error" gpurun_out/pytest_$TAG.log | tail -5
exit $rc
