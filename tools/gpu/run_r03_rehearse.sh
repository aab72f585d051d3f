# round 3: the driver's round-end sequence on the final tree (gpu suite, smoke, default bench line).
set -o pipefail
R="$GRAFT_REPO_ROOT"
O="$R/gpurun_out/rehearse"
mkdir -p "$O"
cd "$R"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > "$O/pytest.log" 2>&1
rc=$?; tail -2 "$O/pytest.log"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 || { tail "$O/smoke.log"; exit 1; }
tail -1 "$O/smoke.log"
timeout -k 10 300 python bench.py > "$O/bench.json" 2> "$O/bench.err" || { tail "$O/bench.err"; exit 1; }
python -c "import json; d=json.load(open('$O/bench.json')); r=d['roofline']; print(d['value'], d['ms_per_step'], d.get('value_full_arithmetic'), r.get('frac'), r.get('frac_unweighted'), d['cpu_baseline']['value'])"
