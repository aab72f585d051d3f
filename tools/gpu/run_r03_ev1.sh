# round 3 evidence, part 1: gpu suite, smoke, default bench line (configs[3]), P7 configs[1] and P61
# configs[2] bench lines, config-5 p-sweeps (syndrome stop; fixed 50 iterations).
set -o pipefail
R="$GRAFT_REPO_ROOT"
O="$R/gpurun_out/ev1"
mkdir -p "$O"
cd "$R"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$O/pytest.log" 2>&1
rc=$?; tail -3 "$O/pytest.log"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 || { tail "$O/smoke.log"; exit 1; }
cat "$O/smoke.log"
timeout -k 10 300 python bench.py > "$O/bench_p61.json" 2> "$O/bench_p61.err" || { tail "$O/bench_p61.err"; exit 1; }
timeout -k 10 120 python bench.py --code p7 --global-batch 65536 --no-cpu > "$O/bench_p7_65536.json" 2> "$O/bench_p7.err" || { tail "$O/bench_p7.err"; exit 1; }
timeout -k 10 120 python bench.py --global-batch 65536 --no-cpu > "$O/bench_p61_65536.json" 2> "$O/bench_p61s.err" || { tail "$O/bench_p61s.err"; exit 1; }
timeout -k 10 120 python bench.py --code p7 --no-cpu > "$O/bench_p7_2e20.json" 2> "$O/bench_p7l.err" || { tail "$O/bench_p7l.err"; exit 1; }
timeout -k 10 300 python tools/psweep.py --out "$O/psweep_syndrome.json" > "$O/psweep_syndrome.log" 2>&1 || { tail "$O/psweep_syndrome.log"; exit 1; }
timeout -k 10 400 python tools/psweep.py --stop fixed --out "$O/psweep_fixed50.json" > "$O/psweep_fixed50.log" 2>&1 || { tail "$O/psweep_fixed50.log"; exit 1; }
for f in bench_p61 bench_p7_65536 bench_p61_65536 bench_p7_2e20; do
  python -c "import json; d=json.load(open('$O/$f.json')); print('$f', d['value'], d['ms_per_step'], d.get('value_full_arithmetic'), d['roofline'].get('frac'))"
done
grep syndromes_per_s "$O/psweep_syndrome.log" | cut -c1-120
grep syndromes_per_s "$O/psweep_fixed50.log" | cut -c1-120
