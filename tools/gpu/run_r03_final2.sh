# round 3 final evidence, part 2 (after profiles/pmc_*.json of this build are in the tree): bench lines
# with the roofline, config-5 profile and sweeps.
set -o pipefail
R="$GRAFT_REPO_ROOT"
O="$R/gpurun_out/final2"
mkdir -p "$O"
cd "$R"
export TMPDIR=/tmp
timeout -k 10 300 python bench.py > "$O/bench_p61.json" 2> "$O/bench_p61.err" || { tail "$O/bench_p61.err"; exit 1; }
timeout -k 10 120 python bench.py --code p7 --global-batch 65536 --no-cpu > "$O/bench_p7_65536.json" 2> "$O/bench_p7.err" || { tail "$O/bench_p7.err"; exit 1; }
timeout -k 10 120 python bench.py --global-batch 65536 --no-cpu > "$O/bench_p61_65536.json" 2> "$O/bench_p61s.err" || { tail "$O/bench_p61s.err"; exit 1; }
timeout -k 10 120 python bench.py --code p7 --no-cpu > "$O/bench_p7_2e20.json" 2> "$O/bench_p7l.err" || { tail "$O/bench_p7l.err"; exit 1; }
for f in bench_p61 bench_p7_65536 bench_p61_65536 bench_p7_2e20; do
  python -c "import json; d=json.load(open('$O/$f.json')); r=d['roofline']; print('$f', d['value'], d['ms_per_step'], d.get('value_full_arithmetic'), r.get('frac'), r.get('frac_unweighted'), r.get('note'))"
done
timeout -k 10 300 python tools/psweep.py --out "$O/psweep_syndrome.json" > "$O/psweep_syndrome.log" 2>&1 || { tail "$O/psweep_syndrome.log"; exit 1; }
timeout -k 10 400 python tools/psweep.py --stop fixed --out "$O/psweep_fixed50.json" > "$O/psweep_fixed50.log" 2>&1 || { tail "$O/psweep_fixed50.log"; exit 1; }
bash tools/gpu/run_mc_profile.sh final 0.002 > "$O/mc_profile.log" 2>&1 || { tail "$O/mc_profile.log"; exit 1; }
tail -8 "$O/mc_profile.log" | cut -c1-200
