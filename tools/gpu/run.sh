#!/bin/bash
# One GPU-box call as a list of steps, each under its own time limit, stopping at the first failure
# (no step runs after a failed, timed-out or crashed one).  Outputs go to gpurun_out/TAG/.
#   bash tools/gpu/run.sh TAG "STEP ARGS..." ...
# Steps:
#   pytest [ARGS]        the GPU suite (-m gpu), or a part of it with -k / file arguments
#   smoke                __graft_entry__.smoke()
#   bench [ARGS]         bench.py ARGS (one JSON line)
#   compare [ARGS]       tools/kbench/compare.py ARGS (A/B of build/variants libraries, one process)
#   psweep [ARGS]        tools/psweep.py ARGS
#   profile NAME [CODES] tools/gpu/run_profile.sh NAME CODES (PMC evidence; EXTRA="..." via env STEP_EXTRA)
#   trace NAME [ARGS]    rocprofv3 --kernel-trace --stats of bench.py ARGS
#   mctrace NAME [ARGS]  rocprofv3 --kernel-trace --stats of tools/psweep.py ARGS
#   exec CMD             any other command (built beforehand on the CPU side)
set -o pipefail
R="$GRAFT_REPO_ROOT"
TAG=$1; shift
O="$R/gpurun_out/$TAG"
mkdir -p "$O"
export TMPDIR=/tmp
cd "$R"
i=0
for spec in "$@"; do
  i=$((i+1))
  read -r step args <<< "$spec"
  echo "== step $i: $spec"
  case "$step" in
    pytest)
      eval timeout -k 10 1500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread "$args" \
          > "$O/pytest_$i.log" 2>&1; rc=$?; tail -3 "$O/pytest_$i.log";;
    smoke)
      timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke_$i.log" 2>&1; rc=$?
      tail -2 "$O/smoke_$i.log";;
    bench)
      timeout -k 10 600 python bench.py $args > "$O/bench_$i.json" 2> "$O/bench_$i.err"; rc=$?
      [ $rc -eq 0 ] && python -c "import json; d=json.load(open('$O/bench_$i.json')); r=d['roofline']; print(d['value'], d['ms_per_step'], d.get('value_full_arithmetic'), r.get('frac'), r.get('frac_unweighted'))"
      [ $rc -ne 0 ] && tail -5 "$O/bench_$i.err";;
    compare)
      timeout -k 10 900 python tools/kbench/compare.py $args > "$O/compare_$i.txt" 2>&1; rc=$?; cat "$O/compare_$i.txt" | grep -v '^{';;
    psweep)
      timeout -k 10 900 python tools/psweep.py $args > "$O/psweep_$i.txt" 2>&1; rc=$?; tail -3 "$O/psweep_$i.txt" | cut -c1-300;;
    profile)
      read -r name codes <<< "$args"
      EXTRA="$STEP_EXTRA" timeout -k 10 1500 bash tools/gpu/run_profile.sh "$name" $codes > "$O/profile_$i.log" 2>&1; rc=$?
      tail -3 "$O/profile_$i.log" | cut -c1-300;;
    trace|mctrace)
      read -r name rest <<< "$args"
      prog="$R/bench.py --no-cpu"; [ "$step" = mctrace ] && prog="$R/tools/psweep.py"
      (cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/$name" -o run -- \
          python3 $prog $rest > "$O/${name}.out" 2> "$O/${name}.err"); rc=$?
      [ $rc -eq 0 ] && cut -d, -f1-4 "$O/$name/run_kernel_stats.csv" | cut -c1-140 | head -12;;
    exec)
      eval timeout -k 10 600 "$args" > "$O/exec_$i.txt" 2>&1; rc=$?; tail -5 "$O/exec_$i.txt" | cut -c1-300;;
    *) echo "unknown step $step"; rc=2;;
  esac
  echo "== step $i rc=$rc"
  [ $rc -ne 0 ] && exit $rc
done
exit 0
