# rocprofv3 evidence for bench.py's rooflines, one workload per spec: a kernel-trace --stats pass
# and five PMC passes (each counter group in its own run, --kernel-trace only beside --pmc), then the
# per-launch / per-syndrome summary bench.py reads (profiles/pmc_<name>.json).
#   bash tools/gpu/run_profile.sh TAG "NAME:BENCH ARGS" ...
# (commas in ARGS stand for spaces) e.g. "p61:" (configs[3]), "p61_131072:--global-batch,131072" (the N = 8
# shard), "p61_hp0:--hard-paths,0"
# (every iteration in full arithmetic), "p7_65536:--code,p7,--global-batch,65536".
# bench.py looks for pmc_<code>_<batch>[_hp0].json, then pmc_<code>[_hp0].json.
set -o pipefail
R="$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-r04}; shift
OUT="$R/gpurun_out/prof_$TAG"
mkdir -p "$OUT"; cd /tmp
for spec in "$@"; do
  name=${spec%%:*}; args=${spec#*:}; args=${args//,/ }
  code=p61; case " $args " in *" --code p7 "*) code=p7;; esac
  D="$OUT/$name"; mkdir -p "$D"
  BENCH="$R/bench.py --no-cpu --no-extras $args"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$D/trace" -o run -- \
      python3 $BENCH --steps 10 --warmup 2 > "$D/bench_trace.json" 2> "$D/trace.err"
  rc=$?; echo "$name trace rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 "$D/trace.err"; exit $rc; fi
  i=0
  for grp in "FETCH_SIZE" "WRITE_SIZE" "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES" \
             "SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES GRBM_GUI_ACTIVE" \
             "SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_INT32 SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT"; do
    i=$((i+1))
    timeout -k 10 -s KILL 180 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d "$D/pmc$i" -o run -- \
        python3 $BENCH --steps 2 --warmup 1 > "$D/bench_pmc$i.json" 2> "$D/pmc$i.err"
    rc=$?; echo "$name pmc$i rc=$rc"
    if [ $rc -ne 0 ]; then tail -5 "$D/pmc$i.err"; exit $rc; fi
  done
  python3 "$R/tools/gpu/pmc_summary.py" --dir "$D" --code "$code" --bench "$D/bench_trace.json" \
      --out "$OUT/pmc_$name.json" > /dev/null || exit 1
  python3 -c "import json; d=json.load(open('$OUT/pmc_$name.json')); print('$name', d['batch'], d.get('hard_paths'), d['kernel_trace_avg_ns'], d.get('valu_issue_frac'), d.get('valu_weighted_issue_frac'), d.get('lds_issue_frac'), d.get('wait_over_issue'), d.get('scratch_bytes_per_lane'), round(d.get('hbm_bytes_per_syndrome', 0)))"
done
