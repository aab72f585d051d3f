# Monte-Carlo (config 5) evidence: the p-sweep, then per p a kernel-trace --stats pass and five PMC
# passes (each counter group in its own run, --kernel-trace only beside --pmc) of one psweep point at the
# sweep's own shape (2^20 samples, one batch), summarised into profiles-ready JSON (mc_pmc_summary.py):
# per kernel its dispatch time, VALU / LDS issue fractions, waits and HBM bytes.
#   [STOP=syndrome|fixed|ref] bash tools/gpu/run_mc_profile.sh TAG [p ...]
# STOP other than syndrome (the config-5 rule) writes pmc_mc_p61_<STOP>_p<P>.json (psweep --stop STOP).
set -o pipefail
R="$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-r05}; shift
PS=${@:-0.002 0.01}
STOP=${STOP:-syndrome}
SFX=""; [ "$STOP" != syndrome ] && SFX="${STOP}_"
OUT="$R/gpurun_out/mc_$TAG"
mkdir -p "$OUT"
cd "$R"
if [ -z "$NO_SWEEP" ]; then
  timeout -k 10 300 python tools/psweep.py --stop $STOP --out "$OUT/psweep_$STOP.json" > "$OUT/psweep_$STOP.txt" 2>&1 || { tail -5 "$OUT/psweep_$STOP.txt"; exit 1; }
  tail -1 "$OUT/psweep_$STOP.txt"
fi
cd /tmp
for P in $PS; do
  D="$OUT/$SFX""p$P"; mkdir -p "$D"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$D/trace" -o run -- \
      python3 "$R/tools/psweep.py" --stop $STOP --ps $P --reps 1 > "$D/trace.out" 2> "$D/trace.err" || { tail -5 "$D/trace.err"; exit 1; }
  i=0
  for grp in "FETCH_SIZE" "WRITE_SIZE" "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES" \
             "SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES GRBM_GUI_ACTIVE" \
             "SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_INT32 SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT"; do
    i=$((i+1))
    timeout -k 10 -s KILL 180 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d "$D/pmc$i" -o run -- \
        python3 "$R/tools/psweep.py" --stop $STOP --ps $P --reps 1 > /dev/null 2> "$D/pmc$i.err"
    rc=$?; echo "p=$P pmc$i rc=$rc"; if [ $rc -ne 0 ]; then tail -5 "$D/pmc$i.err"; exit $rc; fi
  done
  python3 "$R/tools/gpu/mc_pmc_summary.py" --dir "$D" --p $P --stop $STOP --out "$OUT/pmc_mc_p61_$SFX""p$P.json" || exit 1
done
