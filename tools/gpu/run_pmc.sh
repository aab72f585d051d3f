# PMC passes (each counter group in its own rocprofv3 run, --kernel-trace only alongside --pmc)
set -o pipefail
R="$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-r01}
CODE=${2:-p61}
mkdir -p "$R/gpurun_out/pmc_$TAG"; cd /tmp
rocprofv3 -L > "$R/gpurun_out/pmc_list_$TAG.txt" 2>&1 || true
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" "SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_INSTS_SALU" "SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM" "SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_ADD_F32"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d "$R/gpurun_out/pmc_$TAG/p$i" -o run -- python3 "$R/bench.py" --no-cpu --no-full-arith --steps 3 --warmup 1 --code "$CODE" > "$R/gpurun_out/pmc_$TAG/p$i.json" 2> "$R/gpurun_out/pmc_$TAG/p$i.err"
  rc=$?
  echo "pass $i ($grp) rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 "$R/gpurun_out/pmc_$TAG/p$i.err"; fi
  if [ $rc -eq 124 ] || [ $rc -eq 137 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then break; fi
done
ls -R "$R/gpurun_out/pmc_$TAG" | head -40
