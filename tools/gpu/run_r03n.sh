# round 3, call n: order-pass chunk size at P7 configs[1] (QEC_SCHED_CHUNK, separate processes).
set -o pipefail
R="$GRAFT_REPO_ROOT"
O="$R/gpurun_out/r03n"
mkdir -p "$O"
cd "$R"
export TMPDIR=/tmp
for c in 0 128 256 512 1024 2048; do
  QEC_SCHED_CHUNK=$c timeout -k 10 200 python tools/kbench/compare.py --code p7 --batch 65536 --reps 15 cur cur:schedule=0 > "$O/cmp_chunk$c.txt" 2>&1 || { tail "$O/cmp_chunk$c.txt"; exit 1; }
  echo "chunk $c"; grep -v "^{" "$O/cmp_chunk$c.txt" | grep -v amdgpu.ids
done
