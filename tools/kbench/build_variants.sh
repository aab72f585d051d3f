#!/bin/bash
# Build experimental variants of libqecldpc.so into build/variants/<name>/ (same sources,
# different compile flags / macros for bp_decode.hip, triage.hip, schedule.hip and capi.cpp; the other
# objects are shared).
# Used by tools/kbench/compare.py on the GPU box.
#   tools/kbench/build_variants.sh name[:flags] ...     e.g.  cur  pipe:-DQEC_PIPELINE=1
# SRCDIR=dir builds the variants from dir/bp_decode*.hip instead (e.g. an older revision for an A/B;
# the directory also needs qec_device.h and qec_internal.h)
set -e
cd "$(dirname "$0")/../.."
HIPCC=/opt/rocm/bin/hipcc
BASE="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math -fno-slp-vectorize -w"
COMMON=build/variants/_common
mkdir -p $COMMON
common() {
  src=$1; obj=$COMMON/$(basename ${src%.*}).o; shift
  if [ ! -f $obj ] || [ $src -nt $obj ]; then $HIPCC $BASE "$@" -c $src -o $obj; fi
}
common qec_ldpc_amd/csrc/code_model.cpp -x c++ &
common qec_ldpc_amd/csrc/cpu_engine.cpp -x c++ &
common qec_ldpc_amd/csrc/montecarlo.hip &
common qec_ldpc_amd/csrc/bp_sparse.hip &
wait
SRC=${SRCDIR:-qec_ldpc_amd/csrc}
build() {
  name=$1; shift
  out=build/variants/$name
  mkdir -p $out
  $HIPCC $BASE -DQEC_KBENCH_MINIMAL -I qec_ldpc_amd/csrc "$@" -c $SRC/bp_decode.hip -o $out/bp_decode.o
  $HIPCC $BASE -DQEC_KBENCH_MINIMAL -I qec_ldpc_amd/csrc -mllvm -amdgpu-sched-strategy=iterative-minreg "$@" \
      -c $SRC/bp_decode_p61.hip -o $out/bp_decode_p61.o
  $HIPCC $BASE -DQEC_KBENCH_MINIMAL -I qec_ldpc_amd/csrc "$@" -c $SRC/bp_decode_phase.hip -o $out/bp_decode_phase.o
  $HIPCC $BASE -I qec_ldpc_amd/csrc "$@" -c qec_ldpc_amd/csrc/triage.hip -o $out/triage.o
  $HIPCC $BASE -I qec_ldpc_amd/csrc "$@" -c qec_ldpc_amd/csrc/schedule.hip -o $out/schedule.o
  $HIPCC $BASE -I qec_ldpc_amd/csrc -x hip "$@" -c qec_ldpc_amd/csrc/capi.cpp -o $out/capi.o
  $HIPCC --offload-arch=gfx950 -shared -fPIC -o $out/libqecldpc.so $out/bp_decode.o $out/bp_decode_p61.o \
      $out/bp_decode_phase.o $out/triage.o $out/schedule.o $out/capi.o $(ls $COMMON/*.o | grep -v /capi.o)
  echo "built $name"
}
pids=()
while [ $# -gt 0 ]; do
  spec=$1; shift
  name=${spec%%:*}; flags=${spec#*:}
  [ "$flags" = "$spec" ] && flags=""
  flags=${flags//,/ }
  build $name $flags &
  pids+=($!)
  if [ ${#pids[@]} -ge 6 ]; then wait ${pids[0]}; pids=("${pids[@]:1}"); fi
done
wait
