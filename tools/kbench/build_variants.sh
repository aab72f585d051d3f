#!/bin/bash
# Build experimental variants of libqecldpc.so into build/variants/<name>/ (same sources,
# different compile flags / macros).  Used by tools/kbench/compare.py on the GPU box.
set -e
cd "$(dirname "$0")/../.."
HIPCC=/opt/rocm/bin/hipcc
BASE="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math -fno-slp-vectorize -w"
build() {
  name=$1; shift
  out=build/variants/$name
  mkdir -p $out
  $HIPCC $BASE "$@" -c qec_ldpc_amd/csrc/bp_decode.hip -o $out/bp_decode.o &
  $HIPCC $BASE -x c++ -c qec_ldpc_amd/csrc/code_model.cpp -o $out/code_model.o &
  $HIPCC $BASE -c qec_ldpc_amd/csrc/montecarlo.hip -o $out/montecarlo.o &
  $HIPCC $BASE -x hip -c qec_ldpc_amd/csrc/capi.cpp -o $out/capi.o &
  wait
  $HIPCC --offload-arch=gfx950 -shared -fPIC -o $out/libqecldpc.so $out/*.o
  echo "built $name"
}
while [ $# -gt 0 ]; do
  spec=$1; shift
  name=${spec%%:*}; flags=${spec#*:}
  [ "$flags" = "$spec" ] && flags=""
  build $name $flags
done
