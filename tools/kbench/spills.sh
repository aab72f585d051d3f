#!/bin/bash
# Static spill report (scratch instructions, VGPRs) of the decode kernels the library ships:
# the P61 reference/fixed kernels (minreg unit) and the syndrome-stop kernels (main unit).
#   tools/kbench/spills.sh [-DMACRO=...]
cd "$(dirname "$0")/../.."
F="--offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fno-fast-math -fno-slp-vectorize --cuda-device-only -S $*"
/opt/rocm/bin/hipcc $F -mllvm -amdgpu-sched-strategy=iterative-minreg -o /tmp/sp_p61.s qec_ldpc_amd/csrc/bp_decode_p61.hip 2>/dev/null &
/opt/rocm/bin/hipcc $F -DQEC_KBENCH_MINIMAL -o /tmp/sp_main.s qec_ldpc_amd/csrc/bp_decode.hip 2>/dev/null &
wait
python3 tools/kbench/isa_stats.py /tmp/sp_p61.s | sed 's/^/minreg /'
python3 tools/kbench/isa_stats.py /tmp/sp_main.s | sed 's/^/main   /'
