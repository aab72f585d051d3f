#!/bin/bash
# Register / spill report of the P61 fixed-stop decode kernel for a set of compile flags:
#   tools/kbench/regs.sh -DQEC_MASK_SELECT=1 ...
cd "$(dirname "$0")/../.."
out=$(mktemp /tmp/regs.XXXXXX.s)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fno-fast-math -fno-slp-vectorize \
    -DQEC_KBENCH_MINIMAL "$@" --cuda-device-only -S -o $out qec_ldpc_amd/csrc/bp_decode.hip 2>/dev/null
awk '/^_ZN3qec16bp_decode_kernelILi4ELi5ELi10ELi1E.*:/{f=1} f{print} f&&/\.end_amdhsa_kernel/{exit}' $out > $out.k
printf "vgpr=%s spill_vgpr=%s scratch_loads=%s instrs=%s bpermute=%s\n" \
  "$(grep -m1 -oP '\.amdhsa_next_free_vgpr \K\d+' $out.k)" \
  "$(grep -m1 -oP 'VGPRSpill: \K\d+|; NumVGPRsForWavesPerEU: \K\d+' $out.k | head -1)" \
  "$(grep -c scratch_load $out.k)" "$(grep -cE '^\s+[vsd][a-z_0-9]+ ' $out.k)" "$(grep -c ds_bpermute $out.k)"
rm -f $out $out.k
