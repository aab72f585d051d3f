// The P61 reference- and fixed-stop and the P7 syndrome-stop decode kernels, compiled with LLVM's iterative-minreg
// machine scheduler (Makefile: -mllvm -amdgpu-sched-strategy=iterative-minreg, a per-file
// option).  Same source as bp_decode.hip; see the TuneP61 comment there for why and the
// measurements.
#define QEC_P61_MINREG_TU 1
#include "bp_decode.hip"
