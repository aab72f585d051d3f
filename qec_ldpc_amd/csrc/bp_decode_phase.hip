// The instrumented decode kernels of the shipped codes (QEC_OPT_PHASE_STATS): iters[] reports,
// per sector, the iterations spent in each phase (soft | hard << 8 | agreed << 16 | jumped << 24)
// instead of their count.  A translation unit of its own, so the production kernels are compiled
// exactly as without it.  Same source as bp_decode.hip.
#define QEC_PHASE_STATS 1
#define QEC_PHASE_TU 1
#include "bp_decode.hip"
