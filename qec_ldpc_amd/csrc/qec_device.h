// Device helpers shared by the HIP translation units (gfx950 only).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace qec {

// the low bit of each byte of v, byte t -> bit t (the 8 partial products land on distinct bits, so
// no carries: byte t times 2^(56 - 7 s) sits at bit 56 + t for s = t and below bit 56 or above 63
// otherwise)
__device__ __forceinline__ uint32_t pack8(uint64_t v) { return (uint32_t)((v * 0x0102040810204080ull) >> 56); }

// Order this wave's LDS accesses around an exchange between its lanes: a wave's LDS operations
// complete in issue order, and the fences keep the compiler from moving accesses across.
__device__ __forceinline__ void wave_sync()
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

}  // namespace qec
