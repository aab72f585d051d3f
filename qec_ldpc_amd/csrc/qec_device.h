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

// Exponent tables of the QC_LDPC_CSS generator (QEC_LDPC/QEC_LDPC_CSS.cu:37-90) evaluated by the
// compiler: block (r, l) of sector X (Z) is the circulant check (r, i) <-> variable
// (l, (E[r][l] + i) mod P).  The host side checks a code file against the same formula
// (code_model.cpp, generator_exponents) before a kernel specialised on these tables takes it.
template <int J_, int K_, int L_, int P_, int S_, int T_>
struct QcExponents {
    int EX[J_][L_];
    int EZ[K_][L_];
    static constexpr long pw(long base, long e)
    {
        long t = 1;
        for (long i = 0; i < e; ++i) t = (t * base) % P_;
        return t;
    }
    static constexpr QcExponents make()
    {
        QcExponents t{};
        long inv = 1;
        for (long x = 1; x < P_; ++x)
            if ((x * S_) % P_ == 1) { inv = x; break; }
        auto sp = [inv](long p) { return p < 0 ? pw(inv, -p) : pw(S_, p); };
        for (int j = 0; j < J_; ++j)
            for (int l = 0; l < L_; ++l)
                t.EX[j][l] = (int)(((l < L_ / 2) ? sp(l - j) : P_ - (T_ * sp(j - 1 + l)) % P_) % P_);
        for (int k = 0; k < K_; ++k)
            for (int l = 0; l < L_; ++l)
                t.EZ[k][l] = (int)(((((l < L_ / 2) ? (T_ * sp(l - k - 1)) % P_ : P_ - sp(k + l)) % P_) + P_) % P_);
        return t;
    }
};

}  // namespace qec
