// Device pieces of the Monte-Carlo caller shared by montecarlo.hip (sampler, syndromes, statistics)
// and triage.hip (the fused low-p pipeline): the counter-based Philox4x32-10 stream, the gap-walk
// depolarising sampler, the counter layout and the I-P logical check (gfx950 only).
#pragma once
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>

#include "qec_device.h"

namespace qec {

// ---- Philox4x32-10 (Salmon et al., SC'11) -----------------------------------
struct U4 {
    uint32_t x, y, z, w;
};

__host__ __device__ inline U4 philox4x32_10(U4 c, uint32_t k0, uint32_t k1)
{
    for (int r = 0; r < 10; ++r) {
        const uint64_t p0 = (uint64_t)0xD2511F53u * c.x;
        const uint64_t p1 = (uint64_t)0xCD9E8D57u * c.z;
        const uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
        const uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
        c = U4{hi1 ^ c.y ^ k0, lo1, hi0 ^ c.w ^ k1, lo0};
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
    return c;
}


// Depolarising sampler ("gap walk"; restated in numpy by oracle/philox.py).  A qubit is hit with
// probability thr / 2^32, thr = floor(p 2^32) (saturated at 2^32), independently of the others, so
// the number of qubits skipped before the next hit is geometric: P(G >= g) = q^g, q = 1 - thr / 2^32.
// Sample b walks its qubits 0 .. n-1 in order, drawing 32-bit words from Philox calls k = 0, 1, ...
// (counter (b_lo, b_hi, k, kGapSalt), key (seed_lo, seed_hi), word 4k + j = output word j of call
// k): u = next word, G = #{g in 1..n : u < T[g]} with the gap table T[g] = floor(q^g 2^32) (q^g by
// right-to-left binary exponentiation in IEEE double, powsq); skip G qubits; if the walk is still
// inside the sample, the qubit there is hit, of type t = floor(3 w / 2^32) of the next word w
// (0 = X, 1 = Y, 2 = Z; Y sets both bits), and the walk goes on from the next qubit.  A sample at
// p = 0.01 costs ~13 words (four Philox calls) instead of one word per qubit (153 calls for P61).
constexpr uint32_t kGapSalt = 0x6A9C0DE5u;

__host__ __device__ inline double powsq(double q, int g)
{
    double r = 1.0, b = q;
    for (int e = g; e != 0;) {
        if (e & 1) r = r * b;
        e >>= 1;
        if (e != 0) b = b * b;
    }
    return r;
}

struct GapParams {
    uint64_t seed;
    uint64_t thr;     // 0: no qubit is ever hit
    double q;         // 1 - thr / 2^32 (exact)
    float inv_l2q;    // 1 / log2(q) (the gap estimate's scale; -0 for q = 0)
};

__host__ inline GapParams make_gap(uint64_t seed, float p)
{
    const double pd = p;
    GapParams g{seed, pd <= 0.0 ? 0ull : pd >= 1.0 ? (1ull << 32) : (uint64_t)(pd * 4294967296.0), 1.0, 0.0f};
    g.q = (4294967296.0 - (double)g.thr) / 4294967296.0;
    g.inv_l2q = g.thr == 0 ? 0.0f : (float)(1.0 / std::log2(g.q));
    return g;
}

// The gap before the next hit: #{g in 1..n : u < T[g]} (T non-increasing: q^(g+1) < q^g by far more
// than the exponentiation's rounding, so this is the largest g with u < T[g], 0 if none).  A float
// estimate from log2(u / 2^32) / log2(q) lands within a step or two of it; the table walk then
// makes it exact.  T[1..n] in LDS.
__device__ __forceinline__ int gap_of(uint32_t u, const uint32_t* __restrict__ T, int n, float inv_l2q)
{
    if (u >= T[1]) return 0;
    const float x = ((float)u + 0.5f) * 0x1p-32f;
    const float e = __log2f(x) * inv_l2q;
    int g = e >= (float)n ? n : e >= 1.0f ? (int)e : 1;
    while (g < n && u < T[g + 1]) ++g;
    while (u >= T[g]) --g;  // stops at g = 1 at the latest (u < T[1])
    return g;
}

// The walk of one sample (this lane): hit(v, t) for every hit qubit v of type t, in ascending v.
template <class Hit>
__device__ __forceinline__ void gap_walk(const GapParams& gp, uint64_t b, int n, const uint32_t* __restrict__ T,
                                         Hit&& hit)
{
    U4 o{0, 0, 0, 0};
    uint32_t wi = 0, call = 0xFFFFFFFFu;
    auto next = [&]() -> uint32_t {
        const uint32_t k = wi >> 2;
        if (k != call) {
            o = philox4x32_10(U4{(uint32_t)b, (uint32_t)(b >> 32), k, kGapSalt}, (uint32_t)gp.seed,
                              (uint32_t)(gp.seed >> 32));
            call = k;
        }
        const uint32_t j = wi & 3u;
        ++wi;
        return j == 0 ? o.x : j == 1 ? o.y : j == 2 ? o.z : o.w;
    };
    int pos = 0;
    while (true) {
        pos += gap_of(next(), T, n, gp.inv_l2q);
        if (pos >= n) break;
        hit(pos, __umulhi(next(), 3u));
        if (++pos >= n) break;
    }
}

// Build the workgroup's gap table T[1..n] (T[0] unused).
__device__ __forceinline__ void gap_table(const GapParams& gp, int n, uint32_t* __restrict__ T)
{
    for (int g = threadIdx.x + 1; g <= n; g += blockDim.x) T[g] = (uint32_t)(powsq(gp.q, g) * 4294967296.0);
    if (threadIdx.x == 0) T[0] = 0xFFFFFFFFu;
}

// counters, in qec_mc_counters order
enum { C_WITHX, C_WITHZ, C_SYNX, C_SYNZ, C_LOGICAL, C_CORRECTED, C_CONVX, C_CONVZ, C_N };

// CheckLogicalError (Quantum_LDPC_Code.h:126-142): (I-P) r != 0 for the residual r, as the XOR
// of the columns of I-P (restricted to its non-zero rows, cw <= 64 words each; lane k holds word
// k of the sum) at the set bits of r.  A decoded residual is nearly always 0 or sparse, so this
// reads a few columns instead of every row (P61: 678 x 20 words per sample).  res[0..nw) is the
// residual in LDS, the same for every lane; REC: record layout (x bits at [0, 8 nb), z bits at
// [8 nb, 16 nb)), else qubit layout (bit q = qubit q of [x | z]).
constexpr int kMaxWords = 64;  // 2n <= 4096 qubits

// The residual's words are read once (lane k: word k, nw <= 64) and broadcast with readlane, and the
// columns are fetched four at a time, so a sample costs one LDS round trip and about popcount / 4
// global ones instead of one per word and one per set bit.
template <bool REC>
__device__ __forceinline__ bool logical_from_columns(const unsigned long long* res, int nw, int n, int nb,
                                                     const uint64_t* __restrict__ cols, int cw, int lane)
{
    const uint64_t mine = lane < nw ? res[lane] : 0ull;
    const uint32_t lo = (uint32_t)mine, hi = (uint32_t)(mine >> 32);
    const bool col_lane = lane < cw;
    uint64_t acc = 0;
    for (int w = 0; w < nw; ++w) {
        uint64_t bits = ((uint64_t)__builtin_amdgcn_readlane(hi, w) << 32) | __builtin_amdgcn_readlane(lo, w);
        while (bits) {  // uniform
            int q[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                q[u] = -1;
                if (bits) {
                    const int j = __builtin_ctzll(bits);
                    bits &= bits - 1;
                    const int qq = 64 * w + j;
                    q[u] = REC ? (qq < 8 * nb ? qq : n + (qq - 8 * nb)) : qq;
                }
            }
            uint64_t c[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) c[u] = (q[u] >= 0 && col_lane) ? cols[(size_t)q[u] * cw + lane] : 0ull;
            acc ^= (c[0] ^ c[1]) ^ (c[2] ^ c[3]);
        }
    }
    return __any(acc != 0);
}

}  // namespace qec
