// Monte-Carlo caller side on the GPU: what
// DecoderCPU::GetStatistics does around Decode (QEC_LDPC/DecoderCPU.h:392-530),
// batched:
//   * errors: i.i.d. depolarising samples from a counter-based Philox4x32-10 stream
//     (any shard of the sample index space can be generated independently), or the
//     reference's fixed-weight draws (host mt19937 stream, DecoderCPU.h:448-459)
//     expanded on the device;
//   * syndromes: s(r, i) = XOR_l e[l P + (E[r][l] + i) mod P]  (GetSyndromeX/Z,
//     Quantum_LDPC_Code.h:94-124, through the circulant tables), fused with the errors
//     (mc_errors_syndrome_kernel: one wave per sample, errors staged in LDS);
//   * statistics: residual e ^ e_hat bit-packed, I-P logical check
//     (Quantum_LDPC_Code.h:126-142) on bit-packed rows, and the CodeStatistics
//     counters (DecoderCPU.h:464-521) reduced per block.
// These are integer/byte kernels: HBM/L2-bound, not worth MFMA.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>

#include "qec_device.h"
#include "qec_internal.h"

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

constexpr uint32_t kPhiloxSalt = 0x51EC0DE5u;

// Depolarising sampler.  Qubits 4g .. 4g+3 of sample b share one Philox call: counter
// (b_lo, b_hi, g, salt), key (seed_lo, seed_hi), output words w0..w3, word j for qubit 4g + j.
// The qubit is hit iff w < thr = floor(p 2^32) (saturated at 2^32).  Given a hit, w is uniform on
// [0, thr), and its type is t = floor(w mul / 2^64) with mul = min(floor(3 2^64 / thr), 2^64 - 1),
// i.e. floor(3 w / thr) up to the rounding of mul: 0 = X, 1 = Y, 2 = Z, each with probability
// 1/3 to within 1/thr (Y sets both bits).  Four qubits per call: the front end's cost is the
// Philox rounds.  Restated in numpy by oracle/philox.py.
struct Depol {
    uint64_t seed, thr, mul;
};

__host__ inline Depol make_depol(uint64_t seed, float p)
{
    const double pd = p;
    Depol d{seed, pd <= 0.0 ? 0ull : pd >= 1.0 ? (1ull << 32) : (uint64_t)(pd * 4294967296.0), 0};
    if (d.thr >= 3) {
        const unsigned __int128 m = ((unsigned __int128)3 << 64) / d.thr;
        d.mul = m > ~0ull ? ~0ull : (uint64_t)m;
    } else if (d.thr > 0) {
        d.mul = ~0ull;
    }
    return d;
}

// x4 / z4: the four qubits' bits as bytes (byte j = qubit 4g + j)
__device__ __forceinline__ void depolarizing4(const Depol& d, uint64_t sb, uint32_t g, uint32_t& x4, uint32_t& z4)
{
    const U4 o = philox4x32_10(U4{(uint32_t)sb, (uint32_t)(sb >> 32), g, kPhiloxSalt}, (uint32_t)d.seed,
                               (uint32_t)(d.seed >> 32));
    const uint32_t w[4] = {o.x, o.y, o.z, o.w};
    x4 = 0;
    z4 = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        if ((uint64_t)w[j] < d.thr) {
            // floor(w mul / 2^64) = floor((w mul_hi + floor(w mul_lo / 2^32)) / 2^32), no overflow
            const uint64_t hi = (uint64_t)w[j] * (d.mul >> 32) + (((uint64_t)w[j] * (uint32_t)d.mul) >> 32);
            const uint32_t t = (uint32_t)(hi >> 32);
            x4 |= (uint32_t)(t != 2) << (8 * j);
            z4 |= (uint32_t)(t != 0) << (8 * j);
        }
    }
}

// byte form (qec_sample_depolarizing_dev): one thread per four qubits of a sample
__global__ void sample_depolarizing_kernel(Depol d, uint64_t start, long long B, int n, uint8_t* __restrict__ x,
                                           uint8_t* __restrict__ z)
{
    const int ng = (n + 3) / 4;
    const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= B * ng) return;
    const long long b = t / ng;
    const int g = (int)(t - b * ng);
    uint32_t x4, z4;
    depolarizing4(d, start + (uint64_t)b, (uint32_t)g, x4, z4);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int v = 4 * g + j;
        if (v < n) {
            x[b * n + v] = (uint8_t)((x4 >> (8 * j)) & 1u);
            z[b * n + v] = (uint8_t)((z4 >> (8 * j)) & 1u);
        }
    }
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

template <bool REC>
__device__ __forceinline__ bool logical_from_columns(const unsigned long long* res, int nw, int n, int nb,
                                                     const uint64_t* __restrict__ cols, int cw, int lane)
{
    uint64_t acc = 0;
    for (int w = 0; w < nw; ++w) {
        const uint64_t v = res[w];
        uint64_t bits = ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(v >> 32)) << 32) |
                        __builtin_amdgcn_readfirstlane((uint32_t)v);  // uniform: scalar loop below
        while (bits) {
            const int j = __builtin_ctzll(bits);
            bits &= bits - 1;
            int q = 64 * w + j;
            if (REC) q = q < 8 * nb ? q : n + (q - 8 * nb);
            if (lane < cw) acc ^= cols[(size_t)q * cw + lane];
        }
    }
    return __any(acc != 0);
}

// Grid-stride over samples, one wave per sample at a time; each wave keeps its counts in
// registers and the workgroup adds them to `counters` once (same-address atomics from every
// workgroup serialise at L2: 16 384 four-wave workgroups x 8 counters cost ~190 us per 65 536
// samples, profiles/r02/mc_r02f_trace.csv).
constexpr int kStatBlockWaves = 16;
constexpr int kStatMaxBlocks = 512;

__device__ __forceinline__ void stat_flush(unsigned long long (*part)[C_N + 2], const unsigned long long* c, int nc,
                                           unsigned long long* __restrict__ counters)
{
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    if (lane < nc) {
        unsigned long long v = 0;
        for (int k = 0; k < C_N + 2; ++k) v = lane == k ? c[k] : v;
        part[wv][lane] = v;
    }
    __syncthreads();
    if (threadIdx.x < nc) {
        unsigned long long v = 0;
        for (int w = 0; w < kStatBlockWaves; ++w) v += part[w][threadIdx.x];
        if (v) atomicAdd(&counters[threadIdx.x], v);
    }
}

// Residual words are formed with ballots (lane = qubit within a 64-qubit word) and parked in LDS
// for the column test above.
__global__ __launch_bounds__(64 * kStatBlockWaves) void statistics_kernel(
    const uint8_t* __restrict__ x, const uint8_t* __restrict__ z, const uint8_t* __restrict__ eX,
    const uint8_t* __restrict__ eZ, const uint8_t* __restrict__ flags, long long B, int n,
    const uint64_t* __restrict__ imp_cols, int imp_cw, unsigned long long* __restrict__ counters)
{
    __shared__ unsigned long long part[kStatBlockWaves][C_N + 2];
    __shared__ unsigned long long sres[kStatBlockWaves][kMaxWords];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int nw = (2 * n + 63) / 64;
    unsigned long long c[C_N + 2] = {};
    for (long long b = (long long)blockIdx.x * kStatBlockWaves + wv; b < B; b += (long long)gridDim.x * kStatBlockWaves) {
        bool anyX = false, anyZ = false;
        for (int w = 0; w < nw; ++w) {
            const int q = w * 64 + lane;
            bool bit = false;
            if (q < n) {
                const uint8_t xe = x[b * n + q];
                anyX |= xe != 0;
                bit = (xe ^ eX[b * n + q]) & 1;
            } else if (q < 2 * n) {
                const uint8_t ze = z[b * n + q - n];
                anyZ |= ze != 0;
                bit = (ze ^ eZ[b * n + q - n]) & 1;
            }
            const unsigned long long word = __ballot(bit);
            if (lane == 0) sres[wv][w] = word;
        }
        wave_sync();
        const uint8_t f = flags[b];
        const bool dEX = f & QEC_SYNDROME_FAIL_X, dEZ = f & QEC_SYNDROME_FAIL_Z;
        bool logical = false;
        if (!(dEX || dEZ) && imp_cw > 0)  // CheckLogicalError only when no syndrome failure
            logical = logical_from_columns<false>(sres[wv], nw, n, 0, imp_cols, imp_cw, lane);
        wave_sync();  // sres is rewritten by the next sample
        c[C_WITHX] += __any(anyX);
        c[C_WITHZ] += __any(anyZ);
        c[C_SYNX] += dEX;
        c[C_SYNZ] += dEZ;
        c[C_LOGICAL] += !(dEX || dEZ) && logical;
        c[C_CORRECTED] += !(dEX || dEZ) && !logical;
        c[C_CONVX] += (f & QEC_CONVERGENCE_FAIL_X) != 0;
        c[C_CONVZ] += (f & QEC_CONVERGENCE_FAIL_Z) != 0;
    }
    stat_flush(part, c, C_N, counters);
}

// Decision records for the cross-rank gather: per syndrome, eX bit-packed
// (ceil(n/8) bytes, bit j of byte k = qubit 8k + j), then eZ the same way, then the flags byte.
// One thread per output byte; each reads its 8 (contiguous) decision bytes.
__global__ void pack_decisions_kernel(const uint8_t* __restrict__ eX, const uint8_t* __restrict__ eZ,
                                      const uint8_t* __restrict__ flags, long long B, int n,
                                      uint8_t* __restrict__ out)
{
    const int nb = (n + 7) / 8, rec = 2 * nb + 1;
    const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= B * rec) return;
    const long long b = t / rec;
    const int k = (int)(t - b * rec);
    if (k == 2 * nb) {
        out[t] = flags[b];
        return;
    }
    const uint8_t* e = (k < nb ? eX : eZ) + b * n;
    const int q0 = 8 * (k < nb ? k : k - nb);
    uint32_t v = 0;
    for (int j = 0; j < 8 && q0 + j < n; ++j) v |= (uint32_t)(e[q0 + j] & 1) << j;
    out[t] = (uint8_t)v;
}

// ---- fused Monte-Carlo front end ----------------------------------------------------
// One wave per sample, errors staged in LDS (this wave's x and z rows, each zero-padded to
// npad = 8 nb bytes):
//   source PHILOX: the depolarising sampler above, qubit by qubit (nothing read from HBM);
//   source DRAWS:  the reference's W (index, type) draws of the sample (DecoderCPU.h:452-457);
//   source BYTES:  x, z rows [B][n] from HBM.
// Then, from LDS: the syndromes sX, sZ (QC: s(r, i) = XOR_l e[l P + (E[r][l] + i) mod P]; any other
// regular code: the check's variables from the sparse engine's table), and the bit-packed errors
// errp [B][2 nb] in the decision-record layout (x bits, then z bits) for the statistics kernel.
// HBM traffic per P61 sample: 549 B of syndromes + 154 B of packed errors written.
constexpr int kMcWaves = 4;

struct McArgs {
    // sources
    Depol depol;                               // PHILOX
    uint64_t start;
    const int32_t* idx;                        // DRAWS: [B][W] qubit indices
    const uint8_t* type;                       //        [B][W] 0 = X, 1 = Y, 2 = Z
    int W;
    const uint8_t* x;                          // BYTES: [B][n]
    const uint8_t* z;
    // outputs
    uint8_t* sX;                               // [B][mX]
    uint8_t* sZ;                               // [B][mZ]
    uint8_t* errp;                             // [B][2 nb] (nullable)
    const int32_t* chkVar;                     // non-QC codes: [(mX + mZ) L] variables per check
    long long B;
    int n, nb, L, P, J, K, mX, mZ;
    int S;                                     // samples per wave
    uint32_t magicW, magicG, magicG2, magicN, magicM, magicP, magicB;  // ceil(2^32 / d) for the item counts
    int EX[128], EZ[128];
};

// (i, k) = (t / d, t mod d) for the small work-item counts below: magic = ceil(2^32 / d) is exact
// for t d < 2^32 (t < 2^16 and d < 2^16 here); d = 1 (magic 2^32 does not fit) is passed as 0
__device__ __forceinline__ int qdiv(int t, uint32_t magic) { return magic ? (int)__umulhi((uint32_t)t, magic) : t; }

// A wave handles S = max(1, floor(64 / P)) samples (P61: 1, P7: 9), so short codes keep the lanes
// busy; each phase spreads its (sample, item) pairs over the lanes.
// LT: the block-column count L when known at compile time (the shipped codes: 10 and 6), so the
// syndrome's L-term XOR is unrolled with every LDS read in flight at once; 0 = a.L at run time.
template <int SRC, int LT>
__global__ __launch_bounds__(64 * kMcWaves) void mc_errors_syndrome_kernel(const McArgs a)
{
    extern __shared__ __attribute__((aligned(8))) uint8_t mc_smem[];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int S = a.S;
    const long long b0 = ((long long)blockIdx.x * kMcWaves + wv) * S;
    if (b0 >= a.B) return;  // wave-local from here on: no workgroup barrier
    const int ns = (int)(a.B - b0 < S ? a.B - b0 : S);  // samples of this wave
    const int n = a.n, npad = 8 * a.nb;
    uint8_t* __restrict__ stage = mc_smem + (size_t)wv * S * 2 * npad;  // sample s: x at 2 s npad, z after
    if constexpr (SRC == MC_SRC_DRAWS) {
        const int nw = npad / 4;  // zero both rows, a word at a time
        for (int t = lane; t < ns * 2 * nw; t += 64) reinterpret_cast<uint32_t*>(stage)[t] = 0u;
        wave_sync();
        for (int t = lane; t < ns * a.W; t += 64) {
            const int sI = qdiv(t, a.magicW), w = t - sI * a.W;
            const long long b = b0 + sI;
            const int v = a.idx[b * a.W + w];
            const int ty = a.type[b * a.W + w];
            uint8_t* ex = stage + (size_t)sI * 2 * npad;
            if (ty == 0 || ty == 1) ex[v] = 1;  // several draws may hit one qubit: they all store 1
            if (ty == 2 || ty == 1) ex[npad + v] = 1;
        }
    } else if constexpr (SRC == MC_SRC_PHILOX) {
        // four qubits per lane and Philox call, one 32-bit LDS word per row (npad is a multiple of
        // 8, so the padding words are written too, zero past n)
        const int ng = npad / 4;
#pragma unroll 3
        for (int t = lane; t < ns * ng; t += 64) {
            const int sI = qdiv(t, a.magicG), g = t - sI * ng;
            uint32_t x4 = 0, z4 = 0;
            if (4 * g < n) {
                depolarizing4(a.depol, a.start + (uint64_t)(b0 + sI), (uint32_t)g, x4, z4);
                if (4 * g + 4 > n) {
                    const uint32_t keep = 0xFFFFFFFFu >> (8 * (4 * g + 4 - n));
                    x4 &= keep;
                    z4 &= keep;
                }
            }
            uint32_t* row = reinterpret_cast<uint32_t*>(stage + (size_t)sI * 2 * npad);
            row[g] = x4;
            row[ng + g] = z4;
        }
    } else {
        for (int t = lane; t < ns * npad; t += 64) {
            const int sI = qdiv(t, a.magicN), v = t - sI * npad;
            uint8_t xv = 0, zv = 0;
            if (v < n) {
                const long long b = b0 + sI;
                xv = a.x[b * n + v] & 1u;
                zv = a.z[b * n + v] & 1u;
            }
            stage[(size_t)sI * 2 * npad + v] = xv;
            stage[(size_t)sI * 2 * npad + npad + v] = zv;
        }
    }
    wave_sync();
    if (a.chkVar != nullptr) {  // any regular code: the check's variables from the sparse engine's table
        const int m = a.mX + a.mZ;
        for (int t = lane; t < ns * m; t += 64) {
            const int sI = qdiv(t, a.magicM), c = t - sI * m;
            const bool zs = c >= a.mX;
            const uint8_t* e = stage + (size_t)sI * 2 * npad + (zs ? npad : 0);
            const int32_t* vars = a.chkVar + (size_t)c * a.L;
            uint32_t x = 0;
            for (int k = 0; k < a.L; ++k) x ^= e[vars[k]];
            const long long b = b0 + sI;
            if (zs) a.sZ[b * a.mZ + (c - a.mX)] = (uint8_t)(x & 1u); else a.sX[b * a.mX + c] = (uint8_t)(x & 1u);
        }
    } else {
        // QC: the syndrome is the XOR of the H columns of the qubits in error, which are few (a
        // depolarising sample at p = 0.01 hits ~6 of 610): each lane scans its words of the staged
        // rows and, for every set byte, flips that qubit's R checks in an LDS bit set (ds_xor);
        // then lane (sample, i) writes checks (r, i).  The per-check L-term XOR over the staged
        // bytes cost ~450 VALU per P61 sample at any p.
        const int P = a.P, L = LT > 0 ? LT : a.L;
        const int m = a.mX + a.mZ, nsw = (m + 31) / 32;
        uint32_t* __restrict__ syn = reinterpret_cast<uint32_t*>(mc_smem + (size_t)kMcWaves * S * 2 * npad) +
                                     (size_t)wv * S * nsw;
        for (int t = lane; t < ns * nsw; t += 64) syn[t] = 0u;
        wave_sync();
        const int ng = npad / 4;  // 4-byte words per staged row
        for (int t = lane; t < ns * 2 * ng; t += 64) {
            const int sI = qdiv(t, a.magicG2), k = t - sI * 2 * ng;  // word k of [x row | z row]
            uint32_t word = reinterpret_cast<const uint32_t*>(stage + (size_t)sI * 2 * npad)[k];
            if (word == 0u) continue;
            const bool zs = k >= ng;
            const int R = zs ? a.K : a.J;
            const int* E = zs ? a.EZ : a.EX;
            const int c0 = zs ? a.mX : 0;
            uint32_t* sw = syn + (size_t)sI * nsw;
            while (word) {
                const int bt = __builtin_ctz(word) >> 3;
                word &= ~(0xFFu << (8 * bt));
                const int v = 4 * (zs ? k - ng : k) + bt;  // qubit (< n: the padding bytes are zero)
                const int l = v / P, j = v - l * P;
                for (int r = 0; r < R; ++r) {
                    const int d = j - E[r * L + l];
                    const int c = c0 + r * P + (d < 0 ? d + P : d);  // check (r, (j - E) mod P) holds the qubit
                    atomicXor(&sw[c >> 5], 1u << (c & 31));
                }
            }
        }
        wave_sync();
        for (int t = lane; t < ns * P; t += 64) {
            const int sI = qdiv(t, a.magicP), i = t - sI * P;
            const long long b = b0 + sI;
            const uint32_t* sw = syn + (size_t)sI * nsw;
            for (int r = 0; r < a.J + a.K; ++r) {
                const bool zs = r >= a.J;
                const int c = (zs ? a.mX + (r - a.J) * P : r * P) + i;
                const uint8_t x = (uint8_t)((sw[c >> 5] >> (c & 31)) & 1u);
                if (zs) a.sZ[b * a.mZ + (r - a.J) * P + i] = x;
                else a.sX[b * a.mX + r * P + i] = x;
            }
        }
    }
    if (a.errp != nullptr) {
        const int nb2 = 2 * a.nb;
        for (int t = lane; t < ns * nb2; t += 64) {
            const int sI = qdiv(t, a.magicB), k = t - sI * nb2;  // byte k of [x bits | z bits]
            const uint8_t* e = stage + (size_t)sI * 2 * npad + (k < a.nb ? 8 * k : npad + 8 * (k - a.nb));
            a.errp[(b0 + sI) * nb2 + k] = (uint8_t)pack8(*reinterpret_cast<const uint64_t*>(e));
        }
    }
}

// CodeStatistics counters of a batch from bit-packed errors errp [B][2 nb] and decision records
// rec [B][2 nb + 1] (qec_decode_batch_packed_dev): the residual [x ^ eX | z ^ eZ] is their XOR
// over the first 2 nb bytes (record layout), tested by logical_from_columns; optional iteration
// sums (iters [B][2]) into counters[8], counters[9].
// One wave per sample; counters as statistics_kernel (DecoderCPU.h:464-521).
constexpr int kMaxRecWords = 80;  // 2 nb <= 640 bytes

__global__ __launch_bounds__(64 * kStatBlockWaves) void statistics_packed_kernel(
    const uint8_t* __restrict__ errp, const uint8_t* __restrict__ rec, const int32_t* __restrict__ iters, long long B,
    int n, int nb, const uint64_t* __restrict__ imp_cols, int imp_cw, unsigned long long* __restrict__ counters)
{
    __shared__ unsigned long long part[kStatBlockWaves][C_N + 2];
    __shared__ __attribute__((aligned(8))) uint8_t sres[kStatBlockWaves][8 * kMaxRecWords];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int recB = 2 * nb + 1;
    const int nw = (2 * nb + 7) / 8;
    unsigned long long c[C_N + 2] = {};
    for (long long b = (long long)blockIdx.x * kStatBlockWaves + wv; b < B; b += (long long)gridDim.x * kStatBlockWaves) {
        bool anyX = false, anyZ = false;
        for (int t = lane; t < 8 * nw; t += 64) {
            uint8_t r = 0;
            if (t < 2 * nb) {
                const uint8_t e = errp[b * 2 * nb + t];
                if (t < nb) anyX |= e != 0; else anyZ |= e != 0;
                r = e ^ rec[b * recB + t];
            }
            sres[wv][t] = r;
        }
        wave_sync();
        const uint8_t f = rec[b * recB + 2 * nb];
        const bool dEX = f & QEC_SYNDROME_FAIL_X, dEZ = f & QEC_SYNDROME_FAIL_Z;
        bool logical = false;
        if (!(dEX || dEZ) && imp_cw > 0)  // CheckLogicalError only when no syndrome failure
            logical = logical_from_columns<true>(reinterpret_cast<const unsigned long long*>(sres[wv]), nw, n, nb,
                                                 imp_cols, imp_cw, lane);
        wave_sync();
        c[C_WITHX] += __any(anyX);
        c[C_WITHZ] += __any(anyZ);
        c[C_SYNX] += dEX;
        c[C_SYNZ] += dEZ;
        c[C_LOGICAL] += !(dEX || dEZ) && logical;
        c[C_CORRECTED] += !(dEX || dEZ) && !logical;
        c[C_CONVX] += (f & QEC_CONVERGENCE_FAIL_X) != 0;
        c[C_CONVZ] += (f & QEC_CONVERGENCE_FAIL_Z) != 0;
        if (iters != nullptr) {
            c[C_N] += (unsigned)iters[2 * b];
            c[C_N + 1] += (unsigned)iters[2 * b + 1];
        }
    }
    stat_flush(part, c, iters != nullptr ? C_N + 2 : C_N, counters);
}

// ---- launchers --------------------------------------------------------------
static int launch_check(const char* what)
{
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return fail(QEC_ERR_HIP, std::string(what) + ": " + hipGetErrorString(e));
    return QEC_OK;
}

int launch_sample_depolarizing(uint64_t seed, uint64_t start, long long B, int n, float p, uint8_t* x, uint8_t* z,
                               hipStream_t st)
{
    if (B <= 0) return QEC_OK;
    const long long tot = B * ((n + 3) / 4);
    hipLaunchKernelGGL(sample_depolarizing_kernel, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, st,
                       make_depol(seed, p), start, B, n, x, z);
    return launch_check("sample_depolarizing");
}

int launch_mc_errors_syndrome(int src, const McArgsHost& h, hipStream_t st)
{
    if (h.B <= 0) return QEC_OK;
    const Code& c = *h.code;
    McArgs a{};
    a.depol = make_depol(h.seed, h.p);
    a.start = h.start;
    a.idx = h.idx; a.type = h.type; a.W = h.W;
    a.x = h.x; a.z = h.z;
    a.sX = h.sX; a.sZ = h.sZ; a.errp = h.errp;
    a.chkVar = h.chkVar;
    a.B = h.B;
    a.n = c.n; a.nb = (c.n + 7) / 8; a.L = c.L; a.P = c.P; a.J = c.J; a.K = c.K; a.mX = c.mX; a.mZ = c.mZ;
    if (a.chkVar == nullptr) {
        if (!c.is_qc || c.J * c.L > 128 || c.K * c.L > 128) return fail(QEC_ERR_UNSUPPORTED, "mc front end: needs a QC code or a check table");
        for (size_t k = 0; k < c.EX.size(); ++k) a.EX[k] = c.EX[k];
        for (size_t k = 0; k < c.EZ.size(); ++k) a.EZ[k] = c.EZ[k];
    }
    const int npad = 8 * a.nb;
    a.S = (a.chkVar == nullptr && c.P > 0 && c.P < 64) ? 64 / c.P : 1;
    if ((size_t)a.S * (2 * npad + 4 * ((c.mX + c.mZ + 31) / 32)) > 4096) a.S = 1;
    auto magic = [](long long d) { return d > 1 ? (uint32_t)(((1ull << 32) + (uint64_t)d - 1) / (uint64_t)d) : 0u; };
    a.magicW = magic(h.W); a.magicG = magic(npad / 4); a.magicG2 = magic(npad / 2); a.magicN = magic(npad);
    a.magicM = magic(c.mX + c.mZ);
    a.magicP = magic(c.P); a.magicB = magic(2 * a.nb);
    if ((long long)a.S * std::max<long long>({(long long)h.W, npad, (long long)c.mX + c.mZ}) >= 65536)
        return fail(QEC_ERR_UNSUPPORTED, "mc front end: code too long");
    const size_t smem = (size_t)kMcWaves * a.S * (2 * npad + 4 * ((c.mX + c.mZ + 31) / 32));  // error rows + syndrome bits
    if (smem > 64 * 1024) return fail(QEC_ERR_UNSUPPORTED, "mc front end: code too long for the LDS stage");
    const long long per_block = (long long)kMcWaves * a.S;
    const dim3 grid((unsigned)((h.B + per_block - 1) / per_block)), block(64 * kMcWaves);
    auto launch = [&](auto kern) { hipLaunchKernelGGL(kern, grid, block, smem, st, a); };
    const int lt = a.chkVar == nullptr && (c.L == 10 || c.L == 6) ? c.L : 0;
#define QEC_MC_LAUNCH(S)                                                              \
    (lt == 10 ? launch(mc_errors_syndrome_kernel<S, 10>)                              \
              : lt == 6 ? launch(mc_errors_syndrome_kernel<S, 6>) : launch(mc_errors_syndrome_kernel<S, 0>))
    if (src == MC_SRC_PHILOX)
        QEC_MC_LAUNCH(MC_SRC_PHILOX);
    else if (src == MC_SRC_DRAWS)
        QEC_MC_LAUNCH(MC_SRC_DRAWS);
    else
        QEC_MC_LAUNCH(MC_SRC_BYTES);
#undef QEC_MC_LAUNCH
    return launch_check("mc_errors_syndrome");
}

int launch_statistics_packed(const Code& c, const uint64_t* imp_cols, const uint8_t* errp, const uint8_t* rec,
                             const int32_t* iters, long long B, unsigned long long* counters, hipStream_t st)
{
    if (B <= 0) return QEC_OK;
    const int nb = (c.n + 7) / 8;
    if ((2 * nb + 7) / 8 > kMaxRecWords || c.imp_col_words > 64)
        return fail(QEC_ERR_UNSUPPORTED, "packed statistics kernel: code too long");
    const long long blocks = std::min<long long>((B + kStatBlockWaves - 1) / kStatBlockWaves, kStatMaxBlocks);
    hipLaunchKernelGGL(statistics_packed_kernel, dim3((unsigned)blocks), dim3(64 * kStatBlockWaves), 0, st, errp, rec,
                       iters, B, c.n, nb, imp_cols, c.imp_col_words, counters);
    return launch_check("statistics_packed");
}

int launch_statistics(const Code& c, const uint64_t* imp_cols, const uint8_t* x, const uint8_t* z, const uint8_t* eX,
                      const uint8_t* eZ, const uint8_t* flags, long long B, unsigned long long* counters, hipStream_t st)
{
    if (B <= 0) return QEC_OK;
    if (2 * c.n > 64 * kMaxWords || c.imp_col_words > 64) return fail(QEC_ERR_UNSUPPORTED, "statistics kernel: 2n > 4096");
    const long long blocks = std::min<long long>((B + kStatBlockWaves - 1) / kStatBlockWaves, kStatMaxBlocks);
    hipLaunchKernelGGL(statistics_kernel, dim3((unsigned)blocks), dim3(64 * kStatBlockWaves), 0, st, x, z, eX, eZ, flags, B,
                       c.n, imp_cols, c.imp_col_words, counters);
    return launch_check("statistics");
}

int launch_pack_decisions(const uint8_t* eX, const uint8_t* eZ, const uint8_t* flags, long long B, int n, uint8_t* out,
                          hipStream_t st)
{
    if (B <= 0) return QEC_OK;
    const long long total = B * (2 * ((n + 7) / 8) + 1);
    hipLaunchKernelGGL(pack_decisions_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, eX, eZ, flags, B,
                       n, out);
    return launch_check("pack_decisions");
}

}  // namespace qec
