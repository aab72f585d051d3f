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
#include <cmath>
#include <cstdint>
#include <cstdlib>

#include "qec_device.h"
#include "qec_internal.h"
#include "qec_mc.h"

namespace qec {

// byte form (qec_sample_depolarizing_dev): one lane per sample writes the bytes of its hit qubits
// into rows the launcher zeroed
__global__ __launch_bounds__(256) void sample_depolarizing_kernel(GapParams gp, uint64_t start, long long B, int n,
                                                                  uint8_t* __restrict__ x, uint8_t* __restrict__ z)
{
    extern __shared__ uint32_t gap_T[];
    gap_table(gp, n, gap_T);
    __syncthreads();
    const long long s = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= B || gp.thr == 0) return;
    uint8_t* __restrict__ xr = x + s * n;
    uint8_t* __restrict__ zr = z + s * n;
    gap_walk(gp, start + (uint64_t)s, n, gap_T, [&](int v, uint32_t t) {
        if (t != 2) xr[v] = 1;
        if (t != 0) zr[v] = 1;
    });
}

// Grid-stride over samples, one wave per sample at a time; each wave keeps its counts in
// registers and the workgroup adds them to `counters` once (same-address atomics from every
// workgroup serialise at L2: 16 384 four-wave workgroups x 8 counters cost ~190 us per 65 536
// samples, profiles/r02/mc_r02f_psweep_p002_kernel_stats.csv).
constexpr int kStatBlockWaves = 16;
constexpr int kStatMaxBlocks = 256;

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
        bool anyX = false, anyZ = false, anyR = false;  // anyR: wave-uniform (ballots)
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
            anyR |= word != 0ull;
            if (lane == 0) sres[wv][w] = word;
        }
        const uint8_t f = flags[b];
        const bool dEX = f & QEC_SYNDROME_FAIL_X, dEZ = f & QEC_SYNDROME_FAIL_Z;
        bool logical = false;
        if (!(dEX || dEZ) && imp_cw > 0 && anyR) {  // CheckLogicalError only when no syndrome failure
            wave_sync();
            logical = logical_from_columns<false>(sres[wv], nw, n, 0, imp_cols, imp_cw, lane);
            wave_sync();  // sres is rewritten by the next sample
        }
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
//   source DRAWS:  the reference's W (index, type) draws of the sample (DecoderCPU.h:452-457);
//   source BYTES:  x, z rows [B][n] from HBM.
// Then, from LDS: the syndromes sX, sZ (QC: s(r, i) = XOR_l e[l P + (E[r][l] + i) mod P]; any other
// regular code: the check's variables from the sparse engine's table), and the bit-packed errors
// errp [B][2 nb] in the decision-record layout (x bits, then z bits) for the statistics kernel.
// HBM traffic per P61 sample: 549 B of syndromes + 154 B of packed errors written.
constexpr int kMcWaves = 4;

struct McArgs {
    // sources
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

// ---- fused front end for the depolarising sampler (the gap walk) ---------------------
// One lane per sample: the lane walks its sample (gap_walk) and, for every hit, sets the qubit's
// bits in the sample's packed-error words and flips the qubit's checks in its syndrome bit sets
// (both in LDS, this lane's own region of w32 = ew + wX + wZ words: errors in the decision-record
// layout, then the X checks' bits, then the Z checks').  Then the wave writes its samples'
// contiguous output blocks as coalesced dwords (write_block): syndromes as bytes (sX, sZ, the
// public layout) or as bit rows (sXp [B][wX], sZp [B][wZ] words, the Monte-Carlo pipeline's
// layout: 72 instead of 549 B per P61 sample), packed errors at a row stride of 2 nb bytes (the
// public layout) or 4 ew (word-aligned rows, a word copy).  Each lane writing its own sample's
// rows instead (4x fewer instructions, but every store scattered over 64 rows) measured slower:
// 62 vs 41 us per 65 536 P61 samples at p = 0.002.  Nothing but syndromes and packed errors
// reaches HBM, and the sampler costs words per hit, not per qubit.
constexpr int kGapWaves = 4;

struct GapArgs {
    GapParams gp;
    uint64_t start;
    long long B;
    int n, nb, mX, mZ, P, L, J, K;
    int spw;           // samples per wave
    int ew, wX, wZ, w32;  // LDS words per sample: packed errors, X bits, Z bits; total
    int estride;       // errp row stride in bytes: 2 nb or 4 ew
    uint32_t magicX, magicZ, magicE, magicWX, magicWZ, magicEW;  // ceil(2^32 / d)
    uint8_t* sX;       // byte rows (nullable when sXp is given)
    uint8_t* sZ;
    uint32_t* sXp;     // bit rows (nullable)
    uint32_t* sZp;
    uint8_t* errp;     // nullable
    const int32_t* varEdge;  // non-QC codes: n x dvX then n x dvZ edge ids; check = edge / dc
    int dc, dvX, dvZ;
    int EX[128], EZ[128];    // QC codes
};

// Bytes [0, tot) of a wave's output block dst, byte k = f(k): head bytes up to 4-byte alignment,
// then dwords, then the tail (dst is at any alignment).
template <class F>
__device__ __forceinline__ void write_block(uint8_t* __restrict__ dst, int tot, int lane, F&& f)
{
    const int head = min((int)((0u - (uint32_t)(uintptr_t)dst) & 3u), tot);
    if (lane < head) dst[lane] = (uint8_t)f(lane);
    const int body = (tot - head) >> 2;
    uint32_t* __restrict__ d32 = reinterpret_cast<uint32_t*>(dst + head);
#pragma unroll 4
    for (int t = lane; t < body; t += 64) {
        const int k = head + 4 * t;
        d32[t] = f(k) | f(k + 1) << 8 | f(k + 2) << 16 | f(k + 3) << 24;
    }
    const int tail = head + 4 * body + lane;
    if (tail < tot) dst[tail] = (uint8_t)f(tail);
}

// Words [0, tot) of a wave's word-aligned output block, word k = f(k).
template <class F>
__device__ __forceinline__ void write_words(uint32_t* __restrict__ dst, int tot, int lane, F&& f)
{
#pragma unroll 4
    for (int t = lane; t < tot; t += 64) dst[t] = f(t);
}

__global__ __launch_bounds__(64 * kGapWaves) void mc_gap_kernel(const GapArgs a)
{
    extern __shared__ uint32_t gap_smem[];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int n = a.n;
    uint32_t* __restrict__ T = gap_smem;                                            // [n + 1]
    int* __restrict__ E = reinterpret_cast<int*>(gap_smem + n + 1);                 // [(J + K) L], QC
    const int ne = a.varEdge ? 0 : (a.J + a.K) * a.L;
    uint32_t* __restrict__ reg = gap_smem + n + 1 + ne + (size_t)wv * a.spw * a.w32;  // this wave's samples
    gap_table(a.gp, n, T);
    for (int t = threadIdx.x; t < ne; t += blockDim.x) E[t] = t < a.J * a.L ? a.EX[t] : a.EZ[t - a.J * a.L];
    for (int t = lane; t < a.spw * a.w32; t += 64) reg[t] = 0u;
    __syncthreads();
    const long long b0 = ((long long)blockIdx.x * kGapWaves + wv) * a.spw;
    if (b0 >= a.B) return;  // wave-local from here on
    const int ns = (int)(a.B - b0 < a.spw ? a.B - b0 : a.spw);
    const int w32 = a.w32, ew = a.ew, wX = a.wX, wZ = a.wZ;
    if (lane < ns && a.gp.thr != 0) {
        uint32_t* __restrict__ mine = reg + lane * w32;
        uint32_t* __restrict__ synX = mine + ew;
        uint32_t* __restrict__ synZ = synX + wX;
        const int zb = 8 * a.nb, P = a.P, L = a.L;
        gap_walk(a.gp, a.start + (uint64_t)(b0 + lane), n, T, [&](int v, uint32_t t) {
            const bool ex = t != 2, ez = t != 0;
            if (ex) atomicOr(&mine[v >> 5], 1u << (v & 31));
            if (ez) atomicOr(&mine[(zb + v) >> 5], 1u << ((zb + v) & 31));
            if (a.varEdge == nullptr) {
                // QC: qubit (l, j) sits in check (r, (j - E[r][l]) mod P) of each block row r
                const int l = v / P, j = v - l * P;
                if (ex)
                    for (int r = 0; r < a.J; ++r) {
                        const int d = j - E[r * L + l];
                        const int c = r * P + (d < 0 ? d + P : d);
                        atomicXor(&synX[c >> 5], 1u << (c & 31));
                    }
                if (ez)
                    for (int r = 0; r < a.K; ++r) {
                        const int d = j - E[(a.J + r) * L + l];
                        const int c = r * P + (d < 0 ? d + P : d);
                        atomicXor(&synZ[c >> 5], 1u << (c & 31));
                    }
            } else {
                if (ex)
                    for (int k = 0; k < a.dvX; ++k) {
                        const int c = a.varEdge[(size_t)v * a.dvX + k] / a.dc;
                        atomicXor(&synX[c >> 5], 1u << (c & 31));
                    }
                if (ez)
                    for (int k = 0; k < a.dvZ; ++k) {
                        // Z edge ids are offset by mX dc: check mX + c
                        const int c = a.varEdge[(size_t)n * a.dvX + (size_t)v * a.dvZ + k] / a.dc - a.mX;
                        atomicXor(&synZ[c >> 5], 1u << (c & 31));
                    }
            }
        });
    }
    wave_sync();
    if (a.sXp != nullptr) {
        write_words(a.sXp + b0 * wX, ns * wX, lane, [&](int k) {
            const int s = qdiv(k, a.magicWX);
            return reg[s * w32 + ew + (k - s * wX)];
        });
        write_words(a.sZp + b0 * wZ, ns * wZ, lane, [&](int k) {
            const int s = qdiv(k, a.magicWZ);
            return reg[s * w32 + ew + wX + (k - s * wZ)];
        });
    } else {
        write_block(a.sX + b0 * a.mX, ns * a.mX, lane, [&](int k) -> uint32_t {
            const int s = qdiv(k, a.magicX), c = k - s * a.mX;
            return (reg[s * w32 + ew + (c >> 5)] >> (c & 31)) & 1u;
        });
        write_block(a.sZ + b0 * a.mZ, ns * a.mZ, lane, [&](int k) -> uint32_t {
            const int s = qdiv(k, a.magicZ), c = k - s * a.mZ;
            return (reg[s * w32 + ew + wX + (c >> 5)] >> (c & 31)) & 1u;
        });
    }
    if (a.errp != nullptr) {
        if (a.estride == 4 * ew) {
            write_words(reinterpret_cast<uint32_t*>(a.errp) + b0 * ew, ns * ew, lane, [&](int k) {
                const int s = qdiv(k, a.magicEW);
                return reg[s * w32 + (k - s * ew)];
            });
        } else {
            const int eb = 2 * a.nb;
            write_block(a.errp + b0 * eb, ns * eb, lane, [&](int k) -> uint32_t {
                const int s = qdiv(k, a.magicE), c = k - s * eb;
                return (reg[s * w32 + (c >> 2)] >> (8 * (c & 3))) & 0xFFu;
            });
        }
    }
}

// CodeStatistics counters of a batch from bit-packed errors errp [B][2 nb] and decision records
// rec [B][2 nb + 1] (qec_decode_batch_packed_dev): the residual [x ^ eX | z ^ eZ] is their XOR
// over the first 2 nb bytes (record layout), tested by logical_from_columns; optional iteration
// sums (iters [B][2]) into counters[8], counters[9].
// One wave per sample; counters as statistics_kernel (DecoderCPU.h:464-521).  A wave takes U
// samples at a time and issues all their byte loads (NJ per lane and sample) before using any, so
// one memory latency covers U samples; the residual is staged in LDS only for the rare sample that
// needs the I-P columns (no syndrome failure, nonzero residual).  NJ = 0: any code, one sample at
// a time.
constexpr int kMaxRecWords = 80;  // 2 nb <= 640 bytes

template <int NJ, int U>
__global__ __launch_bounds__(64 * kStatBlockWaves) void statistics_packed_kernel(
    const uint8_t* __restrict__ errp, int estride, const uint8_t* __restrict__ rec, const int32_t* __restrict__ iters,
    long long B, int n, int nb, const uint64_t* __restrict__ imp_cols, int imp_cw, unsigned long long* __restrict__ counters)
{
    __shared__ unsigned long long part[kStatBlockWaves][C_N + 2];
    __shared__ __attribute__((aligned(8))) uint8_t sres[kStatBlockWaves][8 * kMaxRecWords];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int recB = 2 * nb + 1;
    const int nw = (2 * nb + 7) / 8;
    const int nj = NJ > 0 ? NJ : (8 * nw + 63) / 64;
    unsigned long long c[C_N + 2] = {};
    const long long step = (long long)gridDim.x * kStatBlockWaves * U;
    for (long long b0 = ((long long)blockIdx.x * kStatBlockWaves + wv) * U; b0 < B; b0 += step) {
        uint32_t any[U];  // per lane and sample: bit 0 x errors, bit 1 z errors, bit 2 residual
        uint8_t f[U];
        // branch-free loads (indices clamped into the batch and the row, results masked after): loads
        // under a condition are each followed by their own wait
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const long long b = b0 + u < B ? b0 + u : B - 1;
            f[u] = rec[b * recB + 2 * nb];
            any[u] = 0;
#pragma unroll
            for (int j = 0; j < (NJ > 0 ? NJ : 1); ++j) {
                for (int jj = j; jj < (NJ > 0 ? j + 1 : nj); ++jj) {
                    const int t = lane + 64 * jj;
                    const int tc = t < 2 * nb ? t : 0;
                    const uint8_t e = errp[b * estride + tc];
                    const uint8_t r = e ^ rec[b * recB + tc];
                    const uint32_t m = (e != 0 ? (t < nb ? 1u : 2u) : 0u) | (r != 0 ? 4u : 0u);
                    any[u] |= t < 2 * nb ? m : 0u;
                }
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const long long b = b0 + u;
            if (b >= B) break;
            const bool dEX = f[u] & QEC_SYNDROME_FAIL_X, dEZ = f[u] & QEC_SYNDROME_FAIL_Z;
            bool logical = false;
            // CheckLogicalError only when no syndrome failure; a zero residual (the decoder found the
            // error itself, the common case) has (I-P) r = 0 without reading a column
            if (!(dEX || dEZ) && imp_cw > 0 && __any(any[u] & 4u)) {
                for (int t = lane; t < 8 * nw; t += 64)
                    sres[wv][t] = t < 2 * nb ? (uint8_t)(errp[b * estride + t] ^ rec[b * recB + t]) : (uint8_t)0;
                wave_sync();
                logical = logical_from_columns<true>(reinterpret_cast<const unsigned long long*>(sres[wv]), nw, n, nb,
                                                     imp_cols, imp_cw, lane);
                wave_sync();
            }
            c[C_WITHX] += __any(any[u] & 1u);
            c[C_WITHZ] += __any(any[u] & 2u);
            c[C_SYNX] += dEX;
            c[C_SYNZ] += dEZ;
            c[C_LOGICAL] += !(dEX || dEZ) && logical;
            c[C_CORRECTED] += !(dEX || dEZ) && !logical;
            c[C_CONVX] += (f[u] & QEC_CONVERGENCE_FAIL_X) != 0;
            c[C_CONVZ] += (f[u] & QEC_CONVERGENCE_FAIL_Z) != 0;
            if (iters != nullptr) {
                c[C_N] += (unsigned)iters[2 * b];
                c[C_N + 1] += (unsigned)iters[2 * b + 1];
            }
        }
    }
    stat_flush(part, c, iters != nullptr ? C_N + 2 : C_N, counters);
}


// The counters with one lane per sample reading its two rows straight from global memory (no LDS
// stage): packed errors and records at word-aligned row strides (the Monte-Carlo pipeline's
// layout: 156-byte rows for P61), EWE / EWR words per row known at compile time so every load of
// both rows is in flight at once (78 per lane for P61).  Lane-per-sample loads touch 64 rows per
// wave instruction, but each line is reused by the row's next words (L1/L2 hits); the wave adds its
// 64 samples' outcomes with ballot popcounts (scalar), so per sample the kernel issues ~2 x 39 loads
// and ~3 x 39 VALU bit operations.
constexpr int kLaneWaves = 16;  // waves per workgroup; one workgroup per CU, grid-stride

template <int EWE, int EWR>
__global__ __launch_bounds__(64 * kLaneWaves) void statistics_lane_kernel(
    const uint32_t* __restrict__ errp, const uint32_t* __restrict__ rec, const int32_t* __restrict__ iters, long long B,
    int n, int nb, const uint64_t* __restrict__ imp_cols, int imp_cw, unsigned long long* __restrict__ counters)
{
    __shared__ unsigned long long part[kLaneWaves][C_N + 2];
    __shared__ unsigned long long sres[kLaneWaves][kMaxRecWords];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int eb = 2 * nb;  // decision bytes of a row; the flags byte follows them in a record
    unsigned long long c[C_N] = {};
    unsigned long long itx = 0, itz = 0;
    const long long step = (long long)gridDim.x * blockDim.x;
    for (long long b0 = (long long)blockIdx.x * blockDim.x + wv * 64; b0 < B; b0 += step) {
        const long long b = b0 + lane;
        const bool valid = b < B;
        const long long bl = valid ? b : B - 1;  // clamped row: every load in bounds, results masked
        uint32_t ev[EWE], rv[EWR];
#pragma unroll
        for (int k = 0; k < EWE; ++k) ev[k] = errp[bl * EWE + k];
#pragma unroll
        for (int k = 0; k < EWR; ++k) rv[k] = rec[bl * EWR + k];
        if (iters != nullptr && valid) {
            const int2 it = *reinterpret_cast<const int2*>(iters + 2 * b);
            itx += (unsigned)it.x;
            itz += (unsigned)it.y;
        }
        uint32_t ax = 0, az = 0, ar = 0;
#pragma unroll
        for (int k = 0; k < (EWE < EWR ? EWE : EWR); ++k) {
            // byte masks of word k: x bytes [0, nb), z bytes [nb, 2 nb) (wave-uniform)
            const int bx = nb - 4 * k, bz = eb - 4 * k;
            const uint32_t mx = bx >= 4 ? ~0u : bx <= 0 ? 0u : (1u << (8 * bx)) - 1u;
            const uint32_t mall = bz >= 4 ? ~0u : bz <= 0 ? 0u : (1u << (8 * bz)) - 1u;
            ax |= ev[k] & mx;
            az |= ev[k] & mall & ~mx;
            ar |= (ev[k] ^ rv[k]) & mall;
        }
        uint32_t f = 0;
#pragma unroll
        for (int k = 0; k < EWR; ++k)
            if (k == eb / 4) f = (rv[k] >> (8 * (eb % 4))) & 0xFFu;
        f = valid ? f : 0u;
        const bool dEX = (f & QEC_SYNDROME_FAIL_X) != 0, dEZ = (f & QEC_SYNDROME_FAIL_Z) != 0;
        unsigned long long need = __ballot(valid && !(dEX || dEZ) && ar != 0u);
        unsigned long long logical = 0;
        if (imp_cw > 0) {
            const int nw = (eb + 7) / 8;  // 64-bit residual words (record layout)
            while (need) {
                const int s = __builtin_ctzll(need);
                need &= need - 1;
                const uint8_t* es = reinterpret_cast<const uint8_t*>(errp + (b0 + s) * EWE);
                const uint8_t* rs = reinterpret_cast<const uint8_t*>(rec + (b0 + s) * EWR);
                if (lane < nw) {
                    uint64_t w = 0;
                    for (int j = 0; j < 8; ++j) {
                        const int t = 8 * lane + j;
                        w |= (t < eb ? (uint64_t)(es[t] ^ rs[t]) : 0ull) << (8 * j);
                    }
                    sres[wv][lane] = w;
                }
                wave_sync();
                if (logical_from_columns<true>(sres[wv], nw, n, nb, imp_cols, imp_cw, lane)) logical |= 1ull << s;
                wave_sync();
            }
        }
        const unsigned long long vm = __ballot(valid), sx = __ballot(dEX), sz = __ballot(dEZ);
        const unsigned long long ok = vm & ~(sx | sz);
        // lanes past the batch end read the clamped row B - 1: their error words are masked here
        // (their flags are already 0)
        c[C_WITHX] += __popcll(vm & __ballot(ax != 0u));
        c[C_WITHZ] += __popcll(vm & __ballot(az != 0u));
        c[C_SYNX] += __popcll(sx);
        c[C_SYNZ] += __popcll(sz);
        c[C_LOGICAL] += __popcll(ok & logical);
        c[C_CORRECTED] += __popcll(ok & ~logical);
        c[C_CONVX] += __popcll(__ballot((f & QEC_CONVERGENCE_FAIL_X) != 0));
        c[C_CONVZ] += __popcll(__ballot((f & QEC_CONVERGENCE_FAIL_Z) != 0));
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
        itx += __shfl_xor(itx, o);
        itz += __shfl_xor(itz, o);
    }
    unsigned long long cc[C_N + 2];
#pragma unroll
    for (int k = 0; k < C_N; ++k) cc[k] = c[k];
    cc[C_N] = itx;
    cc[C_N + 1] = itz;
    if (lane < C_N + 2) {
        unsigned long long v = 0;
#pragma unroll
        for (int k = 0; k < C_N + 2; ++k) v = lane == k ? cc[k] : v;
        part[wv][lane] = v;
    }
    __syncthreads();
    const int nc = iters != nullptr ? C_N + 2 : C_N;
    if (threadIdx.x < nc) {
        unsigned long long v = 0;
        for (int w = 0; w < kLaneWaves; ++w) v += part[w][threadIdx.x];
        if (v) atomicAdd(&counters[threadIdx.x], v);
    }
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
    if (hipMemsetAsync(x, 0, (size_t)B * n, st) != hipSuccess || hipMemsetAsync(z, 0, (size_t)B * n, st) != hipSuccess)
        return fail(QEC_ERR_HIP, "sample_depolarizing: memset failed");
    hipLaunchKernelGGL(sample_depolarizing_kernel, dim3((unsigned)((B + 255) / 256)), dim3(256),
                       (size_t)(n + 1) * sizeof(uint32_t), st, make_gap(seed, p), start, B, n, x, z);
    return launch_check("sample_depolarizing");
}

static uint32_t magic_of(long long d) { return d > 1 ? (uint32_t)(((1ull << 32) + (uint64_t)d - 1) / (uint64_t)d) : 0u; }

// samples per wave of mc_gap_kernel: as many as keep ~8 waves per SIMD busy (8 192 waves), between
// 16 and 64 -- a wave's walk lasts as long as its busiest lane, so more samples per wave cost less
// per sample once there are enough waves (P61, 2^20 samples: 206 / 126 / 124 us at 16 / 32 / 64 per
// wave at p = 0.002, 1109 / 542 us at 16 / 64 at p = 0.05; 65 536 samples: 16 best, 20 vs 22 us at
// 64; profiles/r02/gap_spw_r02s3zn.txt).
static int gap_spw(long long B)
{
    int spw = 16;
    while (spw < 64 && B / (2 * spw) >= 8192) spw *= 2;
    return spw;
}

static int launch_mc_gap(const McArgsHost& h, hipStream_t st)
{
    const Code& c = *h.code;
    GapArgs a{};
    a.gp = make_gap(h.seed, h.p);
    a.start = h.start;
    a.B = h.B;
    a.n = c.n; a.nb = (c.n + 7) / 8; a.mX = c.mX; a.mZ = c.mZ; a.P = c.P; a.L = c.L; a.J = c.J; a.K = c.K;
    a.sX = h.sX; a.sZ = h.sZ; a.sXp = h.sXp; a.sZp = h.sZp; a.errp = h.errp;
    a.varEdge = h.varEdge;
    a.dc = c.L; a.dvX = c.J; a.dvZ = c.K;
    if (a.varEdge == nullptr) {
        if (!c.is_qc || c.J * c.L > 128 || c.K * c.L > 128)
            return fail(QEC_ERR_UNSUPPORTED, "mc front end: needs a QC code or a check table");
        for (size_t k = 0; k < c.EX.size(); ++k) a.EX[k] = c.EX[k];
        for (size_t k = 0; k < c.EZ.size(); ++k) a.EZ[k] = c.EZ[k];
    }
    a.ew = (2 * a.nb + 3) / 4;
    a.wX = (c.mX + 31) / 32;
    a.wZ = (c.mZ + 31) / 32;
    a.w32 = a.ew + a.wX + a.wZ;
    a.estride = h.errp_words ? 4 * a.ew : 2 * a.nb;
    // sample state per wave: what the 64 KiB LDS stage holds beside the gap table T (n + 1 words) and
    // the exponent table E, split over the workgroup's waves (at most gap_spw's choice)
    const int ne = a.varEdge ? 0 : (c.J + c.K) * c.L;
    const long long free_words = 16384LL - ((long long)c.n + 1 + ne);
    const long long spw_fit = free_words > 0 ? free_words / ((long long)kGapWaves * a.w32) : 0;
    if (spw_fit < 1) return fail(QEC_ERR_UNSUPPORTED, "mc front end: code too long for the LDS stage");
    a.spw = (int)std::min<long long>(gap_spw(h.B), spw_fit);
    if ((long long)a.spw * std::max<long long>({(long long)c.mX, (long long)c.mZ, 2LL * a.nb}) >= 65536)
        return fail(QEC_ERR_UNSUPPORTED, "mc front end: code too long");
    a.magicX = magic_of(c.mX); a.magicZ = magic_of(c.mZ); a.magicE = magic_of(2 * a.nb);
    a.magicWX = magic_of(a.wX); a.magicWZ = magic_of(a.wZ); a.magicEW = magic_of(a.ew);
    const size_t smem = 4 * ((size_t)c.n + 1 + ne + (size_t)kGapWaves * a.spw * a.w32);
    if (smem > 64 * 1024) return fail(QEC_ERR_UNSUPPORTED, "mc front end: code too long for the LDS stage");
    const long long per_block = (long long)kGapWaves * a.spw;
    hipLaunchKernelGGL(mc_gap_kernel, dim3((unsigned)((h.B + per_block - 1) / per_block)), dim3(64 * kGapWaves), smem,
                       st, a);
    return launch_check("mc_gap");
}

int launch_mc_errors_syndrome(int src, const McArgsHost& h, hipStream_t st)
{
    if (h.B <= 0) return QEC_OK;
    if (src == MC_SRC_PHILOX) return launch_mc_gap(h, st);
    const Code& c = *h.code;
    McArgs a{};
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
    if (src == MC_SRC_DRAWS)
        QEC_MC_LAUNCH(MC_SRC_DRAWS);
    else
        QEC_MC_LAUNCH(MC_SRC_BYTES);
#undef QEC_MC_LAUNCH
    return launch_check("mc_errors_syndrome");
}

// The row shapes (packed-error stride, record stride) statistics_lane_kernel is instantiated for: the
// shipped codes' word-aligned rows (P61 156 / 156, P7 12 / 16).
bool statistics_lane_shape(int estride, int rec_stride)
{
    return (estride == 156 && rec_stride == 156) || (estride == 12 && rec_stride == 16);
}

int launch_statistics_packed(const Code& c, const uint64_t* imp_cols, const uint8_t* errp, int estride, const uint8_t* rec,
                             const int32_t* iters, long long B, unsigned long long* counters, hipStream_t st,
                             int rec_stride)
{
    if (B <= 0) return QEC_OK;
    const int nb = (c.n + 7) / 8;
    const int recB = rec_stride > 0 ? rec_stride : 2 * nb + 1;
    // word-aligned rows of the shipped codes' sizes: one lane per sample, straight from global memory
    const bool aligned = estride % 4 == 0 && recB % 4 == 0 && (reinterpret_cast<uintptr_t>(errp) & 3) == 0 &&
                         (reinterpret_cast<uintptr_t>(rec) & 3) == 0 && (c.imp_col_words <= 64) &&
                         (2 * nb + 7) / 8 <= kMaxRecWords;
    if (aligned) {
        void (*k)(const uint32_t*, const uint32_t*, const int32_t*, long long, int, int, const uint64_t*, int,
                  unsigned long long*) = nullptr;
        if (estride == 156 && recB == 156) k = statistics_lane_kernel<39, 39>;  // P61 (statistics_lane_shape)
        if (estride == 12 && recB == 16) k = statistics_lane_kernel<3, 4>;      // P7
        if (k) {
            const long long blocks = std::min<long long>((B + 64 * kLaneWaves - 1) / (64 * kLaneWaves), 256);
            hipLaunchKernelGGL(k, dim3((unsigned)blocks), dim3(64 * kLaneWaves), 0, st,
                               reinterpret_cast<const uint32_t*>(errp), reinterpret_cast<const uint32_t*>(rec), iters, B,
                               c.n, nb, imp_cols, c.imp_col_words, counters);
            return launch_check("statistics_lane");
        }
    }
    if (rec_stride > 0 && rec_stride != 2 * nb + 1)
        return fail(QEC_ERR_UNSUPPORTED, "packed statistics: padded record rows need the lane kernel");
    if ((2 * nb + 7) / 8 > kMaxRecWords || c.imp_col_words > 64)
        return fail(QEC_ERR_UNSUPPORTED, "packed statistics kernel: code too long");
    // (an LDS-staged row kernel measured slower than the byte kernel below at P61: 195-304 vs 231 us per
    // 2^20, profiles/r03/)
    const int nj = (8 * ((2 * nb + 7) / 8) + 63) / 64;
    constexpr int U = 4;
    constexpr int maxb = kStatMaxBlocks;
    const long long blocks = std::min<long long>((B + kStatBlockWaves * U - 1) / (kStatBlockWaves * U), maxb);
    auto kern = nj == 1 ? statistics_packed_kernel<1, U> : nj == 3 ? statistics_packed_kernel<3, U> : statistics_packed_kernel<0, 1>;
    hipLaunchKernelGGL(kern, dim3((unsigned)blocks), dim3(64 * kStatBlockWaves), 0, st, errp, estride, rec, iters, B,
                       c.n, nb, imp_cols, c.imp_col_words, counters);
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
