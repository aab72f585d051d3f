// Iteration-0 triage for the syndrome stop rule (hard part 3: active-syndrome
// compaction), on the Monte-Carlo pipeline's bit-row syndromes.
//
// Under QEC_STOP_SYNDROME a sector stops after the first iteration whose hard decision satisfies its
// syndrome.  Iteration 0 starts from q = p' on every edge (DecoderCPU.h:265-267), so after it a
// variable's R outgoing messages, hence its hard decision (DecoderCPU.h:354-373) and whether they all
// lie outside (0.01, 0.99) (:231-246), depend only on the R-bit pattern of its checks' syndrome bits
// (bp_decode.hip, iteration0 / pattern_masks): two 2^R-bit masks, hdpat and cvpat, computed on the
// host from the iteration-0 table with the same float compares.  At low p nearly every sector stops
// there (P61 at p = 0.002: 99 %), yet the decode kernel spends a whole wave (one syndrome) on it.
//
// This kernel decides iteration 0 for 64 syndromes per wave, one lane per syndrome, bit-sliced over
// the P variables of a circulant block: with s_r the P syndrome bits of block row r (bit i = check
// (r, i)), the pattern bit r of variable (l, j) is bit j of rotl(s_r, E[r][l]) (check (r, (j - E) mod P)),
// the block's decisions are hdpat evaluated on those R words (a multiplexer tree, v_bfi), and the
// decision's syndrome on check (r, i) is bit i of XOR_l rotr(hd_l, E[r][l]).  A sector whose syndrome
// matches stops: its record bytes, iteration count (1) and flags are final -- exactly the outputs the
// decode kernel produces for it (tests/test_gpu_triage.py checks that bit for bit).  The others are
// appended to per-sector lists that the decode kernel's list mode then decodes from scratch; the two
// sectors of a syndrome meet in its merge word as in the sector-split launches (done bit + flags).
//
// The fused Monte-Carlo form (mc_fused_kernel, qec_monte_carlo at low p): sampler -> syndrome bits in
// LDS -> this triage -> decision against the sample's hits -> counters, in one kernel; only the
// samples that are not finished there (about 1 % of P61 samples at p = 0.002) reach HBM, for the
// list-mode decode and the survivor statistics (mc_survivor_kernel, which walks the sample again).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdlib>

#include "qec_device.h"
#include "qec_internal.h"
#include "qec_mc.h"

namespace qec {

constexpr int kTriageWaves = 4;

struct TriageMasks {
    uint32_t hdpatX, cvpatX, hdpatZ, cvpatZ;  // bit idx: pattern idx decides 1 / stays outside (0.01, 0.99)
    // the same masks by count when they depend only on the number of unsatisfied checks (symmetric):
    // bit c = the value for patterns with c ones; sym* = 0 when a mask is not symmetric (pattern trees)
    uint32_t hdcntX, cvcntX, hdcntZ, cvcntZ;
    int symX, symZ;
};

struct TriageArgs {
    const uint32_t* sX;  // [B][wX] bit rows (bit c = check c)
    const uint32_t* sZ;  // [B][wZ]
    long long B;
    int wX, wZ, nb, recB;  // recB: record row stride (>= 2 nb + 1)
    TriageMasks m;
    uint8_t* rec;        // [B][recB] decision records
    int32_t* iters;      // [B][2] or null
    uint32_t* merge;     // [B]: done bit (0x100 X, 0x200 Z) + that sector's flags
    int32_t* listX;      // [B] syndromes whose X sector goes on
    int32_t* listZ;
    uint32_t* counts;    // [2] list lengths (zeroed before the launch)
};

// rotations of a P-bit block by compile-time amounts (the shipped codes' generator tables)
template <int P>
__device__ __forceinline__ uint64_t rotl(uint64_t x, int k)
{
    constexpr uint64_t mask = P >= 64 ? ~0ull : (1ull << P) - 1ull;
    return k == 0 ? x : ((x << k) | (x >> (P - k))) & mask;
}
template <int P>
__device__ __forceinline__ uint64_t rotr(uint64_t x, int k)
{
    constexpr uint64_t mask = P >= 64 ? ~0ull : (1ull << P) - 1ull;
    return k == 0 ? x : ((x >> k) | (x << (P - k))) & mask;
}

// f(idx_j) bit-sliced over the P variables: bit j of the result = bit idx_j of pat, idx_j = the bits j
// of v[0..R) (v[r] -> bit r).  A multiplexer tree over v[0] .. v[R-1] (one v_bfi per node and half).
template <int R>
__device__ __forceinline__ uint64_t pattern_eval(uint32_t pat, const uint64_t (&v)[R])
{
    uint64_t t[1 << (R - 1)];
#pragma unroll
    for (int m = 0; m < (1 << (R - 1)); ++m) {
        // leaves 0 / all-ones from the uniform pattern bits (one 32-bit mask serves both halves)
        const uint32_t c0 = 0u - ((pat >> (2 * m)) & 1u), c1 = 0u - ((pat >> (2 * m + 1)) & 1u);
        const uint64_t C0 = ((uint64_t)c0 << 32) | c0, C1 = ((uint64_t)c1 << 32) | c1;
        t[m] = (v[0] & C1) | (~v[0] & C0);
    }
#pragma unroll
    for (int j = 1; j < R; ++j)
#pragma unroll
        for (int m = 0; m < (1 << (R - 1 - j)); ++m) t[m] = (v[j] & t[2 * m + 1]) | (~v[j] & t[2 * m]);
    return t[0];
}

// Bit-sliced count of ones among v[0..R) (R <= 5): b[k] = bit k of the count, per bit position (full
// and half adders on whole words).
template <int R>
__device__ __forceinline__ void count_ones(const uint64_t (&v)[R], uint64_t (&b)[3])
{
    static_assert(R >= 1 && R <= 5, "up to five rows");
    auto fa = [](uint64_t x, uint64_t y, uint64_t z, uint64_t& s, uint64_t& c) {
        s = x ^ y ^ z;
        c = (x & y) | (z & (x ^ y));
    };
    if constexpr (R == 1) {
        b[0] = v[0]; b[1] = 0; b[2] = 0;
    } else if constexpr (R == 2) {
        b[0] = v[0] ^ v[1]; b[1] = v[0] & v[1]; b[2] = 0;
    } else if constexpr (R == 3) {
        fa(v[0], v[1], v[2], b[0], b[1]);
        b[2] = 0;
    } else if constexpr (R == 4) {
        uint64_t s, c;
        fa(v[0], v[1], v[2], s, c);
        b[0] = s ^ v[3];
        const uint64_t c2 = s & v[3];
        b[1] = c ^ c2;
        b[2] = c & c2;
    } else {
        uint64_t s, c, c2;
        fa(v[0], v[1], v[2], s, c);
        fa(s, v[3], v[4], b[0], c2);
        b[1] = c ^ c2;
        b[2] = c & c2;
    }
}

// One sector of this lane's syndrome (its bit row): the decisions hd[l] (bit j = variable (l, j)),
// whether iteration 0 satisfies the syndrome, and whether some message lies inside (0.01, 0.99).
// SYM: the masks are symmetric (hdcnt / cvcnt by count of ones): an adder tree and a 3-level
// multiplexer instead of the 2^R-leaf trees (P61 Z: 16 instead of 124 bit operations per block).
// words of a sector's syndrome bit row (R P bits)
template <int R, int P>
constexpr int row_words() { return (R * P + 31) / 32; }

// The bit row of syndrome b, kW words at a compile-time stride from a 16-byte aligned base
// (launch_triage checks): 16- or 8-byte loads where the row's alignment allows (P61: X 2 x 16 B, Z
// 5 x 8 B instead of 18 dword loads per lane); w[kW], w[kW + 1] = 0.
template <int kW>
__device__ __forceinline__ void load_row(const uint32_t* __restrict__ rows, long long b, uint32_t (&w)[kW + 2])
{
    const uint32_t* __restrict__ row = rows + b * kW;
    if constexpr (kW % 4 == 0) {
#pragma unroll
        for (int k = 0; k < kW; k += 4) {
            const uint4 v = *reinterpret_cast<const uint4*>(row + k);
            w[k] = v.x; w[k + 1] = v.y; w[k + 2] = v.z; w[k + 3] = v.w;
        }
    } else if constexpr (kW % 2 == 0) {
#pragma unroll
        for (int k = 0; k < kW; k += 2) {
            const uint2 v = *reinterpret_cast<const uint2*>(row + k);
            w[k] = v.x; w[k + 1] = v.y;
        }
    } else {
#pragma unroll
        for (int k = 0; k < kW; ++k) w[k] = row[k];
    }
    w[kW] = 0u;
    w[kW + 1] = 0u;
}

template <int R, int L, int P, class EXP, int SEC, bool SYM>
__device__ __forceinline__ bool triage_sector(const uint32_t (&w)[row_words<R, P>() + 2], uint32_t hdpat,
                                              uint32_t cvpat, uint32_t hdcnt, uint32_t cvcnt, uint64_t (&hd)[L],
                                              bool& cvbad)
{
    static_assert(R <= 5 && P <= 64, "patterns in 32 bits, blocks in 64");
    constexpr EXP tab = EXP::make();
    auto E = [&](int r, int l) constexpr { return SEC ? tab.EZ[r][l] : tab.EX[r][l]; };
    constexpr uint64_t mask = P >= 64 ? ~0ull : (1ull << P) - 1ull;
    constexpr uint32_t full = R >= 5 ? 0xFFFFFFFFu : (uint32_t)((1ull << (1 << R)) - 1ull);
    uint64_t s[R];  // block row r: bit i = check (r, i)
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int o = r * P, k = o >> 5, sh = o & 31;
        const uint64_t lo = (uint64_t)w[k] | ((uint64_t)w[k + 1] << 32);
        const uint64_t v = sh == 0 ? lo : (lo >> sh) | ((uint64_t)w[k + 2] << (64 - sh));
        s[r] = v & mask;
    }
    const bool hd_const = hdpat == 0u || hdpat == full;  // uniform: no tree needed
    uint64_t bad = 0;
#pragma unroll
    for (int l = 0; l < L; ++l) {
        uint64_t v[R];  // bit j: syndrome bit of check (r, (j - E[r][l]) mod P) of variable (l, j)
#pragma unroll
        for (int r = 0; r < R; ++r) v[r] = rotl<P>(s[r], E(r, l));
        if constexpr (SYM) {
            uint64_t b[3];
            count_ones<R>(v, b);
            hd[l] = hd_const ? (hdpat ? mask : 0ull) : (pattern_eval<3>(hdcnt, b) & mask);
            if (cvpat != full) bad |= pattern_eval<3>(~cvcnt & 0xFFu, b);
        } else {
            hd[l] = hd_const ? (hdpat ? mask : 0ull) : (pattern_eval<R>(hdpat, v) & mask);
            if (cvpat != full) bad |= pattern_eval<R>(~cvpat, v);
        }
    }
    cvbad = (bad & mask) != 0ull;
    bool ok = true;
#pragma unroll
    for (int r = 0; r < R; ++r) {  // syndrome of the decision: check (r, i) XORs variables (l, (E + i) mod P)
        uint64_t par = 0;
#pragma unroll
        for (int l = 0; l < L; ++l) par ^= rotr<P>(hd[l], E(r, l));
        ok &= par == s[r];
    }
    return ok;
}

// this lane's sector decisions as nb record bytes (bit l P + j of the sector = variable (l, j), bit
// k of byte t = qubit 8 t + k), into its row of the wave's LDS stage
template <int L, int P>
__device__ __forceinline__ void stage_sector(uint8_t* __restrict__ row, int nb, const uint64_t (&hd)[L])
{
    uint64_t acc = 0;  // pending bits (have < 8 of them between blocks)
    int have = 0, out = 0;
#pragma unroll
    for (int l = 0; l < L; ++l) {
        uint64_t lo = acc | (hd[l] << have);
        uint64_t hi = have ? hd[l] >> (64 - have) : 0ull;  // the block's bits past 64 (P + have > 64)
        int tot = have + P;
        while (tot >= 8) {
            row[out++] = (uint8_t)lo;
            lo = (lo >> 8) | (hi << 56);
            hi >>= 8;
            tot -= 8;
        }
        acc = lo;
        have = tot;
    }
    if (have > 0) row[out++] = (uint8_t)acc;
    for (; out < nb; ++out) row[out] = 0;
}

// The whole record (eX bits, eZ bits, flags byte, zero padding) as ndw dwords into this lane's
// dword-aligned row of the stage: dword d takes bits [32 d, 32 d + 32) of the record's bit stream, where
// block l of sector s starts at bit 8 nb s + P l (offsets fold at compile time; every hd block is
// already masked to its P bits).  39 ds_write_b32 per P61 record instead of 155 byte writes.
template <int L, int P>
__device__ __forceinline__ void stage_record_dw(uint32_t* __restrict__ row, int ndw, const uint64_t (&hdX)[L],
                                                const uint64_t (&hdZ)[L], uint32_t flags)
{
    constexpr int nb = (L * P + 7) / 8;
    constexpr int nrec = (2 * nb + 1 + 3) / 4;  // dwords holding bits, the flags byte included
#pragma unroll
    for (int d = 0; d < nrec; ++d) {
        uint32_t w = 0;
#pragma unroll
        for (int s = 0; s < 2; ++s) {
#pragma unroll
            for (int l = 0; l < L; ++l) {
                const int a0 = 32 * d - (8 * nb * s + P * l);  // block bit at this dword's bit 0
                if (a0 >= P || a0 <= -32) continue;
                const uint64_t blk = s ? hdZ[l] : hdX[l];
                w |= a0 >= 0 ? (uint32_t)(blk >> a0) : (uint32_t)(blk << (-a0));
            }
        }
        constexpr int fb = 16 * nb;  // the flags byte's first bit
        if (fb >= 32 * d && fb < 32 * d + 32) w |= flags << (fb - 32 * d);
        row[d] = w;
    }
    for (int d = nrec; d < ndw; ++d) row[d] = 0u;  // row padding
}

// Both sectors of one syndrome: symmetric masks (the usual case) take the adder form; R <= 3 gains
// nothing from it.
template <int J, int K, int L, int P, class EXP>
__device__ __forceinline__ void triage_both(const TriageMasks& m, const uint32_t (&wX)[row_words<J, P>() + 2],
                                            const uint32_t (&wZ)[row_words<K, P>() + 2], uint64_t (&hdX)[L],
                                            uint64_t (&hdZ)[L], bool& cvbX, bool& cvbZ, bool& okX, bool& okZ)
{
    if (J >= 4 && m.symX)
        okX = triage_sector<J, L, P, EXP, 0, J >= 4>(wX, m.hdpatX, m.cvpatX, m.hdcntX, m.cvcntX, hdX, cvbX);
    else
        okX = triage_sector<J, L, P, EXP, 0, false>(wX, m.hdpatX, m.cvpatX, 0u, 0u, hdX, cvbX);
    if (K >= 4 && m.symZ)
        okZ = triage_sector<K, L, P, EXP, 1, K >= 4>(wZ, m.hdpatZ, m.cvpatZ, m.hdcntZ, m.cvcntZ, hdZ, cvbZ);
    else
        okZ = triage_sector<K, L, P, EXP, 1, false>(wZ, m.hdpatZ, m.cvpatZ, 0u, 0u, hdZ, cvbZ);
}

template <int J, int K, int L, int P, int S, int T>
__global__ __launch_bounds__(64 * kTriageWaves) void triage_kernel(const TriageArgs a)
{
    extern __shared__ __attribute__((aligned(16))) uint8_t tri_smem[];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int recB = a.recB, nb = a.nb;
    uint8_t* __restrict__ stage = tri_smem + (size_t)wv * (64 * recB + 16);
    const long long b0 = ((long long)blockIdx.x * kTriageWaves + wv) * 64;
    // every wave reaches the workgroup barriers below (a wave past the batch end does no work)
    const bool wlive = b0 < a.B;
    const int ns = !wlive ? 0 : (int)(a.B - b0 < 64 ? a.B - b0 : 64);
    const long long b = b0 + lane;
    const bool valid = lane < ns;
    const long long bl = valid ? b : wlive ? b0 : 0;  // clamped row (its results are discarded)
    uint64_t hdX[L], hdZ[L];
    bool cvbX = false, cvbZ = false;
    using EXP = QcExponents<J, K, L, P, S, T>;
    uint32_t wX[row_words<J, P>() + 2], wZ[row_words<K, P>() + 2];
    load_row<row_words<J, P>()>(a.sX, bl, wX);
    load_row<row_words<K, P>()>(a.sZ, bl, wZ);
    bool okX, okZ;
    triage_both<J, K, L, P, EXP>(a.m, wX, wZ, hdX, hdZ, cvbX, cvbZ, okX, okZ);
    const bool doneX = valid && okX, doneZ = valid && okZ;
    const uint32_t fX = cvbX ? QEC_CONVERGENCE_FAIL_X : 0u, fZ = cvbZ ? QEC_CONVERGENCE_FAIL_Z : 0u;
    // record rows: both sectors' decisions (a sector that goes on is overwritten by the list decode),
    // the flags byte final when both stopped (else written by the list decode's merge)
    uint8_t* __restrict__ my = stage + lane * recB;
    if (valid) {
        if ((recB & 3) == 0) {  // word-aligned rows (the Monte-Carlo pipeline's): whole dwords
            stage_record_dw<L, P>(reinterpret_cast<uint32_t*>(my), recB >> 2, hdX, hdZ, fX | fZ);
        } else {
            stage_sector<L, P>(my, nb, hdX);
            stage_sector<L, P>(my + nb, nb, hdZ);
            my[2 * nb] = (uint8_t)(fX | fZ);
            for (int k = 2 * nb + 1; k < recB; ++k) my[k] = 0;
        }
    }
    wave_sync();
    // the wave's contiguous block of records: 16-byte stores over its aligned body, bytes at the ends
    {
        uint8_t* __restrict__ g = a.rec + b0 * recB;
        const int tot = ns * recB;
        const uintptr_t g0 = reinterpret_cast<uintptr_t>(g);
        const int head = (int)min((uintptr_t)tot, (16 - (g0 & 15)) & 15);
        const int body = (tot - head) >> 4;
        const int tail0 = head + 16 * body;
        if (lane < head) g[lane] = stage[lane];
        for (int t = lane; t < body; t += 64) {
            const int o = head + 16 * t;
            uint32_t w4[4];
#pragma unroll
            for (int q = 0; q < 4; ++q)
                w4[q] = (uint32_t)stage[o + 4 * q] | (uint32_t)stage[o + 4 * q + 1] << 8 |
                        (uint32_t)stage[o + 4 * q + 2] << 16 | (uint32_t)stage[o + 4 * q + 3] << 24;
            *reinterpret_cast<uint4*>(g + o) = make_uint4(w4[0], w4[1], w4[2], w4[3]);
        }
        if (tail0 + lane < tot) g[tail0 + lane] = stage[tail0 + lane];
    }
    if (valid) {
        if (a.iters != nullptr) *reinterpret_cast<int2*>(a.iters + 2 * b) = make_int2(1, 1);  // list sectors rewrite theirs
        a.merge[b] = (doneX ? 0x100u | fX : 0u) | (doneZ ? 0x200u | fZ : 0u);
    }
    // sectors that go on: appended to the lists with one atomic per workgroup and sector (same-address
    // atomics serialise at L2: one per wave put ~15 k of them on two words per 2^20 batch)
    __shared__ uint32_t wcnt[kTriageWaves][2], wgbase[2];
    const unsigned long long lt = (1ull << lane) - 1ull;
    const unsigned long long gx = __ballot(valid && !okX), gz = __ballot(valid && !okZ);
    if (lane == 0) {
        wcnt[wv][0] = (uint32_t)__popcll(gx);
        wcnt[wv][1] = (uint32_t)__popcll(gz);
    }
    __syncthreads();
    if (threadIdx.x < 2) {
        uint32_t tot = 0;
        for (int w = 0; w < kTriageWaves; ++w) tot += wcnt[w][threadIdx.x];
        wgbase[threadIdx.x] = tot ? atomicAdd(&a.counts[threadIdx.x], tot) : 0u;
    }
    __syncthreads();
    uint32_t baseX = wgbase[0], baseZ = wgbase[1];
    for (int w = 0; w < wv; ++w) {
        baseX += wcnt[w][0];
        baseZ += wcnt[w][1];
    }
    if ((gx >> lane) & 1ull) a.listX[baseX + __popcll(gx & lt)] = (int32_t)b;
    if ((gz >> lane) & 1ull) a.listZ[baseZ + __popcll(gz & lt)] = (int32_t)b;
}

// ---- fused low-p Monte-Carlo pipeline ---------------------------------------------------------
// One lane per sample, 64 samples per wave (DecoderCPU.h:438-521 for each, batched):
//   1. the gap walk (qec_mc.h) of sample start + b: every hit flips its qubit's checks in the lane's
//      syndrome bit rows in LDS (as mc_gap_kernel) and is kept in the lane's hit list (qubit << 2 | type,
//      up to kHitCap of them);
//   2. the iteration-0 triage of both sectors on those rows (triage_both);
//   3. a sample whose two sectors stop there, whose hits fit the list and whose decision equals its
//      error (every hit qubit decided in its sector(s) and nothing else: counts of set bits) is
//      finished here, corrected with iterations 1 + 1 (DecoderCPU.h:464-521); the triage runs sector by
//      sector, so one sector's decisions are live at a time (registers: occupancy);
//   4. any other sample is a survivor: it gets what the triage kernel writes for a syndrome
//      (syndrome rows, record with the iteration-0 decisions, iteration counts, merge word; listX /
//      listZ for the sectors that go on) and is appended to listS; the list-mode decode runs, and
//      mc_survivor_kernel counts the survivors (I-P check included: a stopped survivor whose decision
//      differs from its error is decided there).
// withX / withZ (errors present) are counted here for every sample.
// 4-wave workgroups: six fit a CU's LDS (23 words per lane for P61: rows and up to six hits) and the
// registers are held to six waves per SIMD (measured against 8, 12 and 16-wave workgroups and ten or
// sixteen hits: +2-9 %; a sample with more hits is a survivor); the list appends take one atomic
// per workgroup and list, and the counters are added into 64 rows of partial sums (workgroup mod 64:
// same-address atomics serialise at L2) that mc_survivor_kernel's workgroup 0 adds up
#ifndef QEC_FUSED_WAVES
#define QEC_FUSED_WAVES 4
#endif
#ifndef QEC_FUSED_HITS
#define QEC_FUSED_HITS 6
#endif
#ifndef QEC_FUSED_MINW
#define QEC_FUSED_MINW 6
#endif
constexpr int kFusedWaves = QEC_FUSED_WAVES;
constexpr int kFusedMinWaves = QEC_FUSED_MINW;  // waves per SIMD the registers must allow
constexpr int kHitCap = QEC_FUSED_HITS;  // hits a lane keeps (P61: 1.2 on average at p = 0.002, 3.1 at 0.005)
constexpr uint32_t kXClean = 0x400u;  // merge word: the X sector stopped with the sample's X errors
constexpr int kCountStride = 32;  // words between the three list lengths (separate L2 lines)

struct FusedArgs {
    GapParams gp;
    uint64_t start;  // sample index of batch row 0
    long long B;
    int recB;        // record row stride (a multiple of 4)
    TriageMasks m;
    uint32_t* sX;    // [B][wX] bit rows (survivors only)
    uint32_t* sZ;
    uint8_t* rec;    // [B][recB] (survivors only)
    int32_t* iters;  // [B][2] (survivors only)
    uint32_t* merge; // [B] (survivors only)
    int32_t* listX;
    int32_t* listZ;
    int32_t* listS;
    uint32_t* counts;  // listX, listZ, listS lengths at [0], [kCountStride], [2 kCountStride] (zeroed first)
    const uint64_t* imp_cols;
    int imp_cw;
    unsigned long long* counters;  // [C_N + 2] (iteration sums at C_N, C_N + 1)
    unsigned long long* partials;  // [kPartRows][C_N + 2]: mc_fused_kernel's partial-sum rows (zeroed first)
    int nparts;                    // its grid size
};

// The fused kernel's workgroups add their counters into kPartRows rows of partial sums (row = workgroup
// mod kPartRows: ~64 same-address atomics per counter instead of 4 096, zeroed with the list lengths before
// the kernel); mc_survivor_kernel's workgroup 0 adds the rows into the counters.
constexpr int kPartRows = 64;
static_assert(C_N + 2 == QEC_MC_NCOUNTERS_ALL, "a partial-sum row is the counter vector");

// the workgroup's counters (each wave's ballot popcounts) added into its row of partials
template <int NWAVES>
__device__ __forceinline__ void store_partials(const unsigned long long (&c)[C_N + 2], unsigned long long (*part)[C_N + 2],
                                               unsigned long long* __restrict__ partials)
{
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    if (lane < C_N + 2) {
        unsigned long long v = 0;
#pragma unroll
        for (int k = 0; k < C_N + 2; ++k) v = lane == k ? c[k] : v;
        part[wv][lane] = v;
    }
    __syncthreads();
    if (threadIdx.x < C_N + 2) {
        unsigned long long v = 0;
        for (int w = 0; w < NWAVES; ++w) v += part[w][threadIdx.x];
        if (v) atomicAdd(&partials[(size_t)(blockIdx.x % kPartRows) * (C_N + 2) + threadIdx.x], v);
    }
}

// the wave's counters (ballot popcounts, iteration sums) added to the global ones once per workgroup
template <int NWAVES>
__device__ __forceinline__ void flush_counters(const unsigned long long (&c)[C_N + 2], unsigned long long (*part)[C_N + 2],
                                               unsigned long long* __restrict__ counters)
{
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    if (lane < C_N + 2) {
        unsigned long long v = 0;
#pragma unroll
        for (int k = 0; k < C_N + 2; ++k) v = lane == k ? c[k] : v;
        part[wv][lane] = v;
    }
    __syncthreads();
    if (threadIdx.x < C_N + 2) {
        unsigned long long v = 0;
        for (int w = 0; w < NWAVES; ++w) v += part[w][threadIdx.x];
        if (v) atomicAdd(&counters[threadIdx.x], v);
    }
}

// One sector of this lane's sample, from its syndrome row in LDS: the iteration-0 triage (ok: the
// decision satisfies the syndrome), and whether that decision is exactly the sample's errors in this
// sector -- each hit qubit of the sector (type != Z for X, != X for Z) decided and no other bit set (the
// walk hits a qubit at most once).  Only one sector's decisions are live at a time.
// on_hd(hd, ok, cvb, match) runs while the decisions are live (the survivors' record words).
template <int R, int L, int P, class EXP, int SEC, class F>
__device__ __forceinline__ bool fused_sector(const TriageMasks& m, const uint32_t* __restrict__ syn,
                                             const uint16_t* __restrict__ hits, int nh, bool check, bool& cvb,
                                             bool& match, F&& on_hd)
{
    constexpr int kW = row_words<R, P>();
    uint32_t w[kW + 2];
#pragma unroll
    for (int k = 0; k < kW; ++k) w[k] = syn[k];
    w[kW] = w[kW + 1] = 0u;
    uint64_t hd[L];
    bool ok;
    if (R >= 4 && (SEC ? m.symZ : m.symX))
        ok = triage_sector<R, L, P, EXP, SEC, (R >= 4)>(w, SEC ? m.hdpatZ : m.hdpatX, SEC ? m.cvpatZ : m.cvpatX,
                                                        SEC ? m.hdcntZ : m.hdcntX, SEC ? m.cvcntZ : m.cvcntX, hd, cvb);
    else
        ok = triage_sector<R, L, P, EXP, SEC, false>(w, SEC ? m.hdpatZ : m.hdpatX, SEC ? m.cvpatZ : m.cvpatX, 0u, 0u,
                                                     hd, cvb);
    match = false;
    if (check && ok) {
        int cnt = 0, hs = 0;
        bool mt = true;
#pragma unroll
        for (int l = 0; l < L; ++l) cnt += __popcll(hd[l]);
        for (int h = 0; h < nh; ++h) {
            const int v = hits[h] >> 2, t = hits[h] & 3;
            if (t == (SEC ? 0 : 2)) continue;  // X-only hit in Z, Z-only hit in X
            const int l = v / P, j = v - l * P;
            uint64_t x = 0;
#pragma unroll
            for (int q = 0; q < L; ++q) x = q == l ? hd[q] : x;  // select, not a dynamic register index
            mt &= ((x >> j) & 1ull) != 0ull;
            ++hs;
        }
        match = mt && cnt == hs;
    }
    on_hd(hd, ok, cvb, match);
    return ok;
}

// One sector's record dwords (stage_record_dw's layout: sector s at bits [8 nb s, 8 nb s + n), flags
// byte at bit 16 nb) into the record row, ndw dwords: the X sector keeps the dword it shares with the
// Z sector in carry, the Z sector ORs carry in and writes the flags and the row's padding.
template <int L, int P, int SEC>
__device__ __forceinline__ void stage_sector_dw(uint32_t* __restrict__ row, int ndw, const uint64_t (&hd)[L], uint32_t flags,
                                                uint32_t& carry)
{
    constexpr int n = L * P, nb = (n + 7) / 8, s0 = 8 * nb * SEC;
    constexpr int d0 = s0 / 32, d1 = (s0 + n - 1) / 32;
    constexpr int z0 = 8 * nb / 32;                 // the Z sector's first dword
    constexpr bool shared = (8 * nb) % 32 != 0;     // which also holds the X sector's last bits
    constexpr int fb = 16 * nb;
#pragma unroll
    for (int d = d0; d <= d1; ++d) {
        uint32_t w = 0;
#pragma unroll
        for (int l = 0; l < L; ++l) {
            const int a0 = 32 * d - (s0 + P * l);  // block bit at this dword's bit 0
            if (a0 >= P || a0 <= -32) continue;
            w |= a0 >= 0 ? (uint32_t)(hd[l] >> a0) : (uint32_t)(hd[l] << (-a0));
        }
        if (SEC == 0 && shared && d == z0) {
            carry = w;
            continue;
        }
        if (SEC == 1 && d == d0) w |= carry;
        if (SEC == 1 && fb >= 32 * d && fb < 32 * d + 32) w |= flags << (fb - 32 * d);
        row[d] = w;
    }
    if (SEC == 1)
        for (int d = d1 + 1; d < ndw; ++d) row[d] = (fb >= 32 * d && fb < 32 * d + 32) ? flags << (fb - 32 * d) : 0u;
}

template <int J, int K, int L, int P, int S, int T_>
__global__ __launch_bounds__(64 * kFusedWaves, kFusedMinWaves) void mc_fused_kernel(const FusedArgs a)
{
    using EXP = QcExponents<J, K, L, P, S, T_>;
    constexpr EXP tab = EXP::make();
    constexpr int n = L * P;
    constexpr int kWX = row_words<J, P>(), kWZ = row_words<K, P>();
    constexpr int RS = (kWX + kWZ + (kHitCap + 1) / 2) | 1;  // lane region (odd: the lanes' words in distinct banks)
    __shared__ uint32_t T[n + 1];
    __shared__ int E[(J + K) * L];
    __shared__ uint32_t region[64 * kFusedWaves * RS];
    __shared__ unsigned long long part[kFusedWaves][C_N + 2];
    __shared__ uint32_t wcnt[kFusedWaves][3], wgbase[3];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    gap_table(a.gp, n, T);
    for (int t = threadIdx.x; t < (J + K) * L; t += blockDim.x)
        E[t] = t < J * L ? tab.EX[t / L][t % L] : tab.EZ[(t - J * L) / L][(t - J * L) % L];
    uint32_t* __restrict__ mine = region + threadIdx.x * RS;
    for (int k = 0; k < RS; ++k) mine[k] = 0u;
    __syncthreads();
    const long long b0 = ((long long)blockIdx.x * kFusedWaves + wv) * 64;
    const long long b = b0 + lane;
    const bool valid = b < a.B;
    uint32_t* __restrict__ synX = mine;
    uint32_t* __restrict__ synZ = mine + kWX;
    uint16_t* __restrict__ hits = reinterpret_cast<uint16_t*>(mine + kWX + kWZ);
    int nh = 0;
    bool anyX = false, anyZ = false;
    if (valid && a.gp.thr != 0) {
        gap_walk(a.gp, a.start + (uint64_t)b, n, T, [&](int v, uint32_t t) {
            const bool ex = t != 2, ez = t != 0;
            anyX |= ex;
            anyZ |= ez;
            if (nh < kHitCap) hits[nh] = (uint16_t)(v << 2 | (int)t);
            ++nh;
            // qubit (l, j) sits in check (r, (j - E[r][l]) mod P) of each block row r
            const int l = v / P, j = v - l * P;
            if (ex)
#pragma unroll
                for (int r = 0; r < J; ++r) {
                    const int d = j - E[r * L + l];
                    const int c = r * P + (d < 0 ? d + P : d);
                    atomicXor(&synX[c >> 5], 1u << (c & 31));
                }
            if (ez)
#pragma unroll
                for (int r = 0; r < K; ++r) {
                    const int d = j - E[(J + r) * L + l];
                    const int c = r * P + (d < 0 ? d + P : d);
                    atomicXor(&synZ[c >> 5], 1u << (c & 31));
                }
        });
    }
    const bool fits = valid && nh <= kHitCap;
    // survivors get what the triage kernel writes, sector by sector while its decisions are live
    // (one sector's decisions in registers at a time): the X sector's record words when X is not
    // clean, the Z sector's and the flags for every survivor.  A clean X sector (stopped, decision = errors) of a
    // survivor keeps no record words: merge bit kXClean tells mc_survivor_kernel its residual is 0.
    uint32_t* __restrict__ recrow = reinterpret_cast<uint32_t*>(a.rec + b * a.recB);
    uint32_t carry = 0u, fX = 0u;
    bool cvbX = false, cvbZ = false, mX, mZ;
    const bool okX = fused_sector<J, L, P, EXP, 0>(a.m, synX, hits, nh, fits, cvbX, mX,
                                                   [&](const uint64_t (&hd)[L], bool ok, bool cvb, bool mt) {
                                                       fX = cvb ? QEC_CONVERGENCE_FAIL_X : 0u;
                                                       if (valid && !(fits && ok && mt))
                                                           stage_sector_dw<L, P, 0>(recrow, a.recB >> 2, hd, 0u, carry);
                                                   });
    const bool xclean = fits && okX && mX;
    uint32_t fZ = 0u;
    const bool okZ = fused_sector<K, L, P, EXP, 1>(a.m, synZ, hits, nh, xclean, cvbZ, mZ,
                                                   [&](const uint64_t (&hd)[L], bool ok, bool cvb, bool mt) {
                                                       fZ = cvb ? QEC_CONVERGENCE_FAIL_Z : 0u;
                                                       if (valid && !(xclean && ok && mt))
                                                           stage_sector_dw<L, P, 1>(recrow, a.recB >> 2, hd, fX | fZ, carry);
                                                   });
    // finished: both sectors stop at iteration 0 with the decision equal to the error (corrected)
    const bool done = xclean && okZ && mZ;
    const bool surv = valid && !done;
    if (surv) {  // its syndrome rows, for the list-mode decode
#pragma unroll
        for (int k = 0; k < kWX; ++k) a.sX[b * kWX + k] = synX[k];
#pragma unroll
        for (int k = 0; k < kWZ; ++k) a.sZ[b * kWZ + k] = synZ[k];
        *reinterpret_cast<int2*>(a.iters + 2 * b) = make_int2(1, 1);  // list sectors rewrite theirs
        a.merge[b] = (okX ? 0x100u | fX : 0u) | (okZ ? 0x200u | fZ : 0u) | (xclean ? kXClean : 0u);
    }
    const unsigned long long gs = __ballot(surv), dm = __ballot(done);
    const unsigned long long gx = __ballot(surv && !okX), gz = __ballot(surv && !okZ);
    unsigned long long c[C_N + 2] = {};
    c[C_WITHX] = __popcll(__ballot(valid && anyX));
    c[C_WITHZ] = __popcll(__ballot(valid && anyZ));
    c[C_CORRECTED] = __popcll(dm);
    c[C_CONVX] = __popcll(__ballot(done && cvbX));
    c[C_CONVZ] = __popcll(__ballot(done && cvbZ));
    c[C_N] = c[C_N + 1] = __popcll(dm);  // one iteration per sector
    // list appends: one atomic per workgroup and list (same-address atomics serialise at L2)
    const unsigned long long lt = (1ull << lane) - 1ull;
    if (lane == 0) {
        wcnt[wv][0] = (uint32_t)__popcll(gx);
        wcnt[wv][1] = (uint32_t)__popcll(gz);
        wcnt[wv][2] = (uint32_t)__popcll(gs);
    }
    __syncthreads();
    if (threadIdx.x < 3) {
        uint32_t tot = 0;
        for (int w = 0; w < kFusedWaves; ++w) tot += wcnt[w][threadIdx.x];
        wgbase[threadIdx.x] = tot ? atomicAdd(&a.counts[threadIdx.x * kCountStride], tot) : 0u;
    }
    __syncthreads();
    uint32_t bX = wgbase[0], bZ = wgbase[1], bS = wgbase[2];
    for (int w = 0; w < wv; ++w) {
        bX += wcnt[w][0];
        bZ += wcnt[w][1];
        bS += wcnt[w][2];
    }
    if ((gx >> lane) & 1ull) a.listX[bX + __popcll(gx & lt)] = (int32_t)b;
    if ((gz >> lane) & 1ull) a.listZ[bZ + __popcll(gz & lt)] = (int32_t)b;
    if ((gs >> lane) & 1ull) a.listS[bS + __popcll(gs & lt)] = (int32_t)b;
    store_partials<kFusedWaves>(c, part, a.partials);
}

// The survivors' counters after the list-mode decode: lane per listed sample (grid-stride over
// listS [0, counts[2])); the sample's errors are walked again into the lane's LDS region in the record
// layout, XORed with its record's decisions, and counted as statistics_lane_kernel counts a sample
// (syndrome fails from the flags -- the merge word's low byte --, the I-P check when neither failed and
// the residual is nonzero, convergence fails, both iteration counts).  withX / withZ were counted by
// mc_fused_kernel.
constexpr int kSurvWaves = 4;

// One lane of an I-P check group (CheckLogicalError, Quantum_LDPC_Code.h:126-142, as
// logical_from_columns): word k of the XOR of the I-P columns at the set bits of the residual res[0, nw)
// (u32 words, record layout: x bits at [0, 8 nb), z bits from 8 nb; words: the mask of its nonzero
// words) is nonzero.  Every lane of a group walks the same residual; the columns are fetched eight at
// a time.
template <int L, int P>
__device__ __forceinline__ bool logical_group(const uint32_t* __restrict__ res, uint64_t words, bool active,
                                              const uint64_t* __restrict__ cols, int cw, int k)
{
    constexpr int n = L * P, nb = (n + 7) / 8;
    constexpr int kBatch = 8;  // column fetches in flight
    uint64_t acc = 0;
    if (active && k < cw) {
        while (words) {  // the residual's nonzero words only
            const int w = __builtin_ctzll(words);
            words &= words - 1;
            uint32_t bits = res[w];
            while (bits) {
                int q[kBatch];
#pragma unroll
                for (int u = 0; u < kBatch; ++u) {
                    q[u] = -1;
                    if (bits) {
                        const int qq = 32 * w + __builtin_ctz(bits);
                        bits &= bits - 1;
                        q[u] = qq < 8 * nb ? qq : n + (qq - 8 * nb);
                    }
                }
                uint64_t c[kBatch];
#pragma unroll
                for (int u = 0; u < kBatch; ++u) c[u] = q[u] >= 0 ? cols[(size_t)q[u] * cw + k] : 0ull;
#pragma unroll
                for (int u = 0; u < kBatch; ++u) acc ^= c[u];
            }
        }
    }
    return acc != 0ull;
}

template <int L, int P>
__global__ __launch_bounds__(64 * kSurvWaves) void mc_survivor_kernel(const FusedArgs a)
{
    constexpr int n = L * P, nb = (n + 7) / 8;
    constexpr int NW = (2 * nb + 7) / 8;
    constexpr int RS = (2 * NW) | 1;  // lane region in u32 words (odd stride)
    __shared__ uint32_t T[n + 1];
    __shared__ uint32_t region[64 * kSurvWaves * RS];
    __shared__ unsigned long long part[kSurvWaves][C_N + 2];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    if (blockIdx.x == 0 && threadIdx.x < C_N + 2) {  // mc_fused_kernel's partial-sum rows into the counters
        unsigned long long v = 0;
#pragma unroll 16
        for (int r = 0; r < kPartRows; ++r) v += a.partials[r * (C_N + 2) + threadIdx.x];
        if (v) atomicAdd(&a.counters[threadIdx.x], v);
    }
    const long long cnt = a.counts[2 * kCountStride];
    if ((long long)blockIdx.x * blockDim.x >= cnt) return;  // workgroup-uniform: no survivor for this one
    gap_table(a.gp, n, T);
    __syncthreads();
    uint32_t* __restrict__ mine = region + threadIdx.x * RS;
    unsigned long long c[C_N + 2] = {};
    const long long step = (long long)gridDim.x * blockDim.x;
    // the I-P checks' lane groups: G = 64 / imp_cw samples per pass, lane k of a group sums word k
    const int G = a.imp_cw > 0 ? 64 / a.imp_cw : 1;
    const int g = a.imp_cw > 0 ? lane / a.imp_cw : 0, k = lane - g * a.imp_cw;
    const unsigned long long gmask = a.imp_cw >= 64 ? ~0ull : (1ull << a.imp_cw) - 1ull;
    for (long long i0 = (long long)blockIdx.x * blockDim.x + wv * 64; i0 < cnt; i0 += step) {
        const long long idx = i0 + lane;
        const bool valid = idx < cnt;
        const long long b = valid ? a.listS[idx] : 0;
        // the sample's record words, merge word and iteration counts are loaded before the walk, so
        // their latency overlaps it (the kernel is latency-bound: few survivors per CU)
        const uint32_t* __restrict__ r = reinterpret_cast<const uint32_t*>(a.rec + b * a.recB);
        constexpr int kRW = (2 * nb + 3) / 4;  // record words holding decisions
        static_assert(kRW <= 2 * NW, "the lane region holds the record's words");
        uint32_t rw[kRW];
#pragma unroll
        for (int d = 0; d < kRW; ++d) rw[d] = valid ? r[d] : 0u;
        const uint32_t mw = valid ? a.merge[b] : 0u;
        int2 it2 = make_int2(0, 0);
        if (valid) it2 = *reinterpret_cast<const int2*>(a.iters + 2 * b);
        for (int k = 0; k < RS; ++k) mine[k] = 0u;
        if (valid && a.gp.thr != 0) {
            gap_walk(a.gp, a.start + (uint64_t)b, n, T, [&](int v, uint32_t t) {
                if (t != 2) mine[v >> 5] |= 1u << (v & 31);
                if (t != 0) mine[(8 * nb + v) >> 5] |= 1u << ((8 * nb + v) & 31);
            });
        }
        // residual = errors ^ decisions over the record's 2 nb decision bytes
        const bool xclean = (mw & kXClean) != 0u;  // X residual 0; no X record words
        uint32_t nz = 0;
        uint64_t nzw = 0;  // nonzero residual words
        static_assert(kRW <= 64, "one mask bit per residual word");
#pragma unroll
        for (int d = 0; d < kRW; ++d) {
            const uint32_t rv = rw[d];
            const int rem = 2 * nb - 4 * d;  // decision bytes in word d
            const int xb = n - 32 * d;       // X decision bits in word d
            const uint32_t xm = xb >= 32 ? ~0u : xb <= 0 ? 0u : (1u << xb) - 1u;
            const uint32_t m = (rem >= 4 ? ~0u : rem <= 0 ? 0u : (1u << (8 * rem)) - 1u) & (xclean ? ~xm : ~0u);
            const uint32_t res = (mine[d] ^ rv) & m;
            mine[d] = res;
            nz |= res;
            nzw |= (uint64_t)(res != 0u) << d;
        }
        // the flags: the list-mode decode ORs its sectors' into the merge word, which the fused kernel
        // set to the stopped sectors' (launch_decode_list, merge_only); the record's byte is not merged
        const uint32_t f = mw & 0xFFu;
        const bool sx = (f & QEC_SYNDROME_FAIL_X) != 0, sz = (f & QEC_SYNDROME_FAIL_Z) != 0;
        unsigned long long need = a.imp_cw > 0 ? __ballot(valid && !(sx || sz) && nz != 0u) : 0ull, logical = 0;
        wave_sync();  // the residuals, read across lanes
        while (need) {  // G samples per pass: lane group g (imp_cw lanes) takes the pass's g-th sample
            const unsigned long long pick = need;
            int s = -1;
            for (int q = 0; q < G && need; ++q) {
                const int sl = __builtin_ctzll(need);
                need &= need - 1;
                if (q == g) s = sl;
            }
            const int src = s < 0 ? 0 : s;
            const uint64_t words = ((uint64_t)(uint32_t)__shfl((int)(nzw >> 32), src) << 32) | (uint32_t)__shfl((int)(uint32_t)nzw, src);
            const unsigned long long nzm =
                __ballot(logical_group<L, P>(region + (wv * 64 + src) * RS, words, s >= 0, a.imp_cols, a.imp_cw, k));
            unsigned long long p2 = pick;
            for (int q = 0; q < G && p2; ++q) {
                const int sl = __builtin_ctzll(p2);
                p2 &= p2 - 1;
                if ((nzm >> (q * a.imp_cw)) & gmask) logical |= 1ull << sl;
            }
        }
        const unsigned long long vm = __ballot(valid), bx = __ballot(sx), bz = __ballot(sz);
        const unsigned long long ok = vm & ~(bx | bz);
        c[C_SYNX] += __popcll(bx);
        c[C_SYNZ] += __popcll(bz);
        c[C_LOGICAL] += __popcll(ok & logical);
        c[C_CORRECTED] += __popcll(ok & ~logical);
        c[C_CONVX] += __popcll(__ballot((f & QEC_CONVERGENCE_FAIL_X) != 0));
        c[C_CONVZ] += __popcll(__ballot((f & QEC_CONVERGENCE_FAIL_Z) != 0));
        unsigned long long itx = (unsigned)it2.x, itz = (unsigned)it2.y;
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) {
            itx += __shfl_xor(itx, o);
            itz += __shfl_xor(itz, o);
        }
        c[C_N] += itx;
        c[C_N + 1] += itz;
    }
    flush_counters<kSurvWaves>(c, part, a.counters);
}

using TriageFn = void (*)(const TriageArgs);

// the shipped codes, when the file's tables are its header's generator output (as bp_decode.hip's
// GeneratedShifts variants require)
static TriageFn triage_fn(const Code& c)
{
    TriageFn fn = nullptr;
    if (c.J == 4 && c.K == 5 && c.L == 10 && c.P == 61 && c.sigma == 9 && c.tau == 49) fn = triage_kernel<4, 5, 10, 61, 9, 49>;
    if (c.J == 3 && c.K == 3 && c.L == 6 && c.P == 7 && c.sigma == 2 && c.tau == 3) fn = triage_kernel<3, 3, 6, 7, 2, 3>;
    if (!fn) return nullptr;
    std::vector<int> EX, EZ;
    if (!generator_exponents(c.J, c.K, c.L, c.P, c.sigma, c.tau, EX, EZ) || EX != c.EX || EZ != c.EZ) return nullptr;
    return fn;
}

bool triage_supported(const Code& c) { return c.is_qc && triage_fn(c) != nullptr; }

// pat (bit idx = value for pattern idx of R bits) as a function of the pattern's count of ones: out
// bit c = the value at count c (counts above R: 0); false if two patterns with one count differ
static bool by_count(uint32_t pat, int R, uint32_t& out)
{
    out = 0;
    uint32_t seen = 0;
    for (int idx = 0; idx < (1 << R); ++idx) {
        const int c = __builtin_popcount((unsigned)idx);
        const uint32_t v = (pat >> idx) & 1u;
        if ((seen >> c) & 1u) {
            if (((out >> c) & 1u) != v) return false;
        } else {
            seen |= 1u << c;
            out |= v << c;
        }
    }
    return true;
}

static TriageMasks triage_masks(const Code& c, const uint32_t pats[4])
{
    TriageMasks m{};
    m.hdpatX = pats[0]; m.cvpatX = pats[1]; m.hdpatZ = pats[2]; m.cvpatZ = pats[3];
    m.symX = by_count(pats[0], c.J, m.hdcntX) && by_count(pats[1], c.J, m.cvcntX);
    m.symZ = by_count(pats[2], c.K, m.hdcntZ) && by_count(pats[3], c.K, m.cvcntZ);
    const char* trees = std::getenv("QEC_TRIAGE_TREES");  // tests: force the pattern-tree form
    if (trees && trees[0] == '1') m.symX = m.symZ = 0;
    return m;
}

using FusedFn = void (*)(const FusedArgs);

// the fused kernels of the shipped codes (as triage_fn)
struct FusedFns {
    FusedFn fused, surv;
};
static bool fused_fns(const Code& c, FusedFns& f)
{
    if (!triage_supported(c)) return false;
    if (c.P == 61) f = {mc_fused_kernel<4, 5, 10, 61, 9, 49>, mc_survivor_kernel<10, 61>};
    else f = {mc_fused_kernel<3, 3, 6, 7, 2, 3>, mc_survivor_kernel<6, 7>};
    return true;
}

// workgroups of the fused kernel for a batch of B samples; the
// list lengths' words (counts) span mc_fused_count_words()
long long mc_fused_parts(long long B) { return (B + 64LL * kFusedWaves - 1) / (64LL * kFusedWaves); }
// rows of the partials workspace, zeroed before every fused kernel
int mc_fused_part_rows() { return kPartRows; }
int mc_fused_count_words() { return 2 * kCountStride + 1; }
int mc_fused_count_stride() { return kCountStride; }

bool mc_fused_supported(const Code& c, int rec_stride)
{
    FusedFns f;
    return fused_fns(c, f) && rec_stride % 4 == 0 && rec_stride >= 2 * ((c.n + 7) / 8) + 1 &&
           c.imp_col_words <= 64 && 2 * c.n < (1 << 14);
}

// The fused pipeline's kernels, in stage order on one stream: MC_FUSED_SAMPLE (sample, syndromes,
// triage, the finished samples' statistics, the survivors' triage outputs and lists), then -- after
// the caller's list-mode decode -- MC_FUSED_SURVIVORS (their statistics).  counts must be zeroed
// before the first.
int launch_mc_fused(const Code& c, uint64_t seed, uint64_t start, long long B, float p, const uint32_t pats[4],
                    uint32_t* sX, uint32_t* sZ, uint8_t* rec, int rec_stride, int32_t* iters, uint32_t* merge,
                    int32_t* listX, int32_t* listZ, int32_t* listS, uint32_t* counts, const uint64_t* imp_cols,
                    unsigned long long* counters, unsigned long long* partials, int stage, hipStream_t st)
{
    FusedFns f{};
    if (!mc_fused_supported(c, rec_stride) || !fused_fns(c, f))
        return fail(QEC_ERR_UNSUPPORTED, "mc fused: no kernel for this code or record layout");
    if ((reinterpret_cast<uintptr_t>(sX) | reinterpret_cast<uintptr_t>(sZ)) & 7u || reinterpret_cast<uintptr_t>(iters) & 7u)
        return fail(QEC_ERR_ARG, "mc fused: bit rows and iteration counts must be 8-byte aligned");
    if (B <= 0) return QEC_OK;
    FusedArgs a{};
    a.gp = make_gap(seed, p);
    a.start = start; a.B = B; a.recB = rec_stride;
    a.m = triage_masks(c, pats);
    a.sX = sX; a.sZ = sZ; a.rec = rec; a.iters = iters; a.merge = merge;
    a.listX = listX; a.listZ = listZ; a.listS = listS; a.counts = counts;
    a.imp_cols = imp_cols; a.imp_cw = c.imp_col_words; a.counters = counters;
    a.partials = partials; a.nparts = (int)mc_fused_parts(B);
    if (stage == MC_FUSED_SAMPLE) {
        hipLaunchKernelGGL(f.fused, dim3((unsigned)a.nparts), dim3(64 * kFusedWaves), 0, st, a);
    } else {
        // the survivor count is on the device: a grid for up to every sample, capped (grid-stride)
        int dev = 0, cus = 256;
        if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
            cus <= 0)
            cus = 256;
        const long long per = 64LL * kSurvWaves;
        const long long blocks = std::min<long long>((B + per - 1) / per, 2LL * cus);
        hipLaunchKernelGGL(f.surv, dim3((unsigned)blocks), dim3(64 * kSurvWaves), 0, st, a);
    }
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return fail(QEC_ERR_HIP, std::string("mc fused launch: ") + hipGetErrorString(e));
    return QEC_OK;
}

// Zeroes n 64-bit words on the stream (the fused pipeline's counters and list lengths before a batch):
// a one-workgroup kernel of this library instead of hipMemsetAsync, whose fill launch left ~4 us of
// idle GPU before the next kernel (profiles/r06/ab/cmp_zero_kernel.txt)
__global__ __launch_bounds__(256) void zero_words_kernel(unsigned long long* __restrict__ w, int n,
                                                         unsigned long long* __restrict__ w2, int n2)
{
    for (int i = threadIdx.x; i < n; i += blockDim.x) w[i] = 0ull;
    for (int i = threadIdx.x; i < n2; i += blockDim.x) w2[i] = 0ull;
}

int launch_zero_words(unsigned long long* w, int n, hipStream_t st, unsigned long long* w2, int n2)
{
    if (n <= 0 && n2 <= 0) return QEC_OK;
    hipLaunchKernelGGL(zero_words_kernel, dim3(1), dim3(256), 0, st, w, n, w2, n2);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return fail(QEC_ERR_HIP, std::string("zero words launch: ") + hipGetErrorString(e));
    return QEC_OK;
}

// the kernel loads rows with 16- / 8-byte loads (triage_sector)
bool triage_aligned(const void* sX, const void* sZ)
{
    return ((reinterpret_cast<uintptr_t>(sX) | reinterpret_cast<uintptr_t>(sZ)) & 15u) == 0;
}

int launch_triage(const Code& c, const uint32_t* sX, const uint32_t* sZ, long long B, const uint32_t pats[4],
                  uint8_t* rec, int32_t* iters, uint32_t* merge, int32_t* listX, int32_t* listZ, uint32_t* counts,
                  hipStream_t st, int rec_stride)
{
    TriageFn fn = triage_fn(c);
    if (!fn) return fail(QEC_ERR_UNSUPPORTED, "triage: no kernel for this code");
    if (!triage_aligned(sX, sZ)) return fail(QEC_ERR_ARG, "triage: bit rows must start 16-byte aligned");
    if (B <= 0) return QEC_OK;
    TriageArgs a{};
    a.sX = sX; a.sZ = sZ; a.B = B;
    a.wX = (c.mX + 31) / 32; a.wZ = (c.mZ + 31) / 32;
    a.nb = (c.n + 7) / 8; a.recB = rec_stride > 0 ? rec_stride : 2 * a.nb + 1;
    a.m = triage_masks(c, pats);
    a.rec = rec; a.iters = iters; a.merge = merge; a.listX = listX; a.listZ = listZ; a.counts = counts;
    const long long per_block = 64LL * kTriageWaves;
    const size_t smem = (size_t)kTriageWaves * (64 * a.recB + 16);
    hipLaunchKernelGGL(fn, dim3((unsigned)((B + per_block - 1) / per_block)), dim3(64 * kTriageWaves), smem, st, a);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return fail(QEC_ERR_HIP, std::string("triage launch: ") + hipGetErrorString(e));
    return QEC_OK;
}

}  // namespace qec
