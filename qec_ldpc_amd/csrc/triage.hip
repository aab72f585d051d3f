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
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdlib>

#include "qec_device.h"
#include "qec_internal.h"

namespace qec {

constexpr int kTriageWaves = 4;

struct TriageArgs {
    const uint32_t* sX;  // [B][wX] bit rows (bit c = check c)
    const uint32_t* sZ;  // [B][wZ]
    long long B;
    int wX, wZ, nb, recB;  // recB: record row stride (>= 2 nb + 1)
    uint32_t hdpatX, cvpatX, hdpatZ, cvpatZ;  // bit idx: pattern idx decides 1 / stays outside (0.01, 0.99)
    // the same masks by count when they depend only on the number of unsatisfied checks (symmetric):
    // bit c = the value for patterns with c ones; sym* = 0 when a mask is not symmetric (pattern trees)
    uint32_t hdcntX, cvcntX, hdcntZ, cvcntZ;
    int symX, symZ;
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
template <int R, int L, int P, class EXP, int SEC, bool SYM>
__device__ __forceinline__ bool triage_sector(const uint32_t* __restrict__ rows, long long b, uint32_t hdpat,
                                              uint32_t cvpat, uint32_t hdcnt, uint32_t cvcnt, uint64_t (&hd)[L],
                                              bool& cvbad)
{
    static_assert(R <= 5 && P <= 64, "patterns in 32 bits, blocks in 64");
    constexpr EXP tab = EXP::make();
    auto E = [&](int r, int l) constexpr { return SEC ? tab.EZ[r][l] : tab.EX[r][l]; };
    constexpr uint64_t mask = P >= 64 ? ~0ull : (1ull << P) - 1ull;
    constexpr int kW = (R * P + 31) / 32;  // words of the row
    constexpr uint32_t full = R >= 5 ? 0xFFFFFFFFu : (1u << (1 << R)) - 1u;
    uint32_t w[kW + 2];
    // the row, kW words at a compile-time stride from a 16-byte aligned base (launch_triage checks):
    // 16- or 8-byte loads where the row's alignment allows (P61: X 2 x 16 B, Z 5 x 8 B instead of 18
    // dword loads per lane)
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
    // symmetric masks (the usual case) take the adder form; R <= 3 gains nothing from it
    bool okX, okZ;
    if (J >= 4 && a.symX)
        okX = triage_sector<J, L, P, EXP, 0, J >= 4>(a.sX, bl, a.hdpatX, a.cvpatX, a.hdcntX, a.cvcntX, hdX, cvbX);
    else
        okX = triage_sector<J, L, P, EXP, 0, false>(a.sX, bl, a.hdpatX, a.cvpatX, 0u, 0u, hdX, cvbX);
    if (K >= 4 && a.symZ)
        okZ = triage_sector<K, L, P, EXP, 1, K >= 4>(a.sZ, bl, a.hdpatZ, a.cvpatZ, a.hdcntZ, a.cvcntZ, hdZ, cvbZ);
    else
        okZ = triage_sector<K, L, P, EXP, 1, false>(a.sZ, bl, a.hdpatZ, a.cvpatZ, 0u, 0u, hdZ, cvbZ);
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

// the kernel loads rows with 16- / 8-byte loads (triage_sector)
bool triage_aligned(const void* sX, const void* sZ)
{
    return ((reinterpret_cast<uintptr_t>(sX) | reinterpret_cast<uintptr_t>(sZ)) & 15u) == 0;
}

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
    a.hdpatX = pats[0]; a.cvpatX = pats[1]; a.hdpatZ = pats[2]; a.cvpatZ = pats[3];
    a.symX = by_count(pats[0], c.J, a.hdcntX) && by_count(pats[1], c.J, a.cvcntX);
    a.symZ = by_count(pats[2], c.K, a.hdcntZ) && by_count(pats[3], c.K, a.cvcntZ);
    const char* trees = std::getenv("QEC_TRIAGE_TREES");  // tests: force the pattern-tree form
    if (trees && trees[0] == '1') a.symX = a.symZ = 0;
    a.rec = rec; a.iters = iters; a.merge = merge; a.listX = listX; a.listZ = listZ; a.counts = counts;
    const long long per_block = 64LL * kTriageWaves;
    const size_t smem = (size_t)kTriageWaves * (64 * a.recB + 16);
    hipLaunchKernelGGL(fn, dim3((unsigned)((B + per_block - 1) / per_block)), dim3(64 * kTriageWaves), smem, st, a);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return fail(QEC_ERR_HIP, std::string("triage launch: ") + hipGetErrorString(e));
    return QEC_OK;
}

}  // namespace qec
