// Batched belief-propagation decoding of X and Z syndromes for quasi-cyclic CSS
// codes on MI355X (gfx950, CDNA4).  Replaces the reference's decoding hot path
// DecoderCPU::Decode -> BeliefPropogation -> EqNodeUpdate / VarNodeUpdate /
// CheckConvergence (QEC_LDPC/DecoderCPU.h:150-390) and the never-launched CUDA
// kernels of QEC_LDPC/kernels.cu:33-250.
//
// Design ("wave-circulant"): one 64-lane wavefront owns G = floor(64 / P) whole
// syndrome pairs.  Lane g*P + i of the wave is circulant row i of syndrome g.
//   * check view:  lane i holds, in VGPRs, the message of every edge (r, l, i):
//                  check r*P+i  <->  variable l*P + (E[r][l] + i) mod P.
//                  The check-node update for checks (r, i), r = 0..R-1, is
//                  therefore entirely lane-local.
//   * var view:    variable (l, j) touches edges (r, l, (j - E[r][l]) mod P),
//                  i.e. a rotation of lane index by E[r][l] inside the group.
//                  The variable-node update gathers its R inputs with
//                  ds_bpermute_b32 (forward rotation) and returns the R outputs
//                  with the inverse rotation.
// All messages of one syndrome live in registers for all iterations: HBM traffic
// is only syndromes in and decisions out, so the kernel is VALU-bound rather
// than bound by the 16 B/edge/iteration an HBM-resident flooding schedule moves.
//
// Bit-exactness vs DecoderCPU: every product is the reference's left fold in
// ascending neighbour order (prefix reuse only, never a tree), in IEEE fp32 with
// denormals preserved, -ffp-contract=off, correctly rounded division.  Two
// FMAs are used where they are provably identical to the reference's two-step
// expressions:
//   1.0f - 2.0f*q            == fma(-2, q, 1)          (2q is exact)
//   0.5f*(1.0f -/+ t)        == fma(-/+0.5, t, 0.5)    (halving is exact: |1 -/+ t|
//                                                       is 0 or >= 2^-24, never subnormal)
// The reference computes the syndrome=1 case as 0.5 * (double)(1.0f + t), which is
// the same exact halving of the same fp32 sum.
#include <hip/hip_runtime.h>

#include <atomic>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <type_traits>

#include "qec_device.h"
#include "qec_internal.h"
#include "qec_launch.h"

#pragma clang fp contract(off)

namespace qec {

// Design choices.  Every one below was measured on the chip and is fixed; the measurements of the
// alternatives (and the build flags that selected them, removed in round 6) are in profiles/r0*/ and
// DESIGN.md's changelog.  Each kernel variant carries its own measured choice of lane relabelling,
// mask-selected rotation bases, gather pipelining, short division, zero-skip, hard-message forms and
// occupancy (Tune<> in the variant table below).
//   QEC_PHASE_STATS  instrumented kernels only (bp_decode_phase.hip, QEC_OPT_PHASE_STATS): iters[] reports,
//                    per sector, the iterations spent in each phase (soft | hard << 8 | agreed << 16 |
//                    jumped << 24) instead of the count.  The Makefile builds both states.
#ifndef QEC_PHASE_STATS
#define QEC_PHASE_STATS 0
#endif
// First iteration whose var pass tests whether the sector became hard (iterations 0 and 1 essentially
// never end hard; skipping the test there only delays the exact hard forms, never changes a bit).
constexpr int kTrackFrom = 2;

// Per-variant tuning: minimum waves per SIMD for the register allocator, and the options above.
template <int MINW_, bool RELABEL_, bool ZEROSKIP_, bool FASTDIV_, bool SATURATE_ = false, bool SPLIT_ = false,
          bool MASKSEL_ = false, int PIPE_ = 0, int WPB_ = 4, int SYNW_ = 0, int CG_ = 1, bool ROWB_ = false,
          int MWX_ = 0, int MWZ_ = 0>
struct Tune {
    // sector launches (MODE 3 / 4: one kernel per sector, each compiled for its own sector only): their
    // occupancy, 0 = kMinWaves
    static constexpr int kMinWavesX = MWX_ > 0 ? MWX_ : MINW_;
    static constexpr int kMinWavesZ = MWZ_ > 0 ? MWZ_ : MINW_;
    static constexpr bool kRowBarrier = ROWB_;  // a scheduling barrier after each check-pass row
    static constexpr int kColGroup = CG_;       // columns per division guard in soft var passes
    static constexpr int kMinWaves = MINW_;
    static constexpr int kMinWavesSyn = SYNW_ > 0 ? SYNW_ : MINW_;  // the syndrome-stop kernels
    static constexpr int kWavesPerBlock = WPB_;  // waves per workgroup
    static constexpr bool kMaskSelect = MASKSEL_;  // rotation base chosen by a constant lane mask (rot_addr)
    static constexpr int kPipeline = PIPE_;  // D: the gathers of the next D columns in flight during a column
    static constexpr bool kSplit = SPLIT_;  // QEC_OPT_SECTOR_SPLIT = 1 (auto) splits sectors for this variant
    static constexpr bool kRelabel = RELABEL_;  // spanning-tree lane relabelling (relabel below)
    static constexpr bool kZeroSkip = ZEROSKIP_;  // a column of +0 numerators skips its divisions
    static constexpr bool kFastDiv = FASTDIV_;  // the short division (div_short)
    static constexpr bool kSaturate = SATURATE_;  // the hard-message forms (check_pass_hard, var_pass)
    static constexpr bool kAgreeSyn = false;  // the syndrome stop takes the agreement test (kAgree): never
    static constexpr int kSeqSynWavesX = kMinWavesSyn, kSeqSynWavesZ = kMinWavesSyn;  // sector launches, syndrome stop
};

// The syndrome-stop sector launches of a variant: X at five waves per SIMD where the variant's syndrome
// kernels take fewer (P61: 4 -> 5, +2 %; higher occupancies spill and lose 15-40 %,
// profiles/r06/ab/cmp_occupancy_r06c.txt); Z at the variant's own.
template <class TU>
struct SeqSynTune : TU {
    static constexpr int kSeqSynWavesX = 5 > TU::kMinWavesSyn ? 5 : TU::kMinWavesSyn;
};

// The list-mode (MODE 2) tuning of a variant: its own occupancy (no agreement test, no cycle jump), and
// WPB > 1: workgroups of WPB waves -- every resident wave of a CU -- that take the listed sectors of a
// contiguous share of the list from an LDS counter (bp_decode_kernel).
template <class TU, int LW, int WPB = 0>
struct ListTune : TU {
    static constexpr int kMinWavesSyn = LW;
    static constexpr int kWavesPerBlock = WPB > 0 ? WPB : TU::kWavesPerBlock;
};

// the largest divisor of L not above the variant's column-group size
template <class TU, int L>
constexpr int col_group()
{
    int g = TU::kColGroup < 1 ? 1 : (TU::kColGroup > L ? L : TU::kColGroup);
    while (L % g != 0) --g;
    return g;
}

// Rotations by push, one-group waves (32 < P < 64): a rotation whose pull would wrap a 32-lane half
// (source lane i - s + P for i < s) is made as the same rotation pushed instead (ds_permute_b32, lane i to
// lane i + s mod P).  A wrapping ds_bpermute puts two sources of one half on one LDS bank and costs 7.1
// instead of 6.1 cycles; a push of any shift costs 6.1 (tools/kbench/perm_probe.hip,
// profiles/r05/perm_probe.txt).  The group then sits on the TOP P lanes of the wave, [64 - P, 64), and
// the 64 - P idle lanes below it: when several lanes push to one lane the highest-numbered source wins
// (the ISA's DS_PERMUTE_B32 rule; tools/kbench/permute_collide.hip checks it on the chip), so an idle
// lane's push never overwrites a group lane's (the group's pushes are a bijection on it).  With the group
// on lanes [64 - P, 64) the rotations with s >= P - 31 push (their pulls would wrap the upper half onto
// the group's first lanes, banks shared; their pushes' destinations are distinct banks per half) and pulls
// with s <= P - 32 read distinct banks in both halves.  Multi-group waves (P7) keep their pulls (pushing
// every shift measured -1.8 .. +0.5 %, profiles/r05/cmp_rot_push.txt).

// The first lane of group 0 for compile-time P: with pushed rotations the G = 64 / P groups take the top
// G P lanes and the 64 - G P idle lanes sit below them, else the groups start at lane 0.
template <int P_>
constexpr int group_base()
{
    return (2 * P_ > 64 && P_ < 64) ? 64 - (64 / P_) * P_ : 0;
}

// Rotations by push for compile-time one-group waves (above).
template <class SH>
constexpr bool kPushRot()
{
    return SH::kStatic && 2 * SH::kP > 64 && SH::kP < 64;
}
template <class SH>
constexpr int kGroupBase()
{
    if constexpr (kPushRot<SH>()) return group_base<SH::kP>();
    return 0;
}

// true iff pred holds on every live lane of the wave (lanes outside the batch, or masked off
// by a finished group, do not vote)
__device__ __forceinline__ bool all_live(bool pred, bool live) { return __ballot(live && !pred) == 0ull; }
// The same for a shift provider: with compile-time P > 32 a wave holds one syndrome group whose
// lanes [kGroupBase, kGroupBase + P) are all live once the wave runs (a wave with no syndrome of the batch returns
// at entry), so liveness is a constant lane mask instead of a per-lane predicate.
template <class SH>
__device__ __forceinline__ bool all_live_sh(bool pred, bool live)
{
    if constexpr (SH::kStatic && 2 * SH::kP > 64) {
        constexpr unsigned long long gm = (SH::kP >= 64 ? ~0ull : ((1ull << SH::kP) - 1ull)) << kGroupBase<SH>();
        return (__ballot(!pred) & gm) == 0ull;
    } else {
        return all_live(pred, live);
    }
}

// The hard-message paths need 0 < p' < 1: then every message lies in [0, 1], zeros are +0,
// and q - q*q == 0 exactly iff q is +0 or 1 (NaN fails the test).
__device__ __forceinline__ bool hard_ok(float pp) { return pp > 0.0f && pp < 1.0f; }

constexpr int kMaxRL = 128;  // largest R*L a kernel argument block carries
constexpr int kMaxTab0 = 448;  // iteration-0 table entries, (2^RX RX + 2^RZ RZ), of every instantiated variant
constexpr int kMaxR = 16;
constexpr uint32_t kNonBinary = 1u << 31;  // sbits: a syndrome entry of this lane is not 0 / 1 (load_sbits)
constexpr int kMaxL = 32;

struct BpArgs {
    const uint8_t* sX;  // [B][mX] bytes, or with sbits set [B][wX] words of bits (bit c = check c)
    const uint8_t* sZ;
    int sbits, wX, wZ;
    uint8_t* eX;
    uint8_t* eZ;
    uint8_t* flags;
    int32_t* iters;
    float* q;
    const int32_t* perm;  // dispatch order (schedule.hip): group slot k decodes syndrome perm[k]; null = batch order
    int perm_sectors;     // perm holds the per-sector orders: the Z sector's waves take perm[B + k]
    // packed decision records (qec_decode_batch_packed_dev): per syndrome eX bits, eZ bits (nb bytes
    // each, bit j of byte k = qubit 8k + j), then the flags byte; null = byte outputs eX / eZ / flags
    uint8_t* rec;
    // sector-split launches: one word per syndrome, zeroed before the launch; each sector ORs in its
    // flags plus a done bit and the second one writes the merged flags byte (plain store)
    uint32_t* merge;
    // list mode (MODE 2, after the triage): the syndromes whose X / Z sector goes on, and the two lengths
    const int32_t* listX;
    const int32_t* listZ;
    const uint32_t* counts;
    int mergeOnly;  // list mode for the fused Monte-Carlo pipeline: flags only into merge[] (no record byte)
    int countStride;  // list mode: counts[0] = listX length, counts[countStride] = listZ length
    long long B;
    int P, G, n, mX, mZ;
    int nb, recBytes;  // ceil(n / 8); row stride of the records (2 nb + 1, or padded to whole words)
    float errorProbability;
    int maxIter, stop;
    int hardPaths;  // QEC_HP_* bits: hard-message paths / cycle jump (QEC_OPT_HARD_PATHS, QEC_OPT_CYCLE_JUMP)
    int scaled;     // p' in [2^-20, 1/2] (scaled_ok): var passes with at most 4 factors per fold divide guard-free
    // lane-relabelled circulant tables (see relabel() below)
    // iteration-0 tables of both sectors computed on the host (launch_decode: the same operations,
    // so the same bits, as table0_entry on the device; each workgroup copies them to LDS)
    float tab0[kMaxTab0];
    // zero-syndrome outcome of each sector under the fixed / reference stop (zero_outcome; 0: none):
    // kZsValid | decision bit | conv-fail << 1 | syndrome-fail << 2 | iterations << 8
    uint32_t zs[2];
    int SX[kMaxRL], SZ[kMaxRL];  // rotation of block (r, l) between check and variable views
    int DX[kMaxR], DZ[kMaxR];    // check-view lane lambda holds check (r, (lambda + D[r]) mod P)
    int CX[kMaxL], CZ[kMaxL];    // var-view lane mu holds variable (l, (mu + C[l]) mod P)
};

// ---- lane relabelling ------------------------------------------------------
// Block (r, l) of a sector is the circulant "check (r, i) <-> variable (l, (E[r][l] + i) mod P)".
// Storing check (r, i) in lane (i - D[r]) mod P and variable (l, j) in lane (j - C[l]) mod P
// turns the block's check->variable lane rotation into S[r][l] = (E[r][l] + D[r] - C[l]) mod P.
// With C[l] = E[0][l] and D[r] = (C[0] - E[r][0]) mod P the R + L - 1 blocks of row 0 and
// column 0 need no rotation at all (a spanning tree of the block graph), so those edges skip
// the ds_bpermute in both directions.  Arithmetic (and so every output bit) is unchanged.
inline void relabel(const int* E, int R, int L, int P, bool on, int* S, int* D, int* C)
{
    if (!on) {
        for (int k = 0; k < R * L; ++k) S[k] = E[k];
        for (int r = 0; r < R; ++r) D[r] = 0;
        for (int l = 0; l < L; ++l) C[l] = 0;
        return;
    }
    for (int l = 0; l < L; ++l) C[l] = E[l];
    for (int r = 0; r < R; ++r) D[r] = ((C[0] - E[r * L]) % P + P) % P;
    for (int r = 0; r < R; ++r)
        for (int l = 0; l < L; ++l) S[r * L + l] = ((E[r * L + l] + D[r] - C[l]) % P + P) % P;
}

// ---- shift providers -------------------------------------------------------
// Runtime: exponents read from the kernel-argument block.  table() launders the
// pointer once per iteration so the R*L shift loads and rotation addresses stay
// inside the loop (scalar-cache hits) instead of being hoisted into ~2*R*L
// live registers.
struct RuntimeShifts {
    static constexpr bool kStatic = false;
    static constexpr bool kMaskSelect = false;
    static constexpr int kP = 0;
    __device__ static int P(const BpArgs& a) { return a.P; }
    template <int SEC>
    __device__ static const int* table(const BpArgs& a)
    {
        const int* t = SEC ? a.SZ : a.SX;
        asm volatile("" : "+s"(t));
        return t;
    }
    template <int SEC, int L>
    __device__ static int shift(const int* t, int r, int l) { return t[r * L + l]; }
    template <int SEC>
    __device__ static int rowoff(const BpArgs& a, int r) { return SEC ? a.DZ[r] : a.DX[r]; }
    template <int SEC>
    __device__ static int coloff(const BpArgs& a, int l) { return SEC ? a.CZ[l] : a.CX[l]; }
};

// Compile-time: exponent tables produced by the QC_LDPC_CSS generator formula
// (QEC_LDPC/QEC_LDPC_CSS.cu:37-90) evaluated by the compiler, so every rotation
// address is a loop-invariant constant of the lane index.
template <int J_, int K_, int L_, int P_, int S_, int T_, bool RL_, bool MS_ = false>
struct GeneratedShifts {
    static constexpr bool kStatic = true;
    static constexpr bool kMaskSelect = MS_;  // rotation base by constant lane mask (see rot_addr)
    static constexpr int kP = P_;
    struct Tables {
        int EX[J_][L_];
        int EZ[K_][L_];
        int SX[J_][L_], SZ[K_][L_];
        int DX[J_], DZ[K_];
        int CX[L_], CZ[L_];
    };
    static constexpr Tables make()
    {
        Tables t{};
        constexpr QcExponents<J_, K_, L_, P_, S_, T_> e = QcExponents<J_, K_, L_, P_, S_, T_>::make();
        for (int j = 0; j < J_; ++j)
            for (int l = 0; l < L_; ++l) t.EX[j][l] = e.EX[j][l];
        for (int k = 0; k < K_; ++k)
            for (int l = 0; l < L_; ++l) t.EZ[k][l] = e.EZ[k][l];
        // relabel() on the 2-D tables (same rule, written out for constant evaluation)
        for (int l = 0; l < L_; ++l) { t.CX[l] = RL_ ? t.EX[0][l] : 0; t.CZ[l] = RL_ ? t.EZ[0][l] : 0; }
        for (int r = 0; r < J_; ++r) t.DX[r] = RL_ ? ((t.CX[0] - t.EX[r][0]) % P_ + P_) % P_ : 0;
        for (int r = 0; r < K_; ++r) t.DZ[r] = RL_ ? ((t.CZ[0] - t.EZ[r][0]) % P_ + P_) % P_ : 0;
        for (int r = 0; r < J_; ++r)
            for (int l = 0; l < L_; ++l) t.SX[r][l] = ((t.EX[r][l] + t.DX[r] - t.CX[l]) % P_ + P_) % P_;
        for (int r = 0; r < K_; ++r)
            for (int l = 0; l < L_; ++l) t.SZ[r][l] = ((t.EZ[r][l] + t.DZ[r] - t.CZ[l]) % P_ + P_) % P_;
        return t;
    }
    static constexpr Tables tabs = make();
    __device__ static constexpr int P(const BpArgs&) { return P_; }
    template <int SEC>
    __device__ static const int* table(const BpArgs&) { return nullptr; }
    template <int SEC, int L>
    __device__ static constexpr int shift(const int*, int r, int l) { return SEC ? tabs.SZ[r][l] : tabs.SX[r][l]; }
    template <int SEC>
    __device__ static constexpr int rowoff(const BpArgs&, int r) { return SEC ? tabs.DZ[r] : tabs.DX[r]; }
    template <int SEC>
    __device__ static constexpr int coloff(const BpArgs&, int l) { return SEC ? tabs.CZ[l] : tabs.CX[l]; }
};

// ---- lane helpers ----------------------------------------------------------
__device__ __forceinline__ float bperm(int addr, float v)
{
    return __int_as_float(__builtin_amdgcn_ds_bpermute(addr, __float_as_int(v)));
}
__device__ __forceinline__ int bperm_i(int addr, int v) { return __builtin_amdgcn_ds_bpermute(addr, v); }

// Rotation inside a lane group: the value of lane gb + (i - s) mod P, s in [0, P).
// ds_bpermute selects lane ((addr + offset) >> 2) & 63, so with the two per-lane bases
//   b0 = 4 (gb + i)  and  b1 = b0 + 4P
// the address is (i < s ? b1 : b0) + (256 - 4 s): the constant folds into the
// instruction's offset field and only the base choice costs a VALU op.  For the
// generated (compile-time) tables "i < s" is a constant lane mask held in an SGPR
// pair, so the choice is a single v_cndmask; the runtime tables compare instead.
// s == 0 is the identity and emits nothing.
struct Lane {
    int i, gb;   // in-group index, group base lane
    int b0, b1;  // bpermute bases (laundered once per iteration so they stay cheap to reuse)
    bool live;   // lane belongs to a syndrome of this batch
};

// lanes [g P, g P + s) of every group g, from group_base (the top lanes with pushed rotations)
template <int P_>
__device__ constexpr unsigned long long lanes_below(int s)
{
    unsigned long long m = 0;
    for (int g = 0; g < 64 / P_; ++g)
        for (int k = 0; k < s; ++k) m |= 1ull << (g * P_ + k);
    return m << group_base<P_>();
}


__device__ __forceinline__ int select_lanes(int a, int b, unsigned long long m)
{
    int r;
    asm("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "s"(m));
    return r;
}

// This lane's in-group index, recomputed from the lane id for compile-time P (so ln.i need not stay
// live across a whole sector loop only for the outputs written after it; it spilled at 96 VGPRs).
template <class SH>
__device__ __forceinline__ int lane_i(const Lane& ln)
{
    if constexpr (kPushRot<SH>() && kGroupBase<SH>() > 0) {
        const int lane = (int)__builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
        if constexpr (2 * SH::kP > 64)
            return lane < kGroupBase<SH>() ? lane : lane - kGroupBase<SH>();  // the group on the top lanes
        else
            return lane < kGroupBase<SH>() ? lane : (lane - kGroupBase<SH>()) % SH::kP;
    } else if constexpr (SH::kStatic)
        return (int)__builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u)) % SH::kP;
    else
        return ln.i;
}

// (Rotation masks made at their use with s_bfm_b64 instead of hoisted constants, which spill into VGPR
// lanes: -3.5 % on the headline, profiles/r05/cmp_mask_remat_headline.txt.)
template <class SH>
__device__ __forceinline__ int rot_addr(const Lane& ln, int s)
{
    int base;
    if constexpr (SH::kStatic && SH::kMaskSelect)
        base = select_lanes(ln.b0, ln.b1, lanes_below<SH::kP>(s));
    else
        base = (ln.i < s) ? ln.b1 : ln.b0;  // loop-invariant per s: hoisted by the compiler
    return base + (256 - 4 * s);
}

template <class SH>
__device__ __forceinline__ int rot_i(int v, const Lane& ln, int s)
{
    if constexpr (kPushRot<SH>()) {
        if (s != 0 && (2 * SH::kP < 64 || s >= SH::kP - 31)) {
            // the same rotation as a push: lane i's value goes to lane (i + s) mod P of its group.  The
            // address is (i < P - s ? b1 : b0) + (256 + 4 s - 4 P): lane gb + i + s or gb + i + s - P, mod 64
            int base;
            if constexpr (SH::kMaskSelect)
                base = select_lanes(ln.b0, ln.b1, lanes_below<SH::kP>(SH::kP - s));
            else
                base = (ln.i < SH::kP - s) ? ln.b1 : ln.b0;  // loop-invariant per s: hoisted by the compiler
            return __builtin_amdgcn_ds_permute(base + (256 + 4 * s - 4 * SH::kP), v);
        }
    }
    return s == 0 ? v : bperm_i(rot_addr<SH>(ln, s), v);
}
template <class SH>
__device__ __forceinline__ float rot(float v, const Lane& ln, int s)
{
    return __int_as_float(rot_i<SH>(__float_as_int(v), ln, s));
}
__device__ __forceinline__ int wrap(int x, int P) { return x >= P ? x - P : x; }

// true iff pred holds on every lane of this lane's group [gb, gb+P)
__device__ __forceinline__ bool group_all(bool pred, int gb, int P)
{
    const unsigned long long bad = __ballot(!pred);
    const unsigned long long gm = (P >= 64 ? ~0ull : ((1ull << P) - 1ull)) << gb;
    return (bad & gm) == 0ull;
}
// The same for a shift provider: with compile-time P > 32 a wave holds one group (lanes
// [kGroupBase, kGroupBase + P); the other lanes are never live), so the group mask is a constant rather than a
// per-lane 64-bit value kept live across the whole kernel.
template <class SH>
__device__ __forceinline__ bool group_all_sh(bool pred, const Lane& ln, int P)
{
    if constexpr (SH::kStatic && 2 * SH::kP > 64) {
        constexpr unsigned long long gm = (SH::kP >= 64 ? ~0ull : ((1ull << SH::kP) - 1ull)) << kGroupBase<SH>();
        return (__ballot(!pred) & gm) == 0ull;
    } else {
        return group_all(pred, ln.gb, P);
    }
}

__host__ __device__ __forceinline__ bool outside(float x) { return !(x > 0.01f && x < 0.99f); }
// AND of two wave-uniform (scalar) conditions without a short-circuit branch
__device__ __forceinline__ bool band(bool a, bool b) { return (int)a & (int)b; }

// ---- correctly rounded division, with a short path -----------------------------
// hipcc lowers the IEEE fp32 quotient n / d to 11 instructions:
//   D = div_scale(d), r = rcp(D), e = fma(-D, r, 1), r = fma(e, r, r), N = div_scale(n),
//   q = N r, e = fma(-D, q, N), q = fma(e, r, q), e = fma(-D, q, N), q = div_fmas(e, r, q),
//   q = div_fixup(q, d, n).
// div_scale only rescales (by 2^64) when an operand or the quotient is near the ends of
// the exponent range, and div_fixup only changes special cases (0, inf, NaN, over/underflow);
// with d in [2^-98, 2] and n = +0 or n in [2^-98, d] neither fires.  On that domain the short
// form below (6 instructions) is the correctly rounded quotient:
//   y1 = fma(1 - d rcp(d), rcp(d), rcp(d)) is RN(1/d) -- checked for EVERY d in [2^-98, 2)
//   (all significands, every exponent; d = 2 is exact) by tools/kbench/div_check.hip;
//   q0 = RN(n y1) is then within one ulp of n/d, the residual fma(-d, q0, n) is exact, and
//   by Markstein's theorem q1 = fma(r, y1, q0) = RN(n/d).  The same tool also compares it with
//   the IEEE quotient on 8.6e9 random and near-midpoint pairs of the domain: no difference
//   (profiles/r01/session5/div_check.json).
// The guard below is evaluated for a whole column of divisions and the short path taken only
// when every live lane of the wave passes it; otherwise the full sequence runs.
// (Without the refinement -- q0 = n rcp(d), one residual correction with rcp(d) -- the form is 4
// instructions and would take 9 % of a soft iteration's VALU, but it is not correctly rounded:
// tools/kbench/div4_check.hip finds 47 045 of the 2^46 significand pairs differing from the IEEE
// quotient.)
__device__ __forceinline__ float div_short(float n, float d)
{
    const float y0 = __builtin_amdgcn_rcpf(d);
    const float e = __builtin_fmaf(-d, y0, 1.0f);
    const float y1 = __builtin_fmaf(e, y0, y0);
    const float q0 = n * y1;
    const float r = __builtin_fmaf(-d, q0, n);
    return __builtin_fmaf(r, y1, q0);
}
// n = t1 >= 0 and d = t0 + t1 with t0, t1 products of probabilities in [0, 1] (so d <= 2):
// short path valid iff d >= 2^-98 (a float compare: NaN fails) and n is +0 or >= 2^-98
// (bit patterns of non-negative floats order like unsigned integers; +0 - 1 wraps to the top).
__device__ __forceinline__ bool div_short_ok(float n, float d)
{
    return (d >= 0x1p-98f) & ((__float_as_uint(n) - 1u) >= (__float_as_uint(0x1p-98f) - 1u));
}

// Guard-free short division by scaling (BpArgs::scaled).  Every check->variable message is g =
// RN(0.5 + h t), h = +-1/2, t a float in [-1, 1] (check_pass, table0_entry, or exactly 0 / 1 from the
// hard forms): g = 0 exactly when h t = -1/2, and otherwise 0.5 + h t >= 0.5 (1 - (1 - 2^-24)) = 2^-25,
// so every nonzero g is >= 2^-25, and every nonzero 1 - g is >= 2^-24 (g <= 1 - 2^-24 when g < 1).  A
// numerator with F factors, p' g_a g_b ..., is then +0 or >= p' 2^-25F, a denominator +0 or >=
// (1 - p') 2^-24F: for F <= 4 and p' >= 2^-20 both are normal (>= 2^-120, resp. 2^-97) at every step of
// their folds, and every quotient n / d >= n / 2 is normal too.  Folding from 2^32 p' and 2^32 (1 - p')
// instead therefore gives exactly 2^32 times every fold value (scaling by a power of two commutes with
// rounding in the normal range; nothing reaches 2^33) and the same quotient n / d, on operands
// 2^32 n >= 2^-88 (or +0), 2^32 d in [2^-65, 2^33]: the short form's reciprocal y1 = RN(1/d) depends only
// on d's significand (tools/kbench/div_check.hip verified every one), its residual fma(-d, q0, n) is
// exact (normal, >= 2^-111), so Markstein's correction again gives RN(n / d) -- without any guard.  NaN
// operands give NaN through both forms, +0 numerators +0, 0 / 0 NaN.  F = 5 (the last iteration of a
// five-row sector) keeps the guarded form (its numerators can reach p' 2^-125, subnormal in the
// reference's own fold).  scaled_ok: the launch-wide condition, evaluated on the host (other p' take
// the IEEE division in those passes).
__host__ __device__ inline bool scaled_ok(float pp) { return pp >= 0x1p-20f && pp <= 0.5f; }

// ---- one sector (X: R = J, Z: R = K) ------------------------------------
// EqNodeUpdate (DecoderCPU.h:150-186) for checks (r, i), r = 0..R-1: lane-local.
template <int R, int L, bool RB = false>
__device__ __forceinline__ void check_pass(float (&msg)[R][L], uint32_t sbits)
{
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const float h = ((sbits >> r) & 1u) ? 0.5f : -0.5f;
        float av[L];
#pragma unroll
        for (int l = 0; l < L; ++l) av[l] = __builtin_fmaf(-2.0f, msg[r][l], 1.0f);
        if constexpr (L == 1) {
            msg[r][0] = __builtin_fmaf(h, 1.0f, 0.5f);
        } else {
            float out[L];
            float t0 = av[1];  // 1.0f * a1 == a1
#pragma unroll
            for (int k = 2; k < L; ++k) t0 = t0 * av[k];
            out[0] = __builtin_fmaf(h, t0, 0.5f);
            float pre = av[0];
#pragma unroll
            for (int x = 1; x < L; ++x) {
                float t = pre;
#pragma unroll
                for (int k = x + 1; k < L; ++k) t = t * av[k];
                out[x] = __builtin_fmaf(h, t, 0.5f);
                if (x + 1 < L) pre = pre * av[x];
            }
#pragma unroll
            for (int l = 0; l < L; ++l) msg[r][l] = out[l];
        }
        if constexpr (RB) __builtin_amdgcn_sched_barrier(0);  // rows one at a time (Tune::kRowBarrier)
    }
}

// EqNodeUpdate when every incoming message is exactly +0 or 1.0 (a "hard" sector): then every
// factor 1 - 2q is exactly +1 or -1, every leave-one-out product is exactly (-1)^(ones among
// the others), and 0.5 * (1 -/+ t) is exactly +0 or 1.0 -- i.e. the output is the parity
// s XOR (ones among the others), which on the bit patterns {0, 0x3F800000} is an XOR.
// Bit-identical to check_pass on such inputs.
template <int R, int L>
__device__ __forceinline__ void check_pass_hard(float (&msg)[R][L], uint32_t sbits)
{
    // laundered: the R row seeds below are recomputed at each use (2 VALU each) instead of being
    // hoisted out of the iteration loop into R live registers (which spilled at 96 VGPRs)
    asm volatile("" : "+v"(sbits));
#pragma unroll
    for (int r = 0; r < R; ++r) {
        uint32_t x = ((sbits >> r) & 1u) ? 0x3F800000u : 0u;
#pragma unroll
        for (int l = 0; l < L; ++l) x ^= __float_as_uint(msg[r][l]);
#pragma unroll
        for (int l = 0; l < L; ++l) msg[r][l] = __uint_as_float(x ^ __float_as_uint(msg[r][l]));
    }
}

// The hard decision of one variable (DecoderCPU.h:354-373): some of its R messages q >= 0.5f.  (As the
// maximum of the R messages by v_max3_f32 -- NaN-safe, the messages are probabilities or quiet NaNs --
// and one compare: -0.6 .. +1.1 % on config 5, profiles/r06/ab/cmp_hd_max.txt; not taken.)
template <int R>
__device__ __forceinline__ bool any_ge_half(const float (&q)[R])
{
    bool hd = false;
#pragma unroll
    for (int r = 0; r < R; ++r) hd |= (q[r] >= 0.5f);
    return hd;
}

// Zero numerators.  A numerator n = +0 is harmless: then d = P0 = (1 - p') prod (1 - g_k) over F
// factors, where every 1 - g_k is exact and either 0 or >= 2^-24 (g <= 1 - 2^-24 when g < 1), so
// d is either 0 (0 / 0: NaN from both sequences) or >= (1 - p') 2^(-24 F), which for p' <= 1/2 and
// F <= 5 is >= 2^-121: rcp(d) is finite and the short form returns +0, as +0 / d does.  So with
// zero_ok the guard only has to exclude numerators in (0, 2^-98) (d >= n covers the rest).
template <int R, bool LAST>
__device__ __forceinline__ bool zero_ok(float pp)
{
    constexpr int F = LAST ? R : R - 1;  // factors in a numerator
    return F <= 5 && pp >= 0.0f && pp <= 0.5f;
}

// Syndrome stop with one group per wave (compile-time P > 32): the var pass stores its outgoing messages
// in the variable view (msg[r][l] = variable (l, .)'s message on edge r) instead of rotating each back to
// its check at once.  The stop test needs only the decisions, and the post-processing of a stopped
// sector only the decisions and "every message outside (0.01, 0.99)", which does not depend on the
// layout; so the R L return rotations run (return_pass) only when the sector goes on (or its final
// messages are requested).  At low p most listed sectors stop after one soft iteration.
template <bool HD, class SH>
constexpr bool defer_return()
{
    if constexpr (SH::kStatic) return HD && 2 * SH::kP > 64;
    else return false;
}

// The check view of the messages a deferring var pass left in the variable view.
template <int R, int L, int SEC, class SH>
__device__ __forceinline__ void return_pass(const BpArgs& a, float (&msg)[R][L], Lane& ln)
{
    const int P = SH::P(a);
    const int* et = SH::template table<SEC>(a);
    if constexpr (SH::kMaskSelect) asm volatile("" : "+v"(ln.b0), "+v"(ln.b1));
#pragma unroll
    for (int l = 0; l < L; ++l)
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const int sh = SH::template shift<SEC, L>(et, r, l);
            msg[r][l] = rot<SH>(msg[r][l], ln, sh == 0 ? 0 : P - sh);
        }
}

// VarNodeUpdate (DecoderCPU.h:188-229) for variables (l, i): gather the R incoming
// check messages by forward rotation, update, scatter back by the inverse rotation.
// LAST: the final iteration includes the self message (DecoderCPU.h:216).
// Returns the hard-decision mask (bit l) of the new messages when HD is set.
// hard: in = every incoming (check->variable) message is exactly +0 or 1.0; out = so is every
// outgoing one (only tracked when the hard-message paths are enabled for this launch).
// vagree (out, meaningful when hard comes out set): every variable's R outgoing messages are
// equal (on every live lane), i.e. the new state passes var_pass_agree's test as it stands.
// CG: columns per division guard.  The guard chooses, wave-uniformly, between the short and the
// IEEE division sequence, and each such branch ends a basic block; with CG columns per guard the
// compiler schedules CG columns' products, divisions and rotations as one straight-line block.
// CG > 1 requires soft inputs (hard == false on entry): the hard-input agreement shortcut below
// works column by column.
// SOFT_IN: the caller knows the inputs are soft, so no column takes the agreeing-inputs branch (soft
// passes are straight-line code per column group: P61 headline +3.6 %, P7 +1 %;
// profiles/r03/cmp_soft_straight_*.txt).
template <int R, int L, int SEC, bool LAST, bool HD, class SH, class TU, int CG = 1, bool SOFT_IN = false>
__device__ __forceinline__ uint32_t var_pass(const BpArgs& a, float (&msg)[R][L], const Lane& ln, float pp,
                                             float one_minus_pp, bool& hard, bool& vagree, bool track = true)
{
    static_assert(L % CG == 0, "column groups must tile the L columns");
    const bool hard_in = !SOFT_IN && CG == 1 && hard;
    bool vsame = true;  // this lane's variables: all R outputs equal (float compare: NaN is unequal)
    uint32_t soft_bits = 0;  // OR of bits(q - q*q) over the outputs: 0 iff all are 0 or 1
    constexpr int F = LAST ? R : R - 1;  // factors per fold
    constexpr bool kScalable = TU::kFastDiv && F <= 4;
    const bool scaled = kScalable && a.scaled;  // wave-uniform (see scaled_ok)
    const float fold0 = scaled ? one_minus_pp * 0x1p32f : one_minus_pp, fold1 = scaled ? pp * 0x1p32f : pp;
    const int P = SH::P(a);
    const int* et = SH::template table<SEC>(a);
    uint32_t hdmask = 0;
    // TU::kPipeline = D: the gathers of columns l + 1 .. l + D are in flight while column l is
    // computed, so their ds_bpermute latency hides behind column l's arithmetic in the same wave
    // (the per-group uniform branches below end basic blocks, so the compiler cannot do this).
    constexpr int D = TU::kPipeline > 0 ? (TU::kPipeline < L ? TU::kPipeline : L - 1) : 0;
    constexpr int ND = LAST ? 1 : R;  // distinct outgoing messages per variable (LAST: one, shared)
    float gq[D > 0 ? D : 1][R];  // gq[k]: gathers of column l + 1 + k
    if constexpr (D > 0) {
#pragma unroll
        for (int k = 0; k < D; ++k)
#pragma unroll
            for (int r = 0; r < R; ++r) gq[k][r] = rot<SH>(msg[r][k], ln, SH::template shift<SEC, L>(et, r, k));
    }
#pragma unroll
    for (int l0 = 0; l0 < L; l0 += CG) {
        float gv[CG][R], qv[CG][R];
#pragma unroll
        for (int c = 0; c < CG; ++c) {
            const int l = l0 + c;
            if constexpr (D > 0) {
#pragma unroll
                for (int r = 0; r < R; ++r) gv[c][r] = gq[0][r];
#pragma unroll
                for (int k = 0; k + 1 < D; ++k)
#pragma unroll
                    for (int r = 0; r < R; ++r) gq[k][r] = gq[k + 1][r];
                if (l + D < L) {
#pragma unroll
                    for (int r = 0; r < R; ++r)
                        gq[D - 1][r] = rot<SH>(msg[r][l + D], ln, SH::template shift<SEC, L>(et, r, l + D));
                }
            } else {
#pragma unroll
                for (int r = 0; r < R; ++r) gv[c][r] = rot<SH>(msg[r][l], ln, SH::template shift<SEC, L>(et, r, l));
            }
        }
        // hard inputs: q_j = P1 / (P0 + P1) with every factor 0 or 1 is exactly the common value
        // when all R inputs agree (all 1: p'/p' = 1; all 0: +0/(1-p') = +0); columns where some
        // variable's inputs disagree (0/0 = NaN) take the arithmetic path below
        bool done = false;
        if constexpr (TU::kSaturate && CG == 1) {
            if (hard_in && (LAST || R >= 2)) {
                const uint32_t x0 = __float_as_uint(gv[0][0]);
                bool same = true;
#pragma unroll
                for (int r = 1; r < R; ++r) same &= __float_as_uint(gv[0][r]) == x0;
                if (all_live_sh<SH>(same, ln.live)) {
#pragma unroll
                    for (int r = 0; r < R; ++r) qv[0][r] = gv[0][0];
                    done = true;
                }
            }
        }
        if (!done) {
            // numerators / denominators of the outgoing messages, left folds in ascending k
            float num[CG][ND], den[CG][ND];
#pragma unroll
            for (int c = 0; c < CG; ++c) {
                float bv[R];
#pragma unroll
                for (int r = 0; r < R; ++r) bv[r] = 1.0f - gv[c][r];
                if constexpr (LAST) {
                    float P0 = fold0, P1 = fold1;
#pragma unroll
                    for (int k = 0; k < R; ++k) { P0 = P0 * bv[k]; P1 = P1 * gv[c][k]; }
                    num[c][0] = P1;
                    den[c][0] = P0 + P1;
                } else {
                    float pre0 = fold0, pre1 = fold1;
#pragma unroll
                    for (int j = 0; j < R; ++j) {
                        float t0 = pre0, t1 = pre1;
#pragma unroll
                        for (int k = j + 1; k < R; ++k) { t0 = t0 * bv[k]; t1 = t1 * gv[c][k]; }
                        num[c][j] = t1;
                        den[c][j] = t0 + t1;
                        if (j + 1 < R) { pre0 = pre0 * bv[j]; pre1 = pre1 * gv[c][j]; }
                    }
                }
            }
            float qd[CG][ND];
            bool zero = false, fast = false;
            if constexpr (TU::kZeroSkip) {
                uint32_t nb = 0;
                bool dpos = true;
#pragma unroll
                for (int c = 0; c < CG; ++c)
#pragma unroll
                    for (int j = 0; j < ND; ++j) {
                        nb |= __float_as_uint(num[c][j]);
                        dpos &= den[c][j] > 0.0f;
                    }
                zero = all_live(nb == 0u && dpos, ln.live);
            }
            if constexpr (kScalable) {
                fast = scaled;  // no guard (scaled folds); other p' take the IEEE division
            } else if constexpr (TU::kFastDiv) {
                // numerators outside (0, 2^-98): minima of their bit patterns minus one, +0 wrapping to
                // the top.  The guard assumes every message is a probability in [0, 1] (true by induction
                // for such p', DecoderCPU.h:135-229) and needs zero_ok (p' <= 1/2, a wave-uniform AND, no
                // branch); other p' (p > 3/4, never a decoding regime) always take the IEEE division.
                uint32_t nm = 0xFFFFFFFFu;
#pragma unroll
                for (int c = 0; c < CG; ++c)
#pragma unroll
                    for (int j = 0; j < ND; ++j) nm = min(nm, __float_as_uint(num[c][j]) - 1u);
                fast = band(all_live_sh<SH>(nm >= __float_as_uint(0x1p-98f) - 1u, ln.live), zero_ok<R, LAST>(pp));
            }
            if (zero) {
#pragma unroll
                for (int c = 0; c < CG; ++c)
#pragma unroll
                    for (int j = 0; j < ND; ++j) qd[c][j] = 0.0f;
            } else if (fast) {
#pragma unroll
                for (int c = 0; c < CG; ++c)
#pragma unroll
                    for (int j = 0; j < ND; ++j) qd[c][j] = div_short(num[c][j], den[c][j]);
            } else {
#pragma unroll
                for (int c = 0; c < CG; ++c)
#pragma unroll
                    for (int j = 0; j < ND; ++j) qd[c][j] = num[c][j] / den[c][j];
            }
            if constexpr (TU::kSaturate) {
                if (!zero && track) {
#pragma unroll
                    for (int c = 0; c < CG; ++c) {
#pragma unroll
                        for (int j = 0; j < ND; ++j)
                            soft_bits |= __float_as_uint(__builtin_fmaf(-qd[c][j], qd[c][j], qd[c][j]));
#pragma unroll
                        for (int j = 1; j < ND; ++j) vsame &= qd[c][j] == qd[c][0];
                    }
                }
            }
#pragma unroll
            for (int c = 0; c < CG; ++c)
#pragma unroll
                for (int r = 0; r < R; ++r) qv[c][r] = qd[c][LAST ? 0 : r];
        }  // !done
#pragma unroll
        for (int c = 0; c < CG; ++c) {
            const int l = l0 + c;
            if constexpr (HD) hdmask |= (uint32_t)any_ge_half<R>(qv[c]) << l;
#pragma unroll
            for (int r = 0; r < R; ++r) {
                const int sh = SH::template shift<SEC, L>(et, r, l);
                msg[r][l] = defer_return<HD, SH>() ? qv[c][r] : rot<SH>(qv[c][r], ln, sh == 0 ? 0 : P - sh);
            }
        }
        if constexpr (TU::kSaturate) {
            // a soft output in the first column group already decides that the sector does not turn hard in
            // this pass: the remaining columns skip the hard-state test (its fma and OR per message, compare
            // per variable), which otherwise costs ~9 % of a soft pass (headline +1.1 %, 50 fixed iterations
            // at p = 0.1 +7.7 %, P7 +2.6 %; profiles/r06/ab/cmp_track_early.txt)
            if (l0 == 0 && track && !all_live_sh<SH>(soft_bits == 0u, ln.live)) track = false;
        }
        // a scheduling barrier after each column group: the machine scheduler otherwise hoists work
        // across columns into more live registers (P61 headline +2.8 %, profiles/r03/cmp_col_barrier_*.txt)
        __builtin_amdgcn_sched_barrier(0);
    }
    if constexpr (TU::kSaturate) {
        const bool forms = track && (a.hardPaths & QEC_HP_FORMS) && hard_ok(pp);
        hard = forms && all_live_sh<SH>(soft_bits == 0u, ln.live);
        vagree = hard && all_live_sh<SH>(vsame, ln.live);
    }
    return hdmask;
}

// VarNodeUpdate on a hard sector whose R incoming messages agree for every variable (every
// live lane): then each outgoing message q_j = P1 / (P0 + P1) is the common value (all 1:
// p'/p' = 1; all 0: +0/(1-p') = +0; LAST or R >= 2, see var_pass), so the message sent back on
// edge (r, l) equals the one that arrived on it and the check-view registers are already the
// result.  Gathers every edge into the variable view and tests the agreement; returns false
// (registers untouched) when some variable's inputs differ, and the caller runs var_pass.
template <int R, int L, int SEC, bool HD, class SH>
__device__ __forceinline__ bool var_pass_agree(const BpArgs& a, const float (&msg)[R][L], const Lane& ln,
                                               uint32_t& hdmask)
{
    const int* et = SH::template table<SEC>(a);
    bool same = true;
    uint32_t hd = 0;
#pragma unroll
    for (int l = 0; l < L; ++l) {
        const uint32_t x0 = __float_as_uint(rot<SH>(msg[0][l], ln, SH::template shift<SEC, L>(et, 0, l)));
#pragma unroll
        for (int r = 1; r < R; ++r)
            same &= __float_as_uint(rot<SH>(msg[r][l], ln, SH::template shift<SEC, L>(et, r, l))) == x0;
        if constexpr (HD) hd |= (uint32_t)(x0 == 0x3F800000u) << l;  // q >= 0.5f <=> q == 1.0f here
    }
    hdmask = hd;
    return all_live_sh<SH>(same, ln.live);
}

// CheckConvergence (DecoderCPU.h:231-246) on this lane's edges.
template <int R, int L>
__device__ __forceinline__ bool lane_converged(const float (&msg)[R][L])
{
    bool ok = true;
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
        for (int l = 0; l < L; ++l) ok &= outside(msg[r][l]);
    return ok;
}

// Syndrome of the hard decision (var view, bit l of hdmask) equals the input syndrome
// on this lane's checks (r, i): GetSyndromeX/Z of Decode (DecoderCPU.h:380-384).
template <int R, int L, int SEC, class SH>
__device__ __forceinline__ bool lane_syndrome_ok(const BpArgs& a, uint32_t hdmask, uint32_t sbits, const Lane& ln)
{
    const int P = SH::P(a);
    const int* et = SH::template table<SEC>(a);
    bool match = true;
#pragma unroll
    for (int r = 0; r < R; ++r) {
        uint32_t x = 0;
#pragma unroll
        for (int l = 0; l < L; ++l) {
            const int sh = SH::template shift<SEC, L>(et, r, l);
            x ^= ((uint32_t)rot_i<SH>((int)hdmask, ln, sh == 0 ? 0 : P - sh) >> l) & 1u;
        }
        match &= (x == ((sbits >> r) & 1u));
        // one row's L rotations in flight at a time: all R L at once (the scheduler's choice) held
        // R L results live beside the sector's messages and spilled the syndrome-stop kernels
        __builtin_amdgcn_sched_barrier(0);
    }
    return match && !(sbits & kNonBinary);
}

// The same test for a whole group.  (From ballots and scalar rotations instead of ds_bpermute: 5-8 %
// slower, SALU-bound; profiles/r05/README.md.)
template <int R, int L, int SEC, class SH>
__device__ __forceinline__ bool group_syndrome_ok(const BpArgs& a, uint32_t hdmask, uint32_t sbits, const Lane& ln)
{
    return group_all_sh<SH>(lane_syndrome_ok<R, L, SEC, SH>(a, hdmask, sbits, ln), ln, SH::P(a));
}

// Whether a hard sector first tries the whole-sector agreement test (var_pass_agree, the entry to
// the cycle jump).  Not for the syndrome stop rule: there it costs more than it saves -- with it the
// P61 kernel spills at 128 VGPRs, without it P61 decodes 4-15 % faster at p = 0.1 .. 0.002 and P7
// 7 % (profiles/r02/syn_variants_r02s3h.txt); sectors that never
// satisfy their syndrome then run their hard iterations instead of jumping (same outputs).
// The list-mode kernels (ListTune: their own, lower occupancy, so no spills) take it: they decode the
// few sectors the triage passed on, latency-bound, and the sectors that never satisfy their syndrome
// would otherwise run all their hard iterations to the cap one by one.
template <int STOP, class TU>
constexpr bool kAgree()
{
    return STOP != QEC_STOP_SYNDROME || TU::kAgreeSyn;
}

// Row 0 of the syndrome test is lane-local when every block of row 0 has rotation 0 (the relabelled
// compile-time tables: lane i of the variable view holds exactly the L variables of check (0, i)).
template <int SEC, int L, class SH>
constexpr bool kRow0Local()
{
    if constexpr (!SH::kStatic) {
        return false;
    } else {
        for (int l = 0; l < L; ++l)
            if (SH::template shift<SEC, L>(nullptr, 0, l) != 0) return false;
        return true;
    }
}

// The syndrome stop's repeated-decision skip (iteration) for L columns (the never-seen marker ~0u is no
// decision mask when L < 32)
template <int L>
constexpr bool kSkipSeen() { return L < 32; }

// One BP iteration; returns true if this group stops after it.
// hard: every variable->check message of this sector is exactly +0 or 1.0 (wave-uniform).
// agreed: set when the iteration took the agreement path (hard sector, every variable's inputs
// equal), i.e. it mapped msg to check_pass_hard(msg) (wave-uniform).
// vagree: the new state is hard and each variable's R messages are equal (set on the agreement
// path, where the new state passed that test; tracked by var_pass otherwise).
template <int R, int L, int SEC, int STOP, bool LAST, class SH, class TU>
__device__ __forceinline__ bool iteration(const BpArgs& a, float (&msg)[R][L], uint32_t sbits, int n, Lane& ln,
                                          float pp, float one_minus_pp, bool& hard, bool& agreed, bool& vagree,
                                          uint32_t& hd_out, uint32_t (&seen)[2])
{
    const int P = SH::P(a);
    // launder the permute bases so their per-rotation selects are recomputed inside the
    // loop instead of being hoisted into ~2 R L live registers
    if constexpr (SH::kMaskSelect) asm volatile("" : "+v"(ln.b0), "+v"(ln.b1));
    constexpr bool HD = STOP == QEC_STOP_SYNDROME;
    uint32_t hdmask = 0;
    agreed = false;
    vagree = false;
    bool var_layout = defer_return<HD, SH>();  // the messages are left in the variable view (defer_return)
    if (TU::kSaturate && hard) {
        check_pass_hard<R, L>(msg, sbits);  // outputs are hard too: hard stays set for the var pass
        agreed = kAgree<STOP, TU>() && (LAST || R >= 2) && var_pass_agree<R, L, SEC, HD, SH>(a, msg, ln, hdmask);
        if (agreed) {
            vagree = true;
            var_layout = false;  // the agreement path leaves the check-view registers as they are
        } else {
            // (without the agreement test, a pass whose every column took the agreeing-inputs shortcut could
            // count as the agreement path: 0-6 % slower, profiles/r05/README.md)
            hdmask = var_pass<R, L, SEC, LAST, HD, SH, TU>(a, msg, ln, pp, one_minus_pp, hard, vagree, true);
        }
    } else {
        check_pass<R, L, TU::kRowBarrier>(msg, sbits);
        // the hard-state test is skipped in the first kTrackFrom iterations (they essentially never end
        // hard; skipping only delays the exact hard forms, never changes a bit), and not at all when the
        // hard-message forms are off (QEC_OPT_HARD_PATHS = 0): the test only feeds them (var_pass returns
        // hard = false either way).  hard == false here, so the soft inputs allow column groups and a
        // straight-line pass (var_pass's CG, SOFT_IN).  (One division branch per pass instead of per column
        // group: P61 2x slower, profiles/r03/cmp_soft_straight_*.txt.)
        constexpr int CG = col_group<TU, L>();
        const bool track = (LAST || n >= kTrackFrom) && (a.hardPaths & QEC_HP_FORMS);
        hdmask = var_pass<R, L, SEC, LAST, HD, SH, TU, CG, true>(a, msg, ln, pp, one_minus_pp, hard, vagree, track);
    }
    if constexpr (STOP == QEC_STOP_REF) {
        if (n % 10 == 0) return group_all_sh<SH>(lane_converged<R, L>(msg), ln, P);  // DecoderCPU.h:287-290
    } else if constexpr (STOP == QEC_STOP_SYNDROME) {
        hd_out = hdmask;  // the hard decision of the new state (what the post-processing would compute)
        // The test is a function of the group's hard decisions (and its fixed syndrome): if they equal,
        // group-wide, one of the last two tested decisions, it fails again -- an active group has failed
        // every test so far.  Skipped then (sectors that never satisfy their syndrome mostly repeat one
        // decision or alternate between two).  seen[] holds whole-group tested states: it is updated
        // group-uniformly (kept when the decision is seen[0], else pushed).
        const bool same0 = kSkipSeen<L>() && group_all_sh<SH>(hdmask == seen[0], ln, P);
        bool skip = false;
        if constexpr (kSkipSeen<L>()) skip = all_live_sh<SH>(same0 || group_all_sh<SH>(hdmask == seen[1], ln, P), ln.live);
        // Row 0 first where it is lane-local (kRow0Local): a group that fails there fails the test, so
        // when every active group does, rows 1 .. R - 1 (their rotations) are not needed
        bool stop = false;
        bool row0_fails = false;
        if constexpr (kRow0Local<SEC, L, SH>()) {
            if (!skip) {
                const bool ok0 = ((__popc(hdmask) ^ sbits) & 1u) == 0u && !(sbits & kNonBinary);
                row0_fails = all_live_sh<SH>(!group_all_sh<SH>(ok0, ln, P), ln.live);
            }
        }
        if (!skip && !row0_fails) {
            // launder the bases again: the test's rotations are var_pass's return rotations, whose
            // addresses would otherwise be kept live across the whole var pass for reuse here
            if constexpr (SH::kMaskSelect) asm volatile("" : "+v"(ln.b0), "+v"(ln.b1));
            stop = group_syndrome_ok<R, L, SEC, SH>(a, hdmask, sbits, ln);
        }
        if (kSkipSeen<L>() && !same0) {
            seen[1] = seen[0];
            seen[0] = hdmask;
        }
        // a deferring pass: the check view is needed when the sector goes on to another iteration (one
        // group per wave, so stop is wave-uniform) or its final messages are requested
        if (var_layout && (a.q != nullptr || (!LAST && !stop))) return_pass<R, L, SEC, SH>(a, msg, ln);
        return stop;
    }
    return false;
}

// ---- iteration 0 by table --------------------------------------------------------
// Iteration 0 of BeliefPropogation starts from q = p' on every edge (DecoderCPU.h:265-267).  So
// every factor of every check is a = 1 - 2p', every leave-one-out product is the same left fold
// t = a^(L-1), and each check sends r0 = 0.5 (1 - t) or r1 = 0.5 (1 + t) on all its edges, chosen
// by its syndrome bit.  A variable's R outputs then depend only on the R-bit pattern of its
// checks' syndrome bits:  q0[pattern][j] = P1 / (P0 + P1),  P1 = p' prod_{k != j} r_{bit k},
// P0 = (1 - p') prod_{k != j} (1 - r_{bit k}), ascending k (DecoderCPU.h:210-225).  The workgroup
// builds that 2^R x R table once per sector with exactly the operations check_pass / var_pass
// would run (so the same bits), and iteration 0 becomes gathers of syndrome bits and table reads.
// Not used when iteration 0 is the last one (N = 1: the self message is included).
template <int R, int L>
__host__ __device__ inline float table0_entry(float pp, int e)
{
    const float a = __builtin_fmaf(-2.0f, pp, 1.0f);  // 1.0f - 2.0f*q, as check_pass
    float t = 1.0f;
    if constexpr (L >= 2) {
        t = a;  // 1.0f * a
#pragma unroll
        for (int k = 2; k < L; ++k) t = t * a;
    }
    const float r0 = __builtin_fmaf(-0.5f, t, 0.5f), r1 = __builtin_fmaf(0.5f, t, 0.5f);
    const int idx = e / R, j = e - (e / R) * R;
    float P0 = 1.0f - pp, P1 = pp;
#pragma unroll
    for (int k = 0; k < R; ++k) {
        if (k == j) continue;
        const float g = ((idx >> k) & 1) ? r1 : r0;
        P0 = P0 * (1.0f - g);
        P1 = P1 * g;
    }
    return P1 / (P0 + P1);
}

// Bit idx of hdpat: a variable whose R checks have syndrome pattern idx decides 1 after iteration 0
// (some table entry >= 0.5); of cvpat: its R messages all lie outside (0.01, 0.99).  Called with every
// lane of the wave active (the ballots must see lanes 0 .. 2^R - 1).
template <int R>
__device__ __forceinline__ void pattern_masks(const float* __restrict__ tab, unsigned long long& hdpat,
                                              unsigned long long& cvpat)
{
    const int li = (int)__lane_id();
    bool hp = false, cp = true;
    if (li < (1 << R)) {
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const float t = tab[li * R + r];
            hp |= t >= 0.5f;
            cp &= outside(t);
        }
    }
    hdpat = __ballot(li < (1 << R) && hp);
    cvpat = __ballot(li < (1 << R) && cp);
}

// GO (list mode): the sector is known to go on past iteration 0 -- the triage listed it because its
// iteration-0 hard decision fails the syndrome (triage.hip) -- so only the messages are formed.
template <int R, int L, int SEC, int STOP, class SH, bool GO = false>
__device__ __forceinline__ bool iteration0(const BpArgs& a, float (&msg)[R][L], uint32_t sbits, const Lane& ln,
                                           const float* __restrict__ tab, uint32_t& hd_out, bool& cv_out,
                                           bool& msg_out, unsigned long long hdpat, unsigned long long cvpat)
{
    const int P = SH::P(a);
    const int* et = SH::template table<SEC>(a);
    constexpr bool HD = STOP == QEC_STOP_SYNDROME && !GO;
    msg_out = true;
    if constexpr (HD && L * R <= 64) {
        // Syndrome stop: a variable's hard decision after this iteration, and whether its R
        // messages lie outside (0.01, 0.99), depend only on its syndrome pattern idx, so they come
        // from two 2^R-bit masks before any message is formed; the messages themselves (table
        // reads and return rotations) are only built when some group goes on -- a group that
        // stops here needs just those two bits for its outputs (decode_sector; hdpat / cvpat from
        // pattern_masks).
        uint64_t idxs = 0;
        uint32_t hdmask = 0;
        bool cv = true;
#pragma unroll
        for (int l = 0; l < L; ++l) {
            int idx = 0;
#pragma unroll
            for (int r = 0; r < R; ++r)
                idx |= ((rot_i<SH>((int)sbits, ln, SH::template shift<SEC, L>(et, r, l)) >> r) & 1) << r;
            idxs |= (uint64_t)idx << (R * l);
            hdmask |= (uint32_t)((hdpat >> idx) & 1ull) << l;
            cv &= ((cvpat >> idx) & 1ull) != 0ull;
        }
        const bool stop = group_syndrome_ok<R, L, SEC, SH>(a, hdmask, sbits, ln);
        hd_out = hdmask;
        cv_out = cv;
        msg_out = a.q != nullptr || __any(ln.live && !stop);  // q_final reads the messages
        if (msg_out) {
#pragma unroll
            for (int l = 0; l < L; ++l) {
                const int idx = (int)((idxs >> (R * l)) & ((1u << R) - 1u));
#pragma unroll
                for (int r = 0; r < R; ++r) {
                    const int sh = SH::template shift<SEC, L>(et, r, l);
                    msg[r][l] = rot<SH>(tab[idx * R + r], ln, sh == 0 ? 0 : P - sh);
                }
            }
        }
        return stop;
    }
    uint32_t hdmask = 0;
#pragma unroll
    for (int l = 0; l < L; ++l) {
        int idx = 0;  // syndrome bits of this variable's R checks (var view, row r -> bit r)
#pragma unroll
        for (int r = 0; r < R; ++r)
            idx |= ((rot_i<SH>((int)sbits, ln, SH::template shift<SEC, L>(et, r, l)) >> r) & 1) << r;
        float qv[R];
#pragma unroll
        for (int r = 0; r < R; ++r) qv[r] = tab[idx * R + r];
        if constexpr (HD) hdmask |= (uint32_t)any_ge_half<R>(qv) << l;
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const int sh = SH::template shift<SEC, L>(et, r, l);
            msg[r][l] = rot<SH>(qv[r], ln, sh == 0 ? 0 : P - sh);
        }
    }
    if constexpr (STOP == QEC_STOP_REF) {
        return group_all_sh<SH>(lane_converged<R, L>(msg), ln, P);  // n = 0: DecoderCPU.h:287-290
    } else if constexpr (STOP == QEC_STOP_SYNDROME && !GO) {
        hd_out = hdmask;
        return group_syndrome_ok<R, L, SEC, SH>(a, hdmask, sbits, ln);
    }
    return false;
}

// ---- zero syndrome under the fixed / reference stop ----------------------------------
// A sector whose syndrome is zero keeps every edge's message equal to every other's in every iteration:
// every check sees L equal inputs and syndrome 0, every variable R equal inputs, and each update's
// output depends only on those.  So its decode is a scalar recursion, evaluated on the host with the very
// operations of check_pass / var_pass on equal inputs (same IEEE fp32 operations, -ffp-contract=off:
// every leave-one-out product is a left fold of L - 1 equal factors whatever its prefix reuse; the
// numerators and denominators left folds of R - 1, or R in the last iteration, equal factors; the
// division correctly rounded; the hard forms and cycle jump are bit-identical to it).  The outcome --
// decision (every variable the same), convergence and syndrome flags, iteration count -- is the same
// for every zero-syndrome sector of the launch, which then skips its iterations (decode_sector).
constexpr uint32_t kZsValid = 1u << 31;
template <int R, int L>
uint32_t zero_outcome(float pp, int N, int stop)
{
    if (!(pp > 0.0f && pp < 1.0f) || N < 2 || N > 0xFFFF || stop == QEC_STOP_SYNDROME || QEC_PHASE_STATS)
        return 0u;
    float q = table0_entry<R, L>(pp, 0);  // iteration 0 (syndrome pattern 0), as iteration0
    int it = 1;
    const float one_minus_pp = 1.0f - pp;
    if (!(stop == QEC_STOP_REF && outside(q))) {  // DecoderCPU.h:287-290 at n = 0
        for (int n = 1; n < N; ++n) {
            const float a = __builtin_fmaf(-2.0f, q, 1.0f);
            float t = 1.0f;
            if (L >= 2) {
                t = a;
                for (int k = 2; k < L; ++k) t = t * a;
            }
            const float g = __builtin_fmaf(-0.5f, t, 0.5f);  // syndrome 0: h = -1/2
            const float b = 1.0f - g;
            const int F = n == N - 1 ? R : R - 1;  // the last iteration includes the self message
            float P0 = one_minus_pp, P1 = pp;
            for (int k = 0; k < F; ++k) {
                P0 = P0 * b;
                P1 = P1 * g;
            }
            q = P1 / (P0 + P1);
            ++it;
            if (stop == QEC_STOP_REF && n % 10 == 0 && outside(q)) break;
        }
    }
    const bool d = q >= 0.5f;
    const bool syn_fail = d && (L & 1);  // every check holds L equal decisions, syndrome 0
    return kZsValid | (uint32_t)d | (uint32_t)!outside(q) << 1 | (uint32_t)syn_fail << 2 | (uint32_t)it << 8;
}

// ---- cycle jump --------------------------------------------------------------
// On a hard sector the agreement path maps the check-view registers q to F(q) = check_pass_hard(q):
// row r becomes q ^ c_r with c_r = s_r ^ XOR_l q[r][l] (on the bit patterns {0, 1.0f}).  Then
//   L even: XOR_l F(q)[r][l] = XOR_l q[r][l], so c_r(F(q)) = c_r(q) and F(F(q)) = q;
//   L odd:  c_r(F(q)) = 0, so F(F(q)) = F(q).
// Call a state "agreeing" if it is hard and every variable's R messages are equal -- exactly the
// test var_pass_agree applies to F(q).  If the state S entering iteration n is agreeing and the
// iteration takes the agreement path (F(S) is agreeing), every later state is F(S) or
// F(F(S)) in {S, F(S)}: each is agreeing, so every later iteration (the last one, with the self
// message, included: see var_pass_agree) is F again, and F^k(F(S)) = F^(k mod 2)(F(S)).  S is
// known to be agreeing when it came from the agreement path, or from a var pass whose outputs
// were all 0/1 and equal per variable (var_pass's vagree).  The stop tests repeat too: the
// syndrome rule tested both states already (S when it was produced, F(S) now) and did not stop;
// the reference rule's convergence test holds on every hard state, so it stops at the next
// n' with n' % 10 == 0.  The sector therefore jumps straight to its last executed iteration:
// same registers, same iteration count, same flags as running the iterations one by one
// (bit-identical).
template <int STOP>
__device__ __forceinline__ int cycle_end(int n, int N)
{
    if constexpr (STOP == QEC_STOP_REF) {
        const int next10 = (n / 10 + 1) * 10;  // DecoderCPU.h:287-290
        return next10 < N - 1 ? next10 : N - 1;
    }
    return N - 1;
}

// Syndrome bits of this lane's checks (r, i), r = 0..R-1, as bit r; kNonBinary when one of the
// lane's syndrome bytes is neither 0 nor 1.
template <int R, int SEC, class SH>
__device__ __forceinline__ uint32_t load_sbits(const BpArgs& a, const Lane& ln, uint32_t b, bool in_range)
{
    const int P = SH::P(a);
    const int m = R * P;
    const uint8_t* __restrict__ s = SEC ? a.sZ : a.sX;
    uint32_t sbits = 0;
    if (in_range) {
        if (a.sbits) {  // bit rows (the Monte-Carlo pipeline's layout)
            const uint32_t* __restrict__ w = reinterpret_cast<const uint32_t*>(s) + (size_t)b * (SEC ? a.wZ : a.wX);
#pragma unroll
            for (int r = 0; r < R; ++r) {
                const int c = r * P + wrap(ln.i + SH::template rowoff<SEC>(a, r), P);
                sbits |= ((w[c >> 5] >> (c & 31)) & 1u) << r;
            }
        } else {
            // the check update takes an entry's truthiness (DecoderCPU.h:178) and the syndrome tests
            // compare the entry exactly (:381): an entry other than 0 / 1 decodes as 1 and sets
            // kNonBinary, which fails every syndrome test of the sector (lane_syndrome_ok)
            uint32_t big = 0;
#pragma unroll
            for (int r = 0; r < R; ++r) {
                const uint32_t v = s[(size_t)b * m + r * P + wrap(ln.i + SH::template rowoff<SEC>(a, r), P)];
                sbits |= (uint32_t)(v != 0u) << r;
                big |= v;
            }
            sbits |= big > 1u ? kNonBinary : 0u;
        }
    }
    return sbits;
}

// ---- decision output ---------------------------------------------------------------
// LDS staging of one wave's decisions for the packed records: G groups of npad = 8 nb bytes
// (a syndrome's n decision bytes, zero-padded to whole 8-byte words).
template <int L, class SH>
constexpr int stage_bytes_per_wave()
{
    if constexpr (SH::kStatic) {
        constexpr int n = L * SH::kP;
        return (64 / SH::kP) * ((n + 7) / 8) * 8;
    } else {
        return 64 * (L + 8);  // G (L P + 7) <= 64 L + 7 G for any P <= 64
    }
}

// Hard decisions of this lane's L variables (bit l of hdmask: variable (l, (i + C[l]) mod P)) to
// eX / eZ bytes, or, for a packed launch, through the wave's LDS stage into the record's nb bytes of
// this sector: lane i of a group packs bytes i, i + P, ... (8 staged bytes each, one 8-byte LDS read).
template <int L, int SEC, class SH>
__device__ __forceinline__ void emit_decisions(const BpArgs& a, const Lane& ln, uint32_t b, bool in_range,
                                               uint32_t hdmask, uint8_t* __restrict__ stage)
{
    const int P = SH::P(a);
    const int i = lane_i<SH>(ln);
    if (a.rec == nullptr) {
        uint8_t* __restrict__ e = SEC ? a.eZ : a.eX;
        if (in_range) {
#pragma unroll
            for (int l = 0; l < L; ++l)
                e[b * (long long)a.n + l * P + wrap(i + SH::template coloff<SEC>(a, l), P)] = (uint8_t)((hdmask >> l) & 1u);
        }
        return;
    }
    const int nb = a.nb;
    uint8_t* __restrict__ sg = (SH::kStatic && 2 * SH::kP > 64) ? stage : stage + (ln.gb / P) * (nb * 8);
    if (in_range) {
#pragma unroll
        for (int l = 0; l < L; ++l) sg[l * P + wrap(i + SH::template coloff<SEC>(a, l), P)] = (uint8_t)((hdmask >> l) & 1u);
        for (int k = a.n + i; k < nb * 8; k += P) sg[k] = 0;
    }
    wave_sync();
    if (in_range) {
        uint8_t* __restrict__ out = a.rec + b * (long long)a.recBytes + SEC * nb;
        for (int k = i; k < nb; k += P) out[k] = (uint8_t)pack8(*reinterpret_cast<const uint64_t*>(sg + 8 * k));
    }
    wave_sync();  // the next sector reuses the stage
}

// GO: list mode (the sector is known to go on past iteration 0, see iteration0)
template <int R, int L, int SEC, int STOP, class SH, class TU, bool GO = false>
__device__ __forceinline__ void decode_sector(const BpArgs& a, Lane& ln, uint32_t b, bool in_range, float pp,
                                              uint32_t sbits, const float* __restrict__ tab0, uint32_t& flags,
                                              int& iters_out, uint8_t* __restrict__ stage)
{
    const int i = ln.i;
    const int P = SH::P(a);

    // Zero syndrome under the syndrome stop rule (most sectors at low p: P61 at p = 0.002, 44 %):
    // iteration 0 (by table, see iteration0) sends every edge the pattern-0 entry tab0[r], so the
    // hard decision is 0 when every tab0[r] < 0.5, its syndrome is the input's (0), and the sector
    // stops after that iteration with e = 0, conv = every tab0[r] outside (0.01, 0.99).  The same
    // outputs without the iteration's rotations (not when the final messages are requested).
    if constexpr (STOP == QEC_STOP_SYNDROME && !GO) {
        if (a.maxIter >= 2 && a.q == nullptr && all_live(sbits == 0u, in_range)) {
            bool low = true, cv = true;
#pragma unroll
            for (int r = 0; r < R; ++r) {
                low &= tab0[r] < 0.5f;
                cv &= outside(tab0[r]);
            }
            if (low) {  // wave-uniform (tab0 is the workgroup's)
                emit_decisions<L, SEC, SH>(a, ln, b, in_range, 0u, stage);
                if (!cv) flags |= SEC ? QEC_CONVERGENCE_FAIL_Z : QEC_CONVERGENCE_FAIL_X;
                iters_out = 1;
                return;
            }
        }
    }

    // Zero syndrome under the fixed / reference stop: the launch's precomputed outcome (zero_outcome)
    if constexpr (STOP != QEC_STOP_SYNDROME) {
        const uint32_t zs = a.zs[SEC];
        if (zs != 0u && a.q == nullptr && all_live(sbits == 0u, in_range)) {
            emit_decisions<L, SEC, SH>(a, ln, b, in_range, (zs & 1u) ? (uint32_t)((1ull << L) - 1ull) : 0u, stage);
            if (zs & 2u) flags |= SEC ? QEC_CONVERGENCE_FAIL_Z : QEC_CONVERGENCE_FAIL_X;
            if (zs & 4u) flags |= SEC ? QEC_SYNDROME_FAIL_Z : QEC_SYNDROME_FAIL_X;
            iters_out = (int)((zs >> 8) & 0xFFFFu);
            return;
        }
    }
    // InitVarNodes: every edge starts at p' (DecoderCPU.h:135-148, 265-267)
    float msg[R][L];
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
        for (int l = 0; l < L; ++l) msg[r][l] = pp;

    const float one_minus_pp = 1.0f - pp;
    bool hard = false;  // the initial messages p' are not hard (0 < p' < 1 is required anyway)
    const int N = a.maxIter;
    bool active = in_range;  // group-uniform
    int it = 0;
    int n = 0;
    // in_agree: the state entering the next iteration is hard and every variable's R messages
    // are equal (wave-uniform); st_agreed: this group's current state passed that test (it was
    // produced by the agreement path or is one of a cycle's two states), so the post-processing
    // can read it lane-locally
    bool in_agree = false, st_agreed = false;
    bool agreed = false, vagree = false;
    int ph_soft = 0, ph_hard = 0, ph_agree = 0, ph_jump = 0;  // QEC_PHASE_STATS
    // syndrome stop rule: the hard decision of the last executed iteration and its syndrome test
    // (hd_valid: the current state is that iteration's output, i.e. not reached by a cycle jump).
    // The post-processing's hard decision is the same function of the same messages, and its
    // syndrome test the same test, so they are reused (group-uniform).
    uint32_t hd_last = 0;
    bool syn_last = false, hd_valid = false;
    uint32_t seen[2] = {~0u, ~0u};  // the group's last two tested (failed) hard decisions (iteration's skip)
    // iteration 0 of the syndrome stop may leave the messages unformed (every group stopped there):
    // then cv0 is each lane's convergence test of them (iteration0)
    bool cv0 = true, msg_built = true;
    unsigned long long hdpat = 0, cvpat = 0;
    if constexpr (STOP == QEC_STOP_SYNDROME && !GO) pattern_masks<R>(tab0, hdpat, cvpat);
    if (N >= 2 && active) {  // iteration 0 by table (see iteration0)
        ++it;
        syn_last = iteration0<R, L, SEC, STOP, SH, GO>(a, msg, sbits, ln, tab0, hd_last, cv0, msg_built, hdpat, cvpat);
        hd_valid = true;
        if (STOP == QEC_STOP_SYNDROME && !GO) seen[0] = hd_last;  // tested (a group going on failed it)
        if (syn_last) active = false;
        if constexpr (QEC_PHASE_STATS) ph_soft += 1;
        n = 1;
    }
    // iterations n .. N-2 (DecoderCPU.h:280-291); the last one is peeled below
    for (; n < N - 1; ++n) {
        if (!__any(active)) break;  // DecoderCPU.h:282 (fixed: only after a cycle jump)
        if (active) {
            ++it;
            const bool was_hard = hard;
            syn_last = iteration<R, L, SEC, STOP, false, SH, TU>(a, msg, sbits, n, ln, pp, one_minus_pp, hard, agreed,
                                                                 vagree, hd_last, seen);
            hd_valid = true;
            if (syn_last) active = false;
            if constexpr (QEC_PHASE_STATS) { ph_soft += !was_hard; ph_hard += was_hard && !agreed; ph_agree += agreed; }
            if constexpr (TU::kSaturate) {
                st_agreed = vagree;
                // cycle_end: the state entering this iteration passed the agreement test and this
                // iteration took the agreement path
                if (agreed && in_agree && active && (a.hardPaths & QEC_HP_CYCLE)) {
                    const int last = cycle_end<STOP>(n, N);
                    if ((last - n) & 1) check_pass_hard<R, L>(msg, sbits);
                    it += last - n;
                    if constexpr (QEC_PHASE_STATS) ph_jump = last - n;
                    active = false;
                    hd_valid = false;
                    n = N;  // skips the peeled last iteration too
                }
                in_agree = vagree;
            }
        }
    }
    if (n == N - 1 && active) {
        ++it;
        const bool was_hard = hard;
        syn_last = iteration<R, L, SEC, STOP, true, SH, TU>(a, msg, sbits, n, ln, pp, one_minus_pp, hard, agreed, vagree,
                                                            hd_last, seen);
        hd_valid = true;
        if constexpr (QEC_PHASE_STATS) { ph_soft += !was_hard; ph_hard += was_hard && !agreed; ph_agree += agreed; }
        st_agreed = vagree;
    }

    // ---- post-processing of Decode (DecoderCPU.h:354-384) ----
    asm volatile("" : "+v"(sbits));  // its per-row bits are recomputed here, not held since the sector began
    const int* et = SH::template table<SEC>(a);
    bool conv, syn_ok;
    uint32_t hdmask = 0;  // e[v] of this lane's variables (l, (i + C[l]) mod P), bit l
    if (STOP == QEC_STOP_SYNDROME && all_live(hd_valid, in_range)) {
        // the last iteration's hard decision and syndrome test are the post-processing's
        conv = group_all_sh<SH>(__any(in_range && msg_built) ? lane_converged<R, L>(msg) : cv0, ln, P);
        hdmask = hd_last;
        syn_ok = syn_last;
    } else if (TU::kSaturate && all_live(st_agreed, in_range)) {
        // Every live group's state is hard and each variable's R messages are equal: the hard
        // decision is the value on any one of its edges (row 0's, rotation S[0][l], 0 with the
        // relabelling), the syndrome of that decision on check (r, i) is the XOR of the check's
        // own L messages (each equals its variable's decision), and every message is outside
        // (0.01, 0.99).  Same outputs as the general path below, without its 2 R L rotations.
#pragma unroll
        for (int l = 0; l < L; ++l)
            hdmask |= (uint32_t)(rot<SH>(msg[0][l], ln, SH::template shift<SEC, L>(et, 0, l)) >= 0.5f) << l;
        bool match = true;
#pragma unroll
        for (int r = 0; r < R; ++r) {
            uint32_t x = 0;
#pragma unroll
            for (int l = 0; l < L; ++l) x ^= __float_as_uint(msg[r][l]);
            match &= (x != 0u) == (((sbits >> r) & 1u) != 0u);
        }
        match &= !(sbits & kNonBinary);
        conv = true;
        syn_ok = group_all_sh<SH>(match, ln, P);
    } else {
        conv = group_all_sh<SH>(lane_converged<R, L>(msg), ln, P);
#pragma unroll
        for (int l = 0; l < L; ++l) {
            bool hd = false;  // e[v] = any edge message >= 0.5f (DecoderCPU.h:354-373)
#pragma unroll
            for (int r = 0; r < R; ++r) {
                const int sh = SH::template shift<SEC, L>(et, r, l);
                hd |= rot<SH>(msg[r][l], ln, sh) >= 0.5f;
            }
            hdmask |= (uint32_t)hd << l;
        }
        syn_ok = group_syndrome_ok<R, L, SEC, SH>(a, hdmask, sbits, ln);
    }
    emit_decisions<L, SEC, SH>(a, ln, b, in_range, hdmask, stage);

    if (!syn_ok) flags |= SEC ? QEC_SYNDROME_FAIL_Z : QEC_SYNDROME_FAIL_X;
    if (!conv) flags |= SEC ? QEC_CONVERGENCE_FAIL_Z : QEC_CONVERGENCE_FAIL_X;
    iters_out = QEC_PHASE_STATS ? (ph_soft | ph_hard << 8 | ph_agree << 16 | ph_jump << 24) : it;

    if (a.q != nullptr && in_range) {
        const long long qb = b * (long long)(a.mX + a.mZ) * L + (SEC ? (long long)a.mX * L : 0);
#pragma unroll
        for (int r = 0; r < R; ++r)
#pragma unroll
            for (int l = 0; l < L; ++l)
                a.q[qb + (long long)(r * P + wrap(i + SH::template rowoff<SEC>(a, r), P)) * L + l] = msg[r][l];
    }
}

// The syndrome stop without the hard-message forms: every iteration in soft arithmetic (bit-identical:
// the forms are exact shortcuts).  Under the syndrome stop a sector that turns hard has in practice
// satisfied its syndrome already (P61 at p = 0.02 .. 0.1: no hard iteration among 16 384 syndromes,
// tools/kbench/phase_hist.py, profiles/r06/phase_hist.txt), so tracking the hard state -- an fma and an
// OR per outgoing message and a compare per column in every soft var pass, ~10 % of a P61 soft iteration
// -- and the hard branches' registers are pure cost there: config 5 +2 % (p = 2e-3) .. +10 % (p = 0.1),
// profiles/r06/ab/cmp_syn_soft_vs_hard.txt.
template <class TU>
struct SoftTune : TU {
    static constexpr bool kSaturate = false;
};
// Taken for one-group waves (P61); P7's syndrome-stop kernels (nine groups per wave) keep the forms.
template <int STOP, class SH, class TU>
using StopTune = typename std::conditional<STOP == QEC_STOP_SYNDROME && SH::kStatic && (2 * SH::kP > 64),
                                           SoftTune<TU>, TU>::type;

// MINW: minimum waves per SIMD the register allocator must allow (5 -> <= 96 VGPRs), measured
// per variant with tools/kbench (P61: 5 waves beat 4 by 4 %; see profiles/).
// SPLIT: waves 2k and 2k+1 decode sectors X and Z of group k (adjacent waves; they meet in a global merge word);
// the launch zeroed flags[] and each sector ORs in its bits.  Otherwise one wave decodes both.
template <class TU>
constexpr int waves_per_block() { return TU::kWavesPerBlock; }

// The syndrome pair b (or, with one sector per wave, its sector doX ? X : Z) of this lane's group:
// decode, then the flags byte and iteration counts.  MODE (see bp_decode_kernel) 0: both sectors,
// plain store of the flags; 1 / 2: one sector, the two meet in the syndrome's merge word (atomicOr of
// flags plus a done bit; the second to arrive stores the merged byte); 3: sector X of a sector launch
// (stores its flags in the syndrome's merge word), 4: sector Z of a sector launch, enqueued after the X
// launch on the same stream (stores the flags byte: the merge word OR its own flags).  Modes 3 and 4
// compile one sector only, so each kernel's registers are allocated for that sector alone.
template <int RX, int RZ, int L, int STOP, class SH, class TU, int MODE>
__device__ __forceinline__ void decode_group(const BpArgs& a, const float* __restrict__ tab0, uint8_t* __restrict__ stage,
                                             int i, int gb, uint32_t b, bool in_range, bool doX)
{
    constexpr bool SPLIT = MODE != 0;
    constexpr bool kHasX = MODE != 4, kHasZ = MODE != 3;
    constexpr int kTabX = (1 << RX) * RX;
    // p' = (2/3) p, as the reference writes it (DecoderCPU.h:259)
    const float pp = 2.0f / 3.0f * a.errorProbability;
    const int P = SH::P(a);
    uint32_t flags = 0;
    int itX = 0, itZ = 0;
    Lane ln{i, gb, 4 * (gb + i), 4 * (gb + i + P), in_range};
    const bool runX = kHasX && doX, runZ = kHasZ && (!doX || !SPLIT);
    // list mode: every listed sector goes on past iteration 0 (decode_sector's GO)
    constexpr bool GO = MODE == 2;
    // both sectors' syndrome loads are issued up front: the Z load's latency hides behind X
    const uint32_t sbX = runX ? load_sbits<RX, 0, SH>(a, ln, b, in_range) : 0u;
    const uint32_t sbZ = runZ ? load_sbits<RZ, 1, SH>(a, ln, b, in_range) : 0u;
    if constexpr (kHasX) {
        if (runX) decode_sector<RX, L, 0, STOP, SH, TU, GO>(a, ln, b, in_range, pp, sbX, tab0, flags, itX, stage);
    }
    if constexpr (kHasZ) {
        if (runZ) decode_sector<RZ, L, 1, STOP, SH, TU, GO>(a, ln, b, in_range, pp, sbZ, tab0 + kTabX, flags, itZ, stage);
    }
    if (in_range && lane_i<SH>(ln) == 0) {
        uint8_t* fdst = a.rec != nullptr ? a.rec + b * (long long)a.recBytes + 2 * a.nb : a.flags + b;
        if constexpr (MODE == 0) {
            *fdst = (uint8_t)flags;
        } else if constexpr (MODE == 3) {
            a.merge[b] = flags;  // for the Z launch (a word per syndrome, not the record's byte: one line each)
        } else if constexpr (MODE == 4) {
            *fdst = (uint8_t)(a.merge[b] | flags);  // the X launch's flags (same stream, earlier launch)
        } else if (MODE == 2 && a.mergeOnly) {
            // the fused Monte-Carlo pipeline reads the flags from the merge word itself
            // (mc_survivor_kernel): no returned value to wait for
            __hip_atomic_fetch_or(&a.merge[b], flags, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        } else {
            // the two sectors meet in the syndrome's merge word: whichever finds the other's done
            // bit already set writes the merged byte
            const uint32_t mine = doX ? 0x100u : 0x200u;
            const uint32_t old = atomicOr(&a.merge[b], flags | mine);
            if (old & (0x300u ^ mine)) *fdst = (uint8_t)((old | flags) & 0xFFu);
        }
        if (a.iters != nullptr) {
            if (runX) a.iters[2 * b] = itX;
            if (runZ) a.iters[2 * b + 1] = itZ;
        }
    }
}

// MODE 0: one wave decodes both sectors of its group of G syndromes; 1 (sector split): waves 2k and
// 2k + 1 decode sectors X and Z of group k; 2 (list, after triage.hip): the sectors that went on
// past the triage, listX [0, counts[0]) then listZ [0, counts[1]), G per wave, each wave looping over
// them (the grid does not depend on the lists' device-side lengths); merged as in split mode;
// 3 / 4 (sector launches): sector X, then in a second launch on the same stream sector Z, of group k
// in wave k (decode_group).  (List mode as two launches, one kernel per sector: -8..-12 % at
// p = 5e-3, profiles/r05/cmp_list_sectors54_*.txt, profiles/r06/ab/cmp_occupancy_r06c.txt.)
template <class TU, int STOP, int MODE>
constexpr int min_waves()
{
    if constexpr (MODE == 3) return STOP != QEC_STOP_SYNDROME ? TU::kMinWavesX : TU::kSeqSynWavesX;
    if constexpr (MODE == 4) return STOP != QEC_STOP_SYNDROME ? TU::kMinWavesZ : TU::kSeqSynWavesZ;
    return STOP == QEC_STOP_SYNDROME ? TU::kMinWavesSyn : TU::kMinWaves;
}
template <int RX, int RZ, int L, int STOP, class SH, class TU, int MODE>
__global__ __launch_bounds__(64 * waves_per_block<TU>(), (min_waves<TU, STOP, MODE>()))
void bp_decode_kernel(const BpArgs a)
{
    constexpr bool LIST = MODE == 2;
    constexpr bool SPLIT = MODE == 1 || LIST;
    const int lane = threadIdx.x & 63;
    const long long wave = (long long)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    const int P = SH::P(a);
    const int G = SH::kStatic ? 64 / P : a.G;
    // with pushed rotations the groups sit on the top G P lanes; the idle lanes below them take group
    // index G (never in range), in-group indices 0 .. 63 - G P (in bounds, never stored) and group 0's base
    constexpr int kGB = kGroupBase<SH>();
    const int g = kGB ? (lane < kGB ? G : (lane - kGB) / P) : lane / P;
    const int i = kGB ? (lane < kGB ? lane : lane - kGB - g * P) : lane - g * P;
    const int gb = kGB ? (lane < kGB ? kGB : kGB + g * P) : g * P;
    // iteration-0 tables of both sectors (iteration0), built by the workgroup before any wave leaves
    constexpr int kTabX = (1 << RX) * RX, kTabZ = (1 << RZ) * RZ;
    __shared__ float tab0[kTabX + kTabZ];
    {
        const float ppt = 2.0f / 3.0f * a.errorProbability;
        if constexpr (kTabX + kTabZ <= kMaxTab0) {
            (void)ppt;  // from the host (the same operations: same bits, launch_decode)
            for (int e = threadIdx.x; e < kTabX + kTabZ; e += blockDim.x) tab0[e] = a.tab0[e];
        } else {
            for (int e = threadIdx.x; e < kTabX + kTabZ; e += blockDim.x)
                tab0[e] = e < kTabX ? table0_entry<RX, L>(ppt, e) : table0_entry<RZ, L>(ppt, e - kTabX);
        }
        __syncthreads();
    }
    // this wave's decision stage for packed records (emit_decisions)
    constexpr int kStage = stage_bytes_per_wave<L, SH>();
    __shared__ __attribute__((aligned(8))) uint8_t stage_all[waves_per_block<TU>() * kStage];
    uint8_t* stage = stage_all + (threadIdx.x >> 6) * kStage;
    if constexpr (LIST) {
        const long long nX = a.counts[0], nZ = a.counts[a.countStride];
        const long long wXn = (nX + G - 1) / G, wTot = wXn + (nZ + G - 1) / G;
        const long long nw = (long long)gridDim.x * (blockDim.x >> 6);
        // (the next sectors' list entries and syndrome bits loaded ahead: no gain at p = 2e-3 / 5e-3, -3 %
        // at 1e-2; round 4)
        // With WPB > 1 (ListTune) a workgroup holds every wave of its CU, and they take the sectors of the
        // workgroup's contiguous share one at a time from an LDS counter.  A SIMD issues its oldest wave first,
        // so with a static share per wave the first-launched waves finish their sectors early and the launch
        // ends on the youngest, nearly alone on their SIMDs (P61 at p = 5e-3: busy cycles per wave 0.61 M in
        // the first quarter of the grid, 0.93 M in the last, max / mean 1.7; tools/kbench/list_phases.py):
        // the counter lets a CU's waves finish together.
        constexpr bool kQueue = waves_per_block<TU>() > 1;
        __shared__ uint32_t next;
        long long lo = wave, hi = wTot;
        if constexpr (kQueue) {
            if (threadIdx.x == 0) next = 0u;
            __syncthreads();
            const long long per = (wTot + gridDim.x - 1) / gridDim.x;
            lo = (long long)blockIdx.x * per;
            hi = lo + per < wTot ? lo + per : wTot;
        }
        for (long long t = 0;; ++t) {
            long long vw;
            if constexpr (kQueue) {
                uint32_t k = 0u;
                if (lane == 0) k = __hip_atomic_fetch_add(&next, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                vw = lo + (long long)__builtin_amdgcn_readfirstlane(k);
            } else {
                vw = lo + t * nw;  // a static grid stride
            }
            if (vw >= hi) break;
            const bool doX = vw < wXn;  // wave-uniform
            const long long slot = (doX ? vw : vw - wXn) * G + g;
            const bool in_range = (g < G) && (slot < (doX ? nX : nZ));
            const uint32_t b = in_range ? (uint32_t)(doX ? a.listX : a.listZ)[slot] : 0u;
            // laundered per sector: the rotation addresses derived from the lane index would otherwise
            // be hoisted out of this loop into live registers (they spilled at 3 waves per SIMD)
            int il = i, gbl = gb;
            asm volatile("" : "+v"(il), "+v"(gbl));
            decode_group<RX, RZ, L, STOP, SH, StopTune<STOP, SH, TU>, MODE>(a, tab0, stage, il, gbl, b, in_range, doX);
        }
        return;
    }
    const long long grp = SPLIT ? wave >> 1 : wave;
    const long long slot = grp * G + g;
    const bool in_range = (g < G) && (slot < a.B);
    if (!__any(in_range)) return;
    // the syndrome index in 32 bits (launch_decode caps B below 2^31): a 64-bit index live across both
    // sectors spilled at 96 VGPRs
    const bool doX = MODE == 3 || (MODE != 4 && (!SPLIT || (wave & 1) == 0));  // wave-uniform
    const long long pslot = (a.perm_sectors && !doX) ? slot + a.B : slot;
    const uint32_t b = (in_range && a.perm != nullptr) ? (uint32_t)a.perm[pslot] : (uint32_t)slot;
    decode_group<RX, RZ, L, STOP, SH, StopTune<STOP, SH, TU>, MODE>(a, tab0, stage, i, gb, b, in_range, doX);
}

// ---- variant table ----------------------------------------------------------
using KernelFn = void (*)(const BpArgs);

// The P61 tuning.  Its reference- and fixed-stop kernels are also compiled in a second
// translation unit, bp_decode_p61.hip, under LLVM's iterative-minreg scheduler (the flag is
// per file): 15 instead of 42 spill reloads at 96 VGPRs, fixed stop 0.656 vs 0.700 ms, reference
// stop 0.567 vs 0.613 ms; its syndrome-stop kernel spills more that way (0.517 vs 0.476 ms).
// P7's fixed and reference stops gain nothing, but its syndrome stop does (0.087 vs 0.100 ms)
// (profiles/r01/session7/cmp_s7u_*.txt, cmp_s7v_*.txt).  So those kernels come from there.
// A distinct Tune type keeps the two units' kernels apart (same code, different symbols).
// Sector launches (MODE 3 / 4, QEC_OPT_SECTOR_SPLIT = 3): X alone needs R L = 40 message registers, Z 50.
using TuneP61 = Tune<5, true, false, true, true, false, true, 2, 1, 4, 1, false, 6, 5>;
struct TuneP61MinReg : TuneP61 {};
using ShiftsP61 = GeneratedShifts<4, 5, 10, 61, 9, 49, TuneP61::kRelabel, TuneP61::kMaskSelect>;
// P7: three columns per division guard (col_group): 0.075 vs 0.077 ms at configs[1] (65 536 @ 20), even
// at 2^20 (profiles/r03/cmp_p7_65536_colgroups.txt, cmp_p7_2e20.txt)
// P7 at 7 waves per SIMD (72 VGPRs): its fixed / reference kernels are spill-free there (8: 2-10 B of
// scratch) at the same speed (configs[1] 0.071 vs 0.071 ms, 2^20 0.621 vs 0.618 ms;
// profiles/r04/cmp_p7_waves.txt)
// P7 syndrome-stop kernels at 7 waves (4 B of scratch): 6 waves are spill-free but 3-4 % slower
// (p = 0.05 at 2^20 1.150 vs 1.111 ms; profiles/r04/cmp_p7_syndrome_waves.txt)
using TuneP7 = Tune<7, true, false, true, true, true, false, 2, 1, 7, 3, false, 0, 0>;
struct TuneP7MinReg : TuneP7 {};
using ShiftsP7 = GeneratedShifts<3, 3, 6, 7, 2, 3, TuneP7::kRelabel, TuneP7::kMaskSelect>;
// List mode (MODE 2): P61 at four waves per SIMD (<= 128 VGPRs; three: -5 % at p = 5e-3, -10 % at 1e-2;
// five spill and lose 20-25 %, profiles/r05/, profiles/r06/ab/), P7 at five.
// ... in 16-wave workgroups, one per CU, that take their sectors from an LDS counter (bp_decode_kernel):
// config 5 +12 % at p = 0.01, +6 % at 5e-3, +1 % at 2e-3 over a static grid stride
// (profiles/r06/ab/cmp_list_cu.txt)
using ListTuneP61 = ListTune<TuneP61, 4, 16>;
using ListTuneP7 = ListTune<TuneP7MinReg, 5>;
KernelFn p61_minreg_kernel(int stop, bool split);  // bp_decode_p61.hip
KernelFn p61_minreg_seq_kernel(int stop, int sec); // bp_decode_p61.hip
KernelFn p7_minreg_kernel(int stop, bool split);   // bp_decode_p61.hip
KernelFn p7_minreg_list_kernel();                  // bp_decode_p61.hip

KernelFn phase_kernel(int P, int stop);  // bp_decode_phase.hip

#if defined(QEC_P61_MINREG_TU)
KernelFn p61_minreg_kernel(int stop, bool split)
{
    if (stop == QEC_STOP_REF)
        return split ? bp_decode_kernel<4, 5, 10, QEC_STOP_REF, ShiftsP61, TuneP61MinReg, 1>
                     : bp_decode_kernel<4, 5, 10, QEC_STOP_REF, ShiftsP61, TuneP61MinReg, 0>;
    if (stop == QEC_STOP_FIXED)
        return split ? bp_decode_kernel<4, 5, 10, QEC_STOP_FIXED, ShiftsP61, TuneP61MinReg, 1>
                     : bp_decode_kernel<4, 5, 10, QEC_STOP_FIXED, ShiftsP61, TuneP61MinReg, 0>;
    return nullptr;
}
KernelFn p61_minreg_seq_kernel(int stop, int sec)
{
    if (stop == QEC_STOP_REF)
        return sec ? bp_decode_kernel<4, 5, 10, QEC_STOP_REF, ShiftsP61, TuneP61MinReg, 4>
                   : bp_decode_kernel<4, 5, 10, QEC_STOP_REF, ShiftsP61, TuneP61MinReg, 3>;
    if (stop == QEC_STOP_FIXED)
        return sec ? bp_decode_kernel<4, 5, 10, QEC_STOP_FIXED, ShiftsP61, TuneP61MinReg, 4>
                   : bp_decode_kernel<4, 5, 10, QEC_STOP_FIXED, ShiftsP61, TuneP61MinReg, 3>;
    return nullptr;
}
KernelFn p7_minreg_kernel(int stop, bool split)
{
    if (stop == QEC_STOP_SYNDROME)
        return split ? bp_decode_kernel<3, 3, 6, QEC_STOP_SYNDROME, ShiftsP7, TuneP7MinReg, 1>
                     : bp_decode_kernel<3, 3, 6, QEC_STOP_SYNDROME, ShiftsP7, TuneP7MinReg, 0>;
    return nullptr;
}
KernelFn p7_minreg_list_kernel() { return bp_decode_kernel<3, 3, 6, QEC_STOP_SYNDROME, ShiftsP7, ListTuneP7, 2>; }
#elif defined(QEC_PHASE_TU)
// The instrumented kernels of the shipped codes (QEC_OPT_PHASE_STATS, one wave per syndrome):
// iters[] reports per sector soft | hard << 8 | agreed << 16 | jumped << 24 iterations.
struct TuneP61Phase : TuneP61 {};
struct TuneP7Phase : TuneP7 {};
KernelFn phase_kernel(int P, int stop)
{
    if (P == 61) {
        if (stop == QEC_STOP_REF) return bp_decode_kernel<4, 5, 10, QEC_STOP_REF, ShiftsP61, TuneP61Phase, 0>;
        if (stop == QEC_STOP_FIXED) return bp_decode_kernel<4, 5, 10, QEC_STOP_FIXED, ShiftsP61, TuneP61Phase, 0>;
        return bp_decode_kernel<4, 5, 10, QEC_STOP_SYNDROME, ShiftsP61, TuneP61Phase, 0>;
    }
    if (stop == QEC_STOP_REF) return bp_decode_kernel<3, 3, 6, QEC_STOP_REF, ShiftsP7, TuneP7Phase, 0>;
    if (stop == QEC_STOP_FIXED) return bp_decode_kernel<3, 3, 6, QEC_STOP_FIXED, ShiftsP7, TuneP7Phase, 0>;
    return bp_decode_kernel<3, 3, 6, QEC_STOP_SYNDROME, ShiftsP7, TuneP7Phase, 0>;
}
#else

struct Variant {
    int J, K, L;
    int P, sigma, tau;  // P > 0: specialised to the generator's tables for these parameters
    bool relabel;       // runtime-shift variants: relabel the lane tables at launch
    bool split_auto;    // QEC_OPT_SECTOR_SPLIT = 1 takes the split kernels
    int waves_per_block;
    KernelFn fn[3];     // indexed by stop rule
    KernelFn split[3];  // the same with one wave per sector (nullptr: not instantiated)
    KernelFn phase[3];  // QEC_OPT_PHASE_STATS: instrumented kernels (shipped codes only)
    int (*fill_tab0)(float pp, float* out);  // host iteration-0 tables (kernel arguments)
    uint32_t (*zero_out[2])(float pp, int N, int stop);  // per sector: zero-syndrome outcomes (zero_outcome)
    const char* name;
    KernelFn list = nullptr;  // syndrome stop, list mode (MODE 2: the sectors the triage passed on)
    int min_waves_syn = 1;    // its occupancy (waves per SIMD), for the list launch's grid
    int list_wpb = 1;         // its waves per workgroup
    KernelFn seq[3][2] = {};     // sector launches (MODE 3 / 4): [stop][sector]
    // QEC_OPT_SECTOR_SPLIT = 1 takes the sector launches from this batch on, per stop rule (0: never), and
    // under the syndrome stop only from seq_syn_min_p on
    long long seq_min_batch[3] = {};
    float seq_syn_min_p = 0.0f;
};

// Both sectors' iteration-0 tables on the host, entry for entry what the device's table0_entry
// computes (same IEEE fp32 operations, -ffp-contract=off); returns the entry count, 0 if they do
// not fit the argument block.
template <int J, int K, int L>
static int fill_tab0(float pp, float* out)
{
    constexpr int tx = (1 << J) * J, tz = (1 << K) * K;
    if (tx + tz > kMaxTab0) return 0;
    for (int e = 0; e < tx; ++e) out[e] = table0_entry<J, L>(pp, e);
    for (int e = 0; e < tz; ++e) out[tx + e] = table0_entry<K, L>(pp, e);
    return tx + tz;
}

template <int J, int K, int L, class SH, class TU, bool WITH_SPLIT, class TUL = TU>
static Variant make_variant(int P, int S, int T, const char* name)
{
    Variant v{J, K, L, P, S, T, TU::kRelabel, TU::kSplit && WITH_SPLIT, waves_per_block<TU>(),
              {bp_decode_kernel<J, K, L, QEC_STOP_REF, SH, TU, 0>,
               bp_decode_kernel<J, K, L, QEC_STOP_FIXED, SH, TU, 0>,
               bp_decode_kernel<J, K, L, QEC_STOP_SYNDROME, SH, TU, 0>},
              {nullptr, nullptr, nullptr},
              {nullptr, nullptr, nullptr},
              fill_tab0<J, K, L>,
              {zero_outcome<J, L>, zero_outcome<K, L>},
              name};
    if constexpr (WITH_SPLIT) {
        v.split[QEC_STOP_REF] = bp_decode_kernel<J, K, L, QEC_STOP_REF, SH, TU, 1>;
        v.split[QEC_STOP_FIXED] = bp_decode_kernel<J, K, L, QEC_STOP_FIXED, SH, TU, 1>;
        v.split[QEC_STOP_SYNDROME] = bp_decode_kernel<J, K, L, QEC_STOP_SYNDROME, SH, TU, 1>;
        v.list = bp_decode_kernel<J, K, L, QEC_STOP_SYNDROME, SH, TUL, 2>;
        v.seq[QEC_STOP_REF][0] = bp_decode_kernel<J, K, L, QEC_STOP_REF, SH, TU, 3>;
        v.seq[QEC_STOP_REF][1] = bp_decode_kernel<J, K, L, QEC_STOP_REF, SH, TU, 4>;
        v.seq[QEC_STOP_FIXED][0] = bp_decode_kernel<J, K, L, QEC_STOP_FIXED, SH, TU, 3>;
        v.seq[QEC_STOP_FIXED][1] = bp_decode_kernel<J, K, L, QEC_STOP_FIXED, SH, TU, 4>;
        v.seq[QEC_STOP_SYNDROME][0] = bp_decode_kernel<J, K, L, QEC_STOP_SYNDROME, SH, SeqSynTune<TU>, 3>;
        v.seq[QEC_STOP_SYNDROME][1] = bp_decode_kernel<J, K, L, QEC_STOP_SYNDROME, SH, SeqSynTune<TU>, 4>;
    }
    v.min_waves_syn = TUL::kMinWavesSyn;  // the list launch's grid (launch_decode_list)
    v.list_wpb = waves_per_block<TUL>();
    return v;
}
// Tune<min waves per SIMD, relabel, zero-skip, short division, hard-message paths, sector split,
//      mask-select rotation bases, gather pipelining depth, waves per workgroup, min waves (syndrome stop)>
template <int J, int K, int L, class TU = Tune<1, false, true, true, true>>
static Variant rt()
{
    return make_variant<J, K, L, RuntimeShifts, TU, false>(0, 0, 0, "wave-circulant runtime-shift");
}
template <int J, int K, int L, int P, int S, int T, class TU, class TUL = TU>
static Variant gen()
{
    return make_variant<J, K, L, GeneratedShifts<J, K, L, P, S, T, TU::kRelabel, TU::kMaskSelect>, TU, true, TUL>(
        P, S, T, "wave-circulant generated-shift");
}

// Measured per variant with tools/kbench (profiles/r01/): P61 4 waves + relabel + zero-skip +
// short division 7.11 ms vs 9.46 ms without them; P7 (9 syndromes per wave, so whole-wave
// zero columns are rare) keeps 8 waves and only the short division.  The hard-message paths:
// P61 @ p=0.01 6.24 vs 7.28 ms, @ p=0.05 7.22 vs 9.36 ms; P7 0.186 vs 0.199 ms (session-3 kbench).
// With the hard paths and cycle jump the zero-skip test no longer pays for P61 (0.976 vs 0.987 ms
// @ p=0.01, 2.45 vs 2.81 ms @ p=0.05; session-5 kbench, profiles/r01/session5/cmp_s5m_*.txt),
// and once the hoisted rotation bases spill, selecting them by lane mask wins (P61 0.855 vs
// 0.963 ms, cmp_s5o/s5p).  With the 6-instruction short division and the min-reduced guard P7
// takes the short division again (0.090 vs 0.092 ms, cmp_s6j).  P61 then moves to 5 waves per
// SIMD (96 VGPRs, a few spills) and 2-wave workgroups: fixed stop 0.728 vs 0.751 ms at p = 0.01,
// 1.75 vs 2.16 ms at p = 0.05; its syndrome-stop kernels spill badly at 5 waves (450 scratch
// loads, 1.01 vs 0.50 ms) and keep 4 (profiles/r01/session7/cmp_s7l-n_*.txt).  Round 2: without
// the agreement test (kAgree) the syndrome-stop kernels are spill-free, P61 at 4 waves (125 VGPRs)
// and P7 at 7 (with the lane relabelling and gather pipelining P7 now takes too, 2-5 % faster
// at every stop rule: 260 instead of 456 static ds_bpermute; profiles/r02/p7_variants_r02s3{s,t}.txt).
// With the iteration-0 tables from the host nothing is shared between the waves
// of a workgroup any more, and one-wave workgroups are fastest for both codes (P61 headline 134.0
// vs 131.9M syn/s with two, P7 +3 % vs four; profiles/r02/cmp_wpb_r02s3x.txt).
static Variant gen_p61()
{
    Variant v = gen<4, 5, 10, 61, 9, 49, TuneP61, ListTuneP61>();
    for (int stop : {QEC_STOP_REF, QEC_STOP_FIXED, QEC_STOP_SYNDROME}) v.phase[stop] = phase_kernel(61, stop);
    {
        // the reference- and fixed-stop kernels from the minreg unit (the syndrome stop's spill more there;
        // its sector launches measured +-0, profiles/r05/cmp_syn_seq_waves_*.txt)
        for (int stop : {QEC_STOP_REF, QEC_STOP_FIXED}) {
            v.fn[stop] = p61_minreg_kernel(stop, false);
            v.split[stop] = p61_minreg_kernel(stop, true);
            for (int sec = 0; sec < 2; ++sec) v.seq[stop][sec] = p61_minreg_seq_kernel(stop, sec);
        }
        // sector launches, fixed stop from 2^18 syndromes on: +1.3 % at 262 144, +0.3 % at 524 288, +1.9 % at
        // 2^20, but -2.7 % at 131 072 and -10 % at 65 536 (a second launch tail; profiles/r04/cmp_sector_launch_*.txt);
        // reference stop only at 2^20 (-2.3 % at 2^18, -0.8 % at 2^19, +0.7 % at 2^20); syndrome stop at 2^20 and
        // p >= 0.03 (Monte-Carlo bit rows at 2^20: +1.8 % at p = 0.1, +1 % at 0.05, 0 at 0.02; byte rows at p = 0.01:
        // -6 % at 2^18 and 2^20; profiles/r05/cmp_seq_per_stop*.txt)
        v.seq_min_batch[QEC_STOP_FIXED] = 1LL << 18;
        v.seq_min_batch[QEC_STOP_REF] = 1LL << 20;
        v.seq_min_batch[QEC_STOP_SYNDROME] = 1LL << 20;
        v.seq_syn_min_p = 0.03f;
    }
    return v;
}

static Variant gen_p7()
{
    Variant v = gen<3, 3, 6, 7, 2, 3, TuneP7, ListTuneP7>();
    for (int stop : {QEC_STOP_REF, QEC_STOP_FIXED, QEC_STOP_SYNDROME}) v.phase[stop] = phase_kernel(7, stop);
    v.fn[QEC_STOP_SYNDROME] = p7_minreg_kernel(QEC_STOP_SYNDROME, false);
    v.split[QEC_STOP_SYNDROME] = p7_minreg_kernel(QEC_STOP_SYNDROME, true);
    v.list = p7_minreg_list_kernel();
    v.min_waves_syn = ListTuneP7::kMinWavesSyn;
    v.list_wpb = waves_per_block<ListTuneP7>();
    return v;
}

static const Variant kVariants[] = {
    // specialised: the two code files the reference ships
    gen_p61(),
    gen_p7(),
#ifndef QEC_KBENCH_MINIMAL  // experiment builds (tools/kbench) only compile the shipped-code kernels
    // runtime shifts, any P <= 64 with these block shapes
    rt<4, 5, 10>(),
    rt<3, 3, 6, Tune<6, false, false, true, true>>(),
    rt<2, 3, 6, Tune<6, false, false, true, true>>(),
    rt<3, 4, 8>(),
    rt<4, 4, 8>(),
    rt<3, 5, 10>(),
    rt<4, 6, 12>(),
    rt<2, 2, 4, Tune<8, false, false, true, true>>(),
#endif
};

struct DecodeLaunch {
    const Variant* v;
};

const void* select_variant(const Code& c, std::string& name)
{
    if (!c.is_qc || c.P > 64 || c.P < 1) return nullptr;
    if (c.J * c.L > kMaxRL || c.K * c.L > kMaxRL || c.J > kMaxR || c.K > kMaxR || c.L > kMaxL) return nullptr;
    for (const Variant& v : kVariants) {
        if (v.J != c.J || v.K != c.K || v.L != c.L) continue;
        if (v.P > 0) {
            if (v.P != c.P || v.sigma != c.sigma || v.tau != c.tau) continue;
            std::vector<int> EX, EZ;
            if (!generator_exponents(c.J, c.K, c.L, c.P, c.sigma, c.tau, EX, EZ)) continue;
            if (EX != c.EX || EZ != c.EZ) continue;  // file content differs from its header's generator
        }
        char buf[160];
        snprintf(buf, sizeof buf, "%s J=%d K=%d L=%d P=%d G=%d", v.name, c.J, c.K, c.L, c.P, 64 / c.P);
        name = buf;
        return &v;
    }
    return nullptr;
}

// QEC_OPT_SECTOR_SPLIT: 0 off, 1 the variant's tuned choice, 2 on (runtime-shift variants have
// no split kernels: one wave per syndrome)
// The tuned choice (split_auto) splits batches up to kSplitAutoMaxBatch: the two waves per syndrome
// group help fill the chip when waves are few, and with each sector's waves in the order of that
// sector's weight (schedule.hip, per-sector order) they also group like work: P7 fixed 20 at 2^19
// 0.294 vs 0.342 ms, 2^20 0.500 vs 0.587 ms split vs one wave per group (round 2, total-weight
// order: split lost from 2^19 on, profiles/r02/p7_split_r02s3zz.txt; round 4:
// profiles/r04/cmp_sector_order_*.txt).  Above 2^20 the order pass has more chunks than the fused
// scatter takes and falls back to the total-weight order.
constexpr long long kSplitAutoMaxBatch = (1LL << 20) + 1;

bool decode_uses_split(const void* variant, int stop, int split, long long B);
// Sector launches (QEC_OPT_SECTOR_SPLIT = 3, or 1 as resolved by decode_sector_mode):
// two launches, sector X then sector Z, each kernel compiled for its own sector (no merge words).
static bool decode_uses_seq(const Variant* v, int stop, int split, long long B)
{
    (void)B;
    return split == 3 && v->seq[stop][0] != nullptr && v->seq[stop][1] != nullptr;
}

// QEC_OPT_SECTOR_SPLIT = 1 (the variant's measured choice) resolved for one launch: 3 (sector launches), 2
// (split waves) or 0; other values are returned as they are
int decode_sector_mode(const void* variant, int stop, int split, long long B, float p)
{
    const Variant* v = static_cast<const Variant*>(variant);
    if (split != 1) return split;
    const long long mb = v->seq_min_batch[stop];
    if (mb > 0 && B >= mb && (stop != QEC_STOP_SYNDROME || p >= v->seq_syn_min_p) && v->seq[stop][0] != nullptr &&
        v->seq[stop][1] != nullptr)
        return 3;
    return v->split_auto && B < kSplitAutoMaxBatch && v->split[stop] != nullptr ? 2 : 0;
}

bool decode_needs_merge(const void* variant, int stop, int split, long long B)
{
    const Variant* v = static_cast<const Variant*>(variant);
    return decode_uses_seq(v, stop, split, B) || decode_uses_split(variant, stop, split, B);
}

bool decode_uses_split(const void* variant, int stop, int split, long long B)
{
    const Variant* v = static_cast<const Variant*>(variant);
    if (decode_uses_seq(v, stop, split, B)) return false;
    return split == 2 && v->split[stop] != nullptr;
}

bool decode_has_phase_stats(const void* variant, int stop)
{
    return static_cast<const Variant*>(variant)->phase[stop] != nullptr;
}

int launch_decode(const void* variant, const Code& c, const uint8_t* sX, const uint8_t* sZ, bool sbits, long long B,
                  float errorProbability, int maxIter, int stop, uint8_t* eX, uint8_t* eZ, uint8_t* flags,
                  uint8_t* rec, int32_t* iters, float* q, int hardPaths, const int32_t* perm, int split,
                  uint32_t* merge, bool merge_zeroed, hipStream_t stream, int rec_stride, bool perm_sectors,
                  hipEvent_t done)
{
    const Variant* v = static_cast<const Variant*>(variant);
    if (B <= 0) return QEC_OK;
    if (B >= (1LL << 31)) return fail(QEC_ERR_ARG, "bp_decode: at most 2^31 - 1 syndromes per launch");
    BpArgs a{};
    a.sX = sX; a.sZ = sZ; a.eX = eX; a.eZ = eZ; a.flags = flags; a.iters = iters; a.q = q;
    a.sbits = sbits ? 1 : 0;
    a.wX = (c.mX + 31) / 32;
    a.wZ = (c.mZ + 31) / 32;
    a.rec = rec;
    a.perm = perm;
    a.perm_sectors = perm != nullptr && perm_sectors ? 1 : 0;
    const bool phase = (hardPaths & QEC_HP_PHASE) != 0;
    if (phase && v->phase[stop] == nullptr)
        return fail(QEC_ERR_UNSUPPORTED, "bp_decode: no phase-statistics kernel for this code");
    const int split_opt = split;
    split = !phase && decode_uses_split(variant, stop, split, B) && merge != nullptr;
    if (split) {
        a.merge = merge;
        if (!merge_zeroed && hipMemsetAsync(merge, 0, (size_t)B * sizeof(uint32_t), stream) != hipSuccess)
            return fail(QEC_ERR_HIP, "bp_decode: merge-word memset failed");
    }
    a.B = B;
    a.P = c.P;
    a.G = 64 / c.P;
    a.n = c.n; a.mX = c.mX; a.mZ = c.mZ;
    a.nb = (c.n + 7) / 8;
    a.recBytes = rec_stride > 0 ? rec_stride : 2 * a.nb + 1;
    a.errorProbability = errorProbability;
    a.maxIter = maxIter < 0 ? 0 : maxIter;
    a.stop = stop;
    a.hardPaths = hardPaths & (QEC_HP_FORMS | QEC_HP_CYCLE);
    a.scaled = scaled_ok(2.0f / 3.0f * errorProbability) ? 1 : 0;
    v->fill_tab0(2.0f / 3.0f * errorProbability, a.tab0);  // p' as the kernel forms it
    if (!phase)
        for (int sec = 0; sec < 2; ++sec) a.zs[sec] = v->zero_out[sec](2.0f / 3.0f * errorProbability, a.maxIter, stop);
    relabel(c.EX.data(), c.J, c.L, c.P, v->relabel, a.SX, a.DX, a.CX);
    relabel(c.EZ.data(), c.K, c.L, c.P, v->relabel, a.SZ, a.DZ, a.CZ);
    const int wavesPerBlock = v->waves_per_block;
    const bool seq = !phase && !split && decode_uses_seq(v, stop, split_opt, B);
    const long long waves = (B + a.G - 1) / a.G * (split ? 2 : 1);
    const long long blocks = (waves + wavesPerBlock - 1) / wavesPerBlock;
    if (blocks > 0x7fffffffLL) return fail(QEC_ERR_ARG, "batch too large for one launch");
    if (seq) {  // sector X, then sector Z (which merges X's flags from the merge words) on the same stream
        if (merge == nullptr) return fail(QEC_ERR_ARG, "bp_decode: sector launches need the merge words");
        a.merge = merge;
        for (int sec = 0; sec < 2; ++sec) {
            launch_marked(v->seq[stop][sec], dim3((unsigned)blocks), dim3(64 * wavesPerBlock), 0, stream, nullptr,
                          sec == 1 ? done : nullptr, a);
            hipError_t err = hipGetLastError();
            if (err != hipSuccess) return fail(QEC_ERR_HIP, std::string("bp_decode launch: ") + hipGetErrorString(err));
        }
        return QEC_OK;
    }
    launch_marked(phase ? v->phase[stop] : split ? v->split[stop] : v->fn[stop], dim3((unsigned)blocks),
                  dim3(64 * wavesPerBlock), 0, stream, nullptr, done, a);
    hipError_t err = hipGetLastError();
    if (err != hipSuccess) return fail(QEC_ERR_HIP, std::string("bp_decode launch: ") + hipGetErrorString(err));
    return QEC_OK;
}

bool decode_has_list(const void* variant) { return static_cast<const Variant*>(variant)->list != nullptr; }


// Compute units of the current device (4 SIMDs each), cached per device (the list-mode grid).
static int device_cus()
{
    static std::atomic<int> cached[64] = {};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0) dev = 0;
    if (dev >= 64) dev = 63;
    int c = cached[dev].load(std::memory_order_relaxed);  // every writer stores the same value
    if (c <= 0) {
        if (hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || c <= 0) c = 256;
        cached[dev].store(c, std::memory_order_relaxed);
    }
    return c;
}

// The iteration-0 pattern masks of both sectors (triage.hip): bit idx of hd = pattern idx decides 1
// (some table entry >= 0.5f), of cv = its R messages all lie outside (0.01, 0.99) -- the host table's
// entries under pattern_masks' compares.  pats = {hdX, cvX, hdZ, cvZ}; false if they do not fit.
bool decode_pattern_masks(const void* variant, float errorProbability, uint32_t pats[4])
{
    const Variant* v = static_cast<const Variant*>(variant);
    if (v->J > 5 || v->K > 5) return false;
    float tab[kMaxTab0];
    if (!v->fill_tab0(2.0f / 3.0f * errorProbability, tab)) return false;
    const float* t = tab;
    for (int sec = 0; sec < 2; ++sec) {
        const int R = sec ? v->K : v->J;
        uint32_t hd = 0, cv = 0;
        for (int idx = 0; idx < (1 << R); ++idx) {
            bool h = false, c = true;
            for (int r = 0; r < R; ++r) {
                h |= t[idx * R + r] >= 0.5f;
                c &= !(t[idx * R + r] > 0.01f && t[idx * R + r] < 0.99f);
            }
            hd |= (uint32_t)h << idx;
            cv |= (uint32_t)c << idx;
        }
        pats[2 * sec] = hd;
        pats[2 * sec + 1] = cv;
        t += (1 << R) * R;
    }
    return true;
}

// List-mode decode (syndrome stop, bit-row syndromes, packed records) of the sectors triage.hip
// passed on: listX [0, counts[0]), listZ [0, counts[1]) on the device; at most 2 B sectors.  A
// grid of about one wave per resident slot loops over them.
int launch_decode_list(const void* variant, const Code& c, const uint8_t* sX, const uint8_t* sZ, long long B,
                       float errorProbability, int maxIter, int hardPaths, uint8_t* rec, int32_t* iters,
                       uint32_t* merge, const int32_t* listX, const int32_t* listZ, const uint32_t* counts,
                       hipStream_t stream, int rec_stride, bool merge_only, int count_stride, hipEvent_t done)
{
    const Variant* v = static_cast<const Variant*>(variant);
    if (!v->list) return fail(QEC_ERR_UNSUPPORTED, "bp_decode: no list-mode kernel for this code");
    if (B <= 0) return QEC_OK;
    if (B >= (1LL << 31)) return fail(QEC_ERR_ARG, "bp_decode: at most 2^31 - 1 syndromes per launch");
    BpArgs a{};
    a.sX = sX; a.sZ = sZ; a.sbits = 1;
    a.wX = (c.mX + 31) / 32; a.wZ = (c.mZ + 31) / 32;
    a.rec = rec; a.iters = iters; a.merge = merge;
    a.listX = listX; a.listZ = listZ; a.counts = counts; a.mergeOnly = merge_only ? 1 : 0;
    a.countStride = count_stride;
    a.B = B; a.P = c.P; a.G = 64 / c.P;
    a.n = c.n; a.mX = c.mX; a.mZ = c.mZ;
    a.nb = (c.n + 7) / 8; a.recBytes = rec_stride > 0 ? rec_stride : 2 * a.nb + 1;
    a.errorProbability = errorProbability;
    a.maxIter = maxIter < 0 ? 0 : maxIter;
    a.stop = QEC_STOP_SYNDROME;
    a.hardPaths = hardPaths & (QEC_HP_FORMS | QEC_HP_CYCLE);
    a.scaled = scaled_ok(2.0f / 3.0f * errorProbability) ? 1 : 0;
    v->fill_tab0(2.0f / 3.0f * errorProbability, a.tab0);
    relabel(c.EX.data(), c.J, c.L, c.P, v->relabel, a.SX, a.DX, a.CX);
    relabel(c.EZ.data(), c.K, c.L, c.P, v->relabel, a.SZ, a.DZ, a.CZ);
    // one wave per resident slot of the chip (more rounds of the grid measured no gain,
    // profiles/r03/list_rounds/), each looping over the listed sectors
    const int wpb = v->list_wpb;
    const long long need = (2 * B + a.G - 1) / a.G;
    const long long cap = 4LL * device_cus() * v->min_waves_syn;  // a multiple of wpb for the per-CU workgroups
    const long long waves = need < cap ? need : cap;
    const long long blocks = (waves + wpb - 1) / wpb;
    launch_marked(v->list, dim3((unsigned)blocks), dim3(64 * wpb), 0, stream, nullptr, done, a);
    const hipError_t err = hipGetLastError();
    if (err != hipSuccess) return fail(QEC_ERR_HIP, std::string("bp_decode list launch: ") + hipGetErrorString(err));
    return QEC_OK;
}

#endif  // QEC_P61_MINREG_TU / QEC_PHASE_TU

}  // namespace qec
