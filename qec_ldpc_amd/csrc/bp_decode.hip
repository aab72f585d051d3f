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

#include <cstdint>
#include <cstdio>

#include "qec_internal.h"

#pragma clang fp contract(off)

namespace qec {

constexpr int kMaxRL = 128;  // largest R*L a kernel argument block carries

struct BpArgs {
    const uint8_t* sX;
    const uint8_t* sZ;
    uint8_t* eX;
    uint8_t* eZ;
    uint8_t* flags;
    int32_t* iters;
    float* q;
    long long B;
    int P, G, n, mX, mZ;
    float errorProbability;
    int maxIter, stop;
    int EX[kMaxRL];
    int EZ[kMaxRL];
};

// ---- shift providers -------------------------------------------------------
// Runtime: exponents read from the kernel-argument block.  table() launders the
// pointer once per iteration so the R*L shift loads and rotation addresses stay
// inside the loop (scalar-cache hits) instead of being hoisted into ~2*R*L
// live registers.
struct RuntimeShifts {
    static constexpr bool kStatic = false;
    __device__ static int P(const BpArgs& a) { return a.P; }
    template <int SEC>
    __device__ static const int* table(const BpArgs& a)
    {
        const int* t = SEC ? a.EZ : a.EX;
        asm volatile("" : "+s"(t));
        return t;
    }
    template <int SEC, int L>
    __device__ static int shift(const int* t, int r, int l) { return t[r * L + l]; }
};

// Compile-time: exponent tables produced by the QC_LDPC_CSS generator formula
// (QEC_LDPC/QEC_LDPC_CSS.cu:37-90) evaluated by the compiler, so every rotation
// address is a loop-invariant constant of the lane index.
template <int J_, int K_, int L_, int P_, int S_, int T_>
struct GeneratedShifts {
    static constexpr bool kStatic = true;
    struct Tables {
        int EX[J_][L_];
        int EZ[K_][L_];
    };
    static constexpr long pw(long base, long e)
    {
        long t = 1;
        for (long i = 0; i < e; ++i) t = (t * base) % P_;
        return t;
    }
    static constexpr Tables make()
    {
        Tables t{};
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
    static constexpr Tables tabs = make();
    __device__ static constexpr int P(const BpArgs&) { return P_; }
    template <int SEC>
    __device__ static const int* table(const BpArgs&) { return nullptr; }
    template <int SEC, int L>
    __device__ static constexpr int shift(const int*, int r, int l) { return SEC ? tabs.EZ[r][l] : tabs.EX[r][l]; }
};

// ---- lane helpers ----------------------------------------------------------
__device__ __forceinline__ float bperm(int addr, float v)
{
    return __int_as_float(__builtin_amdgcn_ds_bpermute(addr, __float_as_int(v)));
}
__device__ __forceinline__ int bperm_i(int addr, int v) { return __builtin_amdgcn_ds_bpermute(addr, v); }

// byte address for ds_bpermute: lane (gb + (i - s) mod P), s in [0, P)
__device__ __forceinline__ int rot_addr(int i, int gb, int s, int P)
{
    int t = i - s;
    t += (t < 0) ? P : 0;
    return (gb + t) << 2;
}

// true iff pred holds on every lane of this lane's group [gb, gb+P)
__device__ __forceinline__ bool group_all(bool pred, int gb, int P)
{
    const unsigned long long bad = __ballot(!pred);
    const unsigned long long gm = (P >= 64 ? ~0ull : ((1ull << P) - 1ull)) << gb;
    return (bad & gm) == 0ull;
}

__device__ __forceinline__ bool outside(float x) { return !(x > 0.01f && x < 0.99f); }

// ---- one sector (X: R = J, Z: R = K) ------------------------------------
// EqNodeUpdate (DecoderCPU.h:150-186) for checks (r, i), r = 0..R-1: lane-local.
template <int R, int L>
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
    }
}

// VarNodeUpdate (DecoderCPU.h:188-229) for variables (l, i): gather the R incoming
// check messages by forward rotation, update, scatter back by the inverse rotation.
// LAST: the final iteration includes the self message (DecoderCPU.h:216).
// Returns the hard-decision mask (bit l) of the new messages when HD is set.
template <int R, int L, int SEC, bool LAST, bool HD, class SH>
__device__ __forceinline__ uint32_t var_pass(const BpArgs& a, float (&msg)[R][L], int i, int gb, float pp,
                                             float one_minus_pp)
{
    const int P = SH::P(a);
    const int* et = SH::template table<SEC>(a);
    uint32_t hdmask = 0;
#pragma unroll
    for (int l = 0; l < L; ++l) {
        float gv[R], bv[R], qv[R];
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const int sh = SH::template shift<SEC, L>(et, r, l);
            gv[r] = bperm(rot_addr(i, gb, sh, P), msg[r][l]);
            bv[r] = 1.0f - gv[r];
        }
        if constexpr (LAST) {
            float P0 = one_minus_pp, P1 = pp;
#pragma unroll
            for (int k = 0; k < R; ++k) { P0 = P0 * bv[k]; P1 = P1 * gv[k]; }
            const float q = P1 / (P0 + P1);
#pragma unroll
            for (int r = 0; r < R; ++r) qv[r] = q;
        } else {
            float pre0 = one_minus_pp, pre1 = pp;
#pragma unroll
            for (int j = 0; j < R; ++j) {
                float t0 = pre0, t1 = pre1;
#pragma unroll
                for (int k = j + 1; k < R; ++k) { t0 = t0 * bv[k]; t1 = t1 * gv[k]; }
                qv[j] = t1 / (t0 + t1);
                if (j + 1 < R) { pre0 = pre0 * bv[j]; pre1 = pre1 * gv[j]; }
            }
        }
        if constexpr (HD) {
            bool hd = false;
#pragma unroll
            for (int r = 0; r < R; ++r) hd |= (qv[r] >= 0.5f);
            hdmask |= (uint32_t)hd << l;
        }
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const int sh = SH::template shift<SEC, L>(et, r, l);
            msg[r][l] = bperm(rot_addr(i, gb, sh == 0 ? 0 : P - sh, P), qv[r]);
        }
    }
    return hdmask;
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
__device__ __forceinline__ bool lane_syndrome_ok(const BpArgs& a, uint32_t hdmask, uint32_t sbits, int i, int gb)
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
            x ^= ((uint32_t)bperm_i(rot_addr(i, gb, sh == 0 ? 0 : P - sh, P), (int)hdmask) >> l) & 1u;
        }
        match &= (x == ((sbits >> r) & 1u));
    }
    return match;
}

// One BP iteration; returns true if this group stops after it.
template <int R, int L, int SEC, int STOP, bool LAST, class SH>
__device__ __forceinline__ bool iteration(const BpArgs& a, float (&msg)[R][L], uint32_t sbits, int n, int i, int gb,
                                          float pp, float one_minus_pp)
{
    const int P = SH::P(a);
    check_pass<R, L>(msg, sbits);
    const uint32_t hdmask = var_pass<R, L, SEC, LAST, STOP == QEC_STOP_SYNDROME, SH>(a, msg, i, gb, pp, one_minus_pp);
    if constexpr (STOP == QEC_STOP_REF) {
        if (n % 10 == 0) return group_all(lane_converged<R, L>(msg), gb, P);  // DecoderCPU.h:287-290
    } else if constexpr (STOP == QEC_STOP_SYNDROME) {
        return group_all(lane_syndrome_ok<R, L, SEC, SH>(a, hdmask, sbits, i, gb), gb, P);
    }
    return false;
}

template <int R, int L, int SEC, int STOP, class SH>
__device__ __forceinline__ void decode_sector(const BpArgs& a, int i, int gb, long long b, bool in_range, float pp,
                                              uint32_t& flags, int& iters_out)
{
    const int P = SH::P(a);
    const int m = R * P;
    const uint8_t* __restrict__ s = SEC ? a.sZ : a.sX;

    // syndrome bits of checks (r, i)
    uint32_t sbits = 0;
    if (in_range) {
#pragma unroll
        for (int r = 0; r < R; ++r) sbits |= (uint32_t)(s[b * m + r * P + i] & 1) << r;
    }

    // InitVarNodes: every edge starts at p' (DecoderCPU.h:135-148, 265-267)
    float msg[R][L];
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
        for (int l = 0; l < L; ++l) msg[r][l] = pp;

    const float one_minus_pp = 1.0f - pp;
    const int N = a.maxIter;
    bool active = in_range;  // group-uniform
    int it = 0;
    int n = 0;
    // iterations 0 .. N-2 (DecoderCPU.h:280-291); the last one is peeled below
    for (; n < N - 1; ++n) {
        if constexpr (STOP != QEC_STOP_FIXED) {
            if (!__any(active)) break;  // DecoderCPU.h:282
        }
        if (active) {
            ++it;
            if (iteration<R, L, SEC, STOP, false, SH>(a, msg, sbits, n, i, gb, pp, one_minus_pp)) active = false;
        }
    }
    if (n == N - 1 && active) {
        ++it;
        iteration<R, L, SEC, STOP, true, SH>(a, msg, sbits, n, i, gb, pp, one_minus_pp);
    }

    // ---- post-processing of Decode (DecoderCPU.h:354-384) ----
    const bool conv = group_all(lane_converged<R, L>(msg), gb, P);
    uint8_t* __restrict__ e = SEC ? a.eZ : a.eX;
    const int* et = SH::template table<SEC>(a);
    uint32_t hdmask = 0;
#pragma unroll
    for (int l = 0; l < L; ++l) {
        bool hd = false;  // e[v] = any edge message >= 0.5f (DecoderCPU.h:354-373)
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const int sh = SH::template shift<SEC, L>(et, r, l);
            hd |= bperm(rot_addr(i, gb, sh, P), msg[r][l]) >= 0.5f;
        }
        hdmask |= (uint32_t)hd << l;
        if (in_range) e[b * (long long)a.n + l * P + i] = (uint8_t)hd;
    }
    const bool syn_ok = group_all(lane_syndrome_ok<R, L, SEC, SH>(a, hdmask, sbits, i, gb), gb, P);

    if (!syn_ok) flags |= SEC ? QEC_SYNDROME_FAIL_Z : QEC_SYNDROME_FAIL_X;
    if (!conv) flags |= SEC ? QEC_CONVERGENCE_FAIL_Z : QEC_CONVERGENCE_FAIL_X;
    iters_out = it;

    if (a.q != nullptr && in_range) {
        const long long qb = b * (long long)(a.mX + a.mZ) * L + (SEC ? (long long)a.mX * L : 0);
#pragma unroll
        for (int r = 0; r < R; ++r)
#pragma unroll
            for (int l = 0; l < L; ++l) a.q[qb + (long long)(r * P + i) * L + l] = msg[r][l];
    }
}

template <int RX, int RZ, int L, int STOP, class SH>
__global__ __launch_bounds__(256) void bp_decode_kernel(const BpArgs a)
{
    const int lane = threadIdx.x & 63;
    const long long wave = (long long)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    const int P = SH::P(a);
    const int G = SH::kStatic ? 64 / P : a.G;
    const int g = lane / P;
    const int i = lane - g * P;
    const int gb = g * P;
    const long long b = wave * G + g;
    const bool in_range = (g < G) && (b < a.B);
    if (!__any(in_range)) return;

    // p' = (2/3) p, as the reference writes it (DecoderCPU.h:259)
    const float pp = 2.0f / 3.0f * a.errorProbability;
    uint32_t flags = 0;
    int itX = 0, itZ = 0;
    decode_sector<RX, L, 0, STOP, SH>(a, i, gb, b, in_range, pp, flags, itX);
    decode_sector<RZ, L, 1, STOP, SH>(a, i, gb, b, in_range, pp, flags, itZ);
    if (in_range && i == 0) {
        a.flags[b] = (uint8_t)flags;
        if (a.iters != nullptr) {
            a.iters[2 * b] = itX;
            a.iters[2 * b + 1] = itZ;
        }
    }
}

// ---- variant table ----------------------------------------------------------
using KernelFn = void (*)(const BpArgs);

struct Variant {
    int J, K, L;
    int P, sigma, tau;  // P > 0: specialised to the generator's tables for these parameters
    KernelFn fn[3];     // indexed by stop rule
    const char* name;
};

template <int J, int K, int L, class SH>
static Variant make_variant(int P, int S, int T, const char* name)
{
    return Variant{J, K, L, P, S, T,
                   {bp_decode_kernel<J, K, L, QEC_STOP_REF, SH>, bp_decode_kernel<J, K, L, QEC_STOP_FIXED, SH>,
                    bp_decode_kernel<J, K, L, QEC_STOP_SYNDROME, SH>},
                   name};
}
template <int J, int K, int L>
static Variant rt()
{
    return make_variant<J, K, L, RuntimeShifts>(0, 0, 0, "wave-circulant runtime-shift");
}
template <int J, int K, int L, int P, int S, int T>
static Variant gen()
{
    return make_variant<J, K, L, GeneratedShifts<J, K, L, P, S, T>>(P, S, T, "wave-circulant generated-shift");
}

static const Variant kVariants[] = {
    // specialised: the two code files the reference ships
    gen<4, 5, 10, 61, 9, 49>(),
    gen<3, 3, 6, 7, 2, 3>(),
    // runtime shifts, any P <= 64 with these block shapes
    rt<4, 5, 10>(),
    rt<3, 3, 6>(),
    rt<2, 3, 6>(),
    rt<3, 4, 8>(),
    rt<4, 4, 8>(),
    rt<3, 5, 10>(),
    rt<4, 6, 12>(),
    rt<2, 2, 4>(),
};

struct DecodeLaunch {
    const Variant* v;
};

const void* select_variant(const Code& c, std::string& name)
{
    if (!c.is_qc || c.P > 64 || c.P < 1) return nullptr;
    if (c.J * c.L > kMaxRL || c.K * c.L > kMaxRL) return nullptr;
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

int launch_decode(const void* variant, const Code& c, const uint8_t* sX, const uint8_t* sZ, long long B,
                  float errorProbability, int maxIter, int stop, uint8_t* eX, uint8_t* eZ, uint8_t* flags,
                  int32_t* iters, float* q, hipStream_t stream)
{
    const Variant* v = static_cast<const Variant*>(variant);
    if (B <= 0) return QEC_OK;
    BpArgs a{};
    a.sX = sX; a.sZ = sZ; a.eX = eX; a.eZ = eZ; a.flags = flags; a.iters = iters; a.q = q;
    a.B = B;
    a.P = c.P;
    a.G = 64 / c.P;
    a.n = c.n; a.mX = c.mX; a.mZ = c.mZ;
    a.errorProbability = errorProbability;
    a.maxIter = maxIter < 0 ? 0 : maxIter;
    a.stop = stop;
    for (size_t k = 0; k < c.EX.size(); ++k) a.EX[k] = c.EX[k];
    for (size_t k = 0; k < c.EZ.size(); ++k) a.EZ[k] = c.EZ[k];
    const int wavesPerBlock = 4;
    const long long waves = (B + a.G - 1) / a.G;
    const long long blocks = (waves + wavesPerBlock - 1) / wavesPerBlock;
    if (blocks > 0x7fffffffLL) return fail(QEC_ERR_ARG, "batch too large for one launch");
    hipLaunchKernelGGL(v->fn[stop], dim3((unsigned)blocks), dim3(64 * wavesPerBlock), 0, stream, a);
    hipError_t err = hipGetLastError();
    if (err != hipSuccess) return fail(QEC_ERR_HIP, std::string("bp_decode launch: ") + hipGetErrorString(err));
    return QEC_OK;
}

}  // namespace qec
