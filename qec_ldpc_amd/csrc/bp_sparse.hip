// Sparse-graph BP engine: batched DecoderCPU::Decode (QEC_LDPC/DecoderCPU.h:150-390)
// for ANY code the reference's DecoderCPU accepts -- regular check degree dc = L and
// variable degree J (X) / K (Z), as its constructor assumes (DecoderCPU.h:296-311,
// InitIndexArrays :41-84) -- including codes that are not circulant-permutation QC
// codes, circulant codes with P > 64 and block shapes the wave-circulant engine
// (bp_decode.hip) has no instantiation for.
//
// Design: one workgroup per syndrome pair (grid-stride over the batch).  The X and Z
// Tanner graphs are decoded side by side in one message array, edge-major in the
// reference's own order (check c, slot k = its k-th variable in ascending id), which
// is also the q_final export layout:
//   msg[c * dc + k],  c in [0, mX) for X, [mX, mX + mZ) for Z.
// The array is LDS-resident when it fits (Etot * 4 B + syndrome/hard-decision bytes
// <= 160 KiB per workgroup on gfx950), otherwise it lives in a per-workgroup HBM
// scratch slice (L2-resident in practice).
//   * check pass: thread per check; reads its dc messages (contiguous), forms the
//     leave-one-out products in registers and overwrites them in place.
//   * variable pass: thread per variable; gathers its dv messages through the
//     varEdge table (edge ids in ascending check order), overwrites them in place.
// Each edge is owned by exactly one thread in each pass, so in-place updates are
// race-free; passes are separated by workgroup barriers.
//
// Arithmetic is the same as the wave-circulant engine's (and so the reference's):
// left folds in ascending neighbour order (prefix reuse only), IEEE fp32 with
// denormals, -ffp-contract=off, correctly rounded division, and the two exact FMAs
// documented in bp_decode.hip.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <vector>

#include "../../include/HostDeviceArray.h"
#include "qec_internal.h"

#pragma clang fp contract(off)

namespace qec {

struct SparseArgs {
    const uint8_t* sX;
    const uint8_t* sZ;
    uint8_t* eX;
    uint8_t* eZ;
    uint8_t* flags;
    int32_t* iters;
    float* q;
    const int32_t* chkVar;   // (mX + mZ) x dc: sector-local variable ids, ascending
    const int32_t* varEdge;  // n x dvX (X) then n x dvZ (Z): edge ids, ascending check
    uint8_t* scratch;        // per-workgroup workspace in HBM (nullptr: LDS-resident)
    long long B;
    long long ws_bytes;      // workspace bytes per workgroup
    int n, mX, mZ, dc, dvX, dvZ;
    float errorProbability;
    int maxIter;
};

constexpr int kSparseThreads = 256;

__device__ __forceinline__ bool sp_inside(float x) { return x > 0.01f && x < 0.99f; }

// EqNodeUpdate (DecoderCPU.h:150-186) for one check: out_i = 0.5 -/+ 0.5 * prod_{k != i} (1 - 2 q_k)
template <int MAXDC>
__device__ __forceinline__ void sp_check(float* __restrict__ m, int dc, float h)
{
    float av[MAXDC];
#pragma unroll
    for (int k = 0; k < MAXDC; ++k)
        if (k < dc) av[k] = __builtin_fmaf(-2.0f, m[k], 1.0f);
    float pre = 1.0f;  // av[0] * ... * av[i-1], left fold from 1.0f (1.0f * x == x exactly)
#pragma unroll
    for (int i = 0; i < MAXDC; ++i) {
        if (i < dc) {
            float t = pre;
#pragma unroll
            for (int k = i + 1; k < MAXDC; ++k)
                if (k < dc) t = t * av[k];
            m[i] = __builtin_fmaf(h, t, 0.5f);  // safe in place: av[] already holds every input
            pre = pre * av[i];
        }
    }
}

// VarNodeUpdate (DecoderCPU.h:188-229) for one variable; returns its hard decision
// (any outgoing message >= 0.5f, DecoderCPU.h:354-373).
template <int MAXDV>
__device__ __forceinline__ bool sp_var(float* __restrict__ msg, const int32_t* __restrict__ ve, int dv, float pp,
                                       float omp, bool last)
{
    int idx[MAXDV];
    float g[MAXDV], bv[MAXDV], qv[MAXDV];
#pragma unroll
    for (int j = 0; j < MAXDV; ++j)
        if (j < dv) {
            idx[j] = ve[j];
            g[j] = msg[idx[j]];
            bv[j] = 1.0f - g[j];
        }
    if (last) {  // the final iteration includes the self message (DecoderCPU.h:216)
        float P0 = omp, P1 = pp;
#pragma unroll
        for (int k = 0; k < MAXDV; ++k)
            if (k < dv) { P0 = P0 * bv[k]; P1 = P1 * g[k]; }
        const float qq = P1 / (P0 + P1);
#pragma unroll
        for (int j = 0; j < MAXDV; ++j) qv[j] = qq;
    } else {
        float pre0 = omp, pre1 = pp;
#pragma unroll
        for (int j = 0; j < MAXDV; ++j)
            if (j < dv) {
                float t0 = pre0, t1 = pre1;
#pragma unroll
                for (int k = j + 1; k < MAXDV; ++k)
                    if (k < dv) { t0 = t0 * bv[k]; t1 = t1 * g[k]; }
                qv[j] = t1 / (t0 + t1);
                pre0 = pre0 * bv[j];
                pre1 = pre1 * g[j];
            }
    }
    bool hd = false;
#pragma unroll
    for (int j = 0; j < MAXDV; ++j)
        if (j < dv) {
            msg[idx[j]] = qv[j];
            hd |= qv[j] >= 0.5f;
        }
    return hd;
}

extern __shared__ __attribute__((aligned(16))) uint8_t sp_lds[];

template <int STOP, int MAXDC, int MAXDV, bool LDS>
__global__ __launch_bounds__(kSparseThreads) void bp_sparse_kernel(const SparseArgs a)
{
    const int tid = threadIdx.x, nt = blockDim.x;
    const int n = a.n, mX = a.mX, mZ = a.mZ, m = mX + mZ, dc = a.dc;
    const int EX = mX * dc, E = m * dc;
    uint8_t* ws = LDS ? sp_lds : a.scratch + (long long)blockIdx.x * a.ws_bytes;
    float* msg = reinterpret_cast<float*>(ws);            // E floats
    uint8_t* syn = ws + (size_t)E * sizeof(float);        // m bytes: sX then sZ
    uint8_t* hd = syn + m;                                // 2n bytes: X then Z hard decisions

    const float pp = 2.0f / 3.0f * a.errorProbability;   // DecoderCPU.h:259
    const float omp = 1.0f - pp;
    const int N = a.maxIter < 0 ? 0 : a.maxIter;

    for (long long b = blockIdx.x; b < a.B; b += gridDim.x) {
        // syndromes in, InitVarNodes: every edge starts at p' (DecoderCPU.h:135-148, 265-267)
        // the entry as given: the check update takes its truthiness, the syndrome tests compare it
        // exactly (DecoderCPU.h:178, :381), so an entry other than 0/1 never matches a parity
        for (int c = tid; c < m; c += nt) syn[c] = c < mX ? a.sX[b * mX + c] : a.sZ[b * mZ + (c - mX)];
        for (int e = tid; e < E; e += nt) msg[e] = pp;
        __syncthreads();

        bool actX = true, actZ = true;  // workgroup-uniform
        int itX = 0, itZ = 0;
        for (int it = 0; it < N && (actX || actZ); ++it) {  // BeliefPropogation, DecoderCPU.h:280-291
            const bool last = it == N - 1;
            itX += actX;
            itZ += actZ;
            for (int c = tid; c < m; c += nt) {
                if (c < mX ? !actX : !actZ) continue;
                sp_check<MAXDC>(msg + (size_t)c * dc, dc, syn[c] ? 0.5f : -0.5f);
            }
            __syncthreads();
            for (int v = tid; v < 2 * n; v += nt) {
                const bool z = v >= n;
                if (z ? !actZ : !actX) continue;
                const int dv = z ? a.dvZ : a.dvX;
                const int32_t* ve = a.varEdge + (z ? (size_t)n * a.dvX + (size_t)(v - n) * dv : (size_t)v * dv);
                const bool h = sp_var<MAXDV>(msg, ve, dv, pp, omp, last);
                if (STOP == QEC_STOP_SYNDROME) hd[v] = h;
            }
            __syncthreads();
            if (STOP == QEC_STOP_REF && it % 10 == 0) {  // CheckConvergence, DecoderCPU.h:287-290
                bool bx = false, bz = false;
                for (int e = tid; e < E; e += nt) {
                    const bool in = sp_inside(msg[e]);
                    if (e < EX) bx |= in; else bz |= in;
                }
                const bool anyx = __syncthreads_or(bx), anyz = __syncthreads_or(bz);
                if (actX && !anyx) actX = false;
                if (actZ && !anyz) actZ = false;
            } else if (STOP == QEC_STOP_SYNDROME) {  // hard decision satisfies the syndrome
                bool bx = false, bz = false;
                for (int c = tid; c < m; c += nt) {
                    const bool z = c >= mX;
                    const uint8_t* h = hd + (z ? n : 0);
                    uint32_t x = 0;
                    for (int k = 0; k < dc; ++k) x ^= h[a.chkVar[(size_t)c * dc + k]];
                    if (x != syn[c]) { if (z) bz = true; else bx = true; }
                }
                const bool badx = __syncthreads_or(bx), badz = __syncthreads_or(bz);
                if (actX && !badx) actX = false;
                if (actZ && !badz) actZ = false;
            }
        }

        // ---- post-processing of Decode (DecoderCPU.h:354-384) ----
        bool bx = false, bz = false;
        for (int e = tid; e < E; e += nt) {
            const bool in = sp_inside(msg[e]);
            if (e < EX) bx |= in; else bz |= in;
        }
        for (int v = tid; v < 2 * n; v += nt) {
            const bool z = v >= n;
            const int dv = z ? a.dvZ : a.dvX;
            const int32_t* ve = a.varEdge + (z ? (size_t)n * a.dvX + (size_t)(v - n) * dv : (size_t)v * dv);
            bool h = false;
            for (int j = 0; j < dv; ++j) h |= msg[ve[j]] >= 0.5f;
            hd[v] = h;
            if (z) a.eZ[b * n + (v - n)] = h; else a.eX[b * n + v] = h;
        }
        const bool convFailX = __syncthreads_or(bx), convFailZ = __syncthreads_or(bz);
        bool sx = false, sz = false;
        for (int c = tid; c < m; c += nt) {
            const bool z = c >= mX;
            const uint8_t* h = hd + (z ? n : 0);
            uint32_t x = 0;
            for (int k = 0; k < dc; ++k) x ^= h[a.chkVar[(size_t)c * dc + k]];
            if (x != syn[c]) { if (z) sz = true; else sx = true; }
        }
        const bool synFailX = __syncthreads_or(sx), synFailZ = __syncthreads_or(sz);
        if (a.q != nullptr)
            for (int e = tid; e < E; e += nt) a.q[b * E + e] = msg[e];
        if (tid == 0) {
            uint32_t f = 0;
            if (synFailX) f |= QEC_SYNDROME_FAIL_X;
            if (synFailZ) f |= QEC_SYNDROME_FAIL_Z;
            if (convFailX) f |= QEC_CONVERGENCE_FAIL_X;
            if (convFailZ) f |= QEC_CONVERGENCE_FAIL_Z;
            a.flags[b] = (uint8_t)f;
            if (a.iters != nullptr) { a.iters[2 * b] = itX; a.iters[2 * b + 1] = itZ; }
        }
        __syncthreads();  // the workspace is reused by the next syndrome pair
    }
}

// ---- plan ------------------------------------------------------------------
using SparseFn = void (*)(const SparseArgs);

template <int MAXDC, int MAXDV, bool LDS>
static void sparse_fns(SparseFn (&f)[3])
{
    f[QEC_STOP_REF] = bp_sparse_kernel<QEC_STOP_REF, MAXDC, MAXDV, LDS>;
    f[QEC_STOP_FIXED] = bp_sparse_kernel<QEC_STOP_FIXED, MAXDC, MAXDV, LDS>;
    f[QEC_STOP_SYNDROME] = bp_sparse_kernel<QEC_STOP_SYNDROME, MAXDC, MAXDV, LDS>;
}

struct SparsePlan {
    int n = 0, mX = 0, mZ = 0, dc = 0, dvX = 0, dvZ = 0;
    bool lds = true;
    long long ws_bytes = 0;
    int grid = 0;
    SparseFn fn[3] = {nullptr, nullptr, nullptr};
    DeviceArray<int32_t> chkVar, varEdge;
    DeviceArray<uint8_t> scratch;
    std::string name;
};

// InitIndexArrays (DecoderCPU.h:41-84) for one sector, with the regularity the reference
// assumes checked: row weight dc and column weight dv everywhere.
static bool index_sector(const std::vector<uint8_t>& pcm, int m, int n, int dc, int dv, int edge0, int32_t* chkVar,
                         int32_t* varEdge, std::string& why)
{
    std::vector<int> cnt(n, 0);
    for (int c = 0; c < m; ++c) {
        int k = 0;
        for (int v = 0; v < n; ++v) {
            if (!pcm[(size_t)c * n + v]) continue;
            if (k >= dc || cnt[v] >= dv) { why = "irregular parity-check matrix"; return false; }
            chkVar[(size_t)c * dc + k] = v;
            varEdge[(size_t)v * dv + cnt[v]++] = edge0 + c * dc + k;
            ++k;
        }
        if (k != dc) { why = "irregular parity-check matrix"; return false; }
    }
    for (int v = 0; v < n; ++v)
        if (cnt[v] != dv) { why = "irregular parity-check matrix"; return false; }
    return true;
}

void sparse_plan_free(void* plan) { delete static_cast<SparsePlan*>(plan); }

const char* sparse_plan_name(const void* plan) { return static_cast<const SparsePlan*>(plan)->name.c_str(); }

// Builds the device tables; returns nullptr (with qec_last_error set) if the code is outside
// what the reference decodes or what this engine instantiates.
void* sparse_plan_create(const Code& c, int device)
{
    const int dc = c.L, dvX = c.J, dvZ = c.K, n = c.n, mX = c.mX, mZ = c.mZ;
    if (dc > 32 || dvX > 16 || dvZ > 16) {
        fail(QEC_ERR_UNSUPPORTED, "sparse engine: needs L <= 32 and J, K <= 16");
        return nullptr;
    }
    const long long m = (long long)mX + mZ, E = m * dc;
    std::vector<int32_t> chk((size_t)E), ve((size_t)n * (dvX + dvZ));
    std::string why;
    if (!index_sector(c.pcmX, mX, n, dc, dvX, 0, chk.data(), ve.data(), why) ||
        !index_sector(c.pcmZ, mZ, n, dc, dvZ, mX * dc, chk.data() + (size_t)mX * dc, ve.data() + (size_t)n * dvX,
                      why)) {
        fail(QEC_ERR_UNSUPPORTED, "sparse engine: " + why + " (DecoderCPU assumes row weight L and column weight J/K)");
        return nullptr;
    }
    auto* p = new SparsePlan;
    p->n = n; p->mX = mX; p->mZ = mZ; p->dc = dc; p->dvX = dvX; p->dvZ = dvZ;
    p->ws_bytes = (E * 4 + m + 2LL * n + 15) / 16 * 16;
    p->lds = p->ws_bytes <= 160 * 1024 - 64;
    const int wdc = dc <= 8 ? 8 : dc <= 16 ? 16 : 32;
    const int wdv = std::max(dvX, dvZ) <= 4 ? 4 : std::max(dvX, dvZ) <= 8 ? 8 : 16;
    // instantiated shapes: (8,4) (16,8) (32,16); pick the smallest that covers the code
    if (wdc <= 8 && wdv <= 4) { if (p->lds) sparse_fns<8, 4, true>(p->fn); else sparse_fns<8, 4, false>(p->fn); }
    else if (wdc <= 16 && wdv <= 8) { if (p->lds) sparse_fns<16, 8, true>(p->fn); else sparse_fns<16, 8, false>(p->fn); }
    else { if (p->lds) sparse_fns<32, 16, true>(p->fn); else sparse_fns<32, 16, false>(p->fn); }
    try {
        if (hipSetDevice(device) != hipSuccess) throw std::runtime_error("hipSetDevice");
        int cus = 0;
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || cus <= 0) cus = 256;
        int per_cu = 1;
        if (p->lds) {
            for (SparseFn f : p->fn)
                if (hipFuncSetAttribute(reinterpret_cast<const void*>(f), hipFuncAttributeMaxDynamicSharedMemorySize,
                                        (int)p->ws_bytes) != hipSuccess)
                    throw std::runtime_error("hipFuncSetAttribute(MaxDynamicSharedMemorySize)");
            per_cu = std::max(1, std::min(8, (int)((160 * 1024) / p->ws_bytes)));
        } else {
            per_cu = 4;
        }
        p->grid = cus * per_cu;
        p->chkVar.reserve(chk.size());
        p->varEdge.reserve(ve.size());
        hip_throw(hipMemcpy(p->chkVar.data(), chk.data(), chk.size() * 4, hipMemcpyHostToDevice), "chkVar upload");
        hip_throw(hipMemcpy(p->varEdge.data(), ve.data(), ve.size() * 4, hipMemcpyHostToDevice), "varEdge upload");
        if (!p->lds) p->scratch.reserve((size_t)p->grid * p->ws_bytes);
    } catch (const std::exception& ex) {
        delete p;
        fail(QEC_ERR_HIP, std::string("sparse engine: ") + ex.what());
        return nullptr;
    }
    char buf[192];
    snprintf(buf, sizeof buf, "sparse-graph %s n=%d mX=%d mZ=%d dc=%d dv=%d/%d (%s)", p->lds ? "lds" : "hbm", n, mX, mZ,
             dc, dvX, dvZ, c.describe().c_str());
    p->name = buf;
    return p;
}

const int32_t* sparse_plan_chkvar(const void* plan) { return static_cast<const SparsePlan*>(plan)->chkVar.data(); }
const int32_t* sparse_plan_varedge(const void* plan) { return static_cast<const SparsePlan*>(plan)->varEdge.data(); }

int launch_decode_sparse(void* plan, const uint8_t* sX, const uint8_t* sZ, long long B, float errorProbability,
                         int maxIter, int stop, uint8_t* eX, uint8_t* eZ, uint8_t* flags, int32_t* iters, float* q,
                         hipStream_t stream)
{
    auto* p = static_cast<SparsePlan*>(plan);
    if (B <= 0) return QEC_OK;
    SparseArgs a{};
    a.sX = sX; a.sZ = sZ; a.eX = eX; a.eZ = eZ; a.flags = flags; a.iters = iters; a.q = q;
    a.chkVar = p->chkVar.data();
    a.varEdge = p->varEdge.data();
    a.scratch = p->lds ? nullptr : p->scratch.data();
    a.B = B;
    a.ws_bytes = p->ws_bytes;
    a.n = p->n; a.mX = p->mX; a.mZ = p->mZ; a.dc = p->dc; a.dvX = p->dvX; a.dvZ = p->dvZ;
    a.errorProbability = errorProbability;
    a.maxIter = maxIter;
    const unsigned grid = (unsigned)std::min<long long>(B, p->grid);
    hipLaunchKernelGGL(p->fn[stop], dim3(grid), dim3(kSparseThreads), p->lds ? (size_t)p->ws_bytes : 0, stream, a);
    hipError_t err = hipGetLastError();
    if (err != hipSuccess) return fail(QEC_ERR_HIP, std::string("bp_sparse launch: ") + hipGetErrorString(err));
    return QEC_OK;
}

}  // namespace qec
