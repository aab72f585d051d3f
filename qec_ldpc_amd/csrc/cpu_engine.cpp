// CPU engine of libqecldpc.so (qec_decoder_create with device = -1): DecoderCPU's decode
// (QEC_LDPC/DecoderCPU.h:150-390) for hosts without a GPU and for the reference's unmodified
// `DecoderCPU decoder(code)` call site (include/DecoderCPU.h).  Product code: an independent
// implementation over edge-major tables built from the code's parity-check matrices (the
// reference keeps dense n x m message matrices and pointer tables); the oracle in oracle/ is
// never linked.
//
// Edge e = c dc + k is check c's k-th variable in ascending order (InitIndexArrays,
// DecoderCPU.h:41-84); q[e] is the variable->check message, r[e] the check->variable one.
// Arithmetic is DecoderCPU's, operation for operation, in IEEE binary32 (this unit is built
// with -ffp-contract=off and no fast-math): the left-fold products in ascending neighbour
// order, 1.0f - 2.0f*q, 0.5f*(1 +/- t), P1 / (P0 + P1) (Appendix A of SURVEY.md).
// Samples are independent: a batch is split over std::threads, one workspace each (the
// reference's one decoder per OpenMP thread, DecoderCPU.h:419-438).
#include <algorithm>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "qec_internal.h"

namespace qec {

namespace {

struct CpuSector {
    int m = 0, dc = 0, dv = 0;
    std::vector<int32_t> chk_var;   // [m][dc] variables of each check, ascending
    std::vector<int32_t> var_edge;  // [n][dv] edges of each variable, ascending check
};

struct CpuPlan {
    int n = 0;
    CpuSector sec[2];
};

bool build_sector(const std::vector<uint8_t>& pcm, int m, int n, CpuSector& s, std::string& why)
{
    s.m = m;
    s.dc = 0;
    for (int v = 0; v < n; ++v) s.dc += pcm[v] != 0;  // row 0's weight (DecoderCPU.h:69)
    int dv = 0;
    for (int c = 0; c < m; ++c) dv += pcm[(size_t)c * n] != 0;  // column 0's weight (:77)
    s.dv = dv;
    if (s.dc <= 0 || dv <= 0) { why = "empty row or column"; return false; }
    s.chk_var.assign((size_t)m * s.dc, 0);
    s.var_edge.assign((size_t)n * dv, 0);
    std::vector<int> fill(n, 0);
    for (int c = 0; c < m; ++c) {
        int k = 0;
        for (int v = 0; v < n; ++v) {
            if (!pcm[(size_t)c * n + v]) continue;
            if (k == s.dc || fill[v] == dv) { why = "irregular row or column weights"; return false; }
            s.chk_var[(size_t)c * s.dc + k] = v;
            s.var_edge[(size_t)v * dv + fill[v]++] = c * s.dc + k;  // checks visited in ascending order
            ++k;
        }
        if (k != s.dc) { why = "irregular row weights"; return false; }
    }
    for (int v = 0; v < n; ++v)
        if (fill[v] != dv) { why = "irregular column weights"; return false; }
    return true;
}

inline bool outside(float x) { return !(x > 0.01f && x < 0.99f); }  // CheckConvergence, DecoderCPU.h:231-246

struct Work {
    std::vector<float> q, r;
    std::vector<uint8_t> e;
};

// One sector's BeliefPropogation + the Decode post-processing (DecoderCPU.h:249-292, 354-384).
// Returns the iterations executed; e gets the hard decision, conv / syn_ok the flag tests.
int decode_sector(const CpuSector& S, int n, const uint8_t* syn, float errorProbability, int N, int stop, Work& w,
                  bool& conv_out, bool& syn_ok, float* q_out)
{
    const int m = S.m, dc = S.dc, dv = S.dv;
    const size_t E = (size_t)m * dc;
    float* q = w.q.data();
    float* r = w.r.data();
    uint8_t* e = w.e.data();
    const float pp = (2.0f / 3.0f) * errorProbability;  // DecoderCPU.h:259
    const float one_minus_pp = 1.0f - pp;
    std::fill(q, q + E, pp);  // InitVarNodes (:135-148, 265-267)
    auto hard_decision = [&]() {
        for (int v = 0; v < n; ++v) {
            bool hd = false;
            for (int j = 0; j < dv; ++j) hd |= q[S.var_edge[(size_t)v * dv + j]] >= 0.5f;  // :354-373
            e[v] = hd;
        }
    };
    auto syndrome_ok = [&]() {
        for (int c = 0; c < m; ++c) {
            uint32_t x = 0;
            for (int k = 0; k < dc; ++k) x ^= e[S.chk_var[(size_t)c * dc + k]];
            if ((x & 1u) != syn[c]) return false;  // exact compare (:381): an entry other than 0/1 never matches
        }
        return true;
    };
    bool conv = false;
    int it = 0;
    for (int iter = 0; iter < N; ++iter) {
        if (stop == QEC_STOP_REF && conv) break;  // :282
        ++it;
        // EqNodeUpdate (:150-186)
        for (int c = 0; c < m; ++c) {
            const float* qc = q + (size_t)c * dc;
            float* rc = r + (size_t)c * dc;
            const bool s = syn[c] != 0;  // truthiness (:178)
            for (int i = 0; i < dc; ++i) {
                float t = 1.0f;
                for (int k = 0; k < dc; ++k)
                    if (k != i) t = t * (1.0f - 2.0f * qc[k]);
                rc[i] = s ? 0.5f * (1.0f + t) : 0.5f * (1.0f - t);
            }
        }
        // VarNodeUpdate (:188-229); the last iteration includes the self message (:216)
        const bool last = iter == N - 1;
        for (int v = 0; v < n; ++v) {
            const int32_t* ve = S.var_edge.data() + (size_t)v * dv;
            for (int j = 0; j < dv; ++j) {
                float P0 = one_minus_pp, P1 = pp;
                for (int k = 0; k < dv; ++k) {
                    if (k == j && !last) continue;
                    const float rk = r[ve[k]];
                    P0 = P0 * (1.0f - rk);
                    P1 = P1 * rk;
                }
                q[ve[j]] = P1 / (P0 + P1);
            }
        }
        if (stop == QEC_STOP_REF) {
            if (iter % 10 == 0) {  // :287-290
                conv = true;
                for (size_t k = 0; k < E && conv; ++k) conv = outside(q[k]);
            }
        } else if (stop == QEC_STOP_SYNDROME) {
            hard_decision();
            if (syndrome_ok()) break;
        }
    }
    hard_decision();
    bool c_all = true;
    for (size_t k = 0; k < E && c_all; ++k) c_all = outside(q[k]);  // :375-378
    conv_out = c_all;
    syn_ok = syndrome_ok();  // :380-384
    if (q_out) std::memcpy(q_out, q, E * sizeof(float));
    return it;
}

}  // namespace

void* cpu_plan_create(const Code& c)
{
    auto* p = new CpuPlan;
    p->n = c.n;
    std::string why;
    if (!build_sector(c.pcmX, c.mX, c.n, p->sec[0], why) || !build_sector(c.pcmZ, c.mZ, c.n, p->sec[1], why)) {
        delete p;
        fail(QEC_ERR_UNSUPPORTED, "CPU engine: " + why + " (DecoderCPU assumes regular degrees)");
        return nullptr;
    }
    return p;
}

void cpu_plan_free(void* plan) { delete static_cast<CpuPlan*>(plan); }

int cpu_threads()
{
    const unsigned h = std::thread::hardware_concurrency();
    return h ? (int)h : 1;
}

// Batched Decode on host buffers; outputs in byte form (eX, eZ, flags) and/or packed records.
int cpu_decode_batch(void* plan, const uint8_t* sX, const uint8_t* sZ, long long B, float p, int maxIter, int stop,
                     uint8_t* eX, uint8_t* eZ, uint8_t* flags, uint8_t* rec, int32_t* iters, float* qf, int threads)
{
    const CpuPlan& P = *static_cast<const CpuPlan*>(plan);
    const int n = P.n, nb = (n + 7) / 8;
    const int mX = P.sec[0].m, mZ = P.sec[1].m;
    const size_t qper = (size_t)mX * P.sec[0].dc + (size_t)mZ * P.sec[1].dc;
    if (threads <= 0) threads = cpu_threads();
    threads = (int)std::max<long long>(1, std::min<long long>(threads, B));
    auto run = [&](long long lo, long long hi) {
        Work w;
        const size_t E = std::max((size_t)mX * P.sec[0].dc, (size_t)mZ * P.sec[1].dc);
        w.q.resize(E);
        w.r.resize(E);
        w.e.resize(n);
        for (long long b = lo; b < hi; ++b) {
            uint8_t f = 0;
            for (int sec = 0; sec < 2; ++sec) {
                const CpuSector& S = P.sec[sec];
                bool conv = false, ok = false;
                float* qo = qf ? qf + b * qper + (sec ? (size_t)mX * P.sec[0].dc : 0) : nullptr;
                const int it = decode_sector(S, n, sec ? sZ + b * mZ : sX + b * mX, p, maxIter, stop, w, conv, ok, qo);
                if (!ok) f |= sec ? QEC_SYNDROME_FAIL_Z : QEC_SYNDROME_FAIL_X;
                if (!conv) f |= sec ? QEC_CONVERGENCE_FAIL_Z : QEC_CONVERGENCE_FAIL_X;
                if (iters) iters[2 * b + sec] = it;
                if (rec) {
                    uint8_t* o = rec + b * (2 * nb + 1) + sec * nb;
                    std::memset(o, 0, nb);
                    for (int v = 0; v < n; ++v) o[v >> 3] |= (uint8_t)(w.e[v] << (v & 7));
                } else {
                    std::memcpy((sec ? eZ : eX) + b * n, w.e.data(), n);
                }
            }
            if (rec) rec[b * (2 * nb + 1) + 2 * nb] = f;
            else flags[b] = f;
        }
    };
    if (threads == 1) {
        run(0, B);
    } else {
        std::vector<std::thread> th;
        for (int t = 0; t < threads; ++t) th.emplace_back(run, B * t / threads, B * (t + 1) / threads);
        for (auto& x : th) x.join();
    }
    return QEC_OK;
}

}  // namespace qec
