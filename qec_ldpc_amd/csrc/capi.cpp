// C ABI of libqecldpc.so (declared in include/qec_ldpc.h).
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstring>
#include <memory>
#include <new>
#include <stdexcept>
#include <algorithm>

#include "../../include/HostDeviceArray.h"
#include "qec_internal.h"

namespace qec {
const char* last_error_cstr();
const void* select_variant(const Code& c, std::string& name);
int launch_decode(const void* variant, const Code& c, const uint8_t* sX, const uint8_t* sZ, long long B,
                  float errorProbability, int maxIter, int stop, uint8_t* eX, uint8_t* eZ, uint8_t* flags,
                  int32_t* iters, float* q, int hardPaths, const int32_t* perm, int split, bool flags_zeroed,
                  hipStream_t stream);
size_t schedule_workspace_bytes(long long B, int mX, int mZ);
long long schedule_max_batch();
int launch_schedule(const uint8_t* sX, const uint8_t* sZ, long long B, int mX, int mZ, void* ws,
                    uint8_t* zero_flags, int32_t** perm_out, hipStream_t st);
bool decode_uses_split(const void* variant, int stop, int split);
int launch_sample_depolarizing(uint64_t seed, uint64_t start, long long B, int n, float p, uint8_t* x, uint8_t* z,
                               hipStream_t st);
int launch_errors_from_draws(const int32_t* idx, const uint8_t* type, long long B, int W, int n, uint8_t* x,
                             uint8_t* z, hipStream_t st);
int launch_syndrome(const Code& c, const int32_t* chkVar, const uint8_t* x, const uint8_t* z, long long B,
                    uint8_t* sX, uint8_t* sZ, hipStream_t st);
void* sparse_plan_create(const Code& c, int device);
void sparse_plan_free(void* plan);
const char* sparse_plan_name(const void* plan);
const int32_t* sparse_plan_chkvar(const void* plan);
int launch_decode_sparse(void* plan, const uint8_t* sX, const uint8_t* sZ, long long B, float errorProbability,
                         int maxIter, int stop, uint8_t* eX, uint8_t* eZ, uint8_t* flags, int32_t* iters, float* q,
                         hipStream_t stream);
int launch_pack_decisions(const uint8_t* eX, const uint8_t* eZ, const uint8_t* flags, long long B, int n, uint8_t* out,
                          hipStream_t st);
int launch_statistics(const Code& c, const uint64_t* imp_dev, const uint8_t* x, const uint8_t* z, const uint8_t* eX,
                      const uint8_t* eZ, const uint8_t* flags, long long B, unsigned long long* counters, hipStream_t st);
}  // namespace qec

using namespace qec;

struct qec_code {
    Code c;
};

struct qec_decoder {
    std::shared_ptr<const Code> code;
    int device = 0;
    int engine = QEC_ENGINE_CIRCULANT;
    const void* variant = nullptr;  // wave-circulant kernel variant (bp_decode.hip)
    void* sparse = nullptr;         // sparse-graph plan (bp_sparse.hip)
    std::string variant_name;
    int hard_paths = 1;             // QEC_OPT_HARD_PATHS
    int cycle_jump = 1;             // QEC_OPT_CYCLE_JUMP
    int schedule = 1;               // QEC_OPT_SCHEDULE (0 off, 1 auto, 2 always)
    int sector_split = 1;           // QEC_OPT_SECTOR_SPLIT (0 off, 1 auto, 2 on)
    DeviceArray<uint8_t> sched;     // dispatch-order workspace (schedule.hip)
    hipStream_t stream = nullptr;
    // staging for the host-pointer entry point (DecoderGPU's device vectors, DecoderGPU.h:28-35)
    DeviceArray<uint8_t> sX, sZ, eX, eZ, flags;
    DeviceArray<int32_t> iters;
    DeviceArray<float> q;
    // Monte-Carlo workspace (qec_monte_carlo / qec_get_statistics)
    DeviceArray<uint64_t> imp;  // bit-packed non-zero I-P rows
    DeviceArray<uint8_t> mx, mz, msX, msZ, meX, meZ, mfl, mtype;
    DeviceArray<int32_t> mit, midx;
    DeviceArray<unsigned long long> mcount;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
};

#define QEC_HIP_CHECK(expr)                                                                     \
    do {                                                                                         \
        hipError_t e_ = (expr);                                                                  \
        if (e_ != hipSuccess) return fail(QEC_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(e_)); \
    } while (0)

extern "C" {

const char* qec_last_error(void) { return last_error_cstr(); }
int qec_abi_version(void) { return QEC_LDPC_ABI_VERSION; }

qec_code* qec_code_load(const char* path)
{
    if (!path) { fail(QEC_ERR_ARG, "qec_code_load: null path"); return nullptr; }
    auto* h = new (std::nothrow) qec_code;
    if (!h) { fail(QEC_ERR_NOMEM, "qec_code_load: out of memory"); return nullptr; }
    if (load_code(path, h->c) != QEC_OK) { delete h; return nullptr; }
    return h;
}

qec_code* qec_code_generate(int J, int K, int L, int P, int sigma, int tau)
{
    auto* h = new (std::nothrow) qec_code;
    if (!h) { fail(QEC_ERR_NOMEM, "qec_code_generate: out of memory"); return nullptr; }
    if (generate_code(J, K, L, P, sigma, tau, h->c) != QEC_OK) { delete h; return nullptr; }
    return h;
}

int qec_code_free(qec_code* code)
{
    delete code;
    return QEC_OK;
}

int qec_code_params(const qec_code* h, int* out)
{
    if (!h || !out) return fail(QEC_ERR_ARG, "qec_code_params: null argument");
    const Code& c = h->c;
    const int v[9] = {c.J, c.K, c.L, c.P, c.sigma, c.tau, c.n, c.mX, c.mZ};
    std::memcpy(out, v, sizeof v);
    return QEC_OK;
}

int qec_code_exponents(const qec_code* h, int sector, int* out)
{
    if (!h || !out || (sector != 0 && sector != 1)) return fail(QEC_ERR_ARG, "qec_code_exponents: bad argument");
    if (!h->c.is_qc) return fail(QEC_ERR_UNSUPPORTED, "code is not built from circulant permutation blocks");
    const std::vector<int>& E = sector ? h->c.EZ : h->c.EX;
    std::memcpy(out, E.data(), E.size() * sizeof(int));
    return QEC_OK;
}

int qec_code_pcm(const qec_code* h, int sector, uint8_t* out)
{
    if (!h || !out || (sector != 0 && sector != 1)) return fail(QEC_ERR_ARG, "qec_code_pcm: bad argument");
    const std::vector<uint8_t>& H = sector ? h->c.pcmZ : h->c.pcmX;
    std::memcpy(out, H.data(), H.size());
    return QEC_OK;
}

int qec_code_describe(const qec_code* h, char* buf, size_t len)
{
    if (!h || !buf || !len) return fail(QEC_ERR_ARG, "qec_code_describe: bad argument");
    const std::string s = h->c.describe();
    std::snprintf(buf, len, "%s", s.c_str());
    return QEC_OK;
}

int qec_code_syndrome(const qec_code* h, int sector, const uint8_t* e, size_t B, uint8_t* s)
{
    if (!h || (B && (!e || !s)) || (sector != 0 && sector != 1)) return fail(QEC_ERR_ARG, "qec_code_syndrome: bad argument");
    const Code& c = h->c;
    const int m = sector ? c.mZ : c.mX;
    for (size_t b = 0; b < B; ++b) host_syndrome(c, sector, e + b * c.n, s + b * m);
    return QEC_OK;
}

int qec_code_check_logical(const qec_code* h, const uint8_t* ex, const uint8_t* ez, size_t B, uint8_t* out)
{
    if (!h || (B && (!ex || !ez || !out))) return fail(QEC_ERR_ARG, "qec_code_check_logical: bad argument");
    if (h->c.imp.empty()) return fail(QEC_ERR_UNSUPPORTED, "code has no I-P matrix (generated codes carry none)");
    for (size_t b = 0; b < B; ++b) out[b] = host_check_logical(h->c, ex + b * h->c.n, ez + b * h->c.n) ? 1 : 0;
    return QEC_OK;
}

qec_decoder* qec_decoder_create(const qec_code* h, int device, size_t max_batch)
{
    return qec_decoder_create_engine(h, device, max_batch, QEC_ENGINE_AUTO);
}

qec_decoder* qec_decoder_create_engine(const qec_code* h, int device, size_t max_batch, int engine)
{
    if (!h) { fail(QEC_ERR_ARG, "qec_decoder_create: null code"); return nullptr; }
    if (device < 0) { fail(QEC_ERR_ARG, "qec_decoder_create: the product has no CPU engine; device must be >= 0"); return nullptr; }
    if (engine < QEC_ENGINE_AUTO || engine > QEC_ENGINE_SPARSE) {
        fail(QEC_ERR_ARG, "qec_decoder_create_engine: unknown engine");
        return nullptr;
    }
    std::string name;
    const void* v = engine == QEC_ENGINE_SPARSE ? nullptr : select_variant(h->c, name);
    if (!v && engine == QEC_ENGINE_CIRCULANT) {
        fail(QEC_ERR_UNSUPPORTED, "no wave-circulant kernel for this code shape (" + h->c.describe() +
                                      "): needs circulant-permutation blocks, P <= 64 and an instantiated (J,K,L)");
        return nullptr;
    }
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) {
        fail(QEC_ERR_HIP, "qec_decoder_create: no HIP device available");
        return nullptr;
    }
    if (device >= ndev) { fail(QEC_ERR_ARG, "qec_decoder_create: device ordinal out of range"); return nullptr; }
    if (hipSetDevice(device) != hipSuccess) { fail(QEC_ERR_HIP, "hipSetDevice failed"); return nullptr; }
    auto* d = new (std::nothrow) qec_decoder;
    if (!d) { fail(QEC_ERR_NOMEM, "qec_decoder_create: out of memory"); return nullptr; }
    d->code = std::make_shared<const Code>(h->c);
    d->device = device;
    d->variant = v;
    d->variant_name = name;
    if (!v) {  // AUTO without a wave-circulant kernel, or SPARSE requested
        d->engine = QEC_ENGINE_SPARSE;
        d->sparse = sparse_plan_create(*d->code, device);
        if (!d->sparse) { delete d; return nullptr; }  // error text set by the plan
        d->variant_name = sparse_plan_name(d->sparse);
    }
    if (hipStreamCreateWithFlags(&d->stream, hipStreamNonBlocking) != hipSuccess) {
        delete d;
        fail(QEC_ERR_HIP, "hipStreamCreate failed");
        return nullptr;
    }
    try {
        // the dispatch-order workspace is sized up front so that qec_decode_batch_dev allocates
        // nothing for batches up to max_batch (graph capture); staging grows on demand
        if (max_batch > 0 && d->variant && (long long)max_batch <= schedule_max_batch())
            d->sched.reserve(schedule_workspace_bytes((long long)max_batch, d->code->mX, d->code->mZ));
        if (!d->code->imp_rows.empty()) {
            d->imp.reserve(d->code->imp_rows.size());
            if (hipMemcpy(d->imp.data(), d->code->imp_rows.data(), d->code->imp_rows.size() * sizeof(uint64_t),
                          hipMemcpyHostToDevice) != hipSuccess)
                throw std::runtime_error("I-P upload");
        }
        d->mcount.reserve(QEC_MC_NCOUNTERS);
    } catch (const std::exception& ex) {
        (void)hipStreamDestroy(d->stream);
        delete d;
        fail(QEC_ERR_HIP, std::string("qec_decoder_create: ") + ex.what());
        return nullptr;
    }
    if (hipEventCreate(&d->ev0) != hipSuccess || hipEventCreate(&d->ev1) != hipSuccess) {
        (void)hipStreamDestroy(d->stream);
        delete d;
        fail(QEC_ERR_HIP, "hipEventCreate failed");
        return nullptr;
    }
    return d;
}

int qec_decoder_destroy(qec_decoder* d)
{
    if (!d) return QEC_OK;
    (void)hipSetDevice(d->device);
    if (d->ev0) (void)hipEventDestroy(d->ev0);
    if (d->ev1) (void)hipEventDestroy(d->ev1);
    if (d->stream) (void)hipStreamDestroy(d->stream);
    if (d->sparse) sparse_plan_free(d->sparse);
    delete d;
    return QEC_OK;
}

int qec_decoder_describe(const qec_decoder* d, char* buf, size_t len)
{
    if (!d || !buf || !len) return fail(QEC_ERR_ARG, "qec_decoder_describe: bad argument");
    std::snprintf(buf, len, "%s", d->variant_name.c_str());
    return QEC_OK;
}

int qec_decoder_set_option(qec_decoder* d, int option, int value)
{
    if (!d) return fail(QEC_ERR_ARG, "qec_decoder_set_option: null decoder");
    switch (option) {
    case QEC_OPT_HARD_PATHS: d->hard_paths = value != 0; return QEC_OK;
    case QEC_OPT_CYCLE_JUMP: d->cycle_jump = value != 0; return QEC_OK;
    case QEC_OPT_SCHEDULE:
        if (value < 0 || value > 2) return fail(QEC_ERR_ARG, "qec_decoder_set_option: QEC_OPT_SCHEDULE is 0, 1 or 2");
        d->schedule = value;
        return QEC_OK;
    case QEC_OPT_SECTOR_SPLIT:
        if (value < 0 || value > 2) return fail(QEC_ERR_ARG, "qec_decoder_set_option: QEC_OPT_SECTOR_SPLIT is 0, 1 or 2");
        d->sector_split = value;
        return QEC_OK;
    default: return fail(QEC_ERR_ARG, "qec_decoder_set_option: unknown option");
    }
}

int qec_decoder_get_option(const qec_decoder* d, int option, int* value)
{
    if (!d || !value) return fail(QEC_ERR_ARG, "qec_decoder_get_option: bad argument");
    switch (option) {
    case QEC_OPT_HARD_PATHS: *value = d->hard_paths; return QEC_OK;
    case QEC_OPT_CYCLE_JUMP: *value = d->cycle_jump; return QEC_OK;
    case QEC_OPT_SCHEDULE: *value = d->schedule; return QEC_OK;
    case QEC_OPT_SECTOR_SPLIT: *value = d->sector_split; return QEC_OK;
    default: return fail(QEC_ERR_ARG, "qec_decoder_get_option: unknown option");
    }
}

// QEC_OPT_SCHEDULE = 1 orders batches from this size on (below it the three extra launches
// cost more than the tail they remove)
constexpr long long kScheduleMinBatch = 4096;

static int dispatch_decode(qec_decoder* d, const uint8_t* sX, const uint8_t* sZ, long long B, float p, int maxIter,
                           int stop, uint8_t* eX, uint8_t* eZ, uint8_t* flags, int32_t* iters, float* q, hipStream_t st)
{
    if (d->engine == QEC_ENGINE_SPARSE)
        return launch_decode_sparse(d->sparse, sX, sZ, B, p, maxIter, stop, eX, eZ, flags, iters, q, st);
    const int hp = d->hard_paths ? (QEC_HP_FORMS | (d->cycle_jump ? QEC_HP_CYCLE : 0)) : 0;
    const int32_t* perm = nullptr;
    bool zeroed = false;
    if (B > 1 && B <= schedule_max_batch() && (d->schedule == 2 || (d->schedule == 1 && B >= kScheduleMinBatch))) {
        try {
            d->sched.reserve(schedule_workspace_bytes(B, d->code->mX, d->code->mZ));
        } catch (const std::exception& ex) {
            return fail(QEC_ERR_NOMEM, std::string("decode: dispatch-order workspace: ") + ex.what());
        }
        // a sector-split launch ORs its flags into a zeroed array: the order pass zeroes it
        zeroed = decode_uses_split(d->variant, stop, d->sector_split);
        int32_t* pm = nullptr;
        const int rc = launch_schedule(sX, sZ, B, d->code->mX, d->code->mZ, d->sched.data(), zeroed ? flags : nullptr,
                                       &pm, st);
        if (rc) return rc;
        perm = pm;
    }
    return launch_decode(d->variant, *d->code, sX, sZ, B, p, maxIter, stop, eX, eZ, flags, iters, q, hp, perm,
                         d->sector_split, zeroed, st);
}

static const int32_t* syndrome_table(const qec_decoder* d)
{
    return d->engine == QEC_ENGINE_SPARSE ? sparse_plan_chkvar(d->sparse) : nullptr;
}

static int check_decode_args(const qec_decoder* d, const void* sX, const void* sZ, size_t B, int stop,
                             const void* eX, const void* eZ, const void* flags)
{
    if (!d) return fail(QEC_ERR_ARG, "decode: null decoder");
    if (stop < QEC_STOP_REF || stop > QEC_STOP_SYNDROME) return fail(QEC_ERR_ARG, "decode: unknown stop rule");
    if (B && (!sX || !sZ || !eX || !eZ || !flags)) return fail(QEC_ERR_ARG, "decode: null buffer");
    if (B > (size_t)1 << 40) return fail(QEC_ERR_ARG, "decode: batch too large");
    return QEC_OK;
}

int qec_decode_batch_dev(qec_decoder* d, const uint8_t* sX, const uint8_t* sZ, size_t B, float p, int maxIter,
                         int stop, uint8_t* eX, uint8_t* eZ, uint8_t* flags, int32_t* iters, float* q, void* stream)
{
    int rc = check_decode_args(d, sX, sZ, B, stop, eX, eZ, flags);
    if (rc) return rc;
    QEC_HIP_CHECK(hipSetDevice(d->device));
    return dispatch_decode(d, sX, sZ, (long long)B, p, maxIter, stop, eX, eZ, flags, iters, q,
                           static_cast<hipStream_t>(stream));
}

int qec_decode_batch(qec_decoder* d, const uint8_t* sX, const uint8_t* sZ, size_t B, float p, int maxIter, int stop,
                     uint8_t* eX, uint8_t* eZ, uint8_t* flags, int32_t* iters, float* q)
{
    int rc = check_decode_args(d, sX, sZ, B, stop, eX, eZ, flags);
    if (rc) return rc;
    if (B == 0) return QEC_OK;
    QEC_HIP_CHECK(hipSetDevice(d->device));
    const Code& c = *d->code;
    const size_t qn = (size_t)(c.mX + c.mZ) * c.L;
    try {
        d->sX.reserve(B * c.mX); d->sZ.reserve(B * c.mZ);
        d->eX.reserve(B * c.n); d->eZ.reserve(B * c.n); d->flags.reserve(B);
        if (iters) d->iters.reserve(2 * B);
        if (q) d->q.reserve(B * qn);
    } catch (const std::exception& ex) {
        return fail(QEC_ERR_HIP, std::string("device staging allocation: ") + ex.what());
    }
    hipStream_t st = d->stream;
    QEC_HIP_CHECK(hipMemcpyAsync(d->sX.data(), sX, B * c.mX, hipMemcpyHostToDevice, st));
    QEC_HIP_CHECK(hipMemcpyAsync(d->sZ.data(), sZ, B * c.mZ, hipMemcpyHostToDevice, st));
    rc = dispatch_decode(d, d->sX.data(), d->sZ.data(), (long long)B, p, maxIter, stop, d->eX.data(),
                       d->eZ.data(), d->flags.data(), iters ? d->iters.data() : nullptr, q ? d->q.data() : nullptr, st);
    if (rc) return rc;
    QEC_HIP_CHECK(hipMemcpyAsync(eX, d->eX.data(), B * c.n, hipMemcpyDeviceToHost, st));
    QEC_HIP_CHECK(hipMemcpyAsync(eZ, d->eZ.data(), B * c.n, hipMemcpyDeviceToHost, st));
    QEC_HIP_CHECK(hipMemcpyAsync(flags, d->flags.data(), B, hipMemcpyDeviceToHost, st));
    if (iters) QEC_HIP_CHECK(hipMemcpyAsync(iters, d->iters.data(), 2 * B * sizeof(int32_t), hipMemcpyDeviceToHost, st));
    if (q) QEC_HIP_CHECK(hipMemcpyAsync(q, d->q.data(), B * qn * sizeof(float), hipMemcpyDeviceToHost, st));
    QEC_HIP_CHECK(hipStreamSynchronize(st));
    return QEC_OK;
}

int qec_sample_fixed_weight(uint32_t seed, int W, size_t count, int n, uint8_t* x, uint8_t* z)
{
    if (n <= 0 || W < 0 || (count && (!x || !z))) return fail(QEC_ERR_ARG, "qec_sample_fixed_weight: bad argument");
    Mt19937 g(seed);
    std::memset(x, 0, count * n);
    std::memset(z, 0, count * n);
    for (size_t c = 0; c < count; ++c)
        for (int w = 0; w < W; ++w) {
            const uint32_t index = g.msvc_uniform((uint32_t)n);
            const uint32_t type = g.msvc_uniform(3u);  // x = 0, y = 1, z = 2
            if (type == 0 || type == 1) x[c * n + index] = 1;
            if (type == 2 || type == 1) z[c * n + index] = 1;
        }
    return QEC_OK;
}

static void mc_reserve(qec_decoder* d, size_t B, int W)
{
    const Code& c = *d->code;
    d->mx.reserve(B * c.n); d->mz.reserve(B * c.n);
    d->msX.reserve(B * c.mX); d->msZ.reserve(B * c.mZ);
    d->meX.reserve(B * c.n); d->meZ.reserve(B * c.n);
    d->mfl.reserve(B); d->mit.reserve(2 * B);
    if (W > 0) { d->midx.reserve(B * W); d->mtype.reserve(B * W); }
}

// decode + statistics of the batch already in d->mx / d->mz; adds decode time
static int mc_decode_and_count(qec_decoder* d, long long B, float p, int maxIter, int stop, double& decode_s)
{
    const Code& c = *d->code;
    hipStream_t st = d->stream;
    int rc = launch_syndrome(c, syndrome_table(d), d->mx.data(), d->mz.data(), B, d->msX.data(), d->msZ.data(), st);
    if (rc) return rc;
    QEC_HIP_CHECK(hipEventRecord(d->ev0, st));
    rc = dispatch_decode(d, d->msX.data(), d->msZ.data(), B, p, maxIter, stop, d->meX.data(), d->meZ.data(),
                       d->mfl.data(), d->mit.data(), nullptr, st);
    if (rc) return rc;
    QEC_HIP_CHECK(hipEventRecord(d->ev1, st));
    rc = launch_statistics(c, d->imp.data(), d->mx.data(), d->mz.data(), d->meX.data(), d->meZ.data(), d->mfl.data(), B,
                           d->mcount.data(), st);
    if (rc) return rc;
    QEC_HIP_CHECK(hipEventSynchronize(d->ev1));
    float ms = 0;
    QEC_HIP_CHECK(hipEventElapsedTime(&ms, d->ev0, d->ev1));
    decode_s += ms * 1e-3;
    return QEC_OK;
}

// GetStatistics (DecoderCPU.h:392-530).  The errors are the reference's: W (index, type) draws
// per sample from one mt19937(seed) stream through VS2015's uniform_int_distribution, drawn on
// the host in sample order (the stream is sequential).  Everything after the draws runs on the
// GPU: error expansion, syndromes, decode (reference stop rule), I-P check, counters.
int qec_get_statistics(qec_decoder* d, int W, int numErrors, float p, int maxIter, uint32_t seed, int nThreads,
                       qec_stats* out)
{
    if (!d || !out || numErrors < 0 || W < 0) return fail(QEC_ERR_ARG, "qec_get_statistics: bad argument");
    const Code& c = *d->code;
    if (c.imp.empty()) return fail(QEC_ERR_UNSUPPORTED, "qec_get_statistics: code has no I-P matrix for the logical check");
    if (nThreads < 1) nThreads = 1;
    QEC_HIP_CHECK(hipSetDevice(d->device));
    const auto t0 = std::chrono::high_resolution_clock::now();
    const long tested = (long)(numErrors / nThreads) * nThreads;  // DecoderCPU.h:426,527
    const long CH = 1 << 16;
    const int n = c.n;
    hipStream_t st = d->stream;
    try {
        mc_reserve(d, (size_t)std::min<long>(CH, std::max<long>(tested, 1)), W);
    } catch (const std::exception& ex) {
        return fail(QEC_ERR_HIP, std::string("qec_get_statistics: ") + ex.what());
    }
    QEC_HIP_CHECK(hipMemsetAsync(d->mcount.data(), 0, QEC_MC_NCOUNTERS * sizeof(unsigned long long), st));
    PinnedArray<int32_t> hidx;
    PinnedArray<uint8_t> htype;
    hidx.reserve((size_t)std::min<long>(CH, std::max<long>(tested, 1)) * std::max(W, 1));
    htype.reserve((size_t)std::min<long>(CH, std::max<long>(tested, 1)) * std::max(W, 1));
    Mt19937 g(seed);
    double dec_s = 0;
    for (long base = 0; base < tested; base += CH) {
        const long cnt = std::min(CH, tested - base);
        for (long s = 0; s < cnt; ++s)
            for (int w = 0; w < W; ++w) {
                hidx[s * W + w] = (int32_t)g.msvc_uniform((uint32_t)n);  // index, then type (DecoderCPU.h:452-454)
                htype[s * W + w] = (uint8_t)g.msvc_uniform(3u);
            }
        if (W > 0) {
            QEC_HIP_CHECK(hipMemcpyAsync(d->midx.data(), hidx.data(), (size_t)cnt * W * sizeof(int32_t),
                                         hipMemcpyHostToDevice, st));
            QEC_HIP_CHECK(hipMemcpyAsync(d->mtype.data(), htype.data(), (size_t)cnt * W, hipMemcpyHostToDevice, st));
        }
        int rc = launch_errors_from_draws(d->midx.data(), d->mtype.data(), cnt, W, n, d->mx.data(), d->mz.data(), st);
        if (rc) return rc;
        rc = mc_decode_and_count(d, cnt, p, maxIter, QEC_STOP_REF, dec_s);
        if (rc) return rc;
    }
    unsigned long long cn[QEC_MC_NCOUNTERS];
    QEC_HIP_CHECK(hipMemcpyAsync(cn, d->mcount.data(), sizeof cn, hipMemcpyDeviceToHost, st));
    QEC_HIP_CHECK(hipStreamSynchronize(st));
    const auto t1 = std::chrono::high_resolution_clock::now();
    std::memset(out, 0, sizeof *out);
    out->randSeed = seed;
    out->numErrorsTested = (uint32_t)tested;
    out->numXErrorsTested = (uint32_t)cn[QEC_MC_WITHX];
    out->numZErrorsTested = (uint32_t)cn[QEC_MC_WITHZ];
    out->errorWeight = (uint32_t)W;
    out->corrected = (uint32_t)cn[QEC_MC_CORRECTED];
    out->syndromeErrorsX = (uint32_t)cn[QEC_MC_SYNX];
    out->syndromeErrorsZ = (uint32_t)cn[QEC_MC_SYNZ];
    out->logicalErrors = (uint32_t)cn[QEC_MC_LOGICAL];
    out->convergenceFailX = (uint32_t)cn[QEC_MC_CONVX];
    out->convergenceFailZ = (uint32_t)cn[QEC_MC_CONVZ];
    out->durationMicroSeconds = std::chrono::duration_cast<std::chrono::microseconds>(t1 - t0).count();
    return QEC_OK;
}

int qec_sample_depolarizing_dev(qec_decoder* d, uint64_t seed, uint64_t start, size_t B, float p, uint8_t* x,
                                uint8_t* z, void* stream)
{
    if (!d || (B && (!x || !z))) return fail(QEC_ERR_ARG, "qec_sample_depolarizing_dev: bad argument");
    QEC_HIP_CHECK(hipSetDevice(d->device));
    return launch_sample_depolarizing(seed, start, (long long)B, d->code->n, p, x, z, static_cast<hipStream_t>(stream));
}

int qec_syndrome_dev(qec_decoder* d, const uint8_t* x, const uint8_t* z, size_t B, uint8_t* sX, uint8_t* sZ,
                     void* stream)
{
    if (!d || (B && (!x || !z || !sX || !sZ))) return fail(QEC_ERR_ARG, "qec_syndrome_dev: bad argument");
    QEC_HIP_CHECK(hipSetDevice(d->device));
    return launch_syndrome(*d->code, syndrome_table(d), x, z, (long long)B, sX, sZ, static_cast<hipStream_t>(stream));
}

int qec_pack_decisions_dev(qec_decoder* d, const uint8_t* eX, const uint8_t* eZ, const uint8_t* flags, size_t B,
                           uint8_t* out, void* stream)
{
    if (!d || (B && (!eX || !eZ || !flags || !out))) return fail(QEC_ERR_ARG, "qec_pack_decisions_dev: bad argument");
    if (B > (size_t)1 << 36) return fail(QEC_ERR_ARG, "qec_pack_decisions_dev: batch too large");
    QEC_HIP_CHECK(hipSetDevice(d->device));
    return launch_pack_decisions(eX, eZ, flags, (long long)B, d->code->n, out, static_cast<hipStream_t>(stream));
}

int qec_statistics_dev(qec_decoder* d, const uint8_t* x, const uint8_t* z, const uint8_t* eX, const uint8_t* eZ,
                       const uint8_t* flags, size_t B, uint64_t* counters, void* stream)
{
    if (!d || !counters || (B && (!x || !z || !eX || !eZ || !flags)))
        return fail(QEC_ERR_ARG, "qec_statistics_dev: bad argument");
    if (d->code->imp.empty()) return fail(QEC_ERR_UNSUPPORTED, "qec_statistics_dev: code has no I-P matrix");
    QEC_HIP_CHECK(hipSetDevice(d->device));
    return launch_statistics(*d->code, d->imp.data(), x, z, eX, eZ, flags, (long long)B,
                             reinterpret_cast<unsigned long long*>(counters), static_cast<hipStream_t>(stream));
}

int qec_monte_carlo(qec_decoder* d, uint64_t seed, uint64_t start, uint64_t count, float p, int maxIter, int stop,
                    size_t batch, qec_mc_result* out)
{
    if (!d || !out || (stop < QEC_STOP_REF || stop > QEC_STOP_SYNDROME)) return fail(QEC_ERR_ARG, "qec_monte_carlo: bad argument");
    const Code& c = *d->code;
    if (c.imp.empty()) return fail(QEC_ERR_UNSUPPORTED, "qec_monte_carlo: code has no I-P matrix for the logical check");
    QEC_HIP_CHECK(hipSetDevice(d->device));
    if (batch == 0) batch = 65536;
    const auto t0 = std::chrono::high_resolution_clock::now();
    try {
        mc_reserve(d, (size_t)std::min<uint64_t>(batch, std::max<uint64_t>(count, 1)), 0);
    } catch (const std::exception& ex) {
        return fail(QEC_ERR_HIP, std::string("qec_monte_carlo: ") + ex.what());
    }
    hipStream_t st = d->stream;
    QEC_HIP_CHECK(hipMemsetAsync(d->mcount.data(), 0, QEC_MC_NCOUNTERS * sizeof(unsigned long long), st));
    double dec_s = 0;
    uint64_t itx = 0, itz = 0;
    std::vector<int32_t> hit;
    for (uint64_t base = 0; base < count; base += batch) {
        const long long cnt = (long long)std::min<uint64_t>(batch, count - base);
        int rc = launch_sample_depolarizing(seed, start + base, cnt, c.n, p, d->mx.data(), d->mz.data(), st);
        if (rc) return rc;
        rc = mc_decode_and_count(d, cnt, p, maxIter, stop, dec_s);
        if (rc) return rc;
        hit.resize(2 * (size_t)cnt);
        QEC_HIP_CHECK(hipMemcpyAsync(hit.data(), d->mit.data(), hit.size() * sizeof(int32_t), hipMemcpyDeviceToHost, st));
        QEC_HIP_CHECK(hipStreamSynchronize(st));
        for (long long k = 0; k < cnt; ++k) { itx += hit[2 * k]; itz += hit[2 * k + 1]; }
    }
    unsigned long long cn[QEC_MC_NCOUNTERS];
    QEC_HIP_CHECK(hipMemcpyAsync(cn, d->mcount.data(), sizeof cn, hipMemcpyDeviceToHost, st));
    QEC_HIP_CHECK(hipStreamSynchronize(st));
    const auto t1 = std::chrono::high_resolution_clock::now();
    out->tested = count;
    out->withX = cn[QEC_MC_WITHX]; out->withZ = cn[QEC_MC_WITHZ];
    out->synX = cn[QEC_MC_SYNX]; out->synZ = cn[QEC_MC_SYNZ];
    out->logical = cn[QEC_MC_LOGICAL]; out->corrected = cn[QEC_MC_CORRECTED];
    out->convX = cn[QEC_MC_CONVX]; out->convZ = cn[QEC_MC_CONVZ];
    out->iterationsX = itx; out->iterationsZ = itz;
    out->decodeSeconds = dec_s;
    out->totalSeconds = std::chrono::duration<double>(t1 - t0).count();
    return QEC_OK;
}

}  // extern "C"
