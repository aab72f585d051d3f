// C ABI of libqecldpc.so (declared in include/qec_ldpc.h).
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstring>
#include <memory>
#include <new>
#include <stdexcept>
#include <algorithm>
#include <thread>

#include "../../include/HostDeviceArray.h"
#include "qec_internal.h"

namespace {
// The handle's own events order work on one device (the workspace's cross-stream event) or time it
// (the Monte-Carlo ring); neither needs the system-scope release of a default event record (a cache
// writeback and invalidation between the launches around it; profiles/r06/ab/cmp_event_fence.txt).
constexpr unsigned kEvNoFence = hipEventDisableSystemFence;
}  // namespace

namespace qec {
const char* last_error_cstr();
const void* select_variant(const Code& c, std::string& name);
int launch_decode(const void* variant, const Code& c, const uint8_t* sX, const uint8_t* sZ, bool sbits, long long B,
                  float errorProbability, int maxIter, int stop, uint8_t* eX, uint8_t* eZ, uint8_t* flags,
                  uint8_t* rec, int32_t* iters, float* q, int hardPaths, const int32_t* perm, int split,
                  uint32_t* merge, bool merge_zeroed, hipStream_t stream, int rec_stride = 0, bool perm_sectors = false,
                  hipEvent_t done = nullptr);
size_t schedule_workspace_bytes(long long B, int mX, int mZ);
bool schedule_sector_order(long long B, bool sbits, int mX, int mZ);
long long schedule_max_batch();
long long schedule_local_max_batch();
int launch_schedule(const uint8_t* sX, const uint8_t* sZ, bool sbits, long long B, int mX, int mZ, void* ws,
                    uint32_t* zero_merge, bool want_sectors, int32_t** perm_out, bool* sectors_out, hipStream_t st, int method, uint32_t* bar);
bool decode_uses_split(const void* variant, int stop, int split, long long B);
bool decode_needs_merge(const void* variant, int stop, int split, long long B);
int decode_sector_mode(const void* variant, int stop, int split, long long B, float p);
bool decode_has_list(const void* variant);
bool decode_pattern_masks(const void* variant, float errorProbability, uint32_t pats[4]);
int launch_decode_list(const void* variant, const Code& c, const uint8_t* sX, const uint8_t* sZ, long long B,
                       float errorProbability, int maxIter, int hardPaths, uint8_t* rec, int32_t* iters,
                       uint32_t* merge, const int32_t* listX, const int32_t* listZ, const uint32_t* counts,
                       hipStream_t stream, int rec_stride, bool merge_only, int count_stride, hipEvent_t done = nullptr);
bool triage_supported(const Code& c);
bool triage_aligned(const void* sX, const void* sZ);
int launch_triage(const Code& c, const uint32_t* sX, const uint32_t* sZ, long long B, const uint32_t pats[4],
                  uint8_t* rec, int32_t* iters, uint32_t* merge, int32_t* listX, int32_t* listZ, uint32_t* counts,
                  hipStream_t st, int rec_stride = 0);
bool decode_has_phase_stats(const void* variant, int stop);
int launch_sample_depolarizing(uint64_t seed, uint64_t start, long long B, int n, float p, uint8_t* x, uint8_t* z,
                               hipStream_t st);
int launch_mc_errors_syndrome(int src, const McArgsHost& h, hipStream_t st);
bool statistics_lane_shape(int estride, int rec_stride);
bool mc_fused_supported(const Code& c, int rec_stride);
int launch_mc_fused(const Code& c, uint64_t seed, uint64_t start, long long B, float p, const uint32_t pats[4],
                    uint32_t* sX, uint32_t* sZ, uint8_t* rec, int rec_stride, int32_t* iters, uint32_t* merge,
                    int32_t* listX, int32_t* listZ, int32_t* listS, uint32_t* counts, const uint64_t* imp_cols,
                    unsigned long long* counters, unsigned long long* partials, int stage, hipStream_t st);
long long mc_fused_parts(long long B);
int launch_zero_words(unsigned long long* w, int n, hipStream_t st, unsigned long long* w2 = nullptr, int n2 = 0);
int mc_fused_part_rows();
int mc_fused_count_words();
int mc_fused_count_stride();
// u64 words after the counters that hold the fused pipeline's list lengths
inline int mc_count_u64() { return (mc_fused_count_words() + 3) / 4 * 2; }  // whole 16-byte lines
int launch_statistics_packed(const Code& c, const uint64_t* imp_cols, const uint8_t* errp, int estride, const uint8_t* rec,
                             const int32_t* iters, long long B, unsigned long long* counters, hipStream_t st,
                             int rec_stride = 0);
void* sparse_plan_create(const Code& c, int device);
void sparse_plan_free(void* plan);
const char* sparse_plan_name(const void* plan);
const int32_t* sparse_plan_chkvar(const void* plan);
const int32_t* sparse_plan_varedge(const void* plan);
int launch_decode_sparse(void* plan, const uint8_t* sX, const uint8_t* sZ, long long B, float errorProbability,
                         int maxIter, int stop, uint8_t* eX, uint8_t* eZ, uint8_t* flags, int32_t* iters, float* q,
                         hipStream_t stream);
void* cpu_plan_create(const Code& c);
void cpu_plan_free(void* plan);
int cpu_threads();
int cpu_decode_batch(void* plan, const uint8_t* sX, const uint8_t* sZ, long long B, float p, int maxIter, int stop,
                     uint8_t* eX, uint8_t* eZ, uint8_t* flags, uint8_t* rec, int32_t* iters, float* qf, int threads);
int launch_pack_decisions(const uint8_t* eX, const uint8_t* eZ, const uint8_t* flags, long long B, int n, uint8_t* out,
                          hipStream_t st);
int launch_statistics(const Code& c, const uint64_t* imp_cols, const uint8_t* x, const uint8_t* z, const uint8_t* eX,
                      const uint8_t* eZ, const uint8_t* flags, long long B, unsigned long long* counters, hipStream_t st);
}  // namespace qec

using namespace qec;

struct qec_code {
    Code c;
};


// One decoder handle: a device engine (wave-circulant variant or sparse-graph plan) plus the
// workspaces its entry points share, or a multi-device group of such handles (parts).
// Events owned by a handle (created on first use, destroyed with it on its device).
struct EventSet {
    std::vector<hipEvent_t> ev;
    ~EventSet()
    {
        for (hipEvent_t e : ev) (void)hipEventDestroy(e);
    }
    int make(size_t n, unsigned flags)
    {
        ev.assign(n, nullptr);
        for (auto& e : ev)
            if (hipEventCreateWithFlags(&e, flags) != hipSuccess) return qec::fail(QEC_ERR_HIP, "hipEventCreateWithFlags");
        return QEC_OK;
    }
};

struct qec_decoder {
    std::shared_ptr<const Code> code;
    int device = 0;
    int engine = QEC_ENGINE_CIRCULANT;
    const void* variant = nullptr;  // wave-circulant kernel variant (bp_decode.hip)
    void* sparse = nullptr;         // sparse-graph plan (bp_sparse.hip)
    void* cpu = nullptr;            // CPU engine plan (cpu_engine.cpp), device = -1
    std::string variant_name;
    int hard_paths = 1;             // QEC_OPT_HARD_PATHS
    int cycle_jump = 1;             // QEC_OPT_CYCLE_JUMP
    int schedule = 1;               // QEC_OPT_SCHEDULE (0 off, 1 auto, 2 always, 3 / 4 always, local / one-launch order)
    int sector_split = 1;           // QEC_OPT_SECTOR_SPLIT (0 off, 1 auto, 2 split waves, 3 sector launches)
    int phase_stats = 0;            // QEC_OPT_PHASE_STATS
    int triage = 1;                 // QEC_OPT_TRIAGE
    int last_path = 0;              // QEC_OPT_LAST_PATH: QEC_PATH_* bits of the last decode call
    int mc_time = 1;                // QEC_OPT_MC_DECODE_TIME
    // workspace shared by every launch of this handle (dispatch order, split-flag merge words,
    // sparse byte staging for packed output); ws_ev marks the last launch that used it, so a call
    // on another stream waits for it (stream-ordered reuse)
    DeviceArray<uint8_t> sched;
    DeviceArray<uint32_t> merge;
    DeviceArray<uint32_t> gbar;  // grid-barrier words of the one-launch dispatch order (zeroed at creation)
    DeviceArray<int32_t> tlist;  // triage: listX [B], listZ [B], (fused Monte-Carlo: listS [B]), counts
    hipEvent_t ws_ev = nullptr;
    hipStream_t ws_stream = nullptr;
    bool ws_used = false;
    hipStream_t stream = nullptr;   // the host-pointer and Monte-Carlo entry points' stream
    // staging for the host-pointer entry points (DecoderGPU's device vectors, DecoderGPU.h:28-35)
    DeviceArray<uint8_t> sX, sZ, eX, eZ, flags, rec;
    DeviceArray<int32_t> iters;
    DeviceArray<float> q;
    // Monte-Carlo workspace (qec_monte_carlo / qec_get_statistics)
    DeviceArray<uint64_t> imp_cols;  // I-P by columns over its non-zero rows (Code::imp_cols)
    DeviceArray<uint8_t> msX, msZ, merrp, mrec, mtype;
    DeviceArray<int32_t> mit, midx;
    DeviceArray<unsigned long long> mcount;
    DeviceArray<unsigned long long> mpart;  // fused Monte-Carlo kernel: partial-sum rows of the counters
    PinnedArray<unsigned long long> mhost;  // the counters' host copy (page-locked: an asynchronous copy)
    EventSet mc_ev;  // qec_monte_carlo's ring of decode-time event pairs
    // multi-device group (qec_decoder_create_multi): the parts do the work, this handle only routes
    std::vector<qec_decoder*> parts;

    ~qec_decoder()
    {
        for (qec_decoder* p : parts) delete p;
        if (cpu) cpu_plan_free(cpu);
        if (parts.empty() && !cpu) {
            // the member device arrays are freed after this body, on this device too;
            // qec_decoder_destroy restores the caller's device afterwards
            (void)hipSetDevice(device);
            if (ws_ev) (void)hipEventDestroy(ws_ev);
            if (stream) (void)hipStreamDestroy(stream);
            if (sparse) sparse_plan_free(sparse);
        }
    }
};

#define QEC_HIP_CHECK(expr)                                                                     \
    do {                                                                                         \
        hipError_t e_ = (expr);                                                                  \
        if (e_ != hipSuccess) return fail(QEC_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(e_)); \
    } while (0)

namespace {

// Makes `device` current for the scope of an entry point and restores the caller's device.
struct DeviceGuard {
    int prev = -1;
    hipError_t err;
    explicit DeviceGuard(int device)
    {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        err = hipSetDevice(device);
    }
    ~DeviceGuard()
    {
        if (prev >= 0) (void)hipSetDevice(prev);
    }
};

#define QEC_DEVICE_SCOPE(dev)                                                                      \
    DeviceGuard guard_(dev);                                                                       \
    if (guard_.err != hipSuccess) return fail(QEC_ERR_HIP, std::string("hipSetDevice: ") + hipGetErrorString(guard_.err))

bool capturing(hipStream_t st)
{
    hipStreamCaptureStatus s = hipStreamCaptureStatusNone;
    return hipStreamIsCapturing(st, &s) == hipSuccess && s != hipStreamCaptureStatusNone;
}

// Grow a workspace buffer to n elements.  Refused while `st` is being captured into a graph (an
// allocation there would be invalid): size the decoder with max_batch instead.
template <class T>
int ws_reserve(DeviceArray<T>& a, size_t n, hipStream_t st, const char* what)
{
    if (n <= a.capacity()) return QEC_OK;
    if (capturing(st))
        return fail(QEC_ERR_ARG, std::string(what) + ": the workspace is smaller than this batch and the stream is "
                                                     "being captured; create the decoder with max_batch >= B");
    try {
        a.reserve(n);
    } catch (const std::exception& ex) {
        return fail(QEC_ERR_NOMEM, std::string(what) + ": " + ex.what());
    }
    return QEC_OK;
}

// Stream-ordered use of the handle's workspace: a launch on a stream other than the previous
// one first waits for the previous launch's completion event.  Launches captured into a graph
// neither wait nor record (an event outside the capture cannot be waited on inside it): the
// graph's replays are ordered by its launcher.
int ws_acquire(qec_decoder* d, hipStream_t st)
{
    if (d->ws_used && st != d->ws_stream && !capturing(st)) QEC_HIP_CHECK(hipStreamWaitEvent(st, d->ws_ev, 0));
    return QEC_OK;
}
// The workspace event for the call's last kernel to carry (launch_marked), or null while capturing;
// ws_release(d, st, true) then records nothing more.
hipEvent_t ws_done(qec_decoder* d, hipStream_t st) { return capturing(st) ? nullptr : d->ws_ev; }
int ws_release(qec_decoder* d, hipStream_t st, bool carried = false)
{
    if (capturing(st)) return QEC_OK;
    if (!carried) QEC_HIP_CHECK(hipEventRecord(d->ws_ev, st));
    d->ws_used = true;
    d->ws_stream = st;
    return QEC_OK;
}

std::vector<qec_decoder*> parts_of(qec_decoder* d)
{
    if (d->parts.empty()) return {d};
    return d->parts;
}

// contiguous shard k of n over [0, B): [k B / n, (k + 1) B / n)
long long shard_lo(long long B, int k, int n) { return (long long)((__int128)B * k / n); }

}  // namespace

extern "C" {

const char* qec_last_error(void) { return last_error_cstr(); }
int qec_abi_version(void) { return QEC_LDPC_ABI_VERSION; }
#ifndef QEC_BUILD_ID
#define QEC_BUILD_ID "unknown"
#endif
const char* qec_build_id(void) { return QEC_BUILD_ID; }

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
    if (engine < QEC_ENGINE_AUTO || engine > QEC_ENGINE_CPU) {
        fail(QEC_ERR_ARG, "qec_decoder_create_engine: unknown engine");
        return nullptr;
    }
    if (device < 0 || engine == QEC_ENGINE_CPU) {  // DecoderCPU: host buffers only
        if (device >= 0 || (engine != QEC_ENGINE_AUTO && engine != QEC_ENGINE_CPU)) {
            fail(QEC_ERR_ARG, "qec_decoder_create: the CPU engine is device -1, the GPU engines devices >= 0");
            return nullptr;
        }
        std::unique_ptr<qec_decoder> d(new (std::nothrow) qec_decoder);
        if (!d) { fail(QEC_ERR_NOMEM, "qec_decoder_create: out of memory"); return nullptr; }
        d->code = std::make_shared<const Code>(h->c);
        d->device = -1;
        d->engine = QEC_ENGINE_CPU;
        d->cpu = cpu_plan_create(*d->code);
        if (!d->cpu) return nullptr;
        d->variant_name = "cpu (" + std::to_string(cpu_threads()) + " threads) " + d->code->describe();
        return d.release();
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
    DeviceGuard guard(device);
    if (guard.err != hipSuccess) { fail(QEC_ERR_HIP, "hipSetDevice failed"); return nullptr; }
    std::unique_ptr<qec_decoder> d(new (std::nothrow) qec_decoder);
    if (!d) { fail(QEC_ERR_NOMEM, "qec_decoder_create: out of memory"); return nullptr; }
    d->code = std::make_shared<const Code>(h->c);
    d->device = device;
    d->variant = v;
    d->variant_name = name;
    if (!v) {  // AUTO without a wave-circulant kernel, or SPARSE requested
        d->engine = QEC_ENGINE_SPARSE;
        d->sparse = sparse_plan_create(*d->code, device);
        if (!d->sparse) return nullptr;  // error text set by the plan
        d->variant_name = sparse_plan_name(d->sparse);
    }
    if (hipStreamCreateWithFlags(&d->stream, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreateWithFlags(&d->ws_ev, hipEventDisableTiming | kEvNoFence) != hipSuccess) {
        fail(QEC_ERR_HIP, "qec_decoder_create: stream / event creation failed");
        return nullptr;
    }
    try {
        // the device-pointer workspace is sized up front so that the _dev entry points allocate
        // nothing for batches up to max_batch (graph capture); staging grows on demand
        if (max_batch > 0 && d->variant) {
            if ((long long)max_batch <= schedule_max_batch())
                d->sched.reserve(schedule_workspace_bytes((long long)max_batch, d->code->mX, d->code->mZ));
            d->merge.reserve(max_batch);
        }
        if (max_batch > 0 && d->sparse) {
            d->eX.reserve(max_batch * d->code->n);
            d->eZ.reserve(max_batch * d->code->n);
            d->flags.reserve(max_batch);
        }
        if (!d->code->imp_cols.empty()) {
            d->imp_cols.reserve(d->code->imp_cols.size());
            hip_throw(hipMemcpy(d->imp_cols.data(), d->code->imp_cols.data(), d->code->imp_cols.size() * sizeof(uint64_t),
                                hipMemcpyHostToDevice), "I-P upload");
        }
        // the counters, then the fused pipeline's list lengths: one memset zeroes both per call
        d->mcount.reserve(QEC_MC_NCOUNTERS_ALL + mc_count_u64());
        if (d->variant) {
            d->gbar.reserve(2);
            hip_throw(hipMemset(d->gbar.data(), 0, 2 * sizeof(uint32_t)), "grid-barrier words");
        }
    } catch (const std::exception& ex) {
        fail(QEC_ERR_HIP, std::string("qec_decoder_create: ") + ex.what());
        return nullptr;
    }
    return d.release();
}

qec_decoder* qec_decoder_create_multi(const qec_code* h, const int* devices, int ndevices, size_t max_batch)
{
    if (!h || !devices || ndevices <= 0) { fail(QEC_ERR_ARG, "qec_decoder_create_multi: bad argument"); return nullptr; }
    for (int k = 0; k < ndevices; ++k)
        if (devices[k] < 0) {
            // a CPU-engine part would decode host batches but fail the device-side entry points
            // (statistics, Monte-Carlo) of the group: groups are GPU-only
            fail(QEC_ERR_ARG, "qec_decoder_create_multi: device ordinals must be >= 0 (the CPU engine is device -1 of "
                              "qec_decoder_create)");
            return nullptr;
        }
    std::unique_ptr<qec_decoder> g(new (std::nothrow) qec_decoder);
    if (!g) { fail(QEC_ERR_NOMEM, "qec_decoder_create_multi: out of memory"); return nullptr; }
    for (int k = 0; k < ndevices; ++k) {
        qec_decoder* p = qec_decoder_create(h, devices[k], max_batch);
        if (!p) return nullptr;  // parts created so far are freed with g
        g->parts.push_back(p);
    }
    const qec_decoder* p0 = g->parts[0];
    g->code = p0->code;
    g->device = p0->device;
    g->engine = p0->engine;
    g->variant = p0->variant;
    std::string name = "multi-device [";
    for (int k = 0; k < ndevices; ++k) name += (k ? "," : "") + std::to_string(devices[k]);
    g->variant_name = name + "] " + p0->variant_name;
    return g.release();
}

int qec_decoder_num_parts(const qec_decoder* d)
{
    if (!d) return fail(QEC_ERR_ARG, "qec_decoder_num_parts: null decoder");
    return d->parts.empty() ? 1 : (int)d->parts.size();
}

qec_decoder* qec_decoder_part(qec_decoder* d, int k)
{
    if (!d) { fail(QEC_ERR_ARG, "qec_decoder_part: null decoder"); return nullptr; }
    if (d->parts.empty()) return k == 0 ? d : (fail(QEC_ERR_ARG, "qec_decoder_part: index out of range"), nullptr);
    if (k < 0 || k >= (int)d->parts.size()) { fail(QEC_ERR_ARG, "qec_decoder_part: index out of range"); return nullptr; }
    return d->parts[k];
}

int qec_decoder_device(const qec_decoder* d)
{
    if (!d) return fail(QEC_ERR_ARG, "qec_decoder_device: null decoder");
    return d->device;
}

int qec_decoder_destroy(qec_decoder* d)
{
    // every part's streams, events and device arrays are freed on its own device; the caller's
    // current device is restored afterwards (as every other entry point does)
    int prev = -1;
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    delete d;
    if (prev >= 0) (void)hipSetDevice(prev);
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
    for (qec_decoder* p : d->parts) {
        const int rc = qec_decoder_set_option(p, option, value);
        if (rc) return rc;
    }
    switch (option) {
    case QEC_OPT_HARD_PATHS: d->hard_paths = value != 0; return QEC_OK;
    case QEC_OPT_CYCLE_JUMP: d->cycle_jump = value != 0; return QEC_OK;
    case QEC_OPT_SCHEDULE:
        if (value < 0 || value > 4) return fail(QEC_ERR_ARG, "qec_decoder_set_option: QEC_OPT_SCHEDULE is 0 .. 4");
        d->schedule = value;
        return QEC_OK;
    case QEC_OPT_SECTOR_SPLIT:
        if (value < 0 || value > 3) return fail(QEC_ERR_ARG, "qec_decoder_set_option: QEC_OPT_SECTOR_SPLIT is 0 .. 3");
        d->sector_split = value;
        return QEC_OK;
    case QEC_OPT_PHASE_STATS:
        if (value && (!d->variant || !decode_has_phase_stats(d->variant, QEC_STOP_FIXED)))
            return fail(QEC_ERR_UNSUPPORTED, "qec_decoder_set_option: QEC_OPT_PHASE_STATS needs a shipped code's kernels");
        d->phase_stats = value != 0;
        return QEC_OK;
    case QEC_OPT_TRIAGE:
        if (value < 0 || value > 3) return fail(QEC_ERR_ARG, "qec_decoder_set_option: QEC_OPT_TRIAGE is 0 .. 3");
        d->triage = value;
        return QEC_OK;
    case QEC_OPT_MC_DECODE_TIME: d->mc_time = value != 0; return QEC_OK;
    case QEC_OPT_LAST_PATH: return fail(QEC_ERR_ARG, "qec_decoder_set_option: QEC_OPT_LAST_PATH is read only");
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
    case QEC_OPT_PHASE_STATS: *value = d->phase_stats; return QEC_OK;
    case QEC_OPT_TRIAGE: *value = d->triage; return QEC_OK;
    case QEC_OPT_LAST_PATH: *value = d->parts.empty() ? d->last_path : d->parts[0]->last_path; return QEC_OK;
    case QEC_OPT_MC_DECODE_TIME: *value = d->mc_time; return QEC_OK;
    default: return fail(QEC_ERR_ARG, "qec_decoder_get_option: unknown option");
    }
}

}  // extern "C"

namespace {

// QEC_OPT_SCHEDULE = 1 orders batches from this size on (below it the extra launches cost more
// than the tail they remove) and, with one syndrome per wave (P > 32), up to kScheduleMaxSingle:
// there the order pass reads every syndrome once more (P61: 177 us per 2^20) while the tail it
// removes stays about one long sector (~0.1 ms); P61 at 2^20: 118.7 M/s unordered vs 116.9 M/s,
// at 131 072: 101 M/s vs 113 M/s (profiles/r02/ab_schedule.txt).  Several syndromes per wave (P7)
// always gain: similar syndromes then share waves (1.56 G/s vs 0.88 G/s at 2^20).
// Under the syndrome stop at low p nearly every sector stops at iteration 0 or 1, so there is no
// tail to remove and the pass is pure cost: below kScheduleSyndromeMinP it stays off there
// (P61, 65 536 per batch: p = 0.001 290 vs 266 M/s, 0.002 263 vs 257 off vs on, but 0.005 190 vs
// 197, 0.01 124 vs 143; 262 144 at p = 0.002: 0.450 vs 0.521 ms; profiles/r02/psweep_sched{0,1}_r02s3g.json,
// profiles/r02/cmp_options_r02s3zb.txt).  With sector launches or split waves each sector's waves
// can follow that sector's own weight (schedule_sector_order), which pays for P61 at 2^20 too: the
// bit-row headline 143.1 vs 140.6 M/s ordered vs not (profiles/r04/bench/configs3_*).
constexpr long long kScheduleMinBatch = 4096;
constexpr long long kScheduleMaxSingle = 1LL << 19;
constexpr float kScheduleSyndromeMinP = 0.004f;
constexpr float kTriageMaxP = 0.01f;  // QEC_OPT_TRIAGE = 1 triages syndrome-stop batches up to this p
// QEC_OPT_SECTOR_SPLIT = 1 splits batches above this size only when they get the per-sector order
constexpr long long kSplitOrderedMinBatch = 1LL << 19;

int hard_path_bits(const qec_decoder* d)
{
    return (d->hard_paths ? (QEC_HP_FORMS | (d->cycle_jump ? QEC_HP_CYCLE : 0)) : 0) | (d->phase_stats ? QEC_HP_PHASE : 0);
}

// QEC_OPT_TRIAGE: 1 (auto) and 3 (auto, never the fused Monte-Carlo kernel) up to kTriageMaxP, 2 always
bool triage_on(const qec_decoder* d, float p)
{
    return !d->phase_stats && (d->triage == 2 || ((d->triage == 1 || d->triage == 3) && p <= kTriageMaxP));
}

// One decode launch of a single-device handle on device buffers.  Outputs: byte form (eX, eZ,
// flags) or, with rec non-null, the packed decision records.
// sbits: sX / sZ are bit rows ([B][ceil(m/32)] words, the Monte-Carlo pipeline's layout; wave-circulant
// engine only), else byte rows
// rec_stride: record row stride (0: 2 nb + 1, the public layout; the Monte-Carlo pipeline pads rows to
// whole words for its statistics kernel; wave-circulant engine only)
int dispatch_decode(qec_decoder* d, const uint8_t* sX, const uint8_t* sZ, long long B, float p, int maxIter, int stop,
                    uint8_t* eX, uint8_t* eZ, uint8_t* flags, uint8_t* rec, int32_t* iters, float* q, hipStream_t st,
                    bool sbits = false, int rec_stride = 0)
{
    if (B <= 0) return QEC_OK;
    const Code& c = *d->code;
    int rc = ws_acquire(d, st);
    if (rc) return rc;
    d->last_path = (sbits ? QEC_PATH_BIT_ROWS : 0) | (rec != nullptr ? QEC_PATH_RECORDS : 0);
    if (d->engine == QEC_ENGINE_SPARSE) {
        d->last_path |= QEC_PATH_SPARSE;
        if (sbits) return fail(QEC_ERR_UNSUPPORTED, "decode: bit-row syndromes need the wave-circulant engine");
        if (rec_stride > 0 && rec_stride != 2 * ((c.n + 7) / 8) + 1)
            return fail(QEC_ERR_UNSUPPORTED, "decode: padded record rows need the wave-circulant engine");
        if (rec != nullptr) {  // byte outputs into the handle's staging, then packed
            if ((rc = ws_reserve(d->eX, (size_t)B * c.n, st, "decode")) || (rc = ws_reserve(d->eZ, (size_t)B * c.n, st, "decode")) ||
                (rc = ws_reserve(d->flags, (size_t)B, st, "decode")))
                return rc;
            eX = d->eX.data(); eZ = d->eZ.data(); flags = d->flags.data();
        }
        rc = launch_decode_sparse(d->sparse, sX, sZ, B, p, maxIter, stop, eX, eZ, flags, iters, q, st);
        if (!rc && rec != nullptr) rc = launch_pack_decisions(eX, eZ, flags, B, c.n, rec, st);
        if (rc) return rc;
        return ws_release(d, st);
    }
    const int hp = hard_path_bits(d);
    // syndrome stop on bit rows into records (the Monte-Carlo pipeline): triage iteration 0 for 64
    // syndromes per wave, then decode only the sectors it passes on (triage.hip, list mode)
    // Above p = 0.01 most sectors go on past iteration 0 (P61 at p = 0.02: 2.2 iterations per sector)
    // and the list-mode decode of nearly the whole batch loses to the ordered one-wave-per-syndrome
    // launch (140 vs 178 M syn/s at p = 0.02, 6.4 vs 8.3 at 0.1; 1.47 G vs 0.50 G at 0.002,
    // profiles/r03/psweep_triage.json), so the triage stays off there.
    uint32_t pats[4];
    if (triage_on(d, p) && stop == QEC_STOP_SYNDROME && sbits && rec != nullptr && q == nullptr &&
        maxIter >= 2 && B < (1LL << 31) && decode_has_list(d->variant) && triage_supported(c) && triage_aligned(sX, sZ) &&
        (reinterpret_cast<uintptr_t>(iters) & 7u) == 0 &&  // the triage stores both counts as one 8-byte word
        decode_pattern_masks(d->variant, p, pats)) {
        if ((rc = ws_reserve(d->merge, (size_t)B, st, "decode")) || (rc = ws_reserve(d->tlist, 2 * (size_t)B + 2, st, "decode")))
            return rc;
        int32_t* lX = d->tlist.data();
        int32_t* lZ = lX + B;
        uint32_t* cnt = reinterpret_cast<uint32_t*>(lZ + B);
        QEC_HIP_CHECK(hipMemsetAsync(cnt, 0, 2 * sizeof(uint32_t), st));
        rc = launch_triage(c, reinterpret_cast<const uint32_t*>(sX), reinterpret_cast<const uint32_t*>(sZ), B, pats, rec,
                           iters, d->merge.data(), lX, lZ, cnt, st, rec_stride);
        if (!rc)
            rc = launch_decode_list(d->variant, c, sX, sZ, B, p, maxIter, hp, rec, iters, d->merge.data(), lX, lZ, cnt, st,
                                    rec_stride, false, 1, ws_done(d, st));
        if (rc) return rc;
        d->last_path |= QEC_PATH_TRIAGE;
        return ws_release(d, st, true);
    }
    // QEC_OPT_SECTOR_SPLIT = 1 resolved per launch (the variant's measured choice for this stop, batch and p)
    int split_opt = decode_sector_mode(d->variant, stop, d->sector_split, B, p);
    const bool split_auto = d->sector_split == 1;
    bool split = !d->phase_stats && decode_uses_split(d->variant, stop, split_opt, B);
    bool need_merge = !d->phase_stats && decode_needs_merge(d->variant, stop, split_opt, B);
    const bool single = 2 * c.P > 64;  // one syndrome per wave
    bool sectors = split || need_merge;  // split waves or sector launches
    const bool auto_on = B >= kScheduleMinBatch &&
                         (!single || B <= kScheduleMaxSingle || (sectors && schedule_sector_order(B, sbits, c.mX, c.mZ))) &&
                         !(stop == QEC_STOP_SYNDROME && p < kScheduleSyndromeMinP);
    const bool ordered = B > 1 && B <= schedule_max_batch() && (d->schedule >= 2 || (d->schedule == 1 && auto_on));
    const int method = d->schedule == 3 ? QEC_ORDER_LOCAL : d->schedule == 4 ? QEC_ORDER_ONE_LAUNCH : QEC_ORDER_GLOBAL;
    // The tuned split above kSplitOrderedMinBatch was measured only with the per-sector order (round 2:
    // in total-weight order one wave per group won from 2^19 on); without that order keep one wave per group
    if (split && split_auto && B > kSplitOrderedMinBatch &&
        !(ordered && method == QEC_ORDER_GLOBAL && schedule_sector_order(B, sbits, c.mX, c.mZ))) {
        split_opt = 0;
        split = false;
        need_merge = !d->phase_stats && decode_needs_merge(d->variant, stop, split_opt, B);
        sectors = need_merge;
    }
    if (need_merge && (rc = ws_reserve(d->merge, (size_t)B, st, "decode"))) return rc;
    const int32_t* perm = nullptr;
    bool zeroed = false, perm_sectors = false;
    if (ordered) {
        if ((rc = ws_reserve(d->sched, schedule_workspace_bytes(B, c.mX, c.mZ), st, "decode: dispatch order")))
            return rc;
        int32_t* pm = nullptr;
        // a sector-split launch merges its flags in zeroed words: the order pass zeroes them
        // each sector's waves in the order of its own weight: split waves, or sector launches (need_merge alone)
        rc = launch_schedule(sX, sZ, sbits, B, c.mX, c.mZ, d->sched.data(), split ? d->merge.data() : nullptr, sectors,
                             &pm, &perm_sectors, st, method, d->gbar.data());
        if (rc) return rc;
        perm = pm;
        zeroed = split;
    }
    rc = launch_decode(d->variant, c, sX, sZ, sbits, B, p, maxIter, stop, eX, eZ, flags, rec, iters, q, hp, perm,
                       split_opt, need_merge ? d->merge.data() : nullptr, zeroed, st, rec_stride, perm_sectors,
                       ws_done(d, st));
    if (rc) return rc;
    d->last_path |= (perm ? QEC_PATH_ORDERED : 0) | (perm && perm_sectors ? QEC_PATH_SECTOR_ORDER : 0) |
                    (split ? QEC_PATH_SPLIT_WAVES : 0) | (need_merge && !split ? QEC_PATH_SECTOR_LAUNCHES : 0);
    return ws_release(d, st, true);
}

const int32_t* syndrome_table(const qec_decoder* d)
{
    return d->engine == QEC_ENGINE_SPARSE ? sparse_plan_chkvar(d->sparse) : nullptr;
}

const int32_t* variable_table(const qec_decoder* d)
{
    return d->engine == QEC_ENGINE_SPARSE ? sparse_plan_varedge(d->sparse) : nullptr;
}

int check_decode_args(const qec_decoder* d, const void* sX, const void* sZ, size_t B, int stop)
{
    if (!d) return fail(QEC_ERR_ARG, "decode: null decoder");
    if (stop < QEC_STOP_REF || stop > QEC_STOP_SYNDROME) return fail(QEC_ERR_ARG, "decode: unknown stop rule");
    if (B && (!sX || !sZ)) return fail(QEC_ERR_ARG, "decode: null syndrome buffer");
    if (B > (size_t)1 << 40) return fail(QEC_ERR_ARG, "decode: batch too large");
    return QEC_OK;
}

int single_device_only(const qec_decoder* d, const char* what)
{
    if (d->cpu) return fail(QEC_ERR_UNSUPPORTED, std::string(what) + ": the CPU engine has no device buffers");
    if (!d->parts.empty())
        return fail(QEC_ERR_ARG, std::string(what) + ": device buffers live on one GPU; call it on a part "
                                                     "(qec_decoder_part) of a multi-device decoder");
    return QEC_OK;
}

// Host-buffer decode of one single-device handle (synchronous): stage, decode, copy back.
int decode_host(qec_decoder* d, const uint8_t* sX, const uint8_t* sZ, size_t B, float p, int maxIter, int stop,
                uint8_t* eX, uint8_t* eZ, uint8_t* flags, uint8_t* rec, int32_t* iters, float* q)
{
    if (B == 0) return QEC_OK;
    if (d->cpu) return cpu_decode_batch(d->cpu, sX, sZ, (long long)B, p, maxIter, stop, eX, eZ, flags, rec, iters, q, 0);
    QEC_DEVICE_SCOPE(d->device);
    const Code& c = *d->code;
    const size_t qn = (size_t)(c.mX + c.mZ) * c.L;
    const size_t recB = 2 * (size_t)((c.n + 7) / 8) + 1;
    hipStream_t st = d->stream;
    try {
        d->sX.reserve(B * c.mX); d->sZ.reserve(B * c.mZ);
        if (rec) d->rec.reserve(B * recB);
        else { d->eX.reserve(B * c.n); d->eZ.reserve(B * c.n); d->flags.reserve(B); }
        if (iters) d->iters.reserve(2 * B);
        if (q) d->q.reserve(B * qn);
    } catch (const std::exception& ex) {
        return fail(QEC_ERR_HIP, std::string("device staging allocation: ") + ex.what());
    }
    QEC_HIP_CHECK(hipMemcpyAsync(d->sX.data(), sX, B * c.mX, hipMemcpyHostToDevice, st));
    QEC_HIP_CHECK(hipMemcpyAsync(d->sZ.data(), sZ, B * c.mZ, hipMemcpyHostToDevice, st));
    // the sparse engine's packed path stages its byte outputs in eX/eZ/flags (dispatch_decode)
    int rc = dispatch_decode(d, d->sX.data(), d->sZ.data(), (long long)B, p, maxIter, stop, rec ? nullptr : d->eX.data(),
                             rec ? nullptr : d->eZ.data(), rec ? nullptr : d->flags.data(), rec ? d->rec.data() : nullptr,
                             iters ? d->iters.data() : nullptr, q ? d->q.data() : nullptr, st);
    if (rc) return rc;
    if (rec) {
        QEC_HIP_CHECK(hipMemcpyAsync(rec, d->rec.data(), B * recB, hipMemcpyDeviceToHost, st));
    } else {
        QEC_HIP_CHECK(hipMemcpyAsync(eX, d->eX.data(), B * c.n, hipMemcpyDeviceToHost, st));
        QEC_HIP_CHECK(hipMemcpyAsync(eZ, d->eZ.data(), B * c.n, hipMemcpyDeviceToHost, st));
        QEC_HIP_CHECK(hipMemcpyAsync(flags, d->flags.data(), B, hipMemcpyDeviceToHost, st));
    }
    if (iters) QEC_HIP_CHECK(hipMemcpyAsync(iters, d->iters.data(), 2 * B * sizeof(int32_t), hipMemcpyDeviceToHost, st));
    if (q) QEC_HIP_CHECK(hipMemcpyAsync(q, d->q.data(), B * qn * sizeof(float), hipMemcpyDeviceToHost, st));
    QEC_HIP_CHECK(hipStreamSynchronize(st));
    return QEC_OK;
}

// Host-buffer decode on every part of a handle: contiguous shards, one host thread per part
// (the reference's sample-parallel loop, DecoderCPU.h:419-438, across devices).
int decode_host_parts(qec_decoder* d, const uint8_t* sX, const uint8_t* sZ, size_t B, float p, int maxIter, int stop,
                      uint8_t* eX, uint8_t* eZ, uint8_t* flags, uint8_t* rec, int32_t* iters, float* q)
{
    const std::vector<qec_decoder*> parts = parts_of(d);
    if (parts.size() == 1)
        return decode_host(parts[0], sX, sZ, B, p, maxIter, stop, eX, eZ, flags, rec, iters, q);
    const Code& c = *d->code;
    const size_t qn = (size_t)(c.mX + c.mZ) * c.L;
    const size_t recB = 2 * (size_t)((c.n + 7) / 8) + 1;
    const int np = (int)parts.size();
    std::vector<int> rcs(np, QEC_OK);
    std::vector<std::string> errs(np);
    std::vector<std::thread> th;
    for (int k = 0; k < np; ++k) {
        const size_t lo = (size_t)shard_lo((long long)B, k, np), hi = (size_t)shard_lo((long long)B, k + 1, np);
        th.emplace_back([&, k, lo, hi] {
            rcs[k] = decode_host(parts[k], sX + lo * c.mX, sZ + lo * c.mZ, hi - lo, p, maxIter, stop,
                                 eX ? eX + lo * c.n : nullptr, eZ ? eZ + lo * c.n : nullptr, flags ? flags + lo : nullptr,
                                 rec ? rec + lo * recB : nullptr, iters ? iters + 2 * lo : nullptr, q ? q + lo * qn : nullptr);
            if (rcs[k]) errs[k] = last_error_cstr();
        });
    }
    for (auto& t : th) t.join();
    for (int k = 0; k < np; ++k)
        if (rcs[k]) return fail(rcs[k], "part " + std::to_string(k) + ": " + errs[k]);
    return QEC_OK;
}

}  // namespace

extern "C" {

int qec_decode_batch_dev(qec_decoder* d, const uint8_t* sX, const uint8_t* sZ, size_t B, float p, int maxIter,
                         int stop, uint8_t* eX, uint8_t* eZ, uint8_t* flags, int32_t* iters, float* q, void* stream)
{
    int rc = check_decode_args(d, sX, sZ, B, stop);
    if (rc || (rc = single_device_only(d, "qec_decode_batch_dev"))) return rc;
    if (B && (!eX || !eZ || !flags)) return fail(QEC_ERR_ARG, "decode: null output buffer");
    QEC_DEVICE_SCOPE(d->device);
    return dispatch_decode(d, sX, sZ, (long long)B, p, maxIter, stop, eX, eZ, flags, nullptr, iters, q,
                           static_cast<hipStream_t>(stream));
}

int qec_decode_batch_packed_dev(qec_decoder* d, const uint8_t* sX, const uint8_t* sZ, size_t B, float p, int maxIter,
                                int stop, uint8_t* records, int32_t* iters, float* q, void* stream)
{
    int rc = check_decode_args(d, sX, sZ, B, stop);
    if (rc || (rc = single_device_only(d, "qec_decode_batch_packed_dev"))) return rc;
    if (B && !records) return fail(QEC_ERR_ARG, "decode: null record buffer");
    QEC_DEVICE_SCOPE(d->device);
    return dispatch_decode(d, sX, sZ, (long long)B, p, maxIter, stop, nullptr, nullptr, nullptr, records, iters, q,
                           static_cast<hipStream_t>(stream));
}

int qec_decode_bits_packed_dev(qec_decoder* d, const uint32_t* sX, const uint32_t* sZ, size_t B, float p, int maxIter,
                               int stop, uint8_t* records, int32_t* iters, float* q, void* stream)
{
    int rc = check_decode_args(d, sX, sZ, B, stop);
    if (rc || (rc = single_device_only(d, "qec_decode_bits_packed_dev"))) return rc;
    if (B && !records) return fail(QEC_ERR_ARG, "decode: null record buffer");
    if (d->engine == QEC_ENGINE_SPARSE)
        return fail(QEC_ERR_UNSUPPORTED, "qec_decode_bits_packed_dev: bit-row syndromes need the wave-circulant engine");
    QEC_DEVICE_SCOPE(d->device);
    return dispatch_decode(d, reinterpret_cast<const uint8_t*>(sX), reinterpret_cast<const uint8_t*>(sZ), (long long)B, p,
                           maxIter, stop, nullptr, nullptr, nullptr, records, iters, q, static_cast<hipStream_t>(stream),
                           true);
}

int qec_decode_batch(qec_decoder* d, const uint8_t* sX, const uint8_t* sZ, size_t B, float p, int maxIter, int stop,
                     uint8_t* eX, uint8_t* eZ, uint8_t* flags, int32_t* iters, float* q)
{
    int rc = check_decode_args(d, sX, sZ, B, stop);
    if (rc) return rc;
    if (B && (!eX || !eZ || !flags)) return fail(QEC_ERR_ARG, "decode: null output buffer");
    return decode_host_parts(d, sX, sZ, B, p, maxIter, stop, eX, eZ, flags, nullptr, iters, q);
}

int qec_decode_batch_packed(qec_decoder* d, const uint8_t* sX, const uint8_t* sZ, size_t B, float p, int maxIter,
                            int stop, uint8_t* records, int32_t* iters)
{
    int rc = check_decode_args(d, sX, sZ, B, stop);
    if (rc) return rc;
    if (B && !records) return fail(QEC_ERR_ARG, "decode: null record buffer");
    return decode_host_parts(d, sX, sZ, B, p, maxIter, stop, nullptr, nullptr, nullptr, records, iters, nullptr);
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

}  // extern "C"

namespace {

// Monte-Carlo workspace of one part for batches of up to B samples (W draws each).
int mc_reserve(qec_decoder* d, size_t B, int W)
{
    const Code& c = *d->code;
    const size_t nb = (size_t)(c.n + 7) / 8;
    try {
        // syndromes as bytes or as bit rows, packed errors at 2 nb or word-aligned rows (mc_batch)
        d->msX.reserve(B * std::max<size_t>(c.mX, 4 * ((c.mX + 31) / 32)));
        d->msZ.reserve(B * std::max<size_t>(c.mZ, 4 * ((c.mZ + 31) / 32)));
        d->merrp.reserve(B * 4 * ((2 * nb + 3) / 4)); d->mrec.reserve(B * 4 * ((2 * nb + 1 + 3) / 4));
        d->mit.reserve(2 * B);
        if (W > 0) { d->midx.reserve(B * W); d->mtype.reserve(B * W); }
    } catch (const std::exception& ex) {
        return fail(QEC_ERR_HIP, std::string("Monte-Carlo workspace: ") + ex.what());
    }
    return QEC_OK;
}

// errors (source filled in h by the caller) -> syndromes + packed errors -> packed decode ->
// counters, all enqueued on the part's stream
// zero_counters: the call's first batch (the counters start at 0; one memset with the fused
// pipeline's list lengths, enqueued after the host-side preparation, right before the first kernel)
int mc_batch(qec_decoder* d, McArgsHost h, int src, float p, int maxIter, int stop, bool want_iters,
             hipEvent_t ev0, hipEvent_t ev1, bool zero_counters = false)
{
    hipStream_t st = d->stream;
    const Code& c = *d->code;
    h.code = &c;
    h.chkVar = syndrome_table(d);
    h.varEdge = variable_table(d);
    // the depolarising front end hands the wave-circulant engine its syndromes as bit rows and its
    // packed errors at word-aligned rows (72 + 156 instead of 549 + 154 B per P61 sample)
    const bool bits = src == MC_SRC_PHILOX && d->engine != QEC_ENGINE_SPARSE;
    const int nb = (c.n + 7) / 8;
    const int estride = bits ? 4 * ((2 * nb + 3) / 4) : 2 * nb;
    const int padded = 4 * ((2 * nb + 1 + 3) / 4);
    const int rstride = bits && statistics_lane_shape(estride, padded) ? padded : 2 * nb + 1;
    // the fused low-p pipeline (triage.hip: sampler, syndromes, iteration-0 triage and the finished
    // samples' statistics in one kernel; the list-mode decode and the survivors' statistics after it)
    uint32_t pats[4];
    if (bits && stop == QEC_STOP_SYNDROME && want_iters && d->triage != 3 && triage_on(d, p) && maxIter >= 2 &&
        h.B < (1LL << 31) && decode_has_list(d->variant) && mc_fused_supported(c, rstride) &&
        decode_pattern_masks(d->variant, p, pats)) {
        const long long B = h.B;
        int rc = ws_acquire(d, st);
        if (rc) return rc;
        if ((rc = ws_reserve(d->merge, (size_t)B, st, "monte carlo")) ||
            (rc = ws_reserve(d->tlist, 3 * (size_t)B, st, "monte carlo")) ||
            (rc = ws_reserve(d->mpart, (size_t)mc_fused_part_rows() * QEC_MC_NCOUNTERS_ALL, st, "monte carlo")))
            return rc;
        int32_t* lX = d->tlist.data();
        int32_t* lZ = lX + B;
        int32_t* lS = lZ + B;
        uint32_t* cnt = reinterpret_cast<uint32_t*>(d->mcount.data() + QEC_MC_NCOUNTERS_ALL);  // list lengths
        uint32_t* sXp = reinterpret_cast<uint32_t*>(d->msX.data());
        uint32_t* sZp = reinterpret_cast<uint32_t*>(d->msZ.data());
        // the counters (first batch), the list lengths and the partial-sum rows, in one launch
        const int nz = mc_fused_part_rows() * QEC_MC_NCOUNTERS_ALL;
        rc = zero_counters ? launch_zero_words(d->mcount.data(), QEC_MC_NCOUNTERS_ALL + mc_count_u64(), st, d->mpart.data(), nz)
                           : launch_zero_words(d->mcount.data() + QEC_MC_NCOUNTERS_ALL, mc_count_u64(), st, d->mpart.data(), nz);
        if (rc) return rc;
        // the events here are separate records: carried by the kernels (launch_marked) this pipeline ran
        // 1.5-2.4 % slower at p = 0.001 .. 0.005 (profiles/r06/ab/cmp_event_carry.txt)
        if (ev0) QEC_HIP_CHECK(hipEventRecord(ev0, st));
        auto fused = [&](int stage) {
            return launch_mc_fused(c, h.seed, h.start, B, h.p, pats, sXp, sZp, d->mrec.data(), rstride, d->mit.data(),
                                   d->merge.data(), lX, lZ, lS, cnt, d->imp_cols.data(), d->mcount.data(), d->mpart.data(),
                                   stage, st);
        };
        if ((rc = fused(MC_FUSED_SAMPLE))) return rc;
        rc = launch_decode_list(d->variant, c, d->msX.data(), d->msZ.data(), B, p, maxIter, hard_path_bits(d), d->mrec.data(),
                                d->mit.data(), d->merge.data(), lX, lZ, cnt, st, rstride, true, mc_fused_count_stride());
        if (rc) return rc;
        if (ev1) QEC_HIP_CHECK(hipEventRecord(ev1, st));
        if ((rc = fused(MC_FUSED_SURVIVORS))) return rc;
        return ws_release(d, st);
    }
    if (bits) {
        h.sXp = reinterpret_cast<uint32_t*>(d->msX.data());
        h.sZp = reinterpret_cast<uint32_t*>(d->msZ.data());
        h.errp_words = true;
    } else {
        h.sX = d->msX.data(); h.sZ = d->msZ.data();
    }
    h.errp = d->merrp.data();
    if (zero_counters) QEC_HIP_CHECK(hipMemsetAsync(d->mcount.data(), 0, QEC_MC_NCOUNTERS_ALL * sizeof(unsigned long long), st));
    int rc = launch_mc_errors_syndrome(src, h, st);
    if (rc) return rc;
    if (ev0) QEC_HIP_CHECK(hipEventRecord(ev0, st));
    // records at word-aligned rows (156 instead of 155 B for P61) on the bit-row path where the lane
    // statistics kernel has that row shape (rstride above: it then reads both arrays a word at a time);
    // every other code keeps the public 2 nb + 1 rows, which the other statistics kernel, the triage
    // and the list-mode decode take as they are
    rc = dispatch_decode(d, d->msX.data(), d->msZ.data(), h.B, p, maxIter, stop, nullptr, nullptr, nullptr,
                         d->mrec.data(), want_iters ? d->mit.data() : nullptr, nullptr, st, bits, rstride);
    if (rc) return rc;
    if (ev1) QEC_HIP_CHECK(hipEventRecord(ev1, st));
    return launch_statistics_packed(c, d->imp_cols.data(), d->merrp.data(), estride, d->mrec.data(),
                                    want_iters ? d->mit.data() : nullptr, h.B, d->mcount.data(), st, rstride);
}

// Enqueues the counters' copy into the handle's page-locked host buffer (mhost); valid after the
// stream has been synchronised.
int mc_enqueue_counters(qec_decoder* d)
{
    try {
        d->mhost.reserve(QEC_MC_NCOUNTERS_ALL);
    } catch (const std::exception& ex) {
        return fail(QEC_ERR_HIP, std::string("counter staging allocation: ") + ex.what());
    }
    QEC_HIP_CHECK(hipMemcpyAsync(d->mhost.data(), d->mcount.data(), QEC_MC_NCOUNTERS_ALL * sizeof(unsigned long long),
                                 hipMemcpyDeviceToHost, d->stream));
    return QEC_OK;
}

int mc_fetch_counters(qec_decoder* d, unsigned long long* out)
{
    int rc = mc_enqueue_counters(d);
    if (rc) return rc;
    QEC_HIP_CHECK(hipStreamSynchronize(d->stream));
    std::memcpy(out, d->mhost.data(), QEC_MC_NCOUNTERS_ALL * sizeof(unsigned long long));
    return QEC_OK;
}


// qec_monte_carlo on one part: samples [start, start + count), counters left in d->mcount
int monte_carlo_part(qec_decoder* d, uint64_t seed, uint64_t start, uint64_t count, float p, int maxIter, int stop,
                     size_t batch, double* decode_s)
{
    QEC_DEVICE_SCOPE(d->device);
    hipStream_t st = d->stream;
    int rc = mc_reserve(d, (size_t)std::min<uint64_t>(batch, std::max<uint64_t>(count, 1)), 0);
    if (rc) return rc;
    // decode-kernel time from a ring of event pairs: the host waits only on a pair it reuses,
    // kRing batches behind the launches (no per-batch synchronisation)
    constexpr size_t kRing = 32;
    if (d->mc_ev.ev.empty() && (rc = d->mc_ev.make(2 * kRing, hipEventDefault | kEvNoFence))) return rc;  // once per handle
    EventSet& ev = d->mc_ev;
    double dec = 0;
    uint64_t k = 0;
    auto harvest = [&](size_t slot) -> int {
        QEC_HIP_CHECK(hipEventSynchronize(ev.ev[2 * slot + 1]));
        float ms = 0;
        QEC_HIP_CHECK(hipEventElapsedTime(&ms, ev.ev[2 * slot], ev.ev[2 * slot + 1]));
        dec += ms * 1e-3;
        return QEC_OK;
    };
    for (uint64_t base = 0; base < count; base += batch, ++k) {
        const size_t slot = k % kRing;
        if (d->mc_time && k >= kRing && (rc = harvest(slot))) return rc;
        McArgsHost h;
        h.seed = seed; h.start = start + base; h.p = p;
        h.B = (long long)std::min<uint64_t>(batch, count - base);
        rc = mc_batch(d, h, MC_SRC_PHILOX, p, maxIter, stop, true, d->mc_time ? ev.ev[2 * slot] : nullptr,
                      d->mc_time ? ev.ev[2 * slot + 1] : nullptr, k == 0);
        if (rc) return rc;
    }
    if (k == 0)  // no batch zeroed the counters
        QEC_HIP_CHECK(hipMemsetAsync(d->mcount.data(), 0, QEC_MC_NCOUNTERS_ALL * sizeof(unsigned long long), st));
    // the counters' copy behind the last batch, one synchronisation for the whole run; the remaining
    // event pairs are complete by then (qec_monte_carlo reads the counters from mhost)
    if ((rc = mc_enqueue_counters(d))) return rc;
    QEC_HIP_CHECK(hipStreamSynchronize(st));
    for (uint64_t j = k > kRing ? k - kRing : 0; d->mc_time && j < k; ++j)
        if ((rc = harvest(j % kRing))) return rc;
    *decode_s = dec;
    return QEC_OK;
}

// GetStatistics on the CPU engine: the same draws, host syndromes, CPU decode (reference stop
// rule), host counting (DecoderCPU.h:448-521).
int cpu_statistics(qec_decoder* d, int W, long tested, float p, int maxIter, uint32_t seed, qec_stats* out)
{
    const Code& c = *d->code;
    const int n = c.n;
    const long CH = 1 << 14;
    std::vector<uint8_t> x, z, sx, sz, ex, ez, fl, rx(n), rz(n);
    unsigned long long cn[QEC_MC_NCOUNTERS] = {};
    Mt19937 g(seed);
    for (long base = 0; base < tested; base += CH) {
        const long cnt = std::min(CH, tested - base);
        x.assign((size_t)cnt * n, 0);
        z.assign((size_t)cnt * n, 0);
        for (long s = 0; s < cnt; ++s)
            for (int w = 0; w < W; ++w) {
                const uint32_t v = g.msvc_uniform((uint32_t)n), t = g.msvc_uniform(3u);  // DecoderCPU.h:452-457
                if (t == 0 || t == 1) x[(size_t)s * n + v] = 1;
                if (t == 2 || t == 1) z[(size_t)s * n + v] = 1;
            }
        sx.resize((size_t)cnt * c.mX);
        sz.resize((size_t)cnt * c.mZ);
        for (long s = 0; s < cnt; ++s) {
            host_syndrome(c, 0, &x[(size_t)s * n], &sx[(size_t)s * c.mX]);
            host_syndrome(c, 1, &z[(size_t)s * n], &sz[(size_t)s * c.mZ]);
        }
        ex.resize((size_t)cnt * n);
        ez.resize((size_t)cnt * n);
        fl.resize(cnt);
        const int rc = cpu_decode_batch(d->cpu, sx.data(), sz.data(), cnt, p, maxIter, QEC_STOP_REF, ex.data(), ez.data(),
                                        fl.data(), nullptr, nullptr, nullptr, 0);
        if (rc) return rc;
        for (long s = 0; s < cnt; ++s) {
            bool ax = false, az = false;
            for (int v = 0; v < n; ++v) {
                ax |= x[(size_t)s * n + v] != 0;
                az |= z[(size_t)s * n + v] != 0;
            }
            cn[QEC_MC_WITHX] += ax;
            cn[QEC_MC_WITHZ] += az;
            const bool dEX = fl[s] & QEC_SYNDROME_FAIL_X, dEZ = fl[s] & QEC_SYNDROME_FAIL_Z;
            cn[QEC_MC_SYNX] += dEX;
            cn[QEC_MC_SYNZ] += dEZ;
            if (!(dEX || dEZ)) {
                for (int v = 0; v < n; ++v) {
                    rx[v] = x[(size_t)s * n + v] ^ ex[(size_t)s * n + v];
                    rz[v] = z[(size_t)s * n + v] ^ ez[(size_t)s * n + v];
                }
                ++cn[host_check_logical(c, rx.data(), rz.data()) ? QEC_MC_LOGICAL : QEC_MC_CORRECTED];
            }
            cn[QEC_MC_CONVX] += (fl[s] & QEC_CONVERGENCE_FAIL_X) != 0;
            cn[QEC_MC_CONVZ] += (fl[s] & QEC_CONVERGENCE_FAIL_Z) != 0;
        }
    }
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
    return QEC_OK;
}

}  // namespace

extern "C" {

// GetStatistics (DecoderCPU.h:392-530).  The errors are the reference's: W (index, type) draws
// per sample from one mt19937(seed) stream through VS2015's uniform_int_distribution, drawn on
// the host in sample order (the stream is sequential), into a double-buffered pinned chunk so the
// next chunk is drawn while the devices work on this one.  Each chunk is sharded contiguously
// over the decoder's parts; on each device: errors from the draws + syndromes + packed errors
// (one fused launch), decode (reference stop rule) to packed records, I-P check and counters.
// The counters do not depend on the sample order, so the per-device sums add up exactly.
int qec_get_statistics(qec_decoder* d, int W, int numErrors, float p, int maxIter, uint32_t seed, int nThreads,
                       qec_stats* out)
{
    if (!d || !out || numErrors < 0 || W < 0) return fail(QEC_ERR_ARG, "qec_get_statistics: bad argument");
    const Code& c = *d->code;
    if (c.imp.empty()) return fail(QEC_ERR_UNSUPPORTED, "qec_get_statistics: code has no I-P matrix for the logical check");
    if (nThreads < 1) nThreads = 1;
    const auto t0 = std::chrono::high_resolution_clock::now();
    const long tested = (long)(numErrors / nThreads) * nThreads;  // DecoderCPU.h:426,527
    if (d->cpu) {
        const int rc = cpu_statistics(d, W, tested, p, maxIter, seed, out);
        out->durationMicroSeconds = std::chrono::duration_cast<std::chrono::microseconds>(
                                        std::chrono::high_resolution_clock::now() - t0).count();
        return rc;
    }
    const long CH = 1 << 16;
    const int n = c.n;
    const std::vector<qec_decoder*> parts = parts_of(d);
    const int np = (int)parts.size();
    const long cap = std::max<long>(1, (std::min<long>(CH, std::max<long>(tested, 1)) + np - 1) / np);
    std::vector<EventSet> consumed(2 * np);  // [buffer][part]: the part's copy out of the pinned buffer is done
    for (int j = 0; j < np; ++j) {
        QEC_DEVICE_SCOPE(parts[j]->device);
        int rc = mc_reserve(parts[j], (size_t)cap, W);
        if (rc) return rc;
        QEC_HIP_CHECK(hipMemsetAsync(parts[j]->mcount.data(), 0, QEC_MC_NCOUNTERS_ALL * sizeof(unsigned long long),
                                     parts[j]->stream));
        for (int k = 0; k < 2; ++k)
            if ((rc = consumed[k * np + j].make(1, hipEventDisableTiming))) return rc;
    }
    const size_t draws = (size_t)std::min<long>(CH, std::max<long>(tested, 1)) * std::max(W, 1);
    PinnedArray<int32_t> hidx[2];
    PinnedArray<uint8_t> htype[2];
    try {
        for (int k = 0; k < 2; ++k) { hidx[k].reserve(draws); htype[k].reserve(draws); }
    } catch (const std::exception& ex) {
        return fail(QEC_ERR_HIP, std::string("qec_get_statistics: ") + ex.what());
    }
    Mt19937 g(seed);
    long chunk = 0;
    for (long base = 0; base < tested; base += CH, ++chunk) {
        const int k = (int)(chunk & 1);
        const long cnt = std::min(CH, tested - base);
        if (chunk >= 2)
            for (int j = 0; j < np; ++j) QEC_HIP_CHECK(hipEventSynchronize(consumed[k * np + j].ev[0]));
        for (long s = 0; s < cnt; ++s)
            for (int w = 0; w < W; ++w) {
                hidx[k][s * W + w] = (int32_t)g.msvc_uniform((uint32_t)n);  // index, then type (DecoderCPU.h:452-454)
                htype[k][s * W + w] = (uint8_t)g.msvc_uniform(3u);
            }
        for (int j = 0; j < np; ++j) {
            qec_decoder* pd = parts[j];
            const long lo = (long)shard_lo(cnt, j, np), hi = (long)shard_lo(cnt, j + 1, np);
            if (hi == lo) continue;
            QEC_DEVICE_SCOPE(pd->device);
            hipStream_t st = pd->stream;
            if (W > 0) {
                QEC_HIP_CHECK(hipMemcpyAsync(pd->midx.data(), hidx[k].data() + (size_t)lo * W,
                                             (size_t)(hi - lo) * W * sizeof(int32_t), hipMemcpyHostToDevice, st));
                QEC_HIP_CHECK(hipMemcpyAsync(pd->mtype.data(), htype[k].data() + (size_t)lo * W, (size_t)(hi - lo) * W,
                                             hipMemcpyHostToDevice, st));
            }
            QEC_HIP_CHECK(hipEventRecord(consumed[k * np + j].ev[0], st));
            McArgsHost h;
            h.idx = pd->midx.data(); h.type = pd->mtype.data(); h.W = W;
            h.B = hi - lo;
            const int rc = mc_batch(pd, h, MC_SRC_DRAWS, p, maxIter, QEC_STOP_REF, false, nullptr, nullptr);
            if (rc) return rc;
        }
    }
    unsigned long long cn[QEC_MC_NCOUNTERS_ALL] = {};
    for (qec_decoder* pd : parts) {
        QEC_DEVICE_SCOPE(pd->device);
        unsigned long long part[QEC_MC_NCOUNTERS_ALL];
        const int rc = mc_fetch_counters(pd, part);
        if (rc) return rc;
        for (int k = 0; k < QEC_MC_NCOUNTERS_ALL; ++k) cn[k] += part[k];
    }
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

int qec_monte_carlo(qec_decoder* d, uint64_t seed, uint64_t start, uint64_t count, float p, int maxIter, int stop,
                    size_t batch, qec_mc_result* out)
{
    if (!d || !out || (stop < QEC_STOP_REF || stop > QEC_STOP_SYNDROME)) return fail(QEC_ERR_ARG, "qec_monte_carlo: bad argument");
    if (d->cpu) return fail(QEC_ERR_UNSUPPORTED, "qec_monte_carlo: a device pipeline; the CPU engine has GetStatistics");
    const Code& c = *d->code;
    if (c.imp.empty()) return fail(QEC_ERR_UNSUPPORTED, "qec_monte_carlo: code has no I-P matrix for the logical check");
    if (batch == 0) batch = 65536;
    const auto t0 = std::chrono::high_resolution_clock::now();
    const std::vector<qec_decoder*> parts = parts_of(d);
    const int np = (int)parts.size();
    std::vector<int> rcs(np, QEC_OK);
    std::vector<std::string> errs(np);
    std::vector<double> dec(np, 0.0);
    if (np == 1) {  // one device: no host thread
        rcs[0] = monte_carlo_part(parts[0], seed, start, count, p, maxIter, stop, batch, &dec[0]);
        if (rcs[0]) errs[0] = last_error_cstr();
    } else {
        std::vector<std::thread> th;
        for (int j = 0; j < np; ++j) {
            const uint64_t lo = (uint64_t)shard_lo((long long)count, j, np), hi = (uint64_t)shard_lo((long long)count, j + 1, np);
            th.emplace_back([&, j, lo, hi] {
                rcs[j] = monte_carlo_part(parts[j], seed, start + lo, hi - lo, p, maxIter, stop, batch, &dec[j]);
                if (rcs[j]) errs[j] = last_error_cstr();
            });
        }
        for (auto& t : th) t.join();
    }
    unsigned long long cn[QEC_MC_NCOUNTERS_ALL] = {};
    for (int j = 0; j < np; ++j) {
        if (rcs[j]) return fail(rcs[j], "part " + std::to_string(j) + ": " + errs[j]);
        // monte_carlo_part left the part's counters in its page-locked copy, its stream synchronised
        for (int k = 0; k < QEC_MC_NCOUNTERS_ALL; ++k) cn[k] += parts[j]->mhost[k];
    }
    const auto t1 = std::chrono::high_resolution_clock::now();
    out->tested = count;
    out->withX = cn[QEC_MC_WITHX]; out->withZ = cn[QEC_MC_WITHZ];
    out->synX = cn[QEC_MC_SYNX]; out->synZ = cn[QEC_MC_SYNZ];
    out->logical = cn[QEC_MC_LOGICAL]; out->corrected = cn[QEC_MC_CORRECTED];
    out->convX = cn[QEC_MC_CONVX]; out->convZ = cn[QEC_MC_CONVZ];
    out->iterationsX = cn[QEC_MC_ITERX]; out->iterationsZ = cn[QEC_MC_ITERZ];
    out->decodeSeconds = *std::max_element(dec.begin(), dec.end());
    out->totalSeconds = std::chrono::duration<double>(t1 - t0).count();
    return QEC_OK;
}

int qec_sample_depolarizing_dev(qec_decoder* d, uint64_t seed, uint64_t start, size_t B, float p, uint8_t* x,
                                uint8_t* z, void* stream)
{
    if (!d || (B && (!x || !z))) return fail(QEC_ERR_ARG, "qec_sample_depolarizing_dev: bad argument");
    int rc = single_device_only(d, "qec_sample_depolarizing_dev");
    if (rc) return rc;
    QEC_DEVICE_SCOPE(d->device);
    return launch_sample_depolarizing(seed, start, (long long)B, d->code->n, p, x, z, static_cast<hipStream_t>(stream));
}

int qec_sample_syndrome_dev(qec_decoder* d, uint64_t seed, uint64_t start, size_t B, float p, uint8_t* sX, uint8_t* sZ,
                            uint8_t* errp, void* stream)
{
    if (!d || (B && (!sX || !sZ))) return fail(QEC_ERR_ARG, "qec_sample_syndrome_dev: bad argument");
    int rc = single_device_only(d, "qec_sample_syndrome_dev");
    if (rc) return rc;
    QEC_DEVICE_SCOPE(d->device);
    McArgsHost h;
    h.code = d->code.get();
    h.seed = seed; h.start = start; h.p = p;
    h.sX = sX; h.sZ = sZ; h.errp = errp;
    h.chkVar = syndrome_table(d);
    h.varEdge = variable_table(d);
    h.B = (long long)B;
    return launch_mc_errors_syndrome(MC_SRC_PHILOX, h, static_cast<hipStream_t>(stream));
}

int qec_syndrome_dev(qec_decoder* d, const uint8_t* x, const uint8_t* z, size_t B, uint8_t* sX, uint8_t* sZ,
                     void* stream)
{
    if (!d || (B && (!x || !z || !sX || !sZ))) return fail(QEC_ERR_ARG, "qec_syndrome_dev: bad argument");
    int rc = single_device_only(d, "qec_syndrome_dev");
    if (rc) return rc;
    QEC_DEVICE_SCOPE(d->device);
    McArgsHost h;
    h.code = d->code.get();
    h.x = x; h.z = z;
    h.sX = sX; h.sZ = sZ;
    h.chkVar = syndrome_table(d);
    h.B = (long long)B;
    return launch_mc_errors_syndrome(MC_SRC_BYTES, h, static_cast<hipStream_t>(stream));
}

int qec_pack_decisions_dev(qec_decoder* d, const uint8_t* eX, const uint8_t* eZ, const uint8_t* flags, size_t B,
                           uint8_t* out, void* stream)
{
    if (!d || (B && (!eX || !eZ || !flags || !out))) return fail(QEC_ERR_ARG, "qec_pack_decisions_dev: bad argument");
    if (B > (size_t)1 << 36) return fail(QEC_ERR_ARG, "qec_pack_decisions_dev: batch too large");
    int rc = single_device_only(d, "qec_pack_decisions_dev");
    if (rc) return rc;
    QEC_DEVICE_SCOPE(d->device);
    return launch_pack_decisions(eX, eZ, flags, (long long)B, d->code->n, out, static_cast<hipStream_t>(stream));
}

int qec_statistics_dev(qec_decoder* d, const uint8_t* x, const uint8_t* z, const uint8_t* eX, const uint8_t* eZ,
                       const uint8_t* flags, size_t B, uint64_t* counters, void* stream)
{
    if (!d || !counters || (B && (!x || !z || !eX || !eZ || !flags)))
        return fail(QEC_ERR_ARG, "qec_statistics_dev: bad argument");
    if (d->code->imp.empty()) return fail(QEC_ERR_UNSUPPORTED, "qec_statistics_dev: code has no I-P matrix");
    int rc = single_device_only(d, "qec_statistics_dev");
    if (rc) return rc;
    QEC_DEVICE_SCOPE(d->device);
    return launch_statistics(*d->code, d->imp_cols.data(), x, z, eX, eZ, flags, (long long)B,
                             reinterpret_cast<unsigned long long*>(counters), static_cast<hipStream_t>(stream));
}

int qec_statistics_packed_dev(qec_decoder* d, const uint8_t* errp, const uint8_t* records, const int32_t* iters,
                              size_t B, uint64_t* counters, void* stream)
{
    if (!d || !counters || (B && (!errp || !records))) return fail(QEC_ERR_ARG, "qec_statistics_packed_dev: bad argument");
    if (d->code->imp.empty()) return fail(QEC_ERR_UNSUPPORTED, "qec_statistics_packed_dev: code has no I-P matrix");
    int rc = single_device_only(d, "qec_statistics_packed_dev");
    if (rc) return rc;
    QEC_DEVICE_SCOPE(d->device);
    return launch_statistics_packed(*d->code, d->imp_cols.data(), errp, 2 * ((d->code->n + 7) / 8), records, iters, (long long)B,
                                    reinterpret_cast<unsigned long long*>(counters), static_cast<hipStream_t>(stream));
}

}  // extern "C"
