// C ABI of libqecldpc.so (declared in include/qec_ldpc.h).
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstring>
#include <memory>
#include <new>

#include "../../include/HostDeviceArray.h"
#include "qec_internal.h"

namespace qec {
const char* last_error_cstr();
const void* select_variant(const Code& c, std::string& name);
int launch_decode(const void* variant, const Code& c, const uint8_t* sX, const uint8_t* sZ, long long B,
                  float errorProbability, int maxIter, int stop, uint8_t* eX, uint8_t* eZ, uint8_t* flags,
                  int32_t* iters, float* q, hipStream_t stream);
}  // namespace qec

using namespace qec;

struct qec_code {
    Code c;
};

struct qec_decoder {
    std::shared_ptr<const Code> code;
    int device = 0;
    const void* variant = nullptr;
    std::string variant_name;
    hipStream_t stream = nullptr;
    // staging for the host-pointer entry point (DecoderGPU's device vectors, DecoderGPU.h:28-35)
    DeviceArray<uint8_t> sX, sZ, eX, eZ, flags;
    DeviceArray<int32_t> iters;
    DeviceArray<float> q;
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
    if (!h) { fail(QEC_ERR_ARG, "qec_decoder_create: null code"); return nullptr; }
    if (device < 0) { fail(QEC_ERR_ARG, "qec_decoder_create: the product has no CPU engine; device must be >= 0"); return nullptr; }
    std::string name;
    const void* v = select_variant(h->c, name);
    if (!v) {
        fail(QEC_ERR_UNSUPPORTED, "no GPU kernel for this code shape (" + h->c.describe() +
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
    if (hipStreamCreateWithFlags(&d->stream, hipStreamNonBlocking) != hipSuccess) {
        delete d;
        fail(QEC_ERR_HIP, "hipStreamCreate failed");
        return nullptr;
    }
    (void)max_batch;  // staging grows on demand
    return d;
}

int qec_decoder_destroy(qec_decoder* d)
{
    if (!d) return QEC_OK;
    (void)hipSetDevice(d->device);
    if (d->stream) (void)hipStreamDestroy(d->stream);
    delete d;
    return QEC_OK;
}

int qec_decoder_describe(const qec_decoder* d, char* buf, size_t len)
{
    if (!d || !buf || !len) return fail(QEC_ERR_ARG, "qec_decoder_describe: bad argument");
    std::snprintf(buf, len, "%s", d->variant_name.c_str());
    return QEC_OK;
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
    return launch_decode(d->variant, *d->code, sX, sZ, (long long)B, p, maxIter, stop, eX, eZ, flags, iters, q,
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
    rc = launch_decode(d->variant, c, d->sX.data(), d->sZ.data(), (long long)B, p, maxIter, stop, d->eX.data(),
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

// GetStatistics (DecoderCPU.h:392-530) with the decode batched on the GPU.  Errors are drawn
// from the reference's stream in sample order; counters are order independent.
int qec_get_statistics(qec_decoder* d, int W, int numErrors, float p, int maxIter, uint32_t seed, int nThreads,
                       qec_stats* out)
{
    if (!d || !out || numErrors < 0 || W < 0) return fail(QEC_ERR_ARG, "qec_get_statistics: bad argument");
    const Code& c = *d->code;
    if (c.imp.empty()) return fail(QEC_ERR_UNSUPPORTED, "qec_get_statistics: code has no I-P matrix for the logical check");
    if (nThreads < 1) nThreads = 1;
    const auto t0 = std::chrono::high_resolution_clock::now();
    const long tested = (long)(numErrors / nThreads) * nThreads;  // DecoderCPU.h:426,527
    const long CH = 1 << 16;
    const int n = c.n;
    std::vector<uint8_t> x, z, sx, sz, ex, ez, fl, res(n * 2);
    Mt19937 g(seed);
    std::memset(out, 0, sizeof *out);
    uint64_t withX = 0, withZ = 0, corrected = 0, synX = 0, synZ = 0, logical = 0, convX = 0, convZ = 0;
    for (long base = 0; base < tested; base += CH) {
        const long cnt = std::min(CH, tested - base);
        x.assign((size_t)cnt * n, 0); z.assign((size_t)cnt * n, 0);
        sx.resize((size_t)cnt * c.mX); sz.resize((size_t)cnt * c.mZ);
        ex.resize((size_t)cnt * n); ez.resize((size_t)cnt * n); fl.resize(cnt);
        for (long s = 0; s < cnt; ++s)
            for (int w = 0; w < W; ++w) {
                const uint32_t index = g.msvc_uniform((uint32_t)n);
                const uint32_t type = g.msvc_uniform(3u);
                if (type == 0 || type == 1) x[s * n + index] = 1;
                if (type == 2 || type == 1) z[s * n + index] = 1;
            }
        for (long s = 0; s < cnt; ++s) {
            host_syndrome(c, 0, &x[s * n], &sx[s * c.mX]);
            host_syndrome(c, 1, &z[s * n], &sz[s * c.mZ]);
        }
        int rc = qec_decode_batch(d, sx.data(), sz.data(), cnt, p, maxIter, QEC_STOP_REF, ex.data(), ez.data(),
                                  fl.data(), nullptr, nullptr);
        if (rc) return rc;
        for (long s = 0; s < cnt; ++s) {
            bool ax = false, az = false;
            for (int v = 0; v < n; ++v) { ax |= x[s * n + v] != 0; az |= z[s * n + v] != 0; }
            withX += ax; withZ += az;
            const bool dEX = fl[s] & QEC_SYNDROME_FAIL_X, dEZ = fl[s] & QEC_SYNDROME_FAIL_Z;
            synX += dEX; synZ += dEZ;
            if (!(dEX || dEZ)) {
                for (int v = 0; v < n; ++v) {
                    res[v] = (x[s * n + v] + ex[s * n + v]) % 2;
                    res[n + v] = (z[s * n + v] + ez[s * n + v]) % 2;
                }
                if (host_check_logical(c, res.data(), res.data() + n)) ++logical; else ++corrected;
            }
            convX += (fl[s] & QEC_CONVERGENCE_FAIL_X) != 0;
            convZ += (fl[s] & QEC_CONVERGENCE_FAIL_Z) != 0;
        }
    }
    const auto t1 = std::chrono::high_resolution_clock::now();
    out->randSeed = seed;
    out->numErrorsTested = (uint32_t)tested;
    out->numXErrorsTested = (uint32_t)withX;
    out->numZErrorsTested = (uint32_t)withZ;
    out->errorWeight = (uint32_t)W;
    out->corrected = (uint32_t)corrected;
    out->syndromeErrorsX = (uint32_t)synX;
    out->syndromeErrorsZ = (uint32_t)synZ;
    out->logicalErrors = (uint32_t)logical;
    out->convergenceFailX = (uint32_t)convX;
    out->convergenceFailZ = (uint32_t)convZ;
    out->durationMicroSeconds = std::chrono::duration_cast<std::chrono::microseconds>(t1 - t0).count();
    return QEC_OK;
}

}  // extern "C"
