// Monte-Carlo caller side on the GPU: what
// DecoderCPU::GetStatistics does around Decode (QEC_LDPC/DecoderCPU.h:392-530),
// batched:
//   * errors: i.i.d. depolarising samples from a counter-based Philox4x32-10 stream
//     (any shard of the sample index space can be generated independently), or the
//     reference's fixed-weight draws (host mt19937 stream, DecoderCPU.h:448-459)
//     expanded on the device;
//   * syndromes: s(r, i) = XOR_l e[l P + (E[r][l] + i) mod P]  (GetSyndromeX/Z,
//     Quantum_LDPC_Code.h:94-124, through the circulant tables);
//   * statistics: residual e ^ e_hat bit-packed with ballots, I-P logical check
//     (Quantum_LDPC_Code.h:126-142) on bit-packed rows, and the CodeStatistics
//     counters (DecoderCPU.h:464-521) reduced per block.
// These are integer/byte kernels: HBM/L2-bound, not worth MFMA.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "qec_internal.h"

namespace qec {

// ---- Philox4x32-10 (Salmon et al., SC'11) -----------------------------------
struct U4 {
    uint32_t x, y, z, w;
};

__host__ __device__ inline U4 philox4x32_10(U4 c, uint32_t k0, uint32_t k1)
{
    for (int r = 0; r < 10; ++r) {
        const uint64_t p0 = (uint64_t)0xD2511F53u * c.x;
        const uint64_t p1 = (uint64_t)0xCD9E8D57u * c.z;
        const uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
        const uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
        c = U4{hi1 ^ c.y ^ k0, lo1, hi0 ^ c.w ^ k1, lo0};
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
    return c;
}

constexpr uint32_t kPhiloxSalt = 0x51EC0DE5u;

// Qubit v of sample b: counter (b_lo, b_hi, v, salt), key (seed_lo, seed_hi).
// word x: hit if x < thr (thr = floor(p 2^32), saturated); word y: type = (y * 3) >> 32,
// 0 = X, 1 = Y, 2 = Z.  Restated in numpy by qec_ldpc_amd/synthetic.py.
__global__ void sample_depolarizing_kernel(uint64_t seed, uint64_t start, long long B, int n, uint64_t thr,
                                           uint8_t* __restrict__ x, uint8_t* __restrict__ z)
{
    const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= B * n) return;
    const long long b = t / n;
    const int v = (int)(t - b * n);
    const uint64_t sb = start + (uint64_t)b;
    const U4 o = philox4x32_10(U4{(uint32_t)sb, (uint32_t)(sb >> 32), (uint32_t)v, kPhiloxSalt}, (uint32_t)seed,
                               (uint32_t)(seed >> 32));
    const bool hit = (uint64_t)o.x < thr;
    const uint32_t type = (uint32_t)(((uint64_t)o.y * 3u) >> 32);
    x[t] = (uint8_t)(hit && type != 2);
    z[t] = (uint8_t)(hit && type != 0);
}

// Reference fixed-weight draws (index, type) -> dense errors (x, z pre-zeroed).
__global__ void errors_from_draws_kernel(const int32_t* __restrict__ idx, const uint8_t* __restrict__ type,
                                         long long B, int W, int n, uint8_t* __restrict__ x, uint8_t* __restrict__ z)
{
    const long long b = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= B) return;
    for (int w = 0; w < W; ++w) {
        const int v = idx[b * W + w];
        const int t = type[b * W + w];
        if (t == 0 || t == 1) x[b * n + v] = 1;  // DecoderCPU.h:456-457
        if (t == 2 || t == 1) z[b * n + v] = 1;
    }
}

struct SynArgs {
    const uint8_t* x;
    const uint8_t* z;
    uint8_t* sX;
    uint8_t* sZ;
    long long B;
    int n, L, P, mX, mZ;
    int EX[128], EZ[128];
};

// one thread per (sample, check) over both sectors
__global__ void syndrome_kernel(const SynArgs a)
{
    const int m = a.mX + a.mZ;
    const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= a.B * m) return;
    const long long b = t / m;
    int c = (int)(t - b * m);
    const bool zs = c >= a.mX;
    if (zs) c -= a.mX;
    const int r = c / a.P, i = c - r * a.P;
    const int* E = zs ? a.EZ : a.EX;
    const uint8_t* e = (zs ? a.z : a.x) + b * a.n;
    uint32_t s = 0;
    for (int l = 0; l < a.L; ++l) {
        int j = E[r * a.L + l] + i;
        j -= (j >= a.P) ? a.P : 0;
        s ^= e[l * a.P + j] & 1u;
    }
    (zs ? a.sZ : a.sX)[b * (zs ? a.mZ : a.mX) + c] = (uint8_t)s;
}

// Any regular code (sparse-graph engine): s(c) = XOR_k e[chkVar[c dc + k]], the check's
// variables from the engine's InitIndexArrays table; one thread per (sample, check).
__global__ void syndrome_csr_kernel(const uint8_t* __restrict__ x, const uint8_t* __restrict__ z,
                                    const int32_t* __restrict__ chkVar, long long B, int n, int mX, int mZ, int dc,
                                    uint8_t* __restrict__ sX, uint8_t* __restrict__ sZ)
{
    const int m = mX + mZ;
    const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= B * m) return;
    const long long b = t / m;
    const int c = (int)(t - b * m);
    const bool zs = c >= mX;
    const uint8_t* e = (zs ? z : x) + b * n;
    const int32_t* vars = chkVar + (size_t)c * dc;
    uint32_t s = 0;
    for (int k = 0; k < dc; ++k) s ^= e[vars[k]] & 1u;
    if (zs) sZ[b * mZ + (c - mX)] = (uint8_t)s; else sX[b * mX + c] = (uint8_t)s;
}

// counters, in qec_mc_counters order
enum { C_WITHX, C_WITHZ, C_SYNX, C_SYNZ, C_LOGICAL, C_CORRECTED, C_CONVX, C_CONVZ, C_N };

// One wave per sample.  Residual words are formed with ballots (lane = qubit within a
// 64-qubit word) and parked in LDS, so every lane can test its share of the non-zero
// I-P rows (bit-packed, imp_words u64 per row) for odd parity against them.
constexpr int kStatWaves = 4;
constexpr int kMaxWords = 64;  // 2n <= 4096 qubits

__global__ __launch_bounds__(64 * kStatWaves) void statistics_kernel(
    const uint8_t* __restrict__ x, const uint8_t* __restrict__ z, const uint8_t* __restrict__ eX,
    const uint8_t* __restrict__ eZ, const uint8_t* __restrict__ flags, long long B, int n,
    const uint64_t* __restrict__ imp_rows, int imp_nrows, int imp_words, unsigned long long* __restrict__ counters)
{
    __shared__ unsigned long long part[C_N];
    __shared__ unsigned long long sres[kStatWaves][kMaxWords];
    if (threadIdx.x < C_N) part[threadIdx.x] = 0;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const long long b = (long long)blockIdx.x * kStatWaves + wv;
    const bool live = b < B;
    const int nw = (2 * n + 63) / 64;
    bool anyX = false, anyZ = false;
    if (live) {
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
            if (lane == 0) sres[wv][w] = word;
        }
    }
    __syncthreads();
    if (live) {
        const uint8_t f = flags[b];
        const bool wx = __any(anyX), wz = __any(anyZ);
        const bool dEX = f & QEC_SYNDROME_FAIL_X, dEZ = f & QEC_SYNDROME_FAIL_Z;
        bool logical = false;
        if (!(dEX || dEZ) && imp_nrows > 0) {  // CheckLogicalError only when no syndrome failure
            bool odd = false;
            for (int row = lane; row < imp_nrows; row += 64) {
                const uint64_t* rp = imp_rows + (size_t)row * imp_words;
                unsigned long long acc = 0;
                for (int w = 0; w < imp_words; ++w) acc ^= rp[w] & sres[wv][w];
                odd |= (__popcll(acc) & 1) != 0;
            }
            logical = __any(odd);
        }
        if (lane == 0) {
            atomicAdd(&part[C_WITHX], (unsigned long long)wx);
            atomicAdd(&part[C_WITHZ], (unsigned long long)wz);
            atomicAdd(&part[C_SYNX], (unsigned long long)dEX);
            atomicAdd(&part[C_SYNZ], (unsigned long long)dEZ);
            if (!(dEX || dEZ)) atomicAdd(&part[logical ? C_LOGICAL : C_CORRECTED], 1ull);
            atomicAdd(&part[C_CONVX], (unsigned long long)((f & QEC_CONVERGENCE_FAIL_X) != 0));
            atomicAdd(&part[C_CONVZ], (unsigned long long)((f & QEC_CONVERGENCE_FAIL_Z) != 0));
        }
    }
    __syncthreads();
    if (threadIdx.x < C_N && part[threadIdx.x]) atomicAdd(&counters[threadIdx.x], part[threadIdx.x]);
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
    const double pd = p;
    const uint64_t thr = pd <= 0.0 ? 0ull : pd >= 1.0 ? (1ull << 32) : (uint64_t)(pd * 4294967296.0);
    const long long tot = B * n;
    hipLaunchKernelGGL(sample_depolarizing_kernel, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, st, seed, start, B,
                       n, thr, x, z);
    return launch_check("sample_depolarizing");
}

int launch_errors_from_draws(const int32_t* idx, const uint8_t* type, long long B, int W, int n, uint8_t* x,
                             uint8_t* z, hipStream_t st)
{
    if (B <= 0) return QEC_OK;
    if (hipMemsetAsync(x, 0, (size_t)B * n, st) != hipSuccess || hipMemsetAsync(z, 0, (size_t)B * n, st) != hipSuccess)
        return fail(QEC_ERR_HIP, "errors_from_draws: memset");
    if (W > 0)
        hipLaunchKernelGGL(errors_from_draws_kernel, dim3((unsigned)((B + 255) / 256)), dim3(256), 0, st, idx, type, B,
                           W, n, x, z);
    return launch_check("errors_from_draws");
}

int launch_syndrome(const Code& c, const int32_t* chkVar, const uint8_t* x, const uint8_t* z, long long B,
                    uint8_t* sX, uint8_t* sZ, hipStream_t st)
{
    if (B <= 0) return QEC_OK;
    if (chkVar != nullptr) {
        const long long tot = B * (c.mX + c.mZ);
        hipLaunchKernelGGL(syndrome_csr_kernel, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, st, x, z, chkVar, B,
                           c.n, c.mX, c.mZ, c.L, sX, sZ);
        return launch_check("syndrome_csr");
    }
    if (!c.is_qc || c.J * c.L > 128 || c.K * c.L > 128) return fail(QEC_ERR_UNSUPPORTED, "syndrome kernel: needs a QC code");
    SynArgs a{};
    a.x = x; a.z = z; a.sX = sX; a.sZ = sZ; a.B = B;
    a.n = c.n; a.L = c.L; a.P = c.P; a.mX = c.mX; a.mZ = c.mZ;
    for (size_t k = 0; k < c.EX.size(); ++k) a.EX[k] = c.EX[k];
    for (size_t k = 0; k < c.EZ.size(); ++k) a.EZ[k] = c.EZ[k];
    const long long tot = B * (c.mX + c.mZ);
    hipLaunchKernelGGL(syndrome_kernel, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, st, a);
    return launch_check("syndrome");
}

int launch_statistics(const Code& c, const uint64_t* imp_dev, const uint8_t* x, const uint8_t* z, const uint8_t* eX,
                      const uint8_t* eZ, const uint8_t* flags, long long B, unsigned long long* counters, hipStream_t st)
{
    if (B <= 0) return QEC_OK;
    if (2 * c.n > 64 * kMaxWords) return fail(QEC_ERR_UNSUPPORTED, "statistics kernel: 2n > 4096");
    const int nrows = c.imp_words ? (int)(c.imp_rows.size() / c.imp_words) : 0;
    hipLaunchKernelGGL(statistics_kernel, dim3((unsigned)((B + kStatWaves - 1) / kStatWaves)), dim3(64 * kStatWaves), 0, st,
                       x, z, eX, eZ, flags, B, c.n, imp_dev, nrows, c.imp_words, counters);
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
