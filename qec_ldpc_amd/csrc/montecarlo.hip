// Monte-Carlo caller side on the GPU: what
// DecoderCPU::GetStatistics does around Decode (QEC_LDPC/DecoderCPU.h:392-530),
// batched:
//   * errors: i.i.d. depolarising samples from a counter-based Philox4x32-10 stream
//     (any shard of the sample index space can be generated independently), or the
//     reference's fixed-weight draws (host mt19937 stream, DecoderCPU.h:448-459)
//     expanded on the device;
//   * syndromes: s(r, i) = XOR_l e[l P + (E[r][l] + i) mod P]  (GetSyndromeX/Z,
//     Quantum_LDPC_Code.h:94-124, through the circulant tables), fused with the errors
//     (mc_errors_syndrome_kernel: one wave per sample, errors staged in LDS);
//   * statistics: residual e ^ e_hat bit-packed, I-P logical check
//     (Quantum_LDPC_Code.h:126-142) on bit-packed rows, and the CodeStatistics
//     counters (DecoderCPU.h:464-521) reduced per block.
// These are integer/byte kernels: HBM/L2-bound, not worth MFMA.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "qec_device.h"
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

// ---- fused Monte-Carlo front end ----------------------------------------------------
// One wave per sample, errors staged in LDS (this wave's x and z rows, each zero-padded to
// npad = 8 nb bytes):
//   source PHILOX: the depolarising sampler above, qubit by qubit (nothing read from HBM);
//   source DRAWS:  the reference's W (index, type) draws of the sample (DecoderCPU.h:452-457);
//   source BYTES:  x, z rows [B][n] from HBM.
// Then, from LDS: the syndromes sX, sZ (QC: s(r, i) = XOR_l e[l P + (E[r][l] + i) mod P]; any other
// regular code: the check's variables from the sparse engine's table), and the bit-packed errors
// errp [B][2 nb] in the decision-record layout (x bits, then z bits) for the statistics kernel.
// HBM traffic per P61 sample: 549 B of syndromes + 154 B of packed errors written.
constexpr int kMcWaves = 4;

struct McArgs {
    // sources
    uint64_t seed, start, thr;                 // PHILOX
    const int32_t* idx;                        // DRAWS: [B][W] qubit indices
    const uint8_t* type;                       //        [B][W] 0 = X, 1 = Y, 2 = Z
    int W;
    const uint8_t* x;                          // BYTES: [B][n]
    const uint8_t* z;
    // outputs
    uint8_t* sX;                               // [B][mX]
    uint8_t* sZ;                               // [B][mZ]
    uint8_t* errp;                             // [B][2 nb] (nullable)
    const int32_t* chkVar;                     // non-QC codes: [(mX + mZ) L] variables per check
    long long B;
    int n, nb, L, P, mX, mZ;
    int EX[128], EZ[128];
};

template <int SRC>
__global__ __launch_bounds__(64 * kMcWaves) void mc_errors_syndrome_kernel(const McArgs a)
{
    extern __shared__ __attribute__((aligned(8))) uint8_t mc_smem[];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const long long b = (long long)blockIdx.x * kMcWaves + wv;
    if (b >= a.B) return;  // wave-local from here on: no workgroup barrier
    const int n = a.n, npad = 8 * a.nb;
    uint8_t* __restrict__ ex = mc_smem + (size_t)wv * 2 * npad;
    uint8_t* __restrict__ ez = ex + npad;
    if constexpr (SRC == MC_SRC_DRAWS) {
        for (int v = lane; v < npad; v += 64) { ex[v] = 0; ez[v] = 0; }
        wave_sync();
        for (int w = lane; w < a.W; w += 64) {
            const int v = a.idx[b * a.W + w];
            const int t = a.type[b * a.W + w];
            if (t == 0 || t == 1) ex[v] = 1;  // several draws may hit one qubit: they all store 1
            if (t == 2 || t == 1) ez[v] = 1;
        }
    } else {
        for (int v = lane; v < npad; v += 64) {
            uint8_t xv = 0, zv = 0;
            if (v < n) {
                if constexpr (SRC == MC_SRC_PHILOX) {
                    const uint64_t sb = a.start + (uint64_t)b;
                    const U4 o = philox4x32_10(U4{(uint32_t)sb, (uint32_t)(sb >> 32), (uint32_t)v, kPhiloxSalt},
                                               (uint32_t)a.seed, (uint32_t)(a.seed >> 32));
                    const bool hit = (uint64_t)o.x < a.thr;
                    const uint32_t type = (uint32_t)(((uint64_t)o.y * 3u) >> 32);
                    xv = (uint8_t)(hit && type != 2);
                    zv = (uint8_t)(hit && type != 0);
                } else {
                    xv = a.x[b * n + v] & 1u;
                    zv = a.z[b * n + v] & 1u;
                }
            }
            ex[v] = xv;
            ez[v] = zv;
        }
    }
    wave_sync();
    const int m = a.mX + a.mZ;
    for (int c = lane; c < m; c += 64) {
        const bool zs = c >= a.mX;
        const int cc = zs ? c - a.mX : c;
        const uint8_t* e = zs ? ez : ex;
        uint32_t s = 0;
        if (a.chkVar != nullptr) {
            const int32_t* vars = a.chkVar + (size_t)c * a.L;
            for (int k = 0; k < a.L; ++k) s ^= e[vars[k]];
        } else {
            const int r = cc / a.P, i = cc - r * a.P;
            const int* E = zs ? a.EZ : a.EX;
            for (int l = 0; l < a.L; ++l) {
                int j = E[r * a.L + l] + i;
                j -= (j >= a.P) ? a.P : 0;
                s ^= e[l * a.P + j];
            }
        }
        (zs ? a.sZ + b * a.mZ : a.sX + b * a.mX)[cc] = (uint8_t)(s & 1u);
    }
    if (a.errp != nullptr) {
        for (int t = lane; t < 2 * a.nb; t += 64) {
            const int k = t < a.nb ? t : t - a.nb;
            const uint8_t* e = t < a.nb ? ex : ez;
            a.errp[b * 2 * a.nb + t] = (uint8_t)pack8(*reinterpret_cast<const uint64_t*>(e + 8 * k));
        }
    }
}

// CodeStatistics counters of a batch from bit-packed errors errp [B][2 nb] and decision records
// rec [B][2 nb + 1] (qec_decode_batch_packed_dev): the residual [x ^ eX | z ^ eZ] is their XOR
// over the first 2 nb bytes, tested against the I-P rows packed in the same layout
// (Code::imp_rows_rec); optional iteration sums (iters [B][2]) into counters[8], counters[9].
// One wave per sample; counters as statistics_kernel (DecoderCPU.h:464-521).
constexpr int kMaxRecWords = 80;  // 2 nb <= 640 bytes

__global__ __launch_bounds__(64 * kStatWaves) void statistics_packed_kernel(
    const uint8_t* __restrict__ errp, const uint8_t* __restrict__ rec, const int32_t* __restrict__ iters, long long B,
    int nb, const uint64_t* __restrict__ imp_rows, int imp_nrows, int imp_words, unsigned long long* __restrict__ counters)
{
    __shared__ unsigned long long part[C_N + 2];
    __shared__ __attribute__((aligned(8))) uint8_t sres[kStatWaves][8 * kMaxRecWords];
    if (threadIdx.x < C_N + 2) part[threadIdx.x] = 0;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const long long b = (long long)blockIdx.x * kStatWaves + wv;
    const bool live = b < B;
    const int recB = 2 * nb + 1;
    bool anyX = false, anyZ = false;
    if (live) {
        for (int t = lane; t < 8 * imp_words; t += 64) {
            uint8_t r = 0;
            if (t < 2 * nb) {
                const uint8_t e = errp[b * 2 * nb + t];
                if (t < nb) anyX |= e != 0; else anyZ |= e != 0;
                r = e ^ rec[b * recB + t];
            }
            sres[wv][t] = r;
        }
    }
    __syncthreads();
    if (live) {
        const uint8_t f = rec[b * recB + 2 * nb];
        const bool wx = __any(anyX), wz = __any(anyZ);
        const bool dEX = f & QEC_SYNDROME_FAIL_X, dEZ = f & QEC_SYNDROME_FAIL_Z;
        bool logical = false;
        if (!(dEX || dEZ) && imp_nrows > 0) {  // CheckLogicalError only when no syndrome failure
            const uint64_t* res = reinterpret_cast<const uint64_t*>(sres[wv]);
            bool odd = false;
            for (int row = lane; row < imp_nrows; row += 64) {
                const uint64_t* rp = imp_rows + (size_t)row * imp_words;
                unsigned long long acc = 0;
                for (int w = 0; w < imp_words; ++w) acc ^= rp[w] & res[w];
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
            if (iters != nullptr) {
                atomicAdd(&part[C_N], (unsigned long long)iters[2 * b]);
                atomicAdd(&part[C_N + 1], (unsigned long long)iters[2 * b + 1]);
            }
        }
    }
    __syncthreads();
    const int nc = iters != nullptr ? C_N + 2 : C_N;
    if (threadIdx.x < nc && part[threadIdx.x]) atomicAdd(&counters[threadIdx.x], part[threadIdx.x]);
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

int launch_mc_errors_syndrome(int src, const McArgsHost& h, hipStream_t st)
{
    if (h.B <= 0) return QEC_OK;
    const Code& c = *h.code;
    McArgs a{};
    a.seed = h.seed; a.start = h.start;
    const double pd = h.p;
    a.thr = pd <= 0.0 ? 0ull : pd >= 1.0 ? (1ull << 32) : (uint64_t)(pd * 4294967296.0);
    a.idx = h.idx; a.type = h.type; a.W = h.W;
    a.x = h.x; a.z = h.z;
    a.sX = h.sX; a.sZ = h.sZ; a.errp = h.errp;
    a.chkVar = h.chkVar;
    a.B = h.B;
    a.n = c.n; a.nb = (c.n + 7) / 8; a.L = c.L; a.P = c.P; a.mX = c.mX; a.mZ = c.mZ;
    if (a.chkVar == nullptr) {
        if (!c.is_qc || c.J * c.L > 128 || c.K * c.L > 128) return fail(QEC_ERR_UNSUPPORTED, "mc front end: needs a QC code or a check table");
        for (size_t k = 0; k < c.EX.size(); ++k) a.EX[k] = c.EX[k];
        for (size_t k = 0; k < c.EZ.size(); ++k) a.EZ[k] = c.EZ[k];
    }
    const size_t smem = (size_t)kMcWaves * 2 * 8 * a.nb;
    if (smem > 64 * 1024) return fail(QEC_ERR_UNSUPPORTED, "mc front end: code too long for the LDS stage");
    const dim3 grid((unsigned)((h.B + kMcWaves - 1) / kMcWaves)), block(64 * kMcWaves);
    if (src == MC_SRC_PHILOX)
        hipLaunchKernelGGL(mc_errors_syndrome_kernel<MC_SRC_PHILOX>, grid, block, smem, st, a);
    else if (src == MC_SRC_DRAWS)
        hipLaunchKernelGGL(mc_errors_syndrome_kernel<MC_SRC_DRAWS>, grid, block, smem, st, a);
    else
        hipLaunchKernelGGL(mc_errors_syndrome_kernel<MC_SRC_BYTES>, grid, block, smem, st, a);
    return launch_check("mc_errors_syndrome");
}

int launch_statistics_packed(const Code& c, const uint64_t* imp_rec_dev, const uint8_t* errp, const uint8_t* rec,
                             const int32_t* iters, long long B, unsigned long long* counters, hipStream_t st)
{
    if (B <= 0) return QEC_OK;
    if (c.imp_words_rec > kMaxRecWords) return fail(QEC_ERR_UNSUPPORTED, "packed statistics kernel: 2 ceil(n/8) > 640");
    const int nrows = c.imp_words_rec ? (int)(c.imp_rows_rec.size() / c.imp_words_rec) : 0;
    hipLaunchKernelGGL(statistics_packed_kernel, dim3((unsigned)((B + kStatWaves - 1) / kStatWaves)), dim3(64 * kStatWaves),
                       0, st, errp, rec, iters, B, (c.n + 7) / 8, imp_rec_dev, nrows, c.imp_words_rec, counters);
    return launch_check("statistics_packed");
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
