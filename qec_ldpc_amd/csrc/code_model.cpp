// Host-side code model: the Quantum_LDPC_Code loader, the QC_LDPC_CSS generator,
// circulant extraction, syndromes, the I-P logical check and the reference's
// MSVC-compatible error sampler.  Product code (no oracle dependency).
#include <algorithm>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <sstream>

#include "qec_internal.h"

namespace qec {

namespace {
thread_local std::string g_last_error;

// `stream >> x` until the stream fails (Quantum_LDPC_Code.h:28-41).  Values past
// the matrix size are ignored (the reference would write past its buffer).
void parse_matrix(const std::string& line, std::vector<uint8_t>& dst, size_t cap)
{
    dst.assign(cap, 0);
    const char* p = line.data();
    const char* end = p + line.size();
    size_t idx = 0;
    while (p < end) {
        while (p < end && (*p == ' ' || *p == '\t' || *p == '\r' || *p == '\v' || *p == '\f')) ++p;
        if (p >= end) break;
        bool neg = false;
        if (*p == '-' || *p == '+') { neg = (*p == '-'); ++p; }
        if (p >= end || *p < '0' || *p > '9') break;
        long v = 0;
        while (p < end && *p >= '0' && *p <= '9') v = v * 10 + (*p++ - '0');
        if (idx < cap) dst[idx] = (uint8_t)((neg ? -v : v) != 0);
        ++idx;
    }
}

long pow_mod(long base, long e, long P)
{
    long t = 1;
    for (long i = 0; i < e; ++i) t = (t * base) % P;
    return t;
}
}  // namespace

void set_error(const std::string& msg) { g_last_error = msg; }
int fail(int status, const std::string& msg)
{
    g_last_error = msg;
    return status;
}
const char* last_error_cstr() { return g_last_error.c_str(); }

std::string Code::describe() const
{
    std::ostringstream s;
    s << "[J=" << J << ",K=" << K << ",L=" << L << ",P=" << P << ",s=" << sigma << ",t=" << tau
      << "][[n=" << n << ",k=" << (mZ - mX) << "]]";
    return s.str();
}

// A block is a circulant permutation matrix if row i has its single 1 at column (E + i) mod P.
static bool extract_shifts(const std::vector<uint8_t>& pcm, int R, int L, int P, std::vector<int>& E)
{
    const int n = L * P;
    E.assign((size_t)R * L, 0);
    for (int r = 0; r < R; ++r)
        for (int l = 0; l < L; ++l) {
            int e0 = -1;
            for (int c = 0; c < P; ++c)
                if (pcm[(size_t)(r * P) * n + l * P + c]) {
                    if (e0 >= 0) return false;
                    e0 = c;
                }
            if (e0 < 0) return false;
            for (int i = 0; i < P; ++i)
                for (int c = 0; c < P; ++c) {
                    const bool one = pcm[(size_t)(r * P + i) * n + l * P + c] != 0;
                    if (one != (c == (e0 + i) % P)) return false;
                }
            E[(size_t)r * L + l] = e0;
        }
    return true;
}

void finalize_code(Code& c)
{
    c.n = c.L * c.P;
    c.mX = c.J * c.P;
    c.mZ = c.K * c.P;
    c.is_qc = extract_shifts(c.pcmX, c.J, c.L, c.P, c.EX) && extract_shifts(c.pcmZ, c.K, c.L, c.P, c.EZ);
    if (!c.is_qc) { c.EX.clear(); c.EZ.clear(); }
    c.imp_rows.clear();
    c.imp_words = 0;
    if (!c.imp.empty()) {
        const int N2 = 2 * c.n;
        c.imp_words = (N2 + 63) / 64;
        std::vector<uint64_t> row(c.imp_words);
        for (int i = 0; i < N2; ++i) {
            std::fill(row.begin(), row.end(), 0);
            bool any = false;
            for (int j = 0; j < N2; ++j)
                if (c.imp[(size_t)i * N2 + j]) { row[j >> 6] |= 1ull << (j & 63); any = true; }
            if (any) c.imp_rows.insert(c.imp_rows.end(), row.begin(), row.end());
        }
        // the same test column by column: (I-P) r != 0 iff the XOR of the columns of I-P at the set
        // bits of r, restricted to its non-zero rows, is non-zero.  A decoded residual is almost
        // always 0 or sparse, so the device kernels touch a few columns instead of every row.
        const int nrows = c.imp_words ? (int)(c.imp_rows.size() / c.imp_words) : 0;
        c.imp_col_words = (nrows + 63) / 64;
        c.imp_cols.assign((size_t)N2 * c.imp_col_words, 0);
        int k = 0;
        for (int i = 0; i < N2; ++i) {
            bool any = false;
            for (int j = 0; j < N2 && !any; ++j) any = c.imp[(size_t)i * N2 + j] != 0;
            if (!any) continue;
            for (int j = 0; j < N2; ++j)
                if (c.imp[(size_t)i * N2 + j]) c.imp_cols[(size_t)j * c.imp_col_words + (k >> 6)] |= 1ull << (k & 63);
            ++k;
        }
    }
}

int load_code(const char* path, Code& c)
{
    std::ifstream ifs(path, std::ios::binary);
    if (!ifs.is_open()) return fail(QEC_ERR_IO, std::string("Unable to find code file ") + path);
    std::string params, hc, hd, imp;
    std::getline(ifs, params);
    std::getline(ifs, hc);
    std::getline(ifs, hd);
    std::getline(ifs, imp);
    std::istringstream ps(params);
    if (!(ps >> c.J >> c.K >> c.L >> c.P >> c.sigma >> c.tau))
        return fail(QEC_ERR_FORMAT, std::string("code file has no 'J K L P sigma tau' header: ") + path);
    if (c.J <= 0 || c.K <= 0 || c.L <= 0 || c.P <= 0 || (long)c.L * c.P > (1 << 20))
        return fail(QEC_ERR_FORMAT, "code file header out of range");
    const size_t n = (size_t)c.L * c.P;
    parse_matrix(hc, c.pcmX, (size_t)c.J * c.P * n);
    parse_matrix(hd, c.pcmZ, (size_t)c.K * c.P * n);
    if (!imp.empty()) parse_matrix(imp, c.imp, 4 * n * n);
    else c.imp.clear();
    finalize_code(c);
    return QEC_OK;
}

bool generator_exponents(int J, int K, int L, int P, int sigma, int tau, std::vector<int>& EX, std::vector<int>& EZ)
{
    // sigma^-1: the element of Z_P^* with x*sigma = 1 mod P (QEC_LDPC_CSS.cu:37-39)
    long inv = -1;
    for (long x = 1; x < P; ++x)
        if ((x * sigma) % P == 1) { inv = x; break; }
    if (inv < 0) return false;
    auto spow = [&](long p) { return p < 0 ? pow_mod(inv, -p, P) : pow_mod(sigma, p, P); };
    EX.assign((size_t)J * L, 0);
    EZ.assign((size_t)K * L, 0);
    // HC (QEC_LDPC_CSS.cu:43-65): sigma^(l-j) left half, -(tau sigma^(j-1+l)) right half
    for (int j = 0; j < J; ++j)
        for (int l = 0; l < L; ++l) {
            long t = (l < L / 2) ? spow(l - j) : P - (tau * spow(j - 1 + l)) % P;
            EX[(size_t)j * L + l] = (int)(t % P);
        }
    // HD (QEC_LDPC_CSS.cu:67-90): tau sigma^(l-k-1) left half, -(sigma^(k+l)) right half
    for (int k = 0; k < K; ++k)
        for (int l = 0; l < L; ++l) {
            long t = (l < L / 2) ? (tau * spow(l - k - 1)) % P : P - spow(k + l);
            EZ[(size_t)k * L + l] = (int)(((t % P) + P) % P);
        }
    return true;
}

int generate_code(int J, int K, int L, int P, int sigma, int tau, Code& c)
{
    if (J <= 0 || K <= 0 || L <= 0 || P <= 1 || (long)L * P > (1 << 20))
        return fail(QEC_ERR_ARG, "qec_code_generate: J, K, L must be > 0 and P > 1");
    std::vector<int> EX, EZ;
    if (!generator_exponents(J, K, L, P, sigma, tau, EX, EZ))
        return fail(QEC_ERR_ARG, "qec_code_generate: sigma has no inverse mod P");
    c.J = J; c.K = K; c.L = L; c.P = P; c.sigma = sigma; c.tau = tau;
    const int n = L * P;
    // expand to circulant permutation blocks: col = (E + row % P) % P + l P (QEC_LDPC_CSS.cu:99-131)
    auto expand = [&](const std::vector<int>& E, int R, std::vector<uint8_t>& pcm) {
        pcm.assign((size_t)R * P * n, 0);
        for (int row = 0; row < R * P; ++row)
            for (int l = 0; l < L; ++l)
                pcm[(size_t)row * n + (E[(size_t)(row / P) * L + l] + row % P) % P + l * P] = 1;
    };
    expand(EX, J, c.pcmX);
    expand(EZ, K, c.pcmZ);
    c.imp.clear();
    finalize_code(c);
    return QEC_OK;
}

void host_syndrome(const Code& c, int sector, const uint8_t* e, uint8_t* s)
{
    const int R = sector ? c.K : c.J, P = c.P, L = c.L, n = c.n;
    if (c.is_qc) {
        const std::vector<int>& E = sector ? c.EZ : c.EX;
        for (int r = 0; r < R; ++r)
            for (int i = 0; i < P; ++i) {
                int x = 0;
                for (int l = 0; l < L; ++l) x ^= e[l * P + (E[(size_t)r * L + l] + i) % P] & 1;
                s[r * P + i] = (uint8_t)x;
            }
    } else {
        const std::vector<uint8_t>& H = sector ? c.pcmZ : c.pcmX;
        for (int eq = 0; eq < R * P; ++eq) {
            int x = 0;
            for (int v = 0; v < n; ++v) x += H[(size_t)eq * n + v] * (e[v] & 1);
            s[eq] = (uint8_t)(x % 2);
        }
    }
}

bool host_check_logical(const Code& c, const uint8_t* ex, const uint8_t* ez)
{
    const int W = c.imp_words, n = c.n;
    std::vector<uint64_t> v(W, 0);
    for (int j = 0; j < n; ++j) {
        if (ex[j] & 1) v[j >> 6] |= 1ull << (j & 63);
        if (ez[j] & 1) v[(n + j) >> 6] |= 1ull << ((n + j) & 63);
    }
    const size_t rows = W ? c.imp_rows.size() / W : 0;
    for (size_t r = 0; r < rows; ++r) {
        const uint64_t* row = &c.imp_rows[r * W];
        uint64_t acc = 0;
        for (int w = 0; w < W; ++w) acc ^= row[w] & v[w];
        if (__builtin_popcountll(acc) & 1) return true;
    }
    return false;
}

Mt19937::Mt19937(uint32_t seed)
{
    mt[0] = seed;
    for (int i = 1; i < 624; ++i) mt[i] = 1812433253u * (mt[i - 1] ^ (mt[i - 1] >> 30)) + (uint32_t)i;
    idx = 624;
}

uint32_t Mt19937::next()
{
    if (idx >= 624) {
        for (int i = 0; i < 624; ++i) {
            const uint32_t y = (mt[i] & 0x80000000u) | (mt[(i + 1) % 624] & 0x7fffffffu);
            mt[i] = mt[(i + 397) % 624] ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
        }
        idx = 0;
    }
    uint32_t y = mt[idx++];
    y ^= y >> 11;
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= y >> 18;
    return y;
}

// VS2015 _Rng_from_urng: rejection on [0, 2^32) so that r % N is unbiased.
uint32_t Mt19937::msvc_uniform(uint32_t N)
{
    for (;;) {
        const uint32_t r = next();
        if (r / N < 0xFFFFFFFFu / N || 0xFFFFFFFFu % N == N - 1) return r % N;
    }
}

}  // namespace qec
