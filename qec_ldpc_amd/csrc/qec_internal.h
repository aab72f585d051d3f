// Internal declarations shared by the libqecldpc translation units.
// Not part of the public interface (that is include/qec_ldpc.h).
#pragma once
#include <cstdint>
#include <string>
#include <vector>

#include "../../include/qec_ldpc.h"

namespace qec {

// BpArgs::hardPaths bits (from QEC_OPT_HARD_PATHS / QEC_OPT_CYCLE_JUMP)
enum { QEC_HP_FORMS = 1, QEC_HP_CYCLE = 2, QEC_HP_PHASE = 4 /* launch the instrumented kernel */ };
// dispatch-order method (schedule.hip, launch_schedule): the global counting sort, the one-launch
// chunk-local order or the global sort in one launch with a software grid barrier (both measured
// slower; experiments)
enum { QEC_ORDER_GLOBAL = 0, QEC_ORDER_LOCAL = 1, QEC_ORDER_ONE_LAUNCH = 2 };

// Thread-local last-error text behind qec_last_error().
void set_error(const std::string& msg);
int fail(int status, const std::string& msg);

// Quantum_LDPC_Code (QEC_LDPC/Quantum_LDPC_Code.h:7-150) in circulant form.
// The dense pcmX/pcmZ/iMinusP of the reference are kept for API parity; the
// decoder itself only needs the exponent tables (one shift per P x P block).
struct Code {
    int J = 0, K = 0, L = 0, P = 0, sigma = 0, tau = 0;
    int n = 0, mX = 0, mZ = 0;
    std::vector<uint8_t> pcmX, pcmZ;   // m x n dense, as read / generated
    std::vector<uint8_t> imp;          // 2n x 2n dense I-P (empty for generated codes)
    bool is_qc = false;                // every block a circulant permutation matrix
    std::vector<int> EX, EZ;           // J x L / K x L shifts in [0, P): row i -> col (E + i) mod P
    // Bit-packed I-P rows that are not all-zero (for CheckLogicalError).
    int imp_words = 0;                 // u64 words per packed 2n-bit row
    std::vector<uint64_t> imp_rows;    // nnz_rows x imp_words
    // Columns of I-P over its non-zero rows (2n x imp_col_words, bit k = k-th non-zero row): the
    // device statistics kernels XOR the columns at the residual's set bits.
    int imp_col_words = 0;
    std::vector<uint64_t> imp_cols;
    std::string describe() const;      // operator<< of Quantum_LDPC_Code.h:145-150
};

int load_code(const char* path, Code& out);
int generate_code(int J, int K, int L, int P, int sigma, int tau, Code& out);
// Generator exponent tables (QEC_LDPC/QEC_LDPC_CSS.cu:37-90); returns false if sigma has no inverse.
bool generator_exponents(int J, int K, int L, int P, int sigma, int tau, std::vector<int>& EX, std::vector<int>& EZ);
void finalize_code(Code& c);  // derive circulant tables + packed I-P from the dense matrices

// Host syndrome s = H e mod 2 via the circulant tables (or dense if not QC).
void host_syndrome(const Code& c, int sector, const uint8_t* e, uint8_t* s);
// CheckLogicalError (Quantum_LDPC_Code.h:126-142) on [ex | ez].
bool host_check_logical(const Code& c, const uint8_t* ex, const uint8_t* ez);

// std::mt19937 + VS2015 uniform_int_distribution, the
// stream the reference's published seeds were drawn from.
struct Mt19937 {
    uint32_t mt[624];
    int idx;
    explicit Mt19937(uint32_t seed);
    uint32_t next();
    uint32_t msvc_uniform(uint32_t N);  // uniform_int_distribution<int>(0, N-1)
};

// Host description of a fused Monte-Carlo front-end launch (montecarlo.hip,
// mc_errors_syndrome_kernel, or mc_gap_kernel for PHILOX): error source (MC_SRC_*), syndromes out,
// packed errors out.
enum { MC_SRC_PHILOX = 0, MC_SRC_DRAWS = 1, MC_SRC_BYTES = 2 };
// the fused low-p Monte-Carlo pipeline's stages (triage.hip, launch_mc_fused)
enum { MC_FUSED_SAMPLE = 0, MC_FUSED_SURVIVORS = 1 };
struct McArgsHost {
    const Code* code = nullptr;
    uint64_t seed = 0, start = 0;
    float p = 0.0f;                 // PHILOX
    const int32_t* idx = nullptr;   // DRAWS
    const uint8_t* type = nullptr;
    int W = 0;
    const uint8_t* x = nullptr;     // BYTES
    const uint8_t* z = nullptr;
    uint8_t* sX = nullptr;
    uint8_t* sZ = nullptr;
    uint32_t* sXp = nullptr;        // PHILOX only: syndromes as bit rows [B][ceil(mX/32)] words instead
    uint32_t* sZp = nullptr;
    uint8_t* errp = nullptr;        // [B][2 ceil(n/8)], nullable
    bool errp_words = false;        // PHILOX only: errp rows padded to whole words (4 ceil(2 ceil(n/8) / 4) B)
    const int32_t* chkVar = nullptr;  // non-QC codes: check -> variables (BYTES, DRAWS)
    const int32_t* varEdge = nullptr; // non-QC codes: variable -> edges (PHILOX, the gap walk)
    long long B = 0;
};

}  // namespace qec
