// Quantum_LDPC_Code.h -- C++ face of the code model, same names as
// QEC_LDPC/Quantum_LDPC_Code.h:7-150 (fields J K L P sigma tau n numEqsX numEqsZ,
// pcmX / pcmZ / iMinusP, createFromFile, GetSyndromeX/Z, CheckLogicalError,
// operator<<).  Header-only over the C ABI in qec_ldpc.h; plain C++ (no HIP needed).
#pragma once
#include <cstdint>
#include <memory>
#include <ostream>
#include <string>
#include <vector>

#include "qec_ldpc.h"

#ifndef QEC_INTARRAY1D_DEFINED
#define QEC_INTARRAY1D_DEFINED
typedef std::vector<int> IntArray1d_h;  // cusp::array1d<int, host_memory> in the reference
#endif

// row-major dense int matrix with the cusp::array2d members the reference touches
struct IntArray2d_h {
    int num_rows = 0, num_cols = 0, num_entries = 0;
    std::vector<int> values;
    IntArray2d_h() = default;
    IntArray2d_h(int r, int c) : num_rows(r), num_cols(c), num_entries(r * c), values((size_t)r * c, 0) {}
    int& operator()(int i, int j) { return values[(size_t)i * num_cols + j]; }
    int operator()(int i, int j) const { return values[(size_t)i * num_cols + j]; }
};

class Quantum_LDPC_Code {
public:
    int J, K, L, P, sigma, tau;
    int n;  // number of physical qubits
    int numEqsX, numEqsZ;
    IntArray2d_h pcmX, pcmZ, iMinusP;

    // Quantum_LDPC_Code.h:26-80; throws std::string like the reference (:78)
    static Quantum_LDPC_Code createFromFile(const std::string& file)
    {
        qec_code* h = qec_code_load(file.c_str());
        if (!h) throw std::string(qec_last_error());
        return Quantum_LDPC_Code(h);
    }

    // adopt a handle from qec_code_load / qec_code_generate
    explicit Quantum_LDPC_Code(qec_code* h) : handle_(h, [](qec_code* p) { qec_code_free(p); })
    {
        int v[9];
        qec_code_params(h, v);
        J = v[0]; K = v[1]; L = v[2]; P = v[3]; sigma = v[4]; tau = v[5]; n = v[6]; numEqsX = v[7]; numEqsZ = v[8];
        pcmX = dense(0, numEqsX);
        pcmZ = dense(1, numEqsZ);
    }

    // Quantum_LDPC_Code.h:94-124
    IntArray1d_h GetSyndromeX(const IntArray1d_h& errors) const { return syndrome(0, errors, numEqsX); }
    IntArray1d_h GetSyndromeZ(const IntArray1d_h& errors) const { return syndrome(1, errors, numEqsZ); }

    // Quantum_LDPC_Code.h:126-142: errors = {x_1..x_n, z_1..z_n}
    bool CheckLogicalError(const IntArray1d_h& errors) const
    {
        std::vector<uint8_t> ex(n), ez(n);
        for (int i = 0; i < n; ++i) { ex[i] = (uint8_t)(errors[i] & 1); ez[i] = (uint8_t)(errors[n + i] & 1); }
        uint8_t out = 0;
        if (qec_code_check_logical(handle_.get(), ex.data(), ez.data(), 1, &out) != QEC_OK)
            throw std::string(qec_last_error());
        return out != 0;
    }

    const qec_code* handle() const { return handle_.get(); }

private:
    std::shared_ptr<qec_code> handle_;

    IntArray2d_h dense(int sector, int m) const
    {
        IntArray2d_h a(m, n);
        std::vector<uint8_t> buf((size_t)m * n);
        qec_code_pcm(handle_.get(), sector, buf.data());
        for (size_t k = 0; k < buf.size(); ++k) a.values[k] = buf[k];
        return a;
    }
    IntArray1d_h syndrome(int sector, const IntArray1d_h& errors, int m) const
    {
        std::vector<uint8_t> e(n), s(m);
        for (int i = 0; i < n; ++i) e[i] = (uint8_t)(errors[i] & 1);
        qec_code_syndrome(handle_.get(), sector, e.data(), 1, s.data());
        return IntArray1d_h(s.begin(), s.end());
    }
};

// Quantum_LDPC_Code.h:145-150
inline std::ostream& operator<<(std::ostream& stream, const Quantum_LDPC_Code& code)
{
    stream << "[J=" << code.J << ",K=" << code.K << ",L=" << code.L << ",P=" << code.P << ",s=" << code.sigma
           << ",t=" << code.tau << "][[n=" << code.n << ",k=" << code.numEqsZ - code.numEqsX << "]]";
    return stream;
}
