// Decoder.h -- the reference's abstract decoder interface (QEC_LDPC/Decoder.h:7-48):
// a by-value copy of the code, the ErrorCode bit flags and their operators,
// Decode() and the two GetStatistics overloads.
#pragma once
#include "CodeStatistics.h"
#include "Quantum_LDPC_Code.h"

class Decoder {
protected:
    Quantum_LDPC_Code _code;

public:
    enum ErrorCode {
        SUCCESS = QEC_SUCCESS,
        SYNDROME_FAIL_X = QEC_SYNDROME_FAIL_X,
        SYNDROME_FAIL_Z = QEC_SYNDROME_FAIL_Z,
        SYNDROME_FAIL_XZ = QEC_SYNDROME_FAIL_XZ,
        CONVERGENCE_FAIL_X = QEC_CONVERGENCE_FAIL_X,
        CONVERGENCE_FAIL_Z = QEC_CONVERGENCE_FAIL_Z,
        CONVERGENCE_FAIL_XZ = QEC_CONVERGENCE_FAIL_XZ
    };

    friend inline ErrorCode operator|(const ErrorCode& a, const ErrorCode& b)
    {
        return static_cast<ErrorCode>(static_cast<int>(a) | static_cast<int>(b));
    }
    friend inline ErrorCode operator&(const ErrorCode& a, const ErrorCode& b)
    {
        return static_cast<ErrorCode>(static_cast<int>(a) & static_cast<int>(b));
    }

    explicit Decoder(Quantum_LDPC_Code code) : _code(code) {}

protected:
    // int syndrome entries to the C ABI's bytes keeping the reference's two readings of an entry:
    // its truthiness in the check update (DecoderCPU.h:178) and its exact value in the syndrome
    // comparison (:381) -- 0 -> 0, 1 -> 1, anything else -> 2 (decodes as 1, never matches).
    static std::vector<uint8_t> syndrome_bytes(const IntArray1d_h& s)
    {
        std::vector<uint8_t> out(s.size());
        for (size_t k = 0; k < s.size(); ++k) out[k] = s[k] == 0 ? 0 : s[k] == 1 ? 1 : 2;
        return out;
    }

public:
    virtual ~Decoder() {}

    virtual ErrorCode Decode(const IntArray1d_h& syndromeX, const IntArray1d_h& syndromeZ, float errorProbability,
                             int maxIterations, IntArray1d_h& outErrorsX, IntArray1d_h& outErrorsZ)
    {
        return SUCCESS;
    }
    virtual CodeStatistics GetStatistics(int errorWeight, int numErrors, float errorProbability, int maxIterations) = 0;
    virtual CodeStatistics GetStatistics(int errorWeight, int numErrors, float errorProbability, int maxIterations,
                                         unsigned int seed) = 0;
};
