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
